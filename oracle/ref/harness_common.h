// oracle/ref/harness_common.h -- TEST INFRASTRUCTURE ONLY.
//
// Shared by the two harness drivers that link the reference renderer's own objects
// (see Makefile).  Provides:
//   * the keyed per-pixel RNG that replaces glibc rand() (link-time --wrap=rand), so that the
//     reference becomes deterministic and thread-count independent.  The SAME generator is
//     restated in oracle/restate/rrt_oracle.c and in the HIP kernel
//     (relativistic-ray-tracer_amd/csrc/rrt_rng.h); tests/test_rng.py checks all three agree.
//   * a "scripted" rand mode for function-level known-answer vectors (ref_kat).
//   * a tiny .npy writer for the dumps.
//
// Reference behaviour replaced: random_util.h:11-20 draws `std::rand()/RAND_MAX` from one
// shared, never-seeded glibc stream (non-deterministic under -t > 1).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace harness {

// ---- keyed RNG: splitmix64 finaliser over (seed, x, y) and a per-pixel draw counter ----
static inline uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27; z *= 0x94D049BB133111EBULL;
  z ^= z >> 31; return z;
}
static inline uint64_t pixel_key(uint64_t seed, uint32_t x, uint32_t y) {
  return mix64((((uint64_t)y << 32) | (uint64_t)x) ^ mix64(seed + 0x9E3779B97F4A7C15ULL));
}
// n-th draw of a pixel, in [0, 2^31 - 1] == [0, RAND_MAX] on glibc.
static inline int keyed_rand(uint64_t key, uint32_t n) {
  return (int)(mix64(key + (uint64_t)(n + 1) * 0x9E3779B97F4A7C15ULL) >> 33);
}

enum RandMode { RAND_UNKEYED = 0, RAND_KEYED = 1, RAND_SCRIPTED = 2 };

struct ThreadRng {
  int mode = RAND_UNKEYED;
  uint64_t key = 0;
  uint32_t ctr = 0;
  const int* script = nullptr;  // RAND_SCRIPTED: values returned in order
  size_t script_len = 0;
  // per-query work counters (wrapped reference functions bump these)
  uint64_t bbox_tests = 0, micro_steps = 0, capture_tests = 0;
};
extern thread_local ThreadRng g_rng;

// ---- .npy writer (little-endian, C order) ----
inline void write_npy(const std::string& path, const char* descr, const std::vector<size_t>& shape,
                      const void* data, size_t nbytes) {
  std::string shp = "(";
  for (size_t i = 0; i < shape.size(); ++i) {
    shp += std::to_string(shape[i]);
    if (shape.size() == 1 || i + 1 < shape.size()) shp += ",";
    if (i + 1 < shape.size()) shp += " ";
  }
  shp += ")";
  std::string hdr = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': " + shp + ", }";
  size_t total = 10 + hdr.size() + 1;
  size_t pad = (64 - total % 64) % 64;
  hdr += std::string(pad, ' ');
  hdr += '\n';
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) { std::perror(path.c_str()); std::exit(2); }
  const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
  std::fwrite(magic, 1, 8, f);
  uint16_t hl = (uint16_t)hdr.size();
  std::fwrite(&hl, 2, 1, f);
  std::fwrite(hdr.data(), 1, hdr.size(), f);
  std::fwrite(data, 1, nbytes, f);
  std::fclose(f);
}

}  // namespace harness
