// rrt_rng.h -- keyed per-pixel random stream (host + device).
//
// Replaces the reference's shared, never-seeded glibc stream (random_util.h:11-20:
// `std::rand() / RAND_MAX`, one global state for all worker threads) by a counter-based
// generator keyed on (seed, x, y): draw n of pixel (x, y) is a pure function, so results do not
// depend on thread / wave / GPU schedule.  The oracle harness links the same generator into the
// reference (oracle/ref/harness_common.h), which is what makes per-pixel parity checkable.
// Values lie in [0, 2^31 - 1] = [0, RAND_MAX] so `random_uniform()` keeps its closed [0, 1].
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define RRT_HD __host__ __device__ __forceinline__
#else
#define RRT_HD static inline
#endif

RRT_HD uint64_t rrt_mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27; z *= 0x94D049BB133111EBULL;
  z ^= z >> 31; return z;
}
RRT_HD uint64_t rrt_pixel_key(uint64_t seed, uint32_t x, uint32_t y) {
  return rrt_mix64((((uint64_t)y << 32) | (uint64_t)x) ^ rrt_mix64(seed + 0x9E3779B97F4A7C15ULL));
}
RRT_HD int rrt_keyed_rand(uint64_t key, uint32_t n) {
  return (int)(rrt_mix64(key + (uint64_t)(n + 1) * 0x9E3779B97F4A7C15ULL) >> 33);
}
