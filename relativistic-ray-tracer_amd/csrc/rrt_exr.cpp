// rrt_exr.cpp -- OpenEXR scanline files for the environment map (`-e`, main.cpp:42-79).
// Reader: single-part scanline images, NO_COMPRESSION, HALF or FLOAT channels; writer: the same
// with three FLOAT channels B, G, R (the order EXR files list them in).  Channel mapping follows
// main.cpp:69-75 exactly: R, G, B are the file's channels 2, 1, 0 (whatever their names), so the
// texels equal what the reference's tinyexr path hands to HDRImageBuffer.  Host-only C++.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rrt.h"

namespace {

float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  uint32_t bits;
  if (e == 0) {
    if (m == 0) bits = s;
    else {  // subnormal half -> normal float
      int ee = -1;
      uint32_t mm = m;
      do { ++ee; mm <<= 1; } while (!(mm & 0x400));
      bits = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
    }
  } else if (e == 31) {
    bits = s | 0x7f800000u | (m << 13);
  } else {
    bits = s | ((e - 15 + 127) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

struct Reader {
  const std::vector<unsigned char>& b;
  size_t p = 0;
  bool ok = true;
  explicit Reader(const std::vector<unsigned char>& buf) : b(buf) {}
  bool need(size_t n) { if (p + n > b.size()) ok = false; return ok; }
  template <class T> T get() { T v{}; if (need(sizeof(T))) { std::memcpy(&v, &b[p], sizeof(T)); p += sizeof(T); } return v; }
  std::string str() {
    std::string s;
    while (ok && p < b.size() && b[p]) s += (char)b[p++];
    if (p >= b.size()) ok = false; else ++p;
    return s;
  }
};

struct Channel { std::string name; int32_t type; };

}  // namespace

extern "C" int rrt_exr_load(const char* path, float** texels_out, uint32_t* w_out, uint32_t* h_out) {
  if (!path || !texels_out || !w_out || !h_out) return RRT_E_INVALID;
  *texels_out = nullptr;
  FILE* f = std::fopen(path, "rb");
  if (!f) return RRT_E_IO;
  std::vector<unsigned char> buf;
  {
    unsigned char tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    std::fclose(f);
  }
  Reader r(buf);
  if (r.get<uint32_t>() != 20000630u) return RRT_E_INVALID;  // 0x76, 0x2f, 0x31, 0x01
  const uint32_t version = r.get<uint32_t>();
  if ((version & 0xff) != 2 || (version & ~0xffu) != 0) return RRT_E_INVALID;  // single-part scanline only
  std::vector<Channel> ch;
  int32_t dw[4] = {0, 0, -1, -1};
  int compression = -1, line_order = 0;
  for (;;) {
    std::string name = r.str();
    if (!r.ok) return RRT_E_INVALID;
    if (name.empty()) break;
    std::string type = r.str();
    const int32_t size = r.get<int32_t>();
    if (!r.ok || size < 0 || !r.need((size_t)size)) return RRT_E_INVALID;
    const size_t end = r.p + (size_t)size;
    if (name == "channels" && type == "chlist") {
      for (;;) {
        std::string cn = r.str();
        if (cn.empty() || !r.ok) break;
        Channel c{cn, r.get<int32_t>()};
        r.get<uint8_t>(); r.get<uint8_t>(); r.get<uint8_t>(); r.get<uint8_t>();
        const int32_t xs = r.get<int32_t>(), ys = r.get<int32_t>();
        if (xs != 1 || ys != 1) return RRT_E_INVALID;
        ch.push_back(c);
      }
    } else if (name == "compression") {
      compression = r.get<uint8_t>();
    } else if (name == "dataWindow" && type == "box2i") {
      for (int k = 0; k < 4; ++k) dw[k] = r.get<int32_t>();
    } else if (name == "lineOrder") {
      line_order = r.get<uint8_t>();
    }
    r.p = end;
  }
  if (compression != 0 || ch.size() < 3 || line_order > 1) return RRT_E_INVALID;
  const int64_t W = (int64_t)dw[2] - dw[0] + 1, H = (int64_t)dw[3] - dw[1] + 1;
  if (W <= 0 || H <= 0 || W * H > (int64_t)1 << 28) return RRT_E_INVALID;
  size_t row_bytes = 0;
  for (const Channel& c : ch) {
    if (c.type != 1 && c.type != 2) return RRT_E_INVALID;  // HALF / FLOAT only
    row_bytes += (size_t)W * (c.type == 1 ? 2 : 4);
  }
  std::vector<uint64_t> offsets((size_t)H);
  for (auto& o : offsets) o = r.get<uint64_t>();
  if (!r.ok) return RRT_E_INVALID;
  std::vector<std::vector<float>> plane(ch.size(), std::vector<float>((size_t)(W * H)));
  for (int64_t k = 0; k < H; ++k) {
    r.p = (size_t)offsets[(size_t)k];
    const int32_t y = r.get<int32_t>();
    const int32_t n = r.get<int32_t>();
    if (!r.ok || (size_t)n != row_bytes || y < dw[1] || y > dw[3] || !r.need(row_bytes)) return RRT_E_INVALID;
    const size_t row = (size_t)(y - dw[1]);
    for (size_t c = 0; c < ch.size(); ++c) {
      float* dst = &plane[c][row * (size_t)W];
      for (int64_t x = 0; x < W; ++x) {
        if (ch[c].type == 1) dst[x] = half_to_float(r.get<uint16_t>());
        else dst[x] = r.get<float>();
      }
    }
  }
  float* out = (float*)std::malloc(sizeof(float) * 3 * (size_t)(W * H));
  if (!out) return RRT_E_IO;
  for (size_t i = 0; i < (size_t)(W * H); ++i) {  // main.cpp:69-75: r = images[2], g = [1], b = [0]
    out[3 * i] = plane[2][i];
    out[3 * i + 1] = plane[1][i];
    out[3 * i + 2] = plane[0][i];
  }
  *texels_out = out;
  *w_out = (uint32_t)W;
  *h_out = (uint32_t)H;
  return RRT_OK;
}

extern "C" void rrt_exr_free(float* texels) { std::free(texels); }

extern "C" int rrt_exr_save(const char* path, const float* rgb, uint32_t w, uint32_t h) {
  if (!path || !rgb || !w || !h) return RRT_E_INVALID;
  std::vector<unsigned char> b;
  auto put = [&](const void* p, size_t n) { b.insert(b.end(), (const unsigned char*)p, (const unsigned char*)p + n); };
  auto u32 = [&](uint32_t v) { put(&v, 4); };
  auto i32 = [&](int32_t v) { put(&v, 4); };
  auto cstr = [&](const char* s) { put(s, std::strlen(s) + 1); };
  auto attr = [&](const char* name, const char* type, const std::vector<unsigned char>& v) {
    cstr(name); cstr(type); i32((int32_t)v.size()); put(v.data(), v.size());
  };
  u32(20000630u);
  u32(2u);
  {
    std::vector<unsigned char> v;
    for (const char* n : {"B", "G", "R"}) {
      v.insert(v.end(), n, n + 2);
      const int32_t t = 2;  // FLOAT
      v.insert(v.end(), (const unsigned char*)&t, (const unsigned char*)&t + 4);
      for (int k = 0; k < 4; ++k) v.push_back(0);
      const int32_t one = 1;
      for (int k = 0; k < 2; ++k) v.insert(v.end(), (const unsigned char*)&one, (const unsigned char*)&one + 4);
    }
    v.push_back(0);
    attr("channels", "chlist", v);
  }
  attr("compression", "compression", {0});
  std::vector<unsigned char> box(16);
  const int32_t bx[4] = {0, 0, (int32_t)w - 1, (int32_t)h - 1};
  std::memcpy(box.data(), bx, 16);
  attr("dataWindow", "box2i", box);
  attr("displayWindow", "box2i", box);
  attr("lineOrder", "lineOrder", {0});
  {
    const float par = 1.0f;
    std::vector<unsigned char> v((const unsigned char*)&par, (const unsigned char*)&par + 4);
    attr("pixelAspectRatio", "float", v);
  }
  attr("screenWindowCenter", "v2f", std::vector<unsigned char>(8, 0));
  {
    const float sw = 1.0f;
    std::vector<unsigned char> v((const unsigned char*)&sw, (const unsigned char*)&sw + 4);
    attr("screenWindowWidth", "float", v);
  }
  b.push_back(0);  // end of header
  const size_t row_bytes = (size_t)w * 3 * 4;
  const uint64_t table_end = b.size() + 8ull * h;
  for (uint32_t y = 0; y < h; ++y) {
    const uint64_t off = table_end + (uint64_t)y * (8 + row_bytes);
    put(&off, 8);
  }
  for (uint32_t y = 0; y < h; ++y) {
    i32((int32_t)y);
    i32((int32_t)row_bytes);
    for (int c = 2; c >= 0; --c)  // channels B, G, R
      for (uint32_t x = 0; x < w; ++x) put(&rgb[3 * ((size_t)y * w + x) + c], 4);
  }
  FILE* f = std::fopen(path, "wb");
  if (!f) return RRT_E_IO;
  const bool ok = std::fwrite(b.data(), 1, b.size(), f) == b.size();
  std::fclose(f);
  return ok ? RRT_OK : RRT_E_IO;
}
