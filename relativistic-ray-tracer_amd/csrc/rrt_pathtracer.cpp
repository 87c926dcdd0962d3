// rrt_pathtracer.cpp -- rrt::PathTracer (include/rrt_pathtracer.hpp): the reference's PathTracer
// state machine and image outputs over the C ABI, plus the PNG writer (rrt_write_png).
// Host-only C++; every pixel comes from librrt's HIP kernels through rrt_render.
#include "../../include/rrt_pathtracer.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <sstream>

// ------------------------------------------------------------------------------- PNG writer
// RGBA8, one IDAT holding a zlib stream of stored (uncompressed) deflate blocks, filter 0 on
// every row.  Decoders see the same pixels lodepng::encode (pathtracer.cpp:678) would write.
namespace {
uint32_t crc_table[256];
bool crc_init = false;
uint32_t crc32_update(uint32_t c, const unsigned char* p, size_t n) {
  if (!crc_init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t v = i;
      for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
      crc_table[i] = v;
    }
    crc_init = true;
  }
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c;
}
void be32(std::vector<unsigned char>& b, uint32_t v) {
  b.push_back((unsigned char)(v >> 24)); b.push_back((unsigned char)(v >> 16));
  b.push_back((unsigned char)(v >> 8)); b.push_back((unsigned char)v);
}
void chunk(std::vector<unsigned char>& out, const char* type, const std::vector<unsigned char>& data) {
  be32(out, (uint32_t)data.size());
  const size_t at = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  uint32_t c = crc32_update(0xffffffffu, out.data() + at, 4 + data.size()) ^ 0xffffffffu;
  be32(out, c);
}
}  // namespace

extern "C" int rrt_write_png(const char* path, const uint32_t* rgba, uint32_t w, uint32_t h) {
  if (!path || !rgba || !w || !h) return RRT_E_INVALID;
  std::vector<unsigned char> raw;
  raw.reserve((size_t)h * (1 + 4 * (size_t)w));
  for (uint32_t y = 0; y < h; ++y) {
    raw.push_back(0);  // filter: none
    const unsigned char* row = (const unsigned char*)(rgba + (size_t)y * w);
    raw.insert(raw.end(), row, row + 4 * (size_t)w);
  }
  std::vector<unsigned char> z = {0x78, 0x01};
  uint32_t a = 1, b = 0;  // adler32
  for (unsigned char v : raw) { a = (a + v) % 65521u; b = (b + a) % 65521u; }
  for (size_t off = 0; off < raw.size() || off == 0;) {
    const size_t n = std::min<size_t>(65535, raw.size() - off);
    const bool last = off + n >= raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((unsigned char)(n & 0xff)); z.push_back((unsigned char)(n >> 8));
    z.push_back((unsigned char)(~n & 0xff)); z.push_back((unsigned char)((~n >> 8) & 0xff));
    z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
    off += n;
    if (last) break;
  }
  be32(z, (b << 16) | a);
  std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<unsigned char> ihdr;
  be32(ihdr, w); be32(ihdr, h);
  ihdr.push_back(8); ihdr.push_back(6); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
  chunk(out, "IHDR", ihdr);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  FILE* f = std::fopen(path, "wb");
  if (!f) return RRT_E_IO;
  const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
  std::fclose(f);
  return ok ? RRT_OK : RRT_E_IO;
}

// HDRImageBuffer::toColor + ImageBuffer::update_pixel (image.h:53-62, 183-198): float gamma 2.2,
// exposure sqrt(pow(2, 1)), per channel pow(s * exposure, 1 / gamma), upper clamp (clamp(0.f,
// 1.f, c) is min(1, c): the arguments are in (x, lo, hi) order), * 255 truncated, alpha 255.
extern "C" uint32_t rrt_tonemap_pixel(const float rgb[3]) {
  const float gamma = 2.2f, level = 1.0f;
  const float one_over_gamma = 1.0f / gamma;
  const float exposure = (float)std::sqrt(std::pow(2, level));
  uint32_t p = 0xFF000000u;
  for (int k = 0; k < 3; ++k) {
    float v = std::pow(rgb[k] * exposure, one_over_gamma);
    v = (v < 1.f) ? v : 1.f;  // std::min(1.f, v): NaN -> 1
    p |= ((uint32_t)(v * 255)) << (8 * k);
  }
  return p;
}

namespace rrt {

PathTracer::PathTracer(size_t ns_aa, size_t max_ray_depth, size_t ns_area_light, size_t /*ns_diff*/,
                       size_t /*ns_glsy*/, size_t /*ns_refr*/, size_t /*num_threads*/, size_t samples_per_batch,
                       float max_tolerance, const rrt_envmap_desc* envmap, bool direct_hemisphere_sample,
                       std::string filename, double lensRadius, double focalDistance, int device)
    : ns_aa_(ns_aa), max_ray_depth_(max_ray_depth), ns_area_light_(ns_area_light),
      samples_per_batch_(samples_per_batch), max_tolerance_(max_tolerance),
      direct_hemisphere_(direct_hemisphere_sample), filename_(std::move(filename)), lens_radius_(lensRadius),
      focal_distance_(focalDistance) {
  init({device}, envmap);
}

PathTracer::PathTracer(const std::vector<int>& devices, size_t ns_aa, size_t max_ray_depth, size_t ns_area_light,
                       size_t samples_per_batch, float max_tolerance, const rrt_envmap_desc* envmap,
                       bool direct_hemisphere_sample, std::string filename, double lensRadius, double focalDistance)
    : ns_aa_(ns_aa), max_ray_depth_(max_ray_depth), ns_area_light_(ns_area_light),
      samples_per_batch_(samples_per_batch), max_tolerance_(max_tolerance),
      direct_hemisphere_(direct_hemisphere_sample), filename_(std::move(filename)), lens_radius_(lensRadius),
      focal_distance_(focalDistance) {
  init(devices.empty() ? std::vector<int>{0} : devices, envmap);
}

// one context per device (every setter is applied to all of them); several: a device group
void PathTracer::init(const std::vector<int>& devices, const rrt_envmap_desc* envmap) {
  for (int device : devices) {
    rrt_device_cfg cfg;
    std::memset(&cfg, 0, sizeof(cfg));
    cfg.device = device;
    rrt_ctx* c = nullptr;
    const int rc = rrt_create(&c, &cfg);
    if (rc != RRT_OK) {
      err_ = "rrt_create failed on device " + std::to_string(device) + " (" + std::to_string(rc) + ")";
      return;
    }
    ctxs_.push_back(c);
  }
  ctx_ = ctxs_[0];
  if (ctxs_.size() > 1 && rrt_group_create(ctxs_.data(), (uint32_t)ctxs_.size(), &group_) != RRT_OK) {
    err_ = std::string("rrt_group_create failed: ") + rrt_last_error(ctx_);
    group_ = nullptr;
    return;
  }
  if (envmap && envmap->texels) {  // the reference keeps the pointer; this copy owns the texels
    envmap_texels_.assign(envmap->texels, envmap->texels + (size_t)envmap->width * envmap->height * 3);
    envmap_ = *envmap;
    envmap_.texels = envmap_texels_.data();
    has_envmap_ = true;
    for (rrt_ctx* c : ctxs_)
      if (rrt_set_envmap(c, &envmap_) != RRT_OK) err_ = rrt_last_error(c);
  }
  apply_spacetime();
}

void PathTracer::apply_spacetime() {
  rrt_spacetime_desc st;
  std::memset(&st, 0, sizeof(st));
  st.kind = kerr_spin_ < 0 ? RRT_METRIC_SCHWARZSCHILD : RRT_METRIC_KERR;
  for (int i = 0; i < 3; ++i) st.center[i] = hole_c_[i];
  st.r_s = hole_rs_; st.delta_theta = hole_dt_;
  st.spin = kerr_spin_ < 0 ? 0.0 : kerr_spin_;
  for (int i = 0; i < 3; ++i) st.axis[i] = kerr_axis_[i];
  for (rrt_ctx* c : ctxs_)
    if (rrt_set_spacetime(c, &st) != RRT_OK) err_ = rrt_last_error(c);
}

PathTracer::~PathTracer() {
  stop();
  if (thread_.joinable()) thread_.join();
  if (scene_) rrt_scene_file_free(scene_);
  if (group_) rrt_group_destroy(group_);
  for (rrt_ctx* c : ctxs_) rrt_destroy(c);
}

void PathTracer::set_scene(rrt_scene_file* scene) {
  if (state_ != INIT) return;
  if (scene_ && scene_ != scene) rrt_scene_file_free(scene_);
  scene_ = scene;
  if (!ctx_) { err_ = "no context"; return; }
  for (rrt_ctx* c : ctxs_)
    if (rrt_set_scene(c, rrt_scene_file_desc(scene_)) != RRT_OK) {
      err_ = rrt_last_error(c);
      return;
    }
  if (has_valid_configuration()) state_ = READY;
}

void PathTracer::set_camera(rrt_camera_state* camera) {
  if (state_ != INIT) return;
  camera_ = camera;
  camera_->lensRadius = lens_radius_;  // pathtracer.cpp:126-128
  camera_->focalDistance = focal_distance_;
  rrt_camera_desc d;
  rrt_camera_state_desc(camera_, &d);
  if (!ctx_) { err_ = "no context"; return; }
  for (rrt_ctx* c : ctxs_)
    if (rrt_set_camera(c, &d) != RRT_OK) {
      err_ = rrt_last_error(c);
      return;
    }
  if (has_valid_configuration()) state_ = READY;
}

void PathTracer::set_frame_size(size_t width, size_t height) {
  if (state_ != INIT && state_ != READY) stop();
  frame_w_ = width; frame_h_ = height;
  sample_rgb_.assign(width * height * 3, 0.f);
  sample_cnt_.assign(width * height, 0);
  frame_.resize(width, height);
  render_cell_ = false;
  cell_x0_ = 0; cell_y0_ = 0; cell_x1_ = width; cell_y1_ = height;
  if (has_valid_configuration()) state_ = READY;
}

void PathTracer::set_black_hole(const double center[3], double r_s, double delta_theta) {
  for (int i = 0; i < 3; ++i) hole_c_[i] = center[i];
  hole_rs_ = r_s; hole_dt_ = delta_theta;
  apply_spacetime();
}

void PathTracer::set_kerr(double spin, const double axis[3]) {
  kerr_spin_ = spin;
  if (axis) for (int i = 0; i < 3; ++i) kerr_axis_[i] = axis[i];
  apply_spacetime();
}

rrt_render_params PathTracer::params() const {
  rrt_render_params p;
  rrt_render_params_default(&p);
  p.ns_aa = (uint32_t)ns_aa_;
  p.max_ray_depth = (uint32_t)max_ray_depth_;
  p.ns_area_light = (uint32_t)ns_area_light_;
  p.samples_per_batch = (uint32_t)samples_per_batch_;
  p.max_tolerance = max_tolerance_;
  p.direct_hemisphere = direct_hemisphere_ ? 1u : 0u;
  p.seed = seed_;
  p.frame_w = (uint32_t)frame_w_;
  p.frame_h = (uint32_t)frame_h_;
  return p;
}

void PathTracer::start_raytracing() {
  if (state_ != READY) return;
  if (thread_.joinable()) thread_.join();
  std::fill(sample_rgb_.begin(), sample_rgb_.end(), 0.f);  // sampleBuffer.clear()
  if (!render_cell_) std::fill(frame_.data.begin(), frame_.data.end(), 0u);
  cancel_ = 0;
  state_ = RENDERING;
  thread_ = std::thread(&PathTracer::worker, this);
}

// One dispatcher thread (in place of the reference's worker pool, pathtracer.cpp:611-644):
// the region goes to the GPU -- or to every GPU of the group -- in bands of band_rows_ rows (all
// of it at once by default); the cancel flag is polled between bands (and before each launch).
void PathTracer::worker() {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t x0 = cell_x0_, y0 = cell_y0_, x1 = cell_x1_, y1 = cell_y1_;
  const size_t w = x1 - x0;
  const size_t band = band_rows_ ? band_rows_ : (y1 - y0);
  const rrt_render_params p = params();
  std::vector<float> rgb;
  std::vector<int32_t> cnt;
  bool ok = true;
  for (size_t y = y0; y < y1 && ok; y += band) {
    if (cancel_) { ok = false; break; }
    const size_t h = std::min(band, y1 - y);
    rgb.assign(w * h * 3, 0.f);
    cnt.assign(w * h, 0);
    const int rc = group_ ? rrt_group_render(group_, &p, (uint32_t)x0, (uint32_t)y, (uint32_t)w, (uint32_t)h,
                                             rgb.data(), cnt.data(), &cancel_)
                          : rrt_render(ctx_, &p, (uint32_t)x0, (uint32_t)y, (uint32_t)w, (uint32_t)h, rgb.data(),
                                       cnt.data(), nullptr, nullptr, &cancel_);
    if (rc != RRT_OK) {
      if (rc != RRT_E_CANCELLED) err_ = rrt_last_error(ctx_);
      ok = false;
      break;
    }
    for (size_t j = 0; j < h; ++j) {
      std::memcpy(&sample_rgb_[((y + j) * frame_w_ + x0) * 3], &rgb[j * w * 3], w * 3 * sizeof(float));
      std::memcpy(&sample_cnt_[(y + j) * frame_w_ + x0], &cnt[j * w], w * sizeof(int32_t));
    }
    to_color(x0, y, x1, y + h);
  }
  last_seconds_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  {
    std::lock_guard<std::mutex> lk(m_);
    state_ = ok ? DONE : READY;
  }
  cv_.notify_all();
}

void PathTracer::to_color(size_t x0, size_t y0, size_t x1, size_t y1) {
  for (size_t y = y0; y < y1; ++y)
    for (size_t x = x0; x < x1; ++x) frame_.data[x + y * frame_w_] = rrt_tonemap_pixel(&sample_rgb_[(x + y * frame_w_) * 3]);
}

bool PathTracer::wait_done() {
  std::unique_lock<std::mutex> lk(m_);
  cv_.wait(lk, [this] { return state_ != RENDERING; });
  return state_ == DONE;
}

void PathTracer::stop() {
  if (state_ == RENDERING) {
    cancel_ = 1;
    wait_done();
  }
  if (thread_.joinable()) thread_.join();
  if (state_ == DONE || state_ == VISUALIZE) state_ = READY;
}

void PathTracer::clear() {
  if (state_ != READY) return;
  if (scene_) rrt_scene_file_free(scene_);
  scene_ = nullptr;
  camera_ = nullptr;
  sample_rgb_.clear(); sample_cnt_.clear(); frame_.resize(0, 0);
  frame_w_ = frame_h_ = 0;
  state_ = INIT;
}

void PathTracer::render_to_file(const std::string& filename, size_t x, size_t y, size_t dx, size_t dy) {
  if (x == (size_t)-1) {
    start_raytracing();
    if (!wait_done()) return;
    save_image(filename);
  } else {
    render_cell_ = true;
    cell_x0_ = x; cell_y0_ = y; cell_x1_ = x + dx; cell_y1_ = y + dy;
    ImageBuffer buffer;
    raytrace_cell(buffer);
    save_image(filename, &buffer);
  }
}

void PathTracer::raytrace_cell(ImageBuffer& buffer) {
  const size_t w = cell_x1_ - cell_x0_, h = cell_y1_ - cell_y0_;
  buffer.resize(w, h);
  stop();
  render_cell_ = true;
  start_raytracing();
  if (!wait_done()) return;
  for (size_t y = cell_y0_; y < cell_y1_; ++y)
    for (size_t x = cell_x0_; x < cell_x1_; ++x)
      buffer.data[w * (y - cell_y0_) + (x - cell_x0_)] = frame_.data[x + y * frame_w_];
}

void PathTracer::save_image(std::string filename, const ImageBuffer* buffer) {
  if (state_ != DONE) return;
  if (!buffer) buffer = &frame_;
  if (filename.empty()) {  // <filename>_screenshot_<mon>-<day>_<h>-<m>-<s>.png
    time_t t = time(nullptr);
    tm* lt = localtime(&t);
    std::stringstream ss;
    ss << filename_ << "_screenshot_" << lt->tm_mon + 1 << "-" << lt->tm_mday << "_" << lt->tm_hour << "-"
       << lt->tm_min << "-" << lt->tm_sec << ".png";
    filename = ss.str();
  }
  const size_t w = buffer->w, h = buffer->h;
  std::vector<uint32_t> out(w * h);
  for (size_t i = 0; i < h; ++i)  // bottom-up sampleBuffer rows -> top-down PNG rows
    std::memcpy(&out[i * w], &buffer->data[(h - i - 1) * w], 4 * w);
  for (auto& v : out) v |= 0xFF000000u;
  if (rrt_write_png(filename.c_str(), out.data(), (uint32_t)w, (uint32_t)h) != RRT_OK)
    err_ = "cannot write " + filename;
  save_sampling_rate_image(filename);
}

// pathtracer.cpp:686-717: blue (rate 0) -> green (0.5) -> red (1) per pixel, whole frame
void PathTracer::save_sampling_rate_image(const std::string& filename) {
  const size_t w = frame_w_, h = frame_h_;
  std::vector<uint32_t> out(w * h, 0u);
  for (size_t x = 0; x < w; ++x)
    for (size_t y = 0; y < h; ++y) {
      const float rate = sample_cnt_[y * w + x] * 1.0f / ns_aa_;
      float c[3];
      if (rate <= 0.5) {
        const float r = (0.5 - rate) / 0.5;
        const float s = (float)(1.0 - r);
        c[0] = 0.0f * r + 0.0f * s; c[1] = 0.0f * r + 1.0f * s; c[2] = 1.0f * r + 0.0f * s;
      } else {
        const float r = (1.0 - rate) / 0.5;
        const float s = (float)(1.0 - r);
        c[0] = 0.0f * r + 1.0f * s; c[1] = 1.0f * r + 0.0f * s; c[2] = 0.0f * r + 0.0f * s;
      }
      uint32_t p = 0xFF000000u;
      for (int k = 0; k < 3; ++k) {
        const float v = (c[k] < 1.f) ? c[k] : 1.f;
        p |= ((uint32_t)(v * 255)) << (8 * k);
      }
      out[x + (h - 1 - y) * w] = p;
    }
  const std::string rate = filename.substr(0, filename.size() >= 4 ? filename.size() - 4 : 0) + "_rate.png";
  if (rrt_write_png(rate.c_str(), out.data(), (uint32_t)w, (uint32_t)h) != RRT_OK) err_ = "cannot write " + rate;
}

}  // namespace rrt
