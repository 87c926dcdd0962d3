// rrt_pathtracer.hpp -- the reference's PathTracer surface (pathtracer.h:64-230) in C++ over the
// C ABI of librrt (include/rrt.h), so a caller of CGL::PathTracer (the viewer's Application, or
// main.cpp's windowless path) can switch to the MI355X renderer by changing the type it holds.
//
//   reference                                   here
//   PathTracer(ns_aa, max_ray_depth, ...)       rrt::PathTracer(same 14 parameters, + device)
//   set_scene(StaticScene::Scene*)              set_scene(rrt_scene_file*)   (takes ownership)
//   set_camera(Camera*)                          set_camera(rrt_camera_state*) (not owned; the
//                                                lens parameters are written into it, like :126-128)
//   set_frame_size / start_raytracing / stop /   same names, same state machine (INIT, READY,
//   clear / render_to_file / raytrace_cell /     RENDERING, DONE); the CPU worker pool is replaced
//   save_image / save_sampling_rate_image        by one dispatcher thread that submits whole bands
//                                                of the frame to the GPU -- or, given several
//                                                devices, to all of them (rrt_group: block-cyclic
//                                                tiles, one context per GPU, RCCL gather)
//   sampleBuffer / sampleCountBuffer /           sample_buffer() / sample_count_buffer() /
//   frameBuffer                                  frame_buffer() (same layouts, y = 0 at the bottom)
//   global_black_hole (-B)                       set_black_hole
//
// Rendering is per-pixel identical to the reference under the keyed RNG.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rrt.h"

namespace rrt {

// ImageBuffer (image.h:20-80): RGBA8 packed as uint32 (R in the low byte), row-major
struct ImageBuffer {
  size_t w = 0, h = 0;
  std::vector<uint32_t> data;
  void resize(size_t W, size_t H) { w = W; h = H; data.assign(W * H, 0u); }
};

class PathTracer {
 public:
  enum State { INIT, READY, VISUALIZE, RENDERING, DONE };

  PathTracer(size_t ns_aa = 1, size_t max_ray_depth = 4, size_t ns_area_light = 1, size_t ns_diff = 1,
             size_t ns_glsy = 1, size_t ns_refr = 1, size_t num_threads = 1, size_t samples_per_batch = 32,
             float max_tolerance = 0.05f, const rrt_envmap_desc* envmap = nullptr,
             bool direct_hemisphere_sample = false, std::string filename = "", double lensRadius = 0.25,
             double focalDistance = 4.7, int device = 0);
  // the same over several GPUs (one context each, rrt_group: block-cyclic tiles, RCCL gather)
  PathTracer(const std::vector<int>& devices, size_t ns_aa = 1, size_t max_ray_depth = 4, size_t ns_area_light = 1,
             size_t samples_per_batch = 32, float max_tolerance = 0.05f, const rrt_envmap_desc* envmap = nullptr,
             bool direct_hemisphere_sample = false, std::string filename = "", double lensRadius = 0.25,
             double focalDistance = 4.7);
  ~PathTracer();
  PathTracer(const PathTracer&) = delete;
  PathTracer& operator=(const PathTracer&) = delete;

  void set_scene(rrt_scene_file* scene);          // takes ownership (pathtracer.cpp:95-117)
  void set_camera(rrt_camera_state* camera);      // not owned (:119-134)
  void set_frame_size(size_t width, size_t height);  // (:136-149)
  void set_black_hole(const double center[3], double r_s, double delta_theta);  // -B (main.cpp:139-145)
  // Kerr spin a/M in [0, 1) about `axis` (build-defined); spin < 0: Schwarzschild
  void set_kerr(double spin, const double axis[3] = nullptr);
  void set_seed(uint64_t seed) { seed_ = seed; }  // keyed RNG seed
  void set_band_rows(size_t rows) { band_rows_ = rows; }  // rows per GPU submission (0: whole region)

  void start_raytracing();   // READY -> RENDERING, returns at once (:224-282)
  void stop();               // any running state -> READY (cancels between bands)
  void clear();              // READY -> INIT, drops scene/buffers
  bool wait_done();          // blocks until DONE (true) or stopped (false)
  void render_to_file(const std::string& filename, size_t x = (size_t)-1, size_t y = 0, size_t dx = 0,
                      size_t dy = 0);                                         // (:284-301)
  void raytrace_cell(ImageBuffer& buffer);                                    // (:583-609)
  void save_image(std::string filename = "", const ImageBuffer* buffer = nullptr);  // (:646-684)
  void save_sampling_rate_image(const std::string& filename);                      // (:686-717)

  State state() const { return state_; }
  const std::string& last_error() const { return err_; }
  const std::vector<float>& sample_buffer() const { return sample_rgb_; }        // [h][w][3]
  const std::vector<int32_t>& sample_count_buffer() const { return sample_cnt_; }  // [h][w]
  const ImageBuffer& frame_buffer() const { return frame_; }
  double last_render_seconds() const { return last_seconds_; }

 private:
  bool has_valid_configuration() const { return scene_ && camera_ && frame_w_ && frame_h_; }
  void worker();
  void to_color(size_t x0, size_t y0, size_t x1, size_t y1);
  rrt_render_params params() const;

  size_t ns_aa_, max_ray_depth_, ns_area_light_, samples_per_batch_;
  float max_tolerance_;
  bool direct_hemisphere_;
  std::string filename_;
  double lens_radius_, focal_distance_;
  uint64_t seed_ = 0;
  size_t band_rows_ = 0;

  void init(const std::vector<int>& devices, const rrt_envmap_desc* envmap);
  rrt_ctx* ctx_ = nullptr;           // ctxs_[0]
  std::vector<rrt_ctx*> ctxs_;       // one per device
  rrt_group* group_ = nullptr;       // several devices: the multi-GPU plan
  rrt_scene_file* scene_ = nullptr;
  rrt_camera_state* camera_ = nullptr;
  std::vector<float> envmap_texels_;
  rrt_envmap_desc envmap_{};
  bool has_envmap_ = false;
  double hole_c_[3] = {0.0, 1.0, 0.0}, hole_rs_ = 0.1, hole_dt_ = 0.1;  // blackhole.cpp:5
  double kerr_spin_ = -1.0, kerr_axis_[3] = {0.0, 1.0, 0.0};           // < 0: Schwarzschild
  void apply_spacetime();

  size_t frame_w_ = 0, frame_h_ = 0;
  bool render_cell_ = false;
  size_t cell_x0_ = 0, cell_y0_ = 0, cell_x1_ = 0, cell_y1_ = 0;
  std::vector<float> sample_rgb_;
  std::vector<int32_t> sample_cnt_;
  ImageBuffer frame_;

  std::atomic<State> state_{INIT};
  volatile int cancel_ = 0;
  std::thread thread_;
  std::mutex m_;
  std::condition_variable cv_;
  std::string err_;
  double last_seconds_ = 0.0;
};

}  // namespace rrt
