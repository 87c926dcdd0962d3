// rrt_cli.cpp -- `rrt_render`: the reference's command line (main.cpp:81-188, windowless -f path)
// over rrt::PathTracer and the native COLLADA ingest.  Same flags, same meaning:
//   -s N  camera rays per pixel        -l N  samples per area light     -m N  max ray depth
//   -t N  render threads (accepted; the GPU replaces the worker pool)   -e F  environment map (EXR)
//   -f F  output PNG (+ F_rate.png)    -r W H  frame size              -c F  camera settings file
//   -a N T  adaptive batch / tolerance -H  hemisphere direct lighting  -p X Y DX DY  render a cell
//   -b R  lens radius  -d D  focal distance  -B X Y Z R DTHETA  black hole (centre, r_s, step)
// plus --seed S (keyed RNG seed), --device D and --kerr A [AX AY AZ] (Kerr spin a/M about the
// axis, default +y; build-defined).  The interactive viewer is out of scope: -f is
// required.  Exit codes follow main.cpp (usage -> 1).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rrt.h"
#include "../../include/rrt_pathtracer.hpp"

static void usage(const char* binary) {
  std::printf("Usage: %s [options] <scenefile>\n", binary);
  std::printf("Program Options:\n");
  std::printf("  -s  <INT>        Number of camera rays per pixel\n");
  std::printf("  -l  <INT>        Number of samples per area light\n");
  std::printf("  -t  <INT>        Number of render threads\n");
  std::printf("  -m  <INT>        Maximum ray depth\n");
  std::printf("  -e  <PATH>       Path to environment map\n");
  std::printf("  -f  <FILENAME>   Image (.png) file to save output to in windowless mode\n");
  std::printf("  -r  <INT> <INT>  Width and height of output image (if windowless)\n");
  std::printf("  -c  <PATH>       Camera settings file\n");
  std::printf("  -a  <INT> <FLOAT> Adaptive sampling batch size and tolerance\n");
  std::printf("  -H               Hemisphere sampling for direct lighting\n");
  std::printf("  -p  <X> <Y> <DX> <DY>  Render only a cell of the frame\n");
  std::printf("  -b  <FLOAT>      Lens radius     -d <FLOAT> Focal distance\n");
  std::printf("  -B  <X> <Y> <Z> <R> <DTHETA>  Black hole centre, Schwarzschild radius, step\n");
  std::printf("  --seed <INT>     Keyed RNG seed (default 0)   --device <INT> HIP device\n");
  std::printf("  --devices <D0,D1,...>  Render on several GPUs (block-cyclic tiles, RCCL gather)\n");
  std::printf("  --kerr <A> [<AX> <AY> <AZ>]  Kerr black hole, spin a/M in [0,1) about axis (default 0 1 0)\n");
  std::printf("  -h               Print this help message\n");
}

int main(int argc, char** argv) {
  // AppConfig defaults (application.h:41-65)
  size_t ns_aa = 1, ns_area_light = 1, max_ray_depth = 1, num_threads = 1, samples_per_batch = 32;
  float max_tolerance = 0.05f;
  bool hemi = false;
  double lens_radius = 0.25, focal_distance = 4.7;
  double hole[5] = {0.0, 1.0, 0.0, 0.1, 0.1};  // blackhole.cpp:5
  double kerr_spin = -1.0, kerr_axis[3] = {0.0, 1.0, 0.0};    // --kerr
  size_t w = 0, h = 0, x = (size_t)-1, y = 0, dx = 0, dy = 0;
  std::string filename, cam_settings, envmap_path, scene_path;
  unsigned long long seed = 0;
  int device = 0;
  std::vector<int> devices;  // --devices: several GPUs (rrt_group)
  bool to_file = false;
  auto need = [&](int i, int n) {
    if (i + n >= argc) { usage(argv[0]); std::exit(1); }
  };
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-f") { need(i, 1); to_file = true; filename = argv[++i]; }
    else if (a == "-r") { need(i, 2); w = std::atoi(argv[i + 1]); h = std::atoi(argv[i + 2]); i += 2; }
    else if (a == "-p") {
      need(i, 4);
      x = std::atoi(argv[i + 1]); y = std::atoi(argv[i + 2]); dx = std::atoi(argv[i + 3]); dy = std::atoi(argv[i + 4]);
      i += 4;
    }
    else if (a == "-s") { need(i, 1); ns_aa = std::atoi(argv[++i]); }
    else if (a == "-l") { need(i, 1); ns_area_light = std::atoi(argv[++i]); }
    else if (a == "-t") { need(i, 1); num_threads = std::atoi(argv[++i]); }
    else if (a == "-m") { need(i, 1); max_ray_depth = std::atoi(argv[++i]); }
    else if (a == "-b") { need(i, 1); lens_radius = std::atof(argv[++i]); }
    else if (a == "-d") { need(i, 1); focal_distance = std::atof(argv[++i]); }
    else if (a == "-e") { need(i, 1); envmap_path = argv[++i]; }
    else if (a == "-c") { need(i, 1); cam_settings = argv[++i]; }
    else if (a == "-a") {
      need(i, 2);
      samples_per_batch = std::atoi(argv[i + 1]); max_tolerance = (float)std::atof(argv[i + 2]); i += 2;
    }
    else if (a == "-H") { hemi = true; }
    else if (a == "-B") {
      need(i, 5);
      for (int k = 0; k < 5; ++k) hole[k] = std::atof(argv[i + 1 + k]);
      i += 5;
    }
    else if (a == "--seed") { need(i, 1); seed = std::strtoull(argv[++i], nullptr, 0); }
    else if (a == "--device") { need(i, 1); device = std::atoi(argv[++i]); }
    else if (a == "--devices") {
      need(i, 1);
      const std::string list = argv[++i];
      for (size_t at = 0; at <= list.size();) {
        const size_t comma = std::min(list.find(',', at), list.size());
        devices.push_back(std::atoi(list.substr(at, comma - at).c_str()));
        at = comma + 1;
      }
      device = devices[0];
    }
    else if (a == "--kerr") {
      need(i, 1);
      kerr_spin = std::atof(argv[++i]);
      auto num = [](const char* t) { char* e; std::strtod(t, &e); return *t && !*e; };
      if (i + 3 < argc && num(argv[i + 1]) && num(argv[i + 2]) && num(argv[i + 3])) {
        for (int k = 0; k < 3; ++k) kerr_axis[k] = std::atof(argv[i + 1 + k]);
        i += 3;
      }
    }
    else if (!a.empty() && a[0] == '-') { usage(argv[0]); return 1; }
    else if (scene_path.empty()) scene_path = a;
    else { usage(argv[0]); return 1; }
  }
  if (scene_path.empty()) { usage(argv[0]); return 1; }
  if (!to_file) {
    std::fprintf(stderr, "[rrt_render] the interactive viewer is not part of this build: pass -f <file.png>\n");
    return 1;
  }
  std::string stem = scene_path.substr(scene_path.find_last_of('/') + 1);
  stem = stem.substr(0, stem.find(".dae"));

  // Collada parse + Application::init/load + resize (main.cpp:165-181)
  rrt_collada_options opt;
  rrt_collada_options_default(&opt);
  if (w && h) { opt.screen_w = (uint32_t)w; opt.screen_h = (uint32_t)h; }
  opt.lens_radius = lens_radius;
  opt.focal_distance = focal_distance;
  rrt_scene_file* scene = nullptr;
  rrt_camera_state camera;
  char err[512] = {0};
  int rc = rrt_collada_load(scene_path.c_str(), &opt, &scene, &camera, err, sizeof(err));
  if (rc != RRT_OK) { std::fprintf(stderr, "[rrt_render] %s\n", err); return 2; }
  if (!cam_settings.empty()) {  // Application::load_camera -> Camera::load_settings
    if (rrt_camera_settings_load(cam_settings.c_str(), &camera) != RRT_OK) {
      std::fprintf(stderr, "[rrt_render] cannot read camera settings %s\n", cam_settings.c_str());
      return 2;
    }
    std::printf("[Camera] Loaded settings from %s\n", cam_settings.c_str());
  }
  std::vector<float> env_texels;
  rrt_envmap_desc env{};
  const rrt_envmap_desc* envp = nullptr;
  if (!envmap_path.empty()) {
    uint32_t ew = 0, eh = 0;
    float* t = nullptr;
    if (rrt_exr_load(envmap_path.c_str(), &t, &ew, &eh) != RRT_OK) {  // main.cpp:42-79
      std::fprintf(stderr, "[rrt_render] cannot load environment map %s\n", envmap_path.c_str());
      return 2;
    }
    env_texels.assign(t, t + (size_t)ew * eh * 3);
    rrt_exr_free(t);
    env.width = ew; env.height = eh; env.texels = env_texels.data();
    envp = &env;
  }
  if (devices.empty()) devices.push_back(device);
  rrt::PathTracer pt(devices, ns_aa, max_ray_depth, ns_area_light, samples_per_batch, max_tolerance, envp, hemi, stem,
                     lens_radius, focal_distance);
  (void)num_threads;  // -t: the CPU worker count; the GPU's waves take its place
  pt.set_seed(seed);
  pt.set_black_hole(hole, hole[3], hole[4]);
  if (kerr_spin >= 0) pt.set_kerr(kerr_spin, kerr_axis);
  // Application::set_up_pathtracer (application.cpp:622-628)
  pt.set_camera(&camera);
  pt.set_scene(scene);
  const size_t fw = (size_t)camera.screenW, fh = (size_t)camera.screenH;
  pt.set_frame_size(fw, fh);
  if (!pt.last_error().empty() || pt.state() != rrt::PathTracer::READY) {
    std::fprintf(stderr, "[rrt_render] %s\n", pt.last_error().empty() ? "renderer not ready" : pt.last_error().c_str());
    return 3;
  }
  std::printf("[PathTracer] Rendering %zux%zu, %zu spp on %zu device(s) (first %d)... ", fw, fh, ns_aa,
              devices.size(), devices[0]);
  std::fflush(stdout);
  pt.render_to_file(filename, x, y, dx, dy);
  if (pt.state() != rrt::PathTracer::DONE) {
    std::fprintf(stderr, "\n[rrt_render] render failed: %s\n", pt.last_error().c_str());
    return 3;
  }
  long long samples = 0;
  for (int32_t c : pt.sample_count_buffer()) samples += c;
  std::printf("done (%.4fs, %lld samples, %.1f Msamples/s)\n", pt.last_render_seconds(), samples,
              samples / pt.last_render_seconds() / 1e6);
  std::printf("[PathTracer] %s to file: %s\n", x == (size_t)-1 ? "Job completed, saved" : "Cell job completed, saved",
              filename.c_str());
  return 0;
}
