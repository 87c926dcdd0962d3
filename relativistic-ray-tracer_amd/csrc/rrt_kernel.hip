// rrt_kernel.hip -- general path (any max_ray_depth): one lane = one pixel, the reference's
// recursion unrolled (reference: part1_code.cpp:15-187), plus the small utility kernels
// (tile unpack, tonemap) and the C++ launch shims used by rrt_host.cpp.
//
// Work decomposition: persistent grid; each wave pulls 8x8 pixel blocks (one lane = one pixel,
// the whole adaptive sample loop) from a device atomic over the caller's tile list.  BVH
// traversal is stackless over skip pointers (rrt_internal.h DNode), which visits exactly the
// reference's left-then-right recursion order.  The depth <= 1 hot path runs in the
// sample-parallel batch kernel of rrt_sample.hip instead.
#include "rrt_integrator.h"

#include <cstdlib>
#include <type_traits>

namespace rrt {

template <bool DEEP, bool COUNT, int LEAN, int W = 0, class LV = LevelsPriv>
__device__ __forceinline__ spec est_radiance(const KParams& kp, Rng& g, v3 o, v3 d, Counters& cn, LV lv = LV()) {  // :103-123
  Isect is;
  if (camera_proven_miss<COUNT, LEAN == V_KERR, LEAN == 0, W>(kp, o, d, cn) ||
      !trace<false, COUNT, DEEP, LEAN>(kp, o, d, &is, cn))  // miss: envLight->sample_dir(r), unbent r
    return (!is_lean(LEAN) && kp.env.w) ? env_dir(kp.env, d) : S(0, 0, 0);
  if (LEAN == V_SW && sw_illum(kp) != 2u) {  // ILLUM 0 / 1 / 3 (:108-122)
    const uint32_t il = sw_illum(kp);
    if (il == 0u)  // normal_shading (pathtracer.h:199-201): Spectrum(n) * .5 + Spectrum(.5, .5, .5)
      return S((float)is.n.x, (float)is.n.y, (float)is.n.z) * (float).5 + S(.5f, .5f, .5f);
    if (il == 1u) return one_bounce<COUNT, LEAN, DEEP>(kp, g, is, cn);
    return at_least_one_bounce<COUNT, LEAN>(kp, g, is, cn, lv);
  }
  spec e = emission(kp.bsdfs[is.bsdf]);
  if (kp.max_ray_depth == 0) return e;
  if (!DEEP || kp.max_ray_depth == 1) return e + one_bounce<COUNT, LEAN, DEEP>(kp, g, is, cn);
  return e + at_least_one_bounce<COUNT, general_of(LEAN)>(kp, g, is, cn, lv);
}

// PathTracer::raytrace_pixel (:125-163): ADAPTIVE 1, THIN_LENS 0 -- or, in the V_SW build, as kp.sw says
template <bool DEEP, bool COUNT, int LEAN, int W = 0, class LV = LevelsPriv>
__device__ __forceinline__ spec raytrace_pixel(const KParams& kp, uint32_t x, uint32_t y, int& count, Rng& g, Counters& cn,
                                               LV lv = LV()) {
  spec ret = S(0, 0, 0);
  int n = 0;  // samples taken (the reference's i after its loop; counted explicitly: the
              // `++i; break;` form was miscompiled in the register-starved bounce build)
  double s1 = 0.0, s2 = 0.0;
  const DCamera& cam = kp.cam;
  for (int i = 0; i < (int)kp.ns_aa; ++i) {
    double sx = (double)x, sy = (double)y;
    if (kp.ns_aa == 1) { sx += 0.5; sy += 0.5; }
    else { double jx, jy; g.grid(jx, jy); sx += jx; sy += jy; }
    double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
    double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
    spec s;
    if (LEAN == V_SW && (kp.sw & SW_THIN_LENS)) {
      // Camera::generate_ray_for_thin_lens (camera.cpp:176-184) at the lens sample the grid sampler
      // draws after the jitter (part1_code.cpp:137-139): rndR = its x, rndTheta = its y * 2 * M_PI
      double lx, ly; g.grid(lx, ly);
      const double rnd_theta = ly * 2 * PI_D;
      const double lr = kp.lens_r * sqrt(lx);
      const v3 pl = V(lr * rrt_glibm_cos(rnd_theta), lr * rrt_glibm_sin(rnd_theta), 0);
      const v3 c0 = ld3(cam.c2w0), c1 = ld3(cam.c2w1), c2 = ld3(cam.c2w2);
      const v3 o = ld3(cam.pos) + ((smul(pl.x, c0) + smul(pl.y, c1)) + smul(pl.z, c2));  // pos + c2w * pLens
      const v3 q = V(vx * kp.focal, vy * kp.focal, -1.0 * kp.focal) - pl;                // pinHole * f - pLens
      s = est_radiance<DEEP, COUNT, LEAN, W>(kp, g, o, unit((smul(q.x, c0) + smul(q.y, c1)) + smul(q.z, c2)), cn, lv);
    } else {
      // Camera::generate_ray (part1_code.cpp:182-187)
      v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
      s = est_radiance<DEEP, COUNT, LEAN, W>(kp, g, ld3(cam.pos), unit(w), cn, lv);
    }
    ret = ret + s;
    if (LEAN == V_SW && (kp.sw & SW_NO_ADAPTIVE)) { n = i + 1; continue; }  // ADAPTIVE 0
    double il = illum(s);
    s1 += il;
    s2 += il * il;
    n = i + 1;
    if ((uint32_t)n % kp.samples_per_batch == 0) {
      double avg = s1 / n, sd = sqrt((s2 - avg * s1) / i);
      if (1.96 * sd / sqrt((double)n) <= (double)kp.max_tolerance * avg) break;
    }
  }
  count = n;
  return ret / (float)n;
}

}  // namespace rrt

// ------------------------------------------------------------------ kernels
// DEEP: max_ray_depth >= 2 (bounce loop); COUNT: per-pixel work counters; LEAN: area lights
// only, no microfacet BSDF, importance-sampled direct light (the BASELINE scenes); WAVES: the
// register budget, as minimum waves per SIMD; LVD: 0, or the depth bound of the bounce levels kept
// in LDS (rrt_integrator.h LevelsLds; frames of max_ray_depth <= LVD).
template <bool DEEP, bool COUNT, int LEAN, int WAVES, int LVD = 0>
__global__ __launch_bounds__(256, WAVES) void rrt_render_kernel(const KParams* __restrict__ kpp) {
  const KParams& kp = *kpp;
  using namespace rrt;
  using LV = std::conditional_t<(LVD > 0), LevelsLds<(LVD > 0 ? LVD : 1)>, LevelsPriv>;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t bpt = kp.blocks_per_tile_side;
  const uint32_t tpix = kp.tile_size * kp.tile_size;
  for (;;) {
    uint32_t blk = 0;
    if (lane == 0) blk = atomicAdd(kp.block_counter, kp.claim_list ? 64u : 1u);
    blk = __shfl(blk, 0);
    uint32_t t, lx, ly;
    bool mine;
    if (kp.claim_list) {  // the pixel proof pass's list: 64 listed pixels per claim, one per lane
      const uint32_t n_list = *kp.claim_count;
      if (blk >= n_list) break;
      const uint32_t e = blk + lane;
      mine = e < n_list;
      const uint32_t ix = mine ? (kp.claim_list[e] & 0x7fffffffu) : 0u;
      t = kp.tile_order[ix / tpix];
      const uint32_t r = claim_r(ix % tpix, kp.tile_size);
      lx = r % kp.tile_size; ly = r / kp.tile_size;
    } else {
      if (blk >= kp.n_blocks) break;
      t = blk / (bpt * bpt);
      const uint32_t b = blk % (bpt * bpt);
      lx = (b % bpt) * 8 + (lane & 7u); ly = (b / bpt) * 8 + (lane >> 3);
      mine = true;
    }
    const uint32_t x = kp.tiles[2 * t] + lx, y = kp.tiles[2 * t + 1] + ly;
    if (mine && lx < kp.tile_size && ly < kp.tile_size && x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 &&
        y < kp.clip_y1) {
      Rng g; g.key = rrt_pixel_key(kp.seed, x, y); g.ctr = 0;
      Counters cn = {0, 0, 0, 0};
      int cnt;
      LV lv;
      if constexpr (LVD > 0) {
        __shared__ LevelLds<(LVD > 0 ? LVD : 1)> lvs;
        lv = LV{&lvs, threadIdx.x};
      }
      spec s = raytrace_pixel<DEEP, COUNT, LEAN, 16 * DEEP + 8 * COUNT + WAVES>(kp, x, y, cnt, g, cn, lv);
      const size_t k = (size_t)t * tpix + (size_t)ly * kp.tile_size + lx;
      kp.rgb[3 * k] = s.r; kp.rgb[3 * k + 1] = s.g; kp.rgb[3 * k + 2] = s.b;
      kp.count[k] = cnt;
      if (kp.draws) kp.draws[k] = g.ctr;
      if (COUNT && kp.counters) {
        kp.counters[4 * k] = cn.bbox; kp.counters[4 * k + 1] = cn.micro;
        kp.counters[4 * k + 2] = cn.prim; kp.counters[4 * k + 3] = cn.query;
      }
    }
  }
}

__global__ void rrt_unpack_kernel(const uint32_t* tiles, uint32_t n_tiles, uint32_t ts, uint32_t fw, uint32_t fh,
                                  const float* rgb_p, const int32_t* cnt_p, float* rgb, int32_t* cnt) {
  const size_t tpix = (size_t)ts * ts;
  const size_t total = tpix * n_tiles;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < total; k += (size_t)gridDim.x * blockDim.x) {
    const size_t t = k / tpix, r = k % tpix;
    const uint32_t x = tiles[2 * t] + (uint32_t)(r % ts), y = tiles[2 * t + 1] + (uint32_t)(r / ts);
    if (x < fw && y < fh && (r % ts) < ts) {
      const size_t o = (size_t)y * fw + x;
      rgb[3 * o] = rgb_p[3 * k]; rgb[3 * o + 1] = rgb_p[3 * k + 1]; rgb[3 * o + 2] = rgb_p[3 * k + 2];
      cnt[o] = cnt_p[k];
    }
  }
}

// HDRImageBuffer::toColor (image.h:183-198) + ImageBuffer::update_pixel (image.h:53-62)
__global__ void rrt_tonemap_kernel(uint32_t n, const float* rgb, uint32_t* out, float exposure, float inv_gamma) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    float r = powf(rgb[3 * k] * exposure, inv_gamma);
    float g = powf(rgb[3 * k + 1] * exposure, inv_gamma);
    float b = powf(rgb[3 * k + 2] * exposure, inv_gamma);
    // clamp(0.f, 1.f, c) == std::min(std::max(0.f, 1.f), c) == min(1, c) (misc.h:66-69)
    r = (r < 1.f) ? r : 1.f; g = (g < 1.f) ? g : 1.f; b = (b < 1.f) ? b : 1.f;
    uint32_t p = 0;
    p |= ((uint32_t)(b * 255)) << 16;
    p |= ((uint32_t)(g * 255)) << 8;
    p |= ((uint32_t)(r * 255));
    p |= 0xFF000000u;
    out[k] = p;
  }
}

// The device's restatements of the host C library's functions (rrt_glibm.h), evaluated on n
// arguments: rrt_libm_eval checks them bit for bit against the host's libm (tests/test_gpu_glibm.py).
// fn: 0 sin, 1 cos, 2 acos, 3 atan2(a, b), 4 sinf((float)a), 5 cosf((float)a), 6 exp, 7 log, 8 erf,
// 9 atan, 10 tan
__global__ void rrt_libm_kernel(int fn, uint64_t n, const double* a, const double* b, double* out) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const double x = a[k];
    double r;
    switch (fn) {
      case 0: r = rrt_glibm_sin(x); break;
      case 1: r = rrt_glibm_cos(x); break;
      case 2: r = rrt_glibm_acos(x); break;
      case 3: r = rrt_glibm_atan2(x, b[k]); break;
      case 4: r = rrt_glibm_sinf((float)x); break;
      case 5: r = rrt_glibm_cosf((float)x); break;
      case 6: r = rrt_glibm_exp(x); break;
      case 7: r = rrt_glibm_log(x); break;
      case 8: r = rrt_glibm_erf(x); break;
      case 9: r = rrt_glibm_atan(x); break;
      default: r = rrt_glibm_tan(x); break;
    }
    out[k] = r;
  }
}

// ------------------------------------------------------------------ launch shims (C++ linkage)
// Kernel selection: deep / counting variants are built once (1 wave per SIMD budget); the
// depth <= 1 path has general and LEAN builds at 1..4 waves per SIMD (A/B knob `waves`).
// lean = the kernel variant (rrt_device.h: 0 general, 1/2 LEAN, V_KERR).
hipError_t rrt_launch_render(const KParams& kp, const KParams* d_kp, int deep, int count, int lean, int waves, uint32_t grid,
                             hipStream_t stream) {
#define RRT_LAUNCH(D, C, L, W) hipLaunchKernelGGL((rrt_render_kernel<D, C, L, W>), dim3(grid), dim3(256), 0, stream, d_kp)
  // the bounce levels in LDS (frames of max_ray_depth <= 4; RRT_AB_NO_LEVEL_LDS=1 keeps them private, A/B)
  static const bool no_lv = [] { const char* e = std::getenv("RRT_AB_NO_LEVEL_LDS"); return e && e[0] == '1'; }();
  const bool lv4 = deep && !count && kp.max_ray_depth <= 4u && !no_lv;
  if (lean == rrt::V_SW) {  // the reference's switches as run-time flags: one bounce-capable build
    if (count) RRT_LAUNCH(true, true, rrt::V_SW, 1); else RRT_LAUNCH(true, false, rrt::V_SW, 1);
  } else if (lean == rrt::V_KERR) {  // the Kerr builds (general integrator)
    if (deep) {
      if (count) RRT_LAUNCH(true, true, rrt::V_KERR, 1); else RRT_LAUNCH(true, false, rrt::V_KERR, 1);
    } else if (count) {
      RRT_LAUNCH(false, true, rrt::V_KERR, 1);
    } else {
      RRT_LAUNCH(false, false, rrt::V_KERR, 2);
    }
  } else if (deep) {
    if (count) {
      RRT_LAUNCH(true, true, false, 1);
    } else {
      if (lv4 && (waves == 3 || waves <= 0 || waves > 4)) {
        hipLaunchKernelGGL((rrt_render_kernel<true, false, false, 3, 4>), dim3(grid), dim3(256), 0, stream, d_kp);
        return hipGetLastError();
      }
      switch (waves) {  // register budget (A/B): the bounce build spills below 1 wave/SIMD's 256 VGPRs
        case 2: RRT_LAUNCH(true, false, false, 2); break;
        case 3: RRT_LAUNCH(true, false, false, 3); break;
        case 4: RRT_LAUNCH(true, false, false, 4); break;
        case 1: RRT_LAUNCH(true, false, false, 1); break;
        default: RRT_LAUNCH(true, false, false, 3); break;
      }
    }
  } else if (count) {
    RRT_LAUNCH(false, true, false, 1);
  } else if (lean == 1) {  // LEAN 2 (point lights) runs the general build here
    switch (waves) {
      case 1: RRT_LAUNCH(false, false, true, 1); break;
      case 3: RRT_LAUNCH(false, false, true, 3); break;
      case 4: RRT_LAUNCH(false, false, true, 4); break;
      default: RRT_LAUNCH(false, false, true, 2); break;
    }
  } else {
    if (waves == 1) RRT_LAUNCH(false, false, false, 1); else RRT_LAUNCH(false, false, false, 2);
  }
#undef RRT_LAUNCH
  return hipGetLastError();
}
hipError_t rrt_launch_unpack(const uint32_t* tiles, uint32_t n_tiles, uint32_t ts, uint32_t fw, uint32_t fh,
                             const float* rgb_p, const int32_t* cnt_p, float* rgb, int32_t* cnt, hipStream_t stream) {
  size_t total = (size_t)ts * ts * n_tiles;
  uint32_t grid = (uint32_t)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(rrt_unpack_kernel, dim3(grid), dim3(256), 0, stream, tiles, n_tiles, ts, fw, fh, rgb_p, cnt_p,
                     rgb, cnt);
  return hipGetLastError();
}
hipError_t rrt_launch_libm(int fn, uint64_t n, const double* a, const double* b, double* out, hipStream_t stream) {
  uint64_t grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(rrt_libm_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, fn, n, a, b, out);
  return hipGetLastError();
}
hipError_t rrt_launch_tonemap(uint32_t n, const float* rgb, uint32_t* out, float exposure, float inv_gamma,
                              hipStream_t stream) {
  uint32_t grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(rrt_tonemap_kernel, dim3(grid), dim3(256), 0, stream, n, rgb, out, exposure, inv_gamma);
  return hipGetLastError();
}
