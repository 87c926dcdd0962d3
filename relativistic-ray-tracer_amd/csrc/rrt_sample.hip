// rrt_sample.hip -- the depth <= 1 hot path: one lane = one pixel, one loop iteration = one
// camera sample of every active lane, with per-lane pixel refill at sample boundaries.
//
// Reference: PathTracer::raytrace_pixel (part1_code.cpp:125-163) -> est_radiance_global_illumination
// (:103-123, ILLUM 2, max_ray_depth <= 1) -> estimate_direct_lighting_importance / _hemisphere
// (:15-57) -> BVHAccel::intersect (bvh.cpp:103-138, geodesic march, rrt_device.h query()).
//
// Versus the general kernel (rrt_kernel.hip), which runs a lane's whole adaptive sample loop
// before the wave takes the next 8x8 block (so one 64-sample pixel holds 63 finished lanes):
//   * lanes stay in lock-step per SAMPLE; a lane whose pixel is done takes the next pixel of
//     the wave's pool (an 8x8 block, refilled by one atomic) at the next sample boundary;
//   * state that is cold during a geodesic query (pixel accumulators, the shading record of the
//     camera hit across its shadow rays) lives in LDS, one slot per lane, so the query loops run
//     with fewer live VGPRs (more waves per SIMD hide the long FP64 dependency chains).
#include "rrt_device.h"

namespace rrt {

// per-lane LDS slots, structure-of-arrays (consecutive lanes hit consecutive banks)
struct ColdLds {
  double s1[256], s2[256];
  float rr[256], rg[256], rb[256];
  double hp[3][256], nn[3][256], wo[3][256];
};

template <class T>
__device__ __forceinline__ void lput(T* a, uint32_t i, T v) { ((volatile T*)a)[i] = v; }
template <class T>
__device__ __forceinline__ T lget(const T* a, uint32_t i) { return ((const volatile T*)a)[i]; }

// estimate_direct_lighting_importance (part1_code.cpp:33-57); the camera-hit record is parked in
// LDS across every shadow query and re-read per light sample.
template <bool COUNT, bool LEAN>
__device__ spec direct_importance_lds(const KParams& kp, Rng& g, const Isect& is0, ColdLds& cl, uint32_t t,
                                      Counters& cn) {
  for (int k = 0; k < 3; ++k) {
    lput(cl.hp[k], t, (&is0.hit_p.x)[k]);
    lput(cl.nn[k], t, (&is0.n.x)[k]);
    lput(cl.wo[k], t, (&is0.w_out.x)[k]);
  }
  const uint32_t bsdf = (uint32_t)is0.bsdf;
  spec L = S(0, 0, 0);
  int total = 0;
  for (uint32_t li = 0; li < kp.n_lights; ++li) {
    const uint32_t is_delta_l = kp.lights[li].is_delta;
    const int num = is_delta_l ? 1 : (int)kp.ns_area_light;
    total += num;
    for (int i = 0; i < num; ++i) {
      const v3 hp = V(lget(cl.hp[0], t), lget(cl.hp[1], t), lget(cl.hp[2], t));
      const v3 nn = V(lget(cl.nn[0], t), lget(cl.nn[1], t), lget(cl.nn[2], t));
      const v3 wo = V(lget(cl.wo[0], t), lget(cl.wo[1], t), lget(cl.wo[2], t));
      v3 wi_world; float dist, pdf;
      const spec sample = light_sample_L<LEAN>(kp.lights[li], g, hp, wi_world, dist, pdf);
      const Frame f = coord_space(nn);
      const v3 w_in = to_local(f, wi_world);
      if (w_in.z < 0) continue;
      const spec contrib = ((sample * bsdf_f<LEAN>(kp.bsdfs[bsdf], to_local(f, wo), w_in)) * (float)w_in.z) / pdf;
      if (!query<true, COUNT>(kp, hp + smul(EPS_D, wi_world), wi_world, nullptr, cn)) L = L + contrib;
    }
  }
  return L / (float)total;
}

// estimate_direct_lighting_hemisphere (part1_code.cpp:15-31)
template <bool COUNT>
__device__ spec direct_hemisphere_lds(const KParams& kp, Rng& g, const Isect& is0, ColdLds& cl, uint32_t t,
                                      Counters& cn) {
  for (int k = 0; k < 3; ++k) {
    lput(cl.hp[k], t, (&is0.hit_p.x)[k]);
    lput(cl.nn[k], t, (&is0.n.x)[k]);
    lput(cl.wo[k], t, (&is0.w_out.x)[k]);
  }
  const uint32_t bsdf = (uint32_t)is0.bsdf;
  const int num = (int)(kp.n_lights * kp.ns_area_light);
  spec L = S(0, 0, 0);
  for (int i = 0; i < num; ++i) {
    const v3 hp = V(lget(cl.hp[0], t), lget(cl.hp[1], t), lget(cl.hp[2], t));
    const v3 nn = V(lget(cl.nn[0], t), lget(cl.nn[1], t), lget(cl.nn[2], t));
    const v3 wo = V(lget(cl.wo[0], t), lget(cl.wo[1], t), lget(cl.wo[2], t));
    const Frame f = coord_space(nn);
    const v3 w_in = hemisphere_sample(g);
    const v3 wi_world = to_world(f, w_in);
    const spec fw = bsdf_f(kp.bsdfs[bsdf], to_local(f, wo), w_in);
    Isect is2;
    if (query<false, COUNT>(kp, hp + smul(EPS_D, wi_world), wi_world, &is2, cn))
      L = L + (emission(kp.bsdfs[is2.bsdf]) * fw) * (float)w_in.z;
  }
  return ((L * 2.0f) * (float)PI_D) / (float)num;
}

}  // namespace rrt

// COUNT: per-pixel work counters; LEAN: area lights only, no microfacet BSDF, importance-sampled
// direct light (the BASELINE scenes); WAVES: register budget (minimum waves per SIMD).
template <bool COUNT, bool LEAN, int WAVES>
__global__ __launch_bounds__(256, WAVES) void rrt_sample_kernel(KParams kp) {
  using namespace rrt;
  __shared__ ColdLds cl;
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & 63u;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
  const uint32_t bpt = kp.blocks_per_tile_side;
  const uint32_t tpix = kp.tile_size * kp.tile_size;
  const DCamera& cam = kp.cam;

  uint32_t pool_blk = 0, pool_next = 64;  // wave-uniform pixel pool (one 8x8 block)
  bool pool_empty = false;
  bool have = false;                      // lane holds a pixel
  uint32_t px = 0, py = 0, slot = 0;
  int i = 0;                              // samples done for the lane's pixel
  Rng g; g.key = 0; g.ctr = 0;
  Counters cn = {0, 0, 0, 0};

  for (;;) {
    // ---- refill lanes without a pixel (wave-uniform control flow)
    for (;;) {
      const uint64_t need = __ballot(!have);
      if (need == 0 || pool_empty) break;
      if (pool_next >= 64) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(kp.block_counter, 1u);
        b = __shfl(b, 0);
        if (b >= kp.n_blocks) { pool_empty = true; break; }
        pool_blk = b;
        pool_next = 0;
      }
      const uint32_t avail = 64u - pool_next;
      const uint32_t rank = (uint32_t)__popcll(need & lt_mask);
      if (!have && rank < avail) {
        const uint32_t k = pool_next + rank;
        const uint32_t tl = pool_blk / (bpt * bpt), b = pool_blk % (bpt * bpt);
        const uint32_t lx = (b % bpt) * 8 + (k & 7u), ly = (b / bpt) * 8 + (k >> 3);
        const uint32_t x = kp.tiles[2 * tl] + lx, y = kp.tiles[2 * tl + 1] + ly;
        if (lx < kp.tile_size && ly < kp.tile_size && x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 &&
            y < kp.clip_y1) {
          px = x; py = y; slot = tl * tpix + ly * kp.tile_size + lx;
          g.key = rrt_pixel_key(kp.seed, x, y); g.ctr = 0;
          i = 0;
          cn.bbox = 0; cn.micro = 0; cn.prim = 0; cn.query = 0;
          lput(cl.s1, t, 0.0); lput(cl.s2, t, 0.0);
          lput(cl.rr, t, 0.0f); lput(cl.rg, t, 0.0f); lput(cl.rb, t, 0.0f);
          have = true;
          if (kp.ns_aa == 0) {  // the reference's loop does not run: ret / 0, count 0
            const float r = 0.0f / (float)0;
            kp.rgb[3 * slot] = r; kp.rgb[3 * slot + 1] = r; kp.rgb[3 * slot + 2] = r;
            kp.count[slot] = 0;
            if (kp.draws) kp.draws[slot] = 0;
            have = false;
          }
        }
      }
      const uint32_t n_need = (uint32_t)__popcll(need);
      pool_next += (n_need < avail) ? n_need : avail;
    }
    if (__ballot(have) == 0) break;
    if (!have) continue;

    // ---- one camera sample (raytrace_pixel loop body, part1_code.cpp:131-159)
    double sx = (double)px, sy = (double)py;
    if (kp.ns_aa == 1) { sx += 0.5; sy += 0.5; }
    else { double jx, jy; g.grid(jx, jy); sx += jx; sy += jy; }
    const double cx = sx / kp.frame_w, cy = sy / kp.frame_h;  // Camera::generate_ray (:182-187)
    const double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
    const v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
    spec s = S(0, 0, 0);
    {
      Isect is;
      if (query<false, COUNT>(kp, ld3(cam.pos), unit(w), &is, cn)) {  // est_radiance (:103-123)
        const spec e = emission(kp.bsdfs[is.bsdf]);
        if (kp.max_ray_depth == 0) s = e;
        else if (LEAN) s = e + direct_importance_lds<COUNT, true>(kp, g, is, cl, t, cn);
        else if (kp.direct_hemisphere) s = e + direct_hemisphere_lds<COUNT>(kp, g, is, cl, t, cn);
        else s = e + direct_importance_lds<COUNT, false>(kp, g, is, cl, t, cn);
      }
    }
    const spec ret = S(lget(cl.rr, t), lget(cl.rg, t), lget(cl.rb, t)) + s;
    const double il = illum(s);
    const double s1 = lget(cl.s1, t) + il, s2 = lget(cl.s2, t) + il * il;
    ++i;
    bool stop = i >= (int)kp.ns_aa;
    if ((uint32_t)i % kp.samples_per_batch == 0) {  // ADAPTIVE == 1 (:147-158)
      const double avg = s1 / i, sd = sqrt((s2 - avg * s1) / (i - 1));
      if (1.96 * sd / sqrt((double)i) <= (double)kp.max_tolerance * avg) stop = true;
    }
    if (stop) {
      const spec r = ret / (float)i;
      kp.rgb[3 * slot] = r.r; kp.rgb[3 * slot + 1] = r.g; kp.rgb[3 * slot + 2] = r.b;
      kp.count[slot] = i;
      if (kp.draws) kp.draws[slot] = g.ctr;
      if (COUNT && kp.counters) {
        kp.counters[4 * slot] = cn.bbox; kp.counters[4 * slot + 1] = cn.micro;
        kp.counters[4 * slot + 2] = cn.prim; kp.counters[4 * slot + 3] = cn.query;
      }
      have = false;
    } else {
      lput(cl.s1, t, s1); lput(cl.s2, t, s2);
      lput(cl.rr, t, ret.r); lput(cl.rg, t, ret.g); lput(cl.rb, t, ret.b);
    }
  }
}

hipError_t rrt_launch_sample(const KParams& kp, int count, int lean, int waves, uint32_t grid, hipStream_t stream) {
#define RRT_LAUNCH(C, L, W) hipLaunchKernelGGL((rrt_sample_kernel<C, L, W>), dim3(grid), dim3(256), 0, stream, kp)
  if (count) {
    RRT_LAUNCH(true, false, 1);
  } else if (lean) {
    switch (waves) {
      case 2: RRT_LAUNCH(false, true, 2); break;
      case 4: RRT_LAUNCH(false, true, 4); break;
      case 5: RRT_LAUNCH(false, true, 5); break;
      default: RRT_LAUNCH(false, true, 3); break;
    }
  } else {
    RRT_LAUNCH(false, false, 2);
  }
#undef RRT_LAUNCH
  return hipGetLastError();
}
