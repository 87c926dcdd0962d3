// rrt_path.hip -- the bounce paths (max_ray_depth >= 2) as a ray pool per wave.
//
// Reference: PathTracer::raytrace_pixel (part1_code.cpp:125-163) -> est_radiance_global_illumination
// (:103-123) -> at_least_one_bounce_radiance (:69-101) -> estimate_direct_lighting_importance /
// _hemisphere (:15-57), every ray through BVHAccel::intersect (bvh.cpp:103-138, geodesic march).
//
// Why a pool: one lane per pixel running the whole recursion (rrt_kernel.hip) keeps a lane idle
// whenever its path ended early, missed, or waits on a shadow ray the others do not have -- 21% of
// the VALU lanes active on m3 -- and holds the recursion's per-level terms in registers that spill.
// Here a lane owns a path (one pixel's samples, in order) but does not trace it:
//   * path phase (lane = path): consume the results of the path's rays, run the integrator up to
//     its next rays -- a direct-light ray (R0) and/or a camera or bounce ray (R1) -- and park their
//     directions in LDS.  Every RNG draw happens here, in the reference's order on the path's own
//     counter, so the draws never depend on which lane traces what.
//   * trace phase (lane = ray): the wave's pending rays, R0s first, are dealt one per lane and
//     marched with one shared query call (shadow or closest-hit chosen per lane at run time), the
//     results written back to the owners' LDS slots.  Rays left over wait for the next round.
// A vertex's direct-light rays go out one per round; its last one goes out together with the
// bounce ray (its draws follow the light samples').  The per-level terms of the recursion
// (L_out, the BSDF sample, cos / pdf, the child's emission) go to a global per-path stack and are
// folded back in the reference's order when the path ends (rrt_integrator.h at_least_one_bounce).
// A wave never waits on another wave: no block barrier anywhere.
// No calls in this kernel: a call makes the caller keep its live values in the callee-saved
// registers or spill them, and an out-of-line callee save the ones it touches on every entry --
// the path phase out of line saved ~100 registers to scratch each round.  So the host C library
// restatements (rrt_glibm.h) and the query are inlined here, as is the path phase.
#define RRT_GLIBM_ENTRY __device__ __forceinline__
#define RRT_QUERY_ATTR __device__ __forceinline__
#include "rrt_integrator.h"

// RRT_PATH_FIELDS (rrt_internal.h) floats a level: L_out (3), BSDF sample (3), child emission (3),
// cos, pdf, delta flag

namespace rrt {

struct PathLds {
  double d0[3][256];  // R0: direction of the direct-light ray (origin: the vertex + EPS d)
  double d1[3][256];  // R1: direction of the camera ray or of the bounce ray
  double hp[3][256], nn[3][256], wo[3][256];  // the path's current hit record (its vertex)
  uint8_t bsdf[256];  // (RRT_MAX_BSDFS 64)
  uint8_t res0[256];  // R0: occluded (importance) / hit BSDF + 1, 0 on a miss (hemisphere)
  uint8_t res1[256];  // R1: hit
  uint8_t cam[256];   // R1 is a camera ray
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <class T>
__device__ __forceinline__ void pput(T* a, uint32_t i, T v) { ((volatile T*)a)[i] = v; }
template <class T>
__device__ __forceinline__ T pget(const T* a, uint32_t i) { return ((const volatile T*)a)[i]; }

// the n-th (from 0) set bit of m; n < popcount(m)
__device__ __forceinline__ uint32_t nth_bit(uint64_t m, uint32_t n) {
  uint32_t pos = 0;
#pragma unroll
  for (int w = 32; w > 0; w >>= 1) {
    const uint64_t lo = m & ((1ull << w) - 1ull);
    const uint32_t c = (uint32_t)__popcll(lo);
    if (n >= c) { n -= c; m >>= w; pos += (uint32_t)w; } else { m = lo; }
  }
  return pos;
}

enum : uint32_t { P_IDLE = 0, P_CAM = 1, P_VTX = 2 };
// OwnLds::fl bits; recursion level k in bits 12..15, remaining depth in 16..20, light samples
// drawn at the vertex in 21..31 (the host keeps n_lights x ns_area_light < 2048)
enum : uint32_t { F_R0 = 1u, F_BOUT = 2u, F_LDRAWN = 4u, F_DECIDED = 8u, F_DELTA = 16u };
// the owned path's integrator state between its rounds (lane = path); with PathLds 40 KB a
// block, so four blocks (4 waves/SIMD) fit a CU's 160 KB
struct OwnLds {
  uint32_t ctr[256];     // the pixel's RNG counter (its key is rederived from the pixel)
  uint32_t fl[256];      // vertex progress (F_*), level, depth, light samples drawn
  float lv[3][256];      // the vertex's direct light so far
  float c3[3][256];      // the outstanding R0's contribution (importance) or f (hemisphere)
  float cz[256];         // ... its cos (hemisphere)
};

}  // namespace rrt

// The shadow-ray occlusion proof's build tag for this kernel (rrt_device.h query_nx / occ_exit_call)
#define RRT_OCC_TAG_PATH(WAVES) (512 + (WAVES))

namespace rrt {

// the block's ray slots and owned-path state (one kernel in this unit uses them)
__shared__ PathLds pl;
__shared__ OwnLds ol;

// per-path global slots: level `lv` of the recursion's terms, and the pixel record (level
// max_ray_depth: pixel, output slot, samples, sums, the sample's emission)
__device__ __forceinline__ float* stk(const KParams& kp, uint32_t lv, uint32_t field) {
  return kp.path_stack + ((size_t)(lv * RRT_PATH_FIELDS + field) * (gridDim.x * 256u) + blockIdx.x * 256u + threadIdx.x);
}
__device__ __forceinline__ uint32_t* rec(const KParams& kp, uint32_t field) {
  return (uint32_t*)stk(kp, kp.max_ray_depth, field);
}
// Camera::generate_ray at the sample's jitter (part1_code.cpp:132-141, 182-187) into R1
__device__ __forceinline__ void start_sample(const KParams& kp, Rng& g, uint32_t t) {
  const DCamera& cam = kp.cam;
  const uint32_t pxy = *rec(kp, 0);
  double sx = (double)(pxy & 0xffffu), sy = (double)(pxy >> 16);
  if (kp.ns_aa == 1) { sx += 0.5; sy += 0.5; }
  else { double jx, jy; g.grid(jx, jy); sx += jx; sy += jy; }
  const double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
  const double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
  const v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
  const v3 d = unit(w);
  pput(pl.d1[0], t, d.x); pput(pl.d1[1], t, d.y); pput(pl.d1[2], t, d.z);
  pput(pl.cam, t, (uint8_t)1u);
}

// The path phase of one path whose rays are all back: consume their results and run the
// integrator up to the path's next rays.  Returns the new state (P_*) | R0 pending << 4 | R1
// pending << 5; the rest of the path's state goes back to LDS and its global slots.
template <int W>
__device__ __forceinline__ uint32_t path_phase(const KParams& kp, uint32_t st) {
  const uint32_t t = threadIdx.x;
  const bool deep = kp.max_ray_depth >= 2;
  const bool hemi = kp.direct_hemisphere != 0;
  auto stk = [&](uint32_t lv, uint32_t field) -> float* { return rrt::stk(kp, lv, field); };
  auto rec = [&](uint32_t field) -> uint32_t* { return rrt::rec(kp, field); };
  bool p0 = false, p1 = false;
  uint32_t fl = pget(ol.fl, t);
  bool r0_out = fl & F_R0, b_out = fl & F_BOUT, lights_drawn = fl & F_LDRAWN, decided = fl & F_DECIDED,
       dl = fl & F_DELTA;
  uint32_t k = (fl >> 12) & 15u, depth = (fl >> 16) & 31u, lj = fl >> 21, nsh = 0;
  spec Lv = S(pget(ol.lv[0], t), pget(ol.lv[1], t), pget(ol.lv[2], t));
  const uint32_t pxy = *rec(0);
  Rng g; g.key = rrt_pixel_key(kp.seed, pxy & 0xffffu, pxy >> 16); g.ctr = pget(ol.ctr, t);
  auto vertex_begin = [&]() {  // the hit record in LDS is the vertex
    st = P_VTX;
    dl = is_delta(kp.bsdfs[pget(pl.bsdf, t)]);
    Lv = S(0, 0, 0);
    lj = 0;
    // depth >= 2 takes direct light only at non-delta vertices (:75-77); one_bounce_radiance
    // at depth 1 always samples it (a delta BSDF's f is zero)
    lights_drawn = deep && dl;
    decided = false; b_out = false; r0_out = false;
  };
  bool fin = false;
  spec s = S(0, 0, 0);
  if (st == P_CAM) {  // est_radiance_global_illumination (:103-123) on the camera ray's result
    if (!pget(pl.res1, t)) {
      fin = true;
      if (kp.env.w) s = env_dir(kp.env, V(pget(pl.d1[0], t), pget(pl.d1[1], t), pget(pl.d1[2], t)));
    } else {
      const spec e0 = emission(kp.bsdfs[pget(pl.bsdf, t)]);
      if (kp.max_ray_depth == 0) {
        fin = true;
        s = e0;
      } else {
        ((float*)rec(10))[0] = e0.r; ((float*)rec(11))[0] = e0.g; ((float*)rec(12))[0] = e0.b;
        k = 0;
        depth = kp.max_ray_depth;
        vertex_begin();
      }
    }
  } else if (r0_out) {  // the outstanding direct-light ray's result
    r0_out = false;
    const uint32_t r = pget(pl.res0, t);
    const spec c3 = S(pget(ol.c3[0], t), pget(ol.c3[1], t), pget(ol.c3[2], t));
    if (hemi) {
      if (r) Lv = Lv + (emission(kp.bsdfs[r - 1u]) * c3) * pget(ol.cz, t);
    } else if (!r) {
      Lv = Lv + c3;
    }
  }
  // light samples at the vertex (estimate_direct_lighting_*: n_lights x ns_area_light, one per
  // delta light with importance sampling)
  if (st == P_VTX) {
    if (hemi) {
      nsh = kp.n_lights * kp.ns_area_light;
    } else {
      for (uint32_t l = 0; l < kp.n_lights; ++l) nsh += kp.lights[l].is_delta ? 1u : kp.ns_area_light;
    }
  }
  while (!fin && st == P_VTX) {
    // the vertex's next light samples (:15-57) up to one that needs a ray (R0)
    while (!lights_drawn && lj < nsh) {
      const v3 hp = V(pget(pl.hp[0], t), pget(pl.hp[1], t), pget(pl.hp[2], t));
      const v3 nn = V(pget(pl.nn[0], t), pget(pl.nn[1], t), pget(pl.nn[2], t));
      const v3 wo = V(pget(pl.wo[0], t), pget(pl.wo[1], t), pget(pl.wo[2], t));
      const DBsdf b = kp.bsdfs[pget(pl.bsdf, t)];
      const Frame f = coord_space(nn);
      const uint32_t jj = lj++;
      v3 wi;
      spec c3;
      if (hemi) {
        const v3 w_in = hemisphere_sample(g);
        wi = to_world(f, w_in);
        c3 = bsdf_f(b, to_local(f, wo), w_in);
        pput(ol.cz, t, (float)w_in.z);
      } else {
        uint32_t li = 0, r = jj;  // light and sample of flat index jj
        for (;; ++li) {
          const uint32_t num = kp.lights[li].is_delta ? 1u : kp.ns_area_light;
          if (r < num) break;
          r -= num;
        }
        float dist, pdf;
        const spec smp = light_sample_L<0>(kp.env, kp.lights[li], g, hp, wi, dist, pdf);
        const v3 w_in = to_local(f, wi);
        if (w_in.z < 0) continue;
        c3 = ((smp * bsdf_f<0>(b, to_local(f, wo), w_in)) * (float)w_in.z) / pdf;
      }
      pput(ol.c3[0], t, c3.r); pput(ol.c3[1], t, c3.g); pput(ol.c3[2], t, c3.b);
      pput(pl.d0[0], t, wi.x); pput(pl.d0[1], t, wi.y); pput(pl.d0[2], t, wi.z);
      p0 = true;
      r0_out = true;
      break;
    }
    if (lj >= nsh) lights_drawn = true;
    // the bounce (:85-99) once every light sample is drawn: Russian roulette, the BSDF sample
    if (lights_drawn && !decided) {
      decided = true;
      if (deep && (depth == kp.max_ray_depth || (depth > 1 && g.coin(0.7)))) {
        const v3 nn = V(pget(pl.nn[0], t), pget(pl.nn[1], t), pget(pl.nn[2], t));
        const v3 wo = V(pget(pl.wo[0], t), pget(pl.wo[1], t), pget(pl.wo[2], t));
        const DBsdf b = kp.bsdfs[pget(pl.bsdf, t)];
        const Frame f = coord_space(nn);
        v3 w_in;
        float pdf;
        const spec smp = bsdf_sample_f(b, g, to_local(f, wo), w_in, pdf);
        if (pdf != 0.0f) {
          const v3 wi = to_world(f, w_in);
          pput(pl.d1[0], t, wi.x); pput(pl.d1[1], t, wi.y); pput(pl.d1[2], t, wi.z);
          pput(pl.cam, t, (uint8_t)0u);
          p1 = true;
          b_out = true;
          *stk(k, 3) = smp.r; *stk(k, 4) = smp.g; *stk(k, 5) = smp.b;
          *stk(k, 9) = (float)fabs(w_in.z); *stk(k, 10) = pdf;
        }
      }
    }
    if (p0 || p1) break;
    // the vertex is complete: its direct light, then its bounce's result
    spec Ld = hemi ? ((Lv * 2.0f) * (float)PI_D) / (float)nsh : Lv / (float)nsh;
    if (!deep) {  // max_ray_depth 1: e + one_bounce_radiance
      s = S(*(float*)rec(10), *(float*)rec(11), *(float*)rec(12)) + Ld;
      fin = true;
      break;
    }
    Ld = dl ? S(0, 0, 0) : S(0, 0, 0) + Ld;
    if (b_out && pget(pl.res1, t) && k + 1 < RRT_MAX_DEPTH) {  // the child level
      const spec ce = emission(kp.bsdfs[pget(pl.bsdf, t)]);
      *stk(k, 0) = Ld.r; *stk(k, 1) = Ld.g; *stk(k, 2) = Ld.b;
      *stk(k, 6) = ce.r; *stk(k, 7) = ce.g; *stk(k, 8) = ce.b;
      *stk(k, 11) = dl ? 1.0f : 0.0f;
      ++k;
      --depth;
      vertex_begin();
      continue;
    }
    // fold the levels back up in the reference's order (rrt_integrator.h at_least_one_bounce)
    spec L = Ld;
    for (int j = (int)k - 1; j >= 0; --j) {
      spec Lj = S(*stk(j, 0), *stk(j, 1), *stk(j, 2));
      spec Lc = L;
      if (*stk(j, 11) != 0.0f) Lc = Lc + S(*stk(j, 6), *stk(j, 7), *stk(j, 8));
      Lj = Lj + (((Lc * S(*stk(j, 3), *stk(j, 4), *stk(j, 5))) * *stk(j, 9)) / *stk(j, 10)) / (float)0.7;
      L = Lj;
    }
    s = S(*(float*)rec(10), *(float*)rec(11), *(float*)rec(12)) + L;
    fin = true;
  }
  if (fin) {  // raytrace_pixel's loop body after the sample (:142-158)
    spec ret = S(*(float*)rec(3), *(float*)rec(4), *(float*)rec(5));
    double s1 = __hiloint2double((int)*rec(7), (int)*rec(6)), s2 = __hiloint2double((int)*rec(9), (int)*rec(8));
    const int n = (int)*rec(2) + 1;
    ret = ret + s;
    const double il = illum(s);
    s1 += il;
    s2 += il * il;
    bool stop = n >= (int)kp.ns_aa;
    if ((uint32_t)n % kp.samples_per_batch == 0) {  // ADAPTIVE 1
      const double avg = s1 / n, sd = sqrt((s2 - avg * s1) / (n - 1));
      if (1.96 * sd / sqrt((double)n) <= (double)kp.max_tolerance * avg) stop = true;
    }
    if (stop) {
      const uint32_t slot = *rec(1);
      const spec r = ret / (float)n;
      kp.rgb[3 * slot] = r.r; kp.rgb[3 * slot + 1] = r.g; kp.rgb[3 * slot + 2] = r.b;
      kp.count[slot] = n;
      if (kp.draws) kp.draws[slot] = g.ctr;
      st = P_IDLE;
    } else {
      *(float*)rec(3) = ret.r; *(float*)rec(4) = ret.g; *(float*)rec(5) = ret.b;
      *rec(6) = (uint32_t)__double2loint(s1); *rec(7) = (uint32_t)__double2hiint(s1);
      *rec(8) = (uint32_t)__double2loint(s2); *rec(9) = (uint32_t)__double2hiint(s2);
      *rec(2) = (uint32_t)n;
      start_sample(kp, g, t);
      p1 = true;
      st = P_CAM;
    }
  }
  pput(ol.fl, t, (r0_out ? F_R0 : 0u) | (b_out ? F_BOUT : 0u) | (lights_drawn ? F_LDRAWN : 0u) |
                     (decided ? F_DECIDED : 0u) | (dl ? F_DELTA : 0u) | (k << 12) | (depth << 16) | (lj << 21));
  pput(ol.lv[0], t, Lv.r); pput(ol.lv[1], t, Lv.g); pput(ol.lv[2], t, Lv.b);
  pput(ol.ctr, t, g.ctr);
  return st | (p0 ? 16u : 0u) | (p1 ? 32u : 0u);
}

}  // namespace rrt

#if RRT_PROFILE
// diagnostic build: wave cycles in the path phase, the claims and the trace phase; rounds; rays
// traced; waves (tools/path_profile.py)
__device__ unsigned long long rrt_prof_path[8];
extern "C" int rrt_prof_read_path(unsigned long long* out) {  // out: 8; resets
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rrt_prof_path), sizeof(rrt_prof_path)) != hipSuccess) return -1;
  unsigned long long z[8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(rrt_prof_path), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void rrt_path_kernel(const KParams* __restrict__ kpp0) {
  using namespace rrt;
  const KParams* kpp = kpp0;
  const uint32_t t = threadIdx.x, lane = t & 63u, wb = t - lane;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t n_claims = kpp0->claim_list ? *kpp0->claim_count : kpp0->n_pixels;
  Counters cn = {};

  // loop control stays in registers; the owned path's state lives in LDS (OwnLds) and its
  // global slots, so none of it is live across the trace phase's query
  uint32_t st = P_IDLE;
  bool done = false;            // the claim space is exhausted
  bool p0 = false, p1 = false;  // rays waiting to be traced

#if RRT_PROFILE
  unsigned long long pc_path = 0, pc_claim = 0, pc_trace = 0, pc_rays = 0, pc_rounds = 0;
#endif
  for (;;) {  // one round
    // The launch constants are re-read from the constant cache each round: hoisted out of the loop
    // they would all stay live (in VGPRs, once the SGPRs run out) across the query
    asm volatile("" : "+s"(kpp));
    const KParams& kp = *kpp;
    const uint32_t ts = kp.tile_size, tpix = ts * ts;
    const bool hemi = kp.direct_hemisphere != 0;
    const DCamera& cam = kp.cam;
    auto rec = [&](uint32_t field) -> uint32_t* { return rrt::rec(kp, field); };
#if RRT_PROFILE
    const unsigned long long pc0 = clock64();
#endif
    // ---- path phase: each path whose rays are all back runs to its next rays
    if (st != P_IDLE && !p0 && !p1) {
      const uint32_t r = path_phase<WAVES>(kp, st);
      st = r & 15u;
      p0 = (r >> 4) & 1u;
      p1 = (r >> 5) & 1u;
    }

#if RRT_PROFILE
    const unsigned long long pc1 = clock64();
    pc_path += pc1 - pc0;
#endif
    // ---- claims: one atomic per wave for every path that needs a pixel
    const uint64_t need = __ballot(st == P_IDLE && !done);
    if (need) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(kp.block_counter, (uint32_t)__popcll(need));
      base = __shfl(base, 0);
      if (st == P_IDLE && !done) {
        const uint32_t c = base + (uint32_t)__popcll(need & lt);
        if (c >= n_claims) {
          done = true;
        } else {
          const uint32_t ix = kp.claim_list ? (kp.claim_list[c] & 0x7fffffffu) : c;
          const uint32_t pi = ix < kp.n_pixels ? ix : 0u;
          const uint32_t tl = kp.tile_order[pi / tpix], r = claim_r(pi % tpix, ts);
          const uint32_t x = kp.tiles[2 * tl] + r % ts, y = kp.tiles[2 * tl + 1] + r / ts;
          if (ix < kp.n_pixels && x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 && y < kp.clip_y1) {
            *rec(0) = x | (y << 16);
            *rec(1) = tl * tpix + r;
            *rec(2) = 0u;
            *(float*)rec(3) = 0.0f; *(float*)rec(4) = 0.0f; *(float*)rec(5) = 0.0f;
            *rec(6) = 0u; *rec(7) = 0u; *rec(8) = 0u; *rec(9) = 0u;
            Rng g; g.key = rrt_pixel_key(kp.seed, x, y); g.ctr = 0;
            start_sample(kp, g, t);
            p1 = true;
            st = P_CAM;
            pput(ol.ctr, t, g.ctr);
            pput(ol.fl, t, 0u);
          }
        }
      }
    }
#if RRT_PROFILE
    const unsigned long long pc2 = clock64();
    pc_claim += pc2 - pc1;
#endif
    if (__ballot(st != P_IDLE || !done) == 0) break;

    // ---- trace phase: one ray per lane.  R0 rays first (each reads its vertex before an R1 of the
    // same path may replace it), then the R1 rays of paths waiting on nothing else, then those
    // of paths whose R0 goes out this round.  Every path not counted in the R0s is one slot, so
    // the first two kinds always fit: no ray waits more than one round.
    wave_sync();
    const uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
    const uint64_t b1a = b1 & ~b0, b1b = b1 & b0;
    const uint32_t n0 = (uint32_t)__popcll(b0), n1a = (uint32_t)__popcll(b1a), n1b = (uint32_t)__popcll(b1b);
    if (n0 + n1a + n1b == 0) continue;
    uint32_t rp = 64u;  // the path whose ray this lane traces
    bool rs1 = false;
    if (lane < n0) {
      rp = nth_bit(b0, lane);
    } else if (lane - n0 < n1a) {
      rp = nth_bit(b1a, lane - n0);
      rs1 = true;
    } else if (lane - n0 - n1a < n1b) {
      rp = nth_bit(b1b, lane - n0 - n1a);
      rs1 = true;
    }
    const bool took1 = p1 && (!p0 || n0 + n1a + (uint32_t)__popcll(b1b & lt) < 64u);
    v3 o = V(0, 0, 0), d = V(0, 0, 0);
    bool cray = false, any = false;
    if (rp < 64u) {
      const uint32_t q = wb + rp;
      if (rs1) {
        d = V(pget(pl.d1[0], q), pget(pl.d1[1], q), pget(pl.d1[2], q));
        cray = pget(pl.cam, q) != 0u;
      } else {
        d = V(pget(pl.d0[0], q), pget(pl.d0[1], q), pget(pl.d0[2], q));
        any = !hemi;
      }
      o = cray ? ld3(cam.pos) : V(pget(pl.hp[0], q), pget(pl.hp[1], q), pget(pl.hp[2], q)) + smul(EPS_D, d);
    }
    wave_sync();
    Isect is;
    bool h = false;
    if (rp < 64u) {
      bool known = false;
      if (cray) {
        known = camera_proven_miss<false, false>(kp, o, d, cn);
      } else if (any && kp.occ.on) {
        h = shadow_occluded_proof<RRT_OCC_TAG_PATH(WAVES)>(kp, o, d, kp.hole.steps);
        known = h;
      }
      if (!known) h = query<false, false, false, false>(kp, o, d, &is, cn, any);
      const uint32_t q = wb + rp;
      if (rs1) {
        pput(pl.res1, q, (uint8_t)(h ? 1u : 0u));
        if (h) {
          pput(pl.hp[0], q, is.hit_p.x); pput(pl.hp[1], q, is.hit_p.y); pput(pl.hp[2], q, is.hit_p.z);
          pput(pl.nn[0], q, is.n.x); pput(pl.nn[1], q, is.n.y); pput(pl.nn[2], q, is.n.z);
          pput(pl.wo[0], q, is.w_out.x); pput(pl.wo[1], q, is.w_out.y); pput(pl.wo[2], q, is.w_out.z);
          pput(pl.bsdf, q, (uint8_t)is.bsdf);
        }
      } else {
        pput(pl.res0, q, (uint8_t)(any ? (h ? 1u : 0u) : (h ? (uint32_t)is.bsdf + 1u : 0u)));
      }
    }
    wave_sync();
    p0 = false;  // every R0 was dealt (at most 64)
    if (took1) p1 = false;
#if RRT_PROFILE
    pc_trace += clock64() - pc2;
    pc_rays += min(n0 + n1a + n1b, 64u);
    ++pc_rounds;
#endif
  }
#if RRT_PROFILE
  if (lane == 0) {
    atomicAdd(&rrt_prof_path[0], pc_path); atomicAdd(&rrt_prof_path[1], pc_claim);
    atomicAdd(&rrt_prof_path[2], pc_trace); atomicAdd(&rrt_prof_path[3], pc_rounds);
    atomicAdd(&rrt_prof_path[4], pc_rays); atomicAdd(&rrt_prof_path[5], 1ull);
  }
#endif
}

hipError_t rrt_launch_path(const KParams* d_kp, int waves, uint32_t grid, hipStream_t stream) {
#define RRT_LAUNCH(W) hipLaunchKernelGGL((rrt_path_kernel<W>), dim3(grid), dim3(256), 0, stream, d_kp)
  switch (waves) {
    case 2: RRT_LAUNCH(2); break;
    case 3: RRT_LAUNCH(3); break;
    default: RRT_LAUNCH(4); break;
  }
#undef RRT_LAUNCH
  return hipGetLastError();
}
