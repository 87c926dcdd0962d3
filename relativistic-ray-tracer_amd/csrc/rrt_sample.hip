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
#include "rrt_integrator.h"

namespace rrt {

// per-lane LDS slots, structure-of-arrays (consecutive lanes hit consecutive banks), N lanes per block
template <uint32_t N>
struct ShadeLdsN {  // the camera hit being shaded, parked across its shadow queries
  double hp[3][N], nn[3][N], wo[3][N];
  uint32_t bsdf[N];
  float cr[N], cg[N], cb[N];  // a light sample's contribution, parked across its shadow query
                              // (the batch kernel's fold then reads each sample's radiance here)
};
using ShadeLds = ShadeLdsN<256>;
struct ColdLds : ShadeLds {  // + the per-pixel sums of the lane-per-pixel kernel
  double s1[256], s2[256];
  float rr[256], rg[256], rb[256];
};

template <class T>
__device__ __forceinline__ void lput(T* a, uint32_t i, T v) { ((volatile T*)a)[i] = v; }
template <class T>
__device__ __forceinline__ T lget(const T* a, uint32_t i) { return ((const volatile T*)a)[i]; }

// park a camera-hit record in the lane's LDS slots
template <class SL>
__device__ __forceinline__ void park_hit(SL& cl, uint32_t t, const Isect& is0) {
  for (int k = 0; k < 3; ++k) {
    lput(cl.hp[k], t, (&is0.hit_p.x)[k]);
    lput(cl.nn[k], t, (&is0.n.x)[k]);
    lput(cl.wo[k], t, (&is0.w_out.x)[k]);
  }
  lput(cl.bsdf, t, (uint32_t)is0.bsdf);
}

// estimate_direct_lighting_importance (part1_code.cpp:33-57) for the hit parked in LDS
// (park_hit), re-read per light sample so no hit state stays live across the shadow queries.
// W: the calling kernel build's tag for the out-of-line occlusion proof (rrt_device.h query_nx)
template <bool COUNT, int LEAN, int W = 0, class SL = ShadeLds>
__device__ __forceinline__ spec direct_importance_parked(const KParams& kp, Rng& g, SL& cl, uint32_t t, Counters& cn) {
  const uint32_t bsdf = lget(cl.bsdf, t);
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
      const spec sample = light_sample_L<LEAN>(kp.env, kp.lights[li], g, hp, wi_world, dist, pdf);
      const Frame f = coord_space(nn);
      const v3 w_in = to_local(f, wi_world);
      if (w_in.z < 0) continue;
      const spec contrib = ((sample * bsdf_f<LEAN>(kp.bsdfs[bsdf], to_local(f, wo), w_in)) * (float)w_in.z) / pdf;
      // only the loop state and the RNG stay in registers across the shadow query
      lput(cl.cr, t, contrib.r); lput(cl.cg, t, contrib.g); lput(cl.cb, t, contrib.b);
      if (!query_nx<true, COUNT, LEAN == V_KERR, W, is_lean(LEAN)>(kp, hp + smul(EPS_D, wi_world), wi_world, nullptr, cn))
        L = L + S(lget(cl.cr, t), lget(cl.cg, t), lget(cl.cb, t));
    }
  }
  return L / (float)total;
}
template <bool COUNT, int LEAN, int W = 0>
__device__ __forceinline__ spec direct_importance_lds(const KParams& kp, Rng& g, const Isect& is0, ColdLds& cl, uint32_t t,
                                      Counters& cn) {
  park_hit(cl, t, is0);
  return direct_importance_parked<COUNT, LEAN, W>(kp, g, cl, t, cn);
}

// estimate_direct_lighting_hemisphere (part1_code.cpp:15-31) for the parked hit
template <bool COUNT, int LEAN>
__device__ __forceinline__ spec direct_hemisphere_parked(const KParams& kp, Rng& g, ShadeLds& cl, uint32_t t, Counters& cn) {
  const uint32_t bsdf = lget(cl.bsdf, t);
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
    if (query_nx<false, COUNT, LEAN == V_KERR, 0, is_lean(LEAN)>(kp, hp + smul(EPS_D, wi_world), wi_world, &is2, cn))
      L = L + (emission(kp.bsdfs[is2.bsdf]) * fw) * (float)w_in.z;
  }
  return ((L * 2.0f) * (float)PI_D) / (float)num;
}
template <bool COUNT, int LEAN>
__device__ __forceinline__ spec direct_hemisphere_lds(const KParams& kp, Rng& g, const Isect& is0, ColdLds& cl, uint32_t t,
                                      Counters& cn) {
  park_hit(cl, t, is0);
  return direct_hemisphere_parked<COUNT, LEAN>(kp, g, cl, t, cn);
}

}  // namespace rrt

// The shadow-ray occlusion proof's build tag (rrt_device.h query_nx): the area-light and the
// general builds (cfg1-3; scenes with environment maps or BSDF sampling); not the point-light
// build (cfg4: its frame is the camera rays' -- 98% proven misses -- and carrying the proof's code
// cost it 10%, more than the proof saved) nor the Kerr builds (no planar recurrence).  One tag per
// kernel build (batch kernels; per-sample kernels, counting or not).
#define RRT_OCC_TAG(LEAN, WAVES) ((LEAN) == 1 || (LEAN) == 0 ? 8 * (WAVES) + (LEAN) + 1 : 0)
#define RRT_OCC_TAG_SLOT(LEAN, WAVES) ((LEAN) == 1 || (LEAN) == 0 ? 256 + 8 * (WAVES) + (LEAN) + 1 : 0)
#define RRT_OCC_TAG_S(COUNT, LEAN, WAVES) ((LEAN) == 1 || (LEAN) == 0 ? 64 + ((COUNT) ? 128 : 0) + 8 * (WAVES) + (LEAN) + 1 : 0)

#if RRT_PROFILE
// [0..7] per-phase wave cycles (busiest lane per wave, summed): total, camera queries, micro
// steps, camera walks, miss proofs, shadow queries, shadow walks, -; [8] min start, [9] max end,
// [10] waves, [11] first exhaustion (wall clock); [16..19] batch-kernel phases: claims, chain
// walks, shading, fold; then per-wave end / start / work records
#define RRT_PROF_HDR 24
__device__ unsigned long long rrt_prof[RRT_PROF_HDR];
__device__ unsigned long long rrt_prof_ends[16384], rrt_prof_starts[16384], rrt_prof_work[16384];
// slowest pixels: bucket (pixel slot % 64) keeps max(elapsed wall ticks << 24 | slot)
__device__ unsigned long long rrt_prof_slow[64];
extern "C" int rrt_prof_read_slow(unsigned long long* out) {  // out: 64; resets
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rrt_prof_slow), sizeof(rrt_prof_slow)) != hipSuccess) return -1;
  unsigned long long z[64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(rrt_prof_slow), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// per pixel slot (slot < 2^21, e.g. 1080p): elapsed wall ticks (claim to stop, 24 bits) << 8 | rounds
__device__ uint32_t rrt_prof_px[1u << 21];
// per pixel slot: the wall clock (low 32 bits) when the pixel stopped
__device__ uint32_t rrt_prof_px_end[1u << 21];
extern "C" int rrt_prof_read_px_end(uint32_t* out, uint32_t n) {  // reads min(n, 2^21) slots
  n = n < (1u << 21) ? n : (1u << 21);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rrt_prof_px_end), n * sizeof(uint32_t)) == hipSuccess ? 0 : -1;
}
extern "C" int rrt_prof_read_px(uint32_t* out, uint32_t n) {  // reads and resets min(n, 2^21) slots
  n = n < (1u << 21) ? n : (1u << 21);
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rrt_prof_px), n * sizeof(uint32_t)) != hipSuccess) return -1;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(rrt_prof_px)) != hipSuccess) return -1;
  return hipMemset(p, 0, sizeof(uint32_t) << 21) == hipSuccess ? 0 : -1;
}
extern "C" int rrt_prof_read(unsigned long long* out) {  // out: RRT_PROF_HDR + 3 * 16384
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rrt_prof), sizeof(rrt_prof)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + RRT_PROF_HDR, HIP_SYMBOL(rrt_prof_ends), sizeof(rrt_prof_ends)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + RRT_PROF_HDR + 16384, HIP_SYMBOL(rrt_prof_starts), sizeof(rrt_prof_starts)) != hipSuccess)
    return -1;
  if (hipMemcpyFromSymbol(out + RRT_PROF_HDR + 2 * 16384, HIP_SYMBOL(rrt_prof_work), sizeof(rrt_prof_work)) != hipSuccess)
    return -1;
  unsigned long long z[RRT_PROF_HDR] = {0, 0, 0, 0, 0, 0, 0, 0, ~0ull, 0, 0, ~0ull, 0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(rrt_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

// COUNT: per-pixel work counters; LEAN: area/point lights only, no microfacet BSDF, importance-sampled
// direct light (the BASELINE scenes); WAVES: register budget (minimum waves per SIMD).
// DEEP: max_ray_depth >= 2 (at_least_one_bounce_radiance, part1_code.cpp:69-101) for the general
// build; the pixels then come from the pixel miss proof pass's claim list when it ran
template <bool COUNT, int LEAN, int WAVES, bool DEEP = false>
__global__ __launch_bounds__(256, WAVES) void rrt_sample_kernel(const KParams* __restrict__ kpp) {
  const KParams& kp = *kpp;
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
  uint32_t aud = 0;  // proof audit (COUNT): bit 0 the pixel's miss proof holds, bit 1 its strip's
  int i = 0;                              // samples done for the lane's pixel
  Rng g; g.key = 0; g.ctr = 0;
  Counters cn = {};
#if RRT_PROFILE
  const uint64_t t_start = clock64(), w_start = wall_clock64();  // clock64 is per XCD; wall is global
  uint32_t prof_blocks = 0, prof_samples = 0;
#endif

  for (;;) {
    // ---- refill lanes without a pixel (wave-uniform control flow)
    for (;;) {
      const uint64_t need = __ballot(!have);
      if (need == 0 || pool_empty) break;
      if (pool_next >= 64) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(kp.block_counter, 1u);
        b = __shfl(b, 0);
        // a pool: one 8x8 block of a tile, or 64 entries of the pixel proof pass's claim list
        if (b >= (kp.claim_list ? (*kp.claim_count + 63u) / 64u : kp.n_blocks)) {
          pool_empty = true;
#if RRT_PROFILE
          if (lane == 0) atomicMin(&rrt_prof[11], (unsigned long long)wall_clock64());  // first exhaustion
#endif
          break;
        }
#if RRT_PROFILE
        ++prof_blocks;
#endif
        pool_blk = b;
        pool_next = 0;
      }
      const uint32_t avail = 64u - pool_next;
      const uint32_t rank = (uint32_t)__popcll(need & lt_mask);
      if (!have && rank < avail) {
        const uint32_t k = pool_next + rank;
        uint32_t tl, lx, ly;
        bool listed = true;
        if (kp.claim_list) {
          const uint32_t e = pool_blk * 64u + k;
          listed = e < *kp.claim_count;
          const uint32_t ix = listed ? (kp.claim_list[e] & 0x7fffffffu) : 0u;
          tl = kp.tile_order[ix / tpix];
          const uint32_t r = claim_r(ix % tpix, kp.tile_size);
          lx = r % kp.tile_size; ly = r / kp.tile_size;
        } else {
          tl = pool_blk / (bpt * bpt);
          const uint32_t b = pool_blk % (bpt * bpt);
          lx = (b % bpt) * 8 + (k & 7u); ly = (b / bpt) * 8 + (k >> 3);
        }
        const uint32_t x = kp.tiles[2 * tl] + lx, y = kp.tiles[2 * tl + 1] + ly;
        if (listed && lx < kp.tile_size && ly < kp.tile_size && x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 &&
            y < kp.clip_y1) {
          px = x; py = y; slot = tl * tpix + ly * kp.tile_size + lx;
          g.key = rrt_pixel_key(kp.seed, x, y); g.ctr = 0;
          i = 0;
          cn.bbox = 0; cn.micro = 0; cn.prim = 0; cn.query = 0;
          lput(cl.s1, t, 0.0); lput(cl.s2, t, 0.0);
          lput(cl.rr, t, 0.0f); lput(cl.rg, t, 0.0f); lput(cl.rb, t, 0.0f);
          have = true;
          aud = 0;
          // audit of the pixel pass (rrt_pixel_proof_kernel / rrt_strip_proof_kernel, whose proven
          // pixels the batch kernel never marches): on every 2^audit_shift-th pixel, whether its
          // proofs hold; every camera ray of such a pixel is then marched exactly below
          if (COUNT && kp.audit && kp.miss.on &&
              (rrt_mix64(g.key) & ((1ull << kp.audit_shift) - 1ull)) == 0ull) {
            if (pixel_miss_proof(kp, x, y)) aud |= 1u;
            const uint32_t sx = kp.tiles[2 * tl] + (lx & ~7u), sy = kp.tiles[2 * tl + 1] + (ly & ~7u);
            if (sx >= kp.clip_x0 && sy >= kp.clip_y0 && sx + 8u <= kp.clip_x1 && sy + 8u <= kp.clip_y1 &&
                rect_miss_proof(kp, (double)sx, (double)sy, 8.0, 8.0))
              aud |= 2u;
          }
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
      const v3 wd = unit(w);
      if (!camera_proven_miss<COUNT, LEAN == V_KERR>(kp, ld3(cam.pos), wd, cn) &&
          query<false, COUNT, LEAN == V_KERR, is_lean(LEAN)>(kp, ld3(cam.pos), wd, &is, cn)) {  // est_radiance (:103-123)
        const spec e = emission(kp.bsdfs[is.bsdf]);
        if (kp.max_ray_depth == 0) s = e;
        else if (DEEP && kp.max_ray_depth >= 2) s = e + at_least_one_bounce<COUNT, general_of(LEAN)>(kp, g, is, cn);
        else if (is_lean(LEAN)) s = e + direct_importance_lds<COUNT, LEAN, RRT_OCC_TAG_S(COUNT, LEAN, WAVES)>(kp, g, is, cl, t, cn);
        else if (kp.direct_hemisphere) s = e + direct_hemisphere_lds<COUNT, LEAN>(kp, g, is, cl, t, cn);
        else s = e + direct_importance_lds<COUNT, LEAN, RRT_OCC_TAG_S(COUNT, LEAN, WAVES)>(kp, g, is, cl, t, cn);
      } else if (!is_lean(LEAN) && kp.env.w) {
        s = env_dir(kp.env, unit(w));  // miss: envLight->sample_dir of the unbent camera ray
      }
      if (COUNT && aud) {  // the pixel pass's proofs say this camera ray misses
        Counters c2 = {};
        Isect i2;
        const bool ex = query<false, false, LEAN == V_KERR, is_lean(LEAN)>(kp, ld3(cam.pos), wd, &i2, c2);
        if (aud & 1u) audit_note(kp, RRT_AUDIT_PIXEL, ex);
        if (aud & 2u) audit_note(kp, RRT_AUDIT_STRIP, ex);
      }
    }
    const spec ret = S(lget(cl.rr, t), lget(cl.rg, t), lget(cl.rb, t)) + s;
    const double il = illum(s);
    const double s1 = lget(cl.s1, t) + il, s2 = lget(cl.s2, t) + il * il;
    ++i;
#if RRT_PROFILE
    ++prof_samples;
#endif
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
#if RRT_PROFILE
  // wave time per phase ~ the busiest lane's; summed over waves (tools/phase_profile.py)
  const uint64_t t_end = clock64(), w_end = wall_clock64();
  uint64_t v[8] = {t_end - t_start, cn.t_query, cn.t_micro, cn.t_trav, cn.t_proof, cn.t_squery, cn.t_strav, 0};
  for (int k = 0; k < 8; ++k) {
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t o2 = __shfl_xor(v[k], off);
      v[k] = v[k] > o2 ? v[k] : o2;
    }
    if (lane == 0) atomicAdd(&rrt_prof[k], (unsigned long long)v[k]);
  }
  uint32_t ns = prof_samples;
  for (int off = 32; off > 0; off >>= 1) ns += __shfl_xor(ns, off);
  if (lane == 0) {  // [4] min start, [5] max end, [6] waves, [7] first exhaustion; per-wave records
    atomicMin(&rrt_prof[8], (unsigned long long)w_start);
    atomicMax(&rrt_prof[9], (unsigned long long)w_end);
    const unsigned long long w = atomicAdd(&rrt_prof[10], 1ull) & 16383;
    rrt_prof_ends[w] = w_end;
    rrt_prof_starts[w] = w_start;
    rrt_prof_work[w] = ((unsigned long long)prof_blocks << 32) | ns;
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// rrt_batch_kernel -- sample-parallel depth <= 1 path: a group of G lanes renders G consecutive
// camera samples of ONE pixel at a time (G = samples_per_batch rounded up to a power of two, at
// most 32), so a pixel's 32..64 samples take two group steps instead of 64 sequential lane
// steps, and the lanes of a group march almost identical (jittered) rays.
//
// The reference draws a pixel's samples in sequence from one RNG stream, so sample k starts at
// draw offset O + sum_{j<k} draws_j, and draws_j depends only on whether camera query j hit:
// draws_miss (the jitter) or draws_hit (jitter + the direct-lighting samplers, a per-scene
// constant at depth <= 1).  A group therefore speculates each lane's offset from a hit/miss
// hypothesis, runs the camera queries, recomputes the offsets from the actual hits, and re-runs
// exactly the lanes whose offset was wrong, until every offset is the one the sequential order
// gives (each round fixes at least the first wrong lane).  Shading then runs in parallel, and the
// group leader folds the samples into the pixel sums in sample order (the reference's float /
// double accumulation order) with the adaptive stop test at every samples_per_batch boundary;
// samples past the stop are discarded with their draws.  Results equal the sequential loop's.
// draw-offset slots per group and step: a hit takes Dh / Dm slots (2 with one area light, the
// LEAN builds; 3 with an environment light too), so 32 samples need up to 31 * (Dh / Dm) + 1
template <int LEAN>
struct SlotWindow { static constexpr uint32_t n = rrt::is_lean(LEAN) ? 64u : 128u; };
// striped claim queues: runs of RRT_STRIPE_OF(V) consecutive claims (neighbouring pixels).
// Interleaved A/B (ms/frame): cfg3 (build 1) 20.2 at 32, 20.7 at 16, 20.7 at 8; cfg4 (build 2)
// 20.6 at 32, 20.0 at 16.
#define RRT_STRIPE_OF(V) ((V) == 2 ? 16u : 32u)

// Per-group pixel state, cold during the queries: kept in LDS (one slot per group) so the walks
// run with only the lane's own few speculation registers live.
template <uint32_t NSLOTS>
struct GroupLds {  // group size >= 8: at most 32 groups per 256-thread block
  uint64_t key[32];
  uint32_t px[32], py[32], slot[32], O[32], i[32], hyp[32];
  float rr[32], rg[32], rb[32];
  double s1[32], s2[32];
  // draw-offset slots of the current step (see the camera-query section): state 0 unknown,
  // 1 miss, 2 hit, 3 hit whose record was given up; owner = group lane whose ShadeLds slot holds
  // the hit record
  uint8_t sst[32][NSLOTS], sown[32][NSLOTS];
};

// Heavy pixel hx of the pixel proof pass's heavy list (rrt_device.h pixel_heavy),
// rendered by one block of NW waves: its 64 NW consecutive draw-offset slots per round, in
// parallel.  Sample k of a pixel starts at draw offset Dm * m_k with m_0 = 0 and m_{k+1} = m_k +
// (hit_k ? Dh / Dm : 1) (the slots below, counted from the pixel's first draw), so slot m's
// sample -- the camera ray from its jitter draws, then est_radiance_global_illumination with the
// draws that follow -- is the same whichever sample lands on it.  After a round the block folds
// the chain of samples over the computed slots in sample order, with the adaptive stop at each
// step's end (raytrace_pixel, part1_code.cpp:136-158; the batch kernel's group-leader fold, so the
// result is the same), and the next round starts at the first slot the chain has not reached.
// With 128 slots a 64-sample pixel (two 32-sample steps, a hit taking two slots) takes one round,
// where the batch kernel's speculation takes four to seven (pixels that straddle the capture
// boundary).  Every thread runs the fold on the same LDS values, so control stays block-uniform.
// The body stays out of line: inlined into the batch kernel, an earlier (per-wave) form of it hung
// on the first heavy pixel of bunny_B1_160x120_s16 while the out-of-line build rendered it
// bit-exactly (tools/probe_case.py; cause not found); called out of line from the batch kernel,
// it doubled the group loop's spills (cfg3 batch kernel 17.3 -> 33.5 ms), hence its own kernel.
// The same block also takes continuations (ContRec, from the batch kernel): a pixel some of whose
// steps are already folded, resumed from its sums and draw offset.
// LDS: the parked hit records (ShadeLdsN, the batch kernel's own `cl` when its blocks take
// continuations) and HeavyState (over the batch kernel's group records there).
template <int NW>
struct HeavyState {
  float r[64 * NW], g[64 * NW], b[64 * NW];  // each slot's sample radiance
  uint64_t hits[NW];  // each wave's ballot of hits
  // the claimed pixel (thread 0 writes it between block barriers): position, output slot, samples
  // folded, first slot (draw offset / Dm) and the sums so far
  double s1, s2;
  float r0, g0, b0;
  uint32_t x, y, slot, i, m0;
  uint32_t go;
};
template <int NW>
struct HeavyLds {
  rrt::ShadeLdsN<64 * NW> sh;  // parked hit records (direct_importance_parked)
  HeavyState<NW> hs;
};
// Thread 0: the pixel proof pass's heavy-list entry k as a fresh pixel
template <int NW>
__device__ __forceinline__ void heavy_take_listed(const KParams& kp, HeavyState<NW>& hs, uint32_t k) {
  const uint32_t ts = kp.tile_size, tpix = ts * ts;
  const uint32_t ix = kp.heavy_list[k];
  const uint32_t tl = kp.tile_order[ix / tpix], r = claim_r(ix % tpix, ts);
  hs.x = kp.tiles[2 * tl] + r % ts; hs.y = kp.tiles[2 * tl + 1] + r / ts; hs.slot = tl * tpix + r;
  hs.i = 0; hs.m0 = 0; hs.r0 = 0.0f; hs.g0 = 0.0f; hs.b0 = 0.0f; hs.s1 = 0.0; hs.s2 = 0.0;
}
// Thread 0: continuation record h once its writer has published it (seq), as the pixel to resume
template <int NW>
__device__ __forceinline__ void heavy_take_cont(const KParams& kp, HeavyState<NW>& hs, uint32_t h) {
  ContRec* rc = kp.cont + h;
  while (__hip_atomic_load(&rc->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != kp.cont_seq)
    __builtin_amdgcn_s_sleep(2);  // reserved by a running batch wave, whose stores are on their way
  hs.x = rc->x; hs.y = rc->y; hs.slot = rc->slot; hs.i = rc->i; hs.m0 = rc->O / kp.draws_miss;
  hs.r0 = rc->r; hs.g0 = rc->g; hs.b0 = rc->b; hs.s1 = rc->s1; hs.s2 = rc->s2;
}
__device__ __forceinline__ uint32_t cont_word(const KParams& kp, int w) {
  return __hip_atomic_load(kp.cont_ctl + RRT_QUEUE_STRIDE * w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Thread 0: take the oldest published record without waiting (true: hs holds it)
template <int NW>
__device__ __forceinline__ bool cont_try_take(const KParams& kp, HeavyState<NW>& hs) {
  const uint32_t hd = cont_word(kp, RRT_CONT_HEAD);
  uint32_t e = hd;
  if (hd < min(cont_word(kp, RRT_CONT_TAIL), kp.cont_cap) &&
      __hip_atomic_compare_exchange_strong(kp.cont_ctl + RRT_QUEUE_STRIDE * RRT_CONT_HEAD, &e, hd + 1u, __ATOMIC_RELAXED,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
    heavy_take_cont(kp, hs, hd);
    return true;
  }
  return false;
}
// Thread 0 of a block waiting for a continuation: counts itself idle (cont_ctl[RRT_CONT_IDLE],
// which lets the batch kernel's groups hand pixels over) while it waits, takes the next published
// record (true), or gives up (false) once every batch wave is past its last pixel -- no record
// can come then -- or after cont_ticks without one.  It never waits for anything else: a launch's
// kernels may run in any order the hardware picks, and the drain launch behind them renders any
// record left untaken.
template <int NW>
__device__ bool cont_wait_take(const KParams& kp, HeavyState<NW>& hs) {
  uint32_t* const cc = kp.cont_ctl;
  atomicAdd(cc + RRT_QUEUE_STRIDE * RRT_CONT_IDLE, 1u);
  const uint64_t since = wall_clock64();
  bool got = false;
  for (;;) {
    if (cont_try_take(kp, hs)) { got = true; break; }
    const bool fin = __hip_atomic_load(cc + RRT_QUEUE_STRIDE * RRT_CONT_DONE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >=
                     kp.batch_waves;
    if (fin && cont_word(kp, RRT_CONT_HEAD) < min(cont_word(kp, RRT_CONT_TAIL), kp.cont_cap)) continue;  // published before
    if (fin || wall_clock64() - since > kp.cont_ticks) break;
    __builtin_amdgcn_s_sleep(16);
  }
  atomicSub(cc + RRT_QUEUE_STRIDE * RRT_CONT_IDLE, 1u);
  return got;
}
template <int LEAN, int W, int NW>
__device__ __noinline__ void heavy_pixel_block(const KParams& kp, rrt::ShadeLdsN<64 * NW>& sh, HeavyState<NW>& hs,
                                               uint32_t t, rrt::Counters& cn) {
  using namespace rrt;
  constexpr uint32_t NS = 64u * NW;  // slots per round
  const uint32_t Dm = kp.draws_miss, Dh = kp.draws_hit, S1 = Dh / Dm;
  const DCamera& cam = kp.cam;
  const uint32_t x = hs.x, y = hs.y, slot = hs.slot;
  const uint64_t key = rrt_pixel_key(kp.seed, x, y);
  spec ret = S(hs.r0, hs.g0, hs.b0);
  double s1 = hs.s1, s2 = hs.s2;
  uint32_t i = hs.i, m0 = hs.m0;  // samples folded; the round's first slot
  for (;;) {
    // the chain of the ns_aa - i samples left spans at most S1 (ns_aa - i) slots: lanes beyond
    // that are never reached by the fold and stay idle
    const uint32_t lim = S1 * (kp.ns_aa - i);
    const uint32_t sl = m0 + t;
    Rng g; g.key = key; g.ctr = sl * Dm;
    double jx, jy; g.grid(jx, jy);  // Camera::generate_ray (part1_code.cpp:182-187) at the slot's jitter
    const double sx = (double)x + jx, sy = (double)y + jy;
    const double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
    const double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
    const v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
    const v3 wd = unit(w);
    Isect is;
    const bool hit = t < lim && !camera_proven_miss<false, false>(kp, ld3(cam.pos), wd, cn) &&
                     query_nx<false, false, false>(kp, ld3(cam.pos), wd, &is, cn);
    spec s = S(0, 0, 0);
    if (hit) {
      park_hit(sh, t, is);
      g.ctr = sl * Dm + Dm;
      const spec e = emission(kp.bsdfs[lget(sh.bsdf, t)]);
      if (kp.max_ray_depth == 0) s = e;
      else s = e + direct_importance_parked<false, LEAN, W>(kp, g, sh, t, cn);
    }
    const uint64_t hb = __ballot(hit);
    if ((t & 63u) == 0) hs.hits[t >> 6] = hb;
    hs.r[t] = s.r; hs.g[t] = s.g; hs.b[t] = s.b;
    __syncthreads();
    // the chain over the computed slots and the ordered fold (every thread alike)
    uint32_t m = 0;  // slot relative to m0
    bool st = false;
    while (m < NS) {
      const spec sk = S(hs.r[m], hs.g[m], hs.b[m]);
      if (sk.r != 0.0f || sk.g != 0.0f || sk.b != 0.0f) {  // zero samples: identities on the sums
        ret = ret + sk;
        const double il = illum(sk);
        s1 += il;
        s2 += il * il;
      }
      ++i;
      m += ((hs.hits[m >> 6] >> (m & 63u)) & 1ull) ? S1 : 1u;
      st = i >= kp.ns_aa;
      if (i % kp.samples_per_batch == 0) {  // ADAPTIVE == 1 (:147-158)
        const double avg = s1 / i, sd = sqrt((s2 - avg * s1) / (i - 1));
        if (1.96 * sd / sqrt((double)i) <= (double)kp.max_tolerance * avg) st = true;
      }
      if (st) break;
    }
    m0 += m;
    __syncthreads();  // the fold's reads before the next round's writes
    if (st) break;
  }
  if (t == 0) {
    const spec rr = ret / (float)i;
    kp.rgb[3 * slot] = rr.r; kp.rgb[3 * slot + 1] = rr.g; kp.rgb[3 * slot + 2] = rr.b;
    kp.count[slot] = (int32_t)i;
    if (kp.draws) kp.draws[slot] = m0 * Dm;
  }
}

// The heavy pixels' kernel (heavy pixels), launched after the pixel proof pass on
// the context's high-priority side stream, beside the batch kernel, which leaves room for its
// blocks (rrt_host.cpp): each block of NW waves takes heavy pixels one at a time, at issue
// priority 3 -- first the pass's heavy list, then (kp.cont, blocks below kp.cont_waiters)
// continuations from the batch kernel (cont_wait_take).  mode RRT_HEAVY_DRAIN: the launch behind
// the batch and heavy kernels on the main stream, which renders the records nobody took.
template <int LEAN, int HW, int NW>
__global__ __launch_bounds__(64 * NW, HW) void rrt_heavy_kernel(const KParams* __restrict__ kpp, int mode) {
  const bool drain = mode == RRT_HEAVY_DRAIN;
  const KParams& kp = *kpp;
  using namespace rrt;
  __shared__ HeavyLds<NW> hl;
  HeavyState<NW>& hs = hl.hs;
  const uint32_t t = threadIdx.x;
  Counters cn = {};
  const uint32_t nh = mode != RRT_HEAVY_LIST ? 0u : min(*kp.heavy_count, kp.heavy_cap);
  const bool waiter = kp.cont && mode == RRT_HEAVY_LIST && blockIdx.x < kp.cont_waiters;
  bool listed = mode == RRT_HEAVY_LIST;  // (thread 0's)
  __builtin_amdgcn_s_setprio(3);
#if RRT_PROFILE
  volatile uint32_t* wd = kp.wd ? kp.wd + RRT_WD_HEAVY + 4u * (blockIdx.x & 0x7fffu) : nullptr;
  uint32_t wd_it = 0;
#endif
  for (;;) {
    if (t == 0) {
      bool go = false;
      if (listed) {
        const uint32_t k = atomicAdd(kp.heavy_count + 1, 1u);
        if (k < nh) { heavy_take_listed(kp, hs, k); go = true; }
        else listed = false;
      }
      if (!go && kp.cont && drain) {  // behind both kernels: every reserved record is written
        const uint32_t h = atomicAdd(kp.cont_ctl + RRT_QUEUE_STRIDE * RRT_CONT_HEAD, 1u);
        if (h < min(cont_word(kp, RRT_CONT_TAIL), kp.cont_cap)) { heavy_take_cont(kp, hs, h); go = true; }
      } else if (!go && waiter) {
        go = cont_wait_take(kp, hs);
      }
      hs.go = go ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t go = hs.go;
    __syncthreads();  // every thread has read the claim before thread 0 claims again
#if RRT_PROFILE
    if (wd && t == 0) { wd[0] = ++wd_it; wd[1] = nh; wd[2] = hs.slot; wd[3] = 0x11u; }
#endif
    if (!go) break;
#if RRT_PROFILE
    const uint64_t w_h = wall_clock64();
    const uint32_t pslot = hs.slot;
#endif
    heavy_pixel_block<LEAN, RRT_OCC_TAG_SLOT(LEAN, HW) ? RRT_OCC_TAG_SLOT(LEAN, HW) + 32 * NW : 0, NW>(kp, hl.sh, hs, t, cn);
#if RRT_PROFILE
    if (wd && t == 0) wd[3] = 0x12u;  // pixel done
    if (t == 0 && pslot < (1u << 21)) {  // elapsed ticks; "rounds" 1
      rrt_prof_px[pslot] = ((uint32_t)min(wall_clock64() - w_h, (uint64_t)0xffffff) << 8) | 1u;
      rrt_prof_px_end[pslot] = (uint32_t)wall_clock64();
    }
#endif
  }
#if RRT_PROFILE
  if (wd && t == 0) wd[3] = 0xdeadu;  // exited
#endif
}

// waves/SIMD budget 4 or 5; NW waves per pixel (1, 2 or 4); grid in blocks; mode RRT_HEAVY_*
hipError_t rrt_launch_heavy(const KParams* d_kp, int lean, int waves, int nw, uint32_t grid, int mode, hipStream_t stream) {
#define RRT_LAUNCH_H(L, W, N) hipLaunchKernelGGL((rrt_heavy_kernel<L, W, N>), dim3(grid), dim3(64 * N), 0, stream, d_kp, mode)
  if (lean == 1) {
    if (waves == 5) {
      if (nw == 1) RRT_LAUNCH_H(1, 5, 1); else if (nw == 4) RRT_LAUNCH_H(1, 5, 4); else RRT_LAUNCH_H(1, 5, 2);
    } else {
      if (nw == 1) RRT_LAUNCH_H(1, 4, 1); else if (nw == 4) RRT_LAUNCH_H(1, 4, 4); else RRT_LAUNCH_H(1, 4, 2);
    }
  } else if (lean == 2) {
    if (nw == 4) RRT_LAUNCH_H(2, 4, 4); else RRT_LAUNCH_H(2, 4, 2);
  } else {
    return hipErrorInvalidValue;
  }
#undef RRT_LAUNCH_H
  return hipGetLastError();
}

// Continuations.  A group leader whose pixel did not stop at an adaptive check and
// has at least kp.cont_min_left samples to go hands it to a heavy block when one is waiting for
// work and no record already waits for it: it reserves record k, writes the pixel's state there and
// publishes it (seq, release).  The heavy block resumes the fold from that state with its 64 NW
// slots per round, so the result is the one the group would have reached.  false: keep the pixel.
__device__ __forceinline__ bool cont_push(const KParams& kp, uint32_t x, uint32_t y, uint32_t slot, uint32_t i,
                                          uint32_t O, rrt::spec ret, double s1, double s2) {
  uint32_t* const cc = kp.cont_ctl;
  const uint32_t idle = __hip_atomic_load(cc + RRT_QUEUE_STRIDE * RRT_CONT_IDLE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (idle == 0) return false;
  const uint32_t tl = __hip_atomic_load(cc + RRT_QUEUE_STRIDE * RRT_CONT_TAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t hd = __hip_atomic_load(cc + RRT_QUEUE_STRIDE * RRT_CONT_HEAD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((int32_t)(tl - hd) >= (int32_t)idle || tl >= kp.cont_cap) return false;
  const uint32_t k = atomicAdd(cc + RRT_QUEUE_STRIDE * RRT_CONT_TAIL, 1u);
  if (k >= kp.cont_cap) return false;
  ContRec* rc = kp.cont + k;
  rc->s1 = s1; rc->s2 = s2; rc->r = ret.r; rc->g = ret.g; rc->b = ret.b;
  rc->x = x; rc->y = y; rc->slot = slot; rc->i = i; rc->O = O;
  __hip_atomic_store(&rc->seq, kp.cont_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}
// a batch wave is past its last pixel (it hands over no more): once all are, waiting blocks stop
__device__ __forceinline__ void cont_wave_done(const KParams& kp, uint32_t lane) {
  if (kp.cont && lane == 0)
    __hip_atomic_fetch_add(kp.cont_ctl + RRT_QUEUE_STRIDE * RRT_CONT_DONE, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

template <int LEAN, int WAVES>
__global__ __launch_bounds__(256, WAVES) void rrt_batch_kernel(const KParams* __restrict__ kpp) {
  const KParams& kp = *kpp;
  using namespace rrt;
  __shared__ ShadeLds cl;
  constexpr uint32_t RRT_SLOTS = SlotWindow<LEAN>::n;
  constexpr uint32_t STRIPE = RRT_STRIPE_OF(LEAN);
  // the claim space (a multiple of 64 pixels: tiles of 8k x 8k) must hold whole stripes
  static_assert(STRIPE > 0 && 64u % STRIPE == 0, "RRT_STRIPE must divide 64");
  __shared__ GroupLds<RRT_SLOTS> gs;
  float* const fr = cl.cr;  // per-lane sample radiance for the ordered fold (free after shading)
  float* const fg = cl.cg;
  float* const fb = cl.cb;
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & 63u;
  const uint32_t G = kp.group;
  const uint32_t gl = lane & (G - 1u);
  const uint32_t gbase = lane - gl;
  const uint32_t gid = t / G;  // group slot in GroupLds
  const uint32_t ts = kp.tile_size, tpix = ts * ts;
  const uint32_t Dm = kp.draws_miss, Dh = kp.draws_hit;
  const DCamera& cam = kp.cam;
  Counters cn = {};
#if RRT_PROFILE
  const uint64_t t_start = clock64(), w_start = wall_clock64();
  uint32_t prof_blocks = 0, prof_samples = 0;  // pixels claimed, query rounds
  uint32_t px_rounds = 0, px_steps = 0;           // of the group's current pixel
#endif

  // Room for the heavy pixels' kernel (launched beside this one on the side stream): the grid is
  // the resident block count, and its top blocks -- as many as the heavy pixels the pass listed
  // need, in batch blocks of 4 waves -- leave at once, so the heavy kernel's blocks take their
  // slots whichever kernel the hardware dispatched first.  A launch with no heavy pixels keeps
  // every block (the heavy kernel's blocks then start at its end and find the list empty).
  // With continuations the heavy blocks wait for work the whole launch: kp.cont_room blocks at least.
  if (kp.heavy_grid) {
    const uint32_t nh = min(*kp.heavy_count, kp.heavy_cap);
    const uint32_t need = max((min(nh, kp.heavy_grid) * kp.heavy_nw + 3u) / 4u, kp.cont_room);
    if (blockIdx.x + min(need, gridDim.x - 1u) >= gridDim.x) {
      cont_wave_done(kp, lane);
      return;
    }
  }
  bool have = false, done = false;
  uint32_t q = blockIdx.x % kp.n_queues, q_left = kp.n_queues;  // claim queue (group leaders)

  uint64_t t_claim = 0;  // when the group claimed its pixel (wall clock)
#if RRT_PROFILE
  volatile uint32_t* wd = kp.wd ? kp.wd + 4u * ((blockIdx.x * (blockDim.x >> 6) + (t >> 6)) & 0x7fffu) : nullptr;
  uint32_t wd_it = 0;
#endif

  for (;;) {
#if RRT_PROFILE
    if (wd && lane == 0) { wd[0] = ++wd_it; wd[1] = (have ? 1u : 0u) | (done ? 2u : 0u); wd[3] = 0x21u; }
#endif
    // ---- claim a pixel (one atomic per group)
    RRT_T0(tc0);
    // The wave's group leaders that need a pixel claim together: one atomic takes as many
    // consecutive claims as there are leaders (2 with the BASELINE group size), lane 0 issues it.
    const uint64_t needers = __ballot(gl == 0 && !have && !done);
    if (needers) {
      // claim space: every pixel slot, or the pixel proof's list padded to whole stripes (the
      // padding claims no pixel); read here, not held through the kernel
      const uint32_t n_list = kp.claim_list ? *kp.claim_count + (kp.claim_back ? kp.claim_count[1] : 0u) : 0u;
      const uint32_t npx = kp.claim_list ? (n_list + STRIPE - 1) / STRIPE * STRIPE : kp.n_pixels;
      uint64_t pending = needers;
      uint32_t p = npx + 1;  // npx + 1: this group did not claim
      while (pending) {
        const uint32_t want = (uint32_t)__popcll(pending);
        uint32_t base = 0, got = 0, out = 0, qc = 0;
        if (lane == 0) {  // this XCD's queue first, then the others in turn (KParams::q_end)
          if (q_left == 0) {  // every queue found empty before
            out = 1;
          } else {
            // striped queues: queue q holds the runs q, q + nq, q + 2 nq, ... of STRIPE
            // consecutive claims (n_pixels is a multiple of 64: tiles of 8k x 8k pixels)
            const uint32_t nq = kp.n_queues;
            const uint32_t qb = kp.q_stripe ? 0u : (q ? kp.q_end[q - 1] : 0u);
            const uint32_t qn = kp.q_stripe ? (npx / STRIPE - q + nq - 1) / nq * STRIPE
                                            : (kp.claim_list ? npx : kp.q_end[q] - qb);
            const uint32_t k = atomicAdd(kp.block_counter + RRT_QUEUE_STRIDE * q, want);
            if (k < qn) {
              base = qb + k; got = min(want, qn - k); qc = q;
            } else if (--q_left == 0) {
              out = 1;
            } else {
              q = q + 1 == nq ? 0u : q + 1;
            }
          }
        }
        base = __shfl(base, 0); got = __shfl(got, 0); out = __shfl(out, 0); qc = __shfl(qc, 0);
        const uint32_t rank = (uint32_t)__popcll(pending & ((1ull << gbase) - 1ull));  // pending leaders before mine
        const bool mine = (pending >> gbase) & 1ull;
        if (mine && rank < got) {
          const uint32_t ix = base + rank;
          p = kp.q_stripe ? ((ix / STRIPE) * kp.n_queues + qc) * STRIPE + ix % STRIPE : ix;
        }
        if (mine && out) p = npx;
        pending = out ? 0ull : (got >= want ? 0ull : pending & ~__ballot(gl == 0 && mine && rank < got));
      }
      q = __shfl(q, 0);
      q_left = __shfl(q_left, 0);
      p = __shfl(p, (int)gbase);
      if (p == npx + 1) {
        // (the group kept its pixel)
      } else if (p >= npx) {
        done = true;
#if RRT_PROFILE
        if (gl == 0) atomicMin(&rrt_prof[11], (unsigned long long)wall_clock64());
#endif
      } else {
#if RRT_PROFILE
        ++prof_blocks;
#endif
        // a list entry: pixel claim index | hint << 31 (rrt_pixel_proof_kernel)
        // (claim_back: the front part's entries, then the back part's from the list's end)
        const uint32_t n_front = kp.claim_list ? *kp.claim_count : 0u;
        const uint32_t ent = !kp.claim_list ? p
                             : p < n_front ? kp.claim_list[p]
                             : p < n_list ? kp.claim_list[kp.claim_back ? kp.n_pixels - 1u - (p - n_front) : p]
                             : kp.n_pixels;
        const uint32_t ix = kp.claim_list ? (ent & 0x7fffffffu) : ent;
        const uint32_t pi = ix < kp.n_pixels ? ix : 0u;
        const uint32_t tl = kp.tile_order[pi / tpix], r = claim_r(pi % tpix, ts), lx = r % ts, ly = r / ts;
        const uint32_t x = kp.tiles[2 * tl] + lx, y = kp.tiles[2 * tl + 1] + ly;
        if (ix < kp.n_pixels && x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 && y < kp.clip_y1) {
          if (gl == 0) {
            const uint32_t slot = tl * tpix + r;
            lput(gs.px, gid, x); lput(gs.py, gid, y); lput(gs.slot, gid, slot);
            lput(gs.key, gid, rrt_pixel_key(kp.seed, x, y));
            if (kp.first) {  // sample 0 from rrt_first_kernel; its hit status is the hypothesis
              const KParams::FirstSample f0 = kp.first[slot];
              const spec s0 = S(f0.r, f0.g, f0.b);
              const spec ret = S(0, 0, 0) + s0;
              const double il = illum(s0);
              lput(gs.rr, gid, ret.r); lput(gs.rg, gid, ret.g); lput(gs.rb, gid, ret.b);
              lput(gs.s1, gid, 0.0 + il); lput(gs.s2, gid, 0.0 + il * il);
              lput(gs.i, gid, 1u); lput(gs.O, gid, f0.hit ? Dh : Dm); lput(gs.hyp, gid, f0.hit);
            } else {
              lput(gs.O, gid, 0u); lput(gs.i, gid, 0u);
              // The first step's hypothesis: "miss" without the pixel proof's list; for a listed
              // pixel (one whose camera rays are not all proven misses) the list entry's hint (its
              // central ray is no proven miss).  A/B: "miss" / "hit" / hint for every listed pixel:
              // cfg3 23.9 / 22.6 / 20.5 ms, cfg4 - / 19.8 / 20.1
              const uint32_t hyp0 = !kp.claim_list ? 0u : (ent >> 31);
              lput(gs.hyp, gid, hyp0);
              lput(gs.rr, gid, 0.0f); lput(gs.rg, gid, 0.0f); lput(gs.rb, gid, 0.0f);
              lput(gs.s1, gid, 0.0); lput(gs.s2, gid, 0.0);
            }
          }
          have = true;
          t_claim = wall_clock64();
#if RRT_PROFILE
          px_rounds = 0; px_steps = 0;
#endif
        }
      }
    }
    RRT_ACC(t_claim, tc0);
    if (__ballot(!done) == 0) break;
    // Tail latency: a pixel whose rounds are long (the costliest ones -- long walks next to the
    // hole and the geometry) keeps its wave busy long after the claim queue runs dry.  A wave
    // whose oldest pixel has been running for a while takes issue priority over the other waves
    // of its SIMD, so the costliest pixels finish early instead of forming the frame's tail.
    auto tail_prio = [&]() {
      const uint64_t age = have ? wall_clock64() - t_claim : 0;
      if (__ballot(age > 4ull * kp.prio_ticks)) __builtin_amdgcn_s_setprio(3);
      else if (__ballot(age > kp.prio_ticks)) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(0);
    };
    tail_prio();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- camera queries by draw-offset slot.  Sample k of the step starts at draw offset
    // O + Dm * m_k, where slot m_0 = 0 and m_{k+1} = m_k + (hit_k ? Dh / Dm : 1): a slot's ray
    // (its jitter draws) is the same whichever sample lands on it, so slot results are shared.
    // Round 1 computes the slots of the hypothesis (all samples hit or all miss, as the pixel's
    // last sample); every round then walks the chain over the known slots and hands the first
    // unknown slot -- and the unknown ones after it -- to lanes whose slot is off the chain.
    // Each round resolves at least one more sample; all-hit and all-miss pixels take one round,
    // mixed ones two or three.  A chain that leaves the slot window ends the step early (the
    // next step continues it).
    const int done_i = (int)lget(gs.i, gid);
    const int to_check = (int)kp.samples_per_batch - done_i % (int)kp.samples_per_batch;
    const int left = min((int)kp.ns_aa - done_i, to_check);
    const uint32_t S1 = Dh / Dm;  // slots a hit consumes
    const uint32_t O0 = lget(gs.O, gid);
    for (uint32_t m = gl; m < RRT_SLOTS; m += G) lput(&gs.sst[gid][0], m, (uint8_t)0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t my = RRT_SLOTS;  // slot to compute this round (RRT_SLOTS: none)
    if (have && (int)gl < left) {
      const uint32_t m0 = gl * (lget(gs.hyp, gid) ? S1 : 1u);
      if (m0 < RRT_SLOTS) my = m0;
    }
    // the camera query of slot sl (Camera::generate_ray, part1_code.cpp:182-187, at its jitter)
    auto slot_query = [&](uint32_t sl, Isect* is) -> bool {
      Rng g; g.key = lget(gs.key, gid); g.ctr = O0 + sl * Dm;
      double jx, jy; g.grid(jx, jy);
      const double sx = (double)lget(gs.px, gid) + jx, sy = (double)lget(gs.py, gid) + jy;
      const double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
      const double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
      const v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
      const v3 wd = unit(w);
      if (camera_proven_miss<false, LEAN == V_KERR>(kp, ld3(cam.pos), wd, cn)) return false;
      return query_nx<false, false, LEAN == V_KERR, 0, is_lean(LEAN)>(kp, ld3(cam.pos), wd, is, cn);
    };
    const uint64_t gmask = (G >= 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;  // this group's lanes
    const uint64_t lt = ((1ull << lane) - 1ull) & gmask;                         // group lanes before me
    uint32_t held = RRT_SLOTS;  // slot whose hit record this lane's ShadeLds slot holds
    uint32_t mk = 0;            // slot of this lane's sample (lane gl = sample gl of the step)
    bool hk = false;
    int n_step = 0;             // samples the step resolves
    bool resolved = !have;      // (group-uniform)
    for (int round = 0;; ++round) {
      const bool need = my < RRT_SLOTS;
#if RRT_PROFILE
      if (wd && lane == 0) { wd[1] = (have ? 1u : 0u) | (done ? 2u : 0u) | ((uint32_t)round << 8); wd[2] = lget(gs.slot, gid); wd[3] = 0x22u; }
#endif
      if (__ballot(need) == 0) break;
      if (round > 0) tail_prio();
#if RRT_PROFILE
      ++prof_samples;
      ++px_rounds;
#endif
      bool h = false;
      if (need) {
        Isect is;
        h = slot_query(my, &is);
        if (h) park_hit(cl, t, is);  // nothing of the hit stays live across later rounds
        held = my;
        lput(&gs.sst[gid][0], my, (uint8_t)(h ? 2 : 1));
        lput(&gs.sown[gid][0], my, (uint8_t)gl);
      }
      if (round == 0) {  // the hypothesis held for every sample: the chain is its slots
        const uint64_t comp = __ballot(need) & gmask, hb = __ballot(need && h) & gmask;
        const bool hyp1 = lget(gs.hyp, gid) != 0;
        if (!resolved && (int)__popcll(comp) == left && hb == (hyp1 ? comp : 0ull)) {
          resolved = true;
          n_step = left;
          if (need) mk = my;
          hk = h;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      my = RRT_SLOTS;
      if (resolved) continue;
      RRT_T0(tw0);
      // walk the chain over the known slots (group-uniform)
      uint32_t m = 0;
      int k = 0, kh = 0;
      bool on_chain = false;
      for (; k < left && m < RRT_SLOTS; ++k) {
        const uint32_t st = lget(&gs.sst[gid][0], m);
        if (st == 0) break;
        on_chain |= m == held;
        if (k == (int)gl) { mk = m; hk = st >= 2; }
        kh += st >= 2;
        m += st >= 2 ? S1 : 1u;
      }
      n_step = k;
      const bool open = have && k < left && m < RRT_SLOTS;  // unresolved samples remain
      resolved = !open;
      // Lanes off the chain take the unknown slots along the continuation (an unknown slot taken
      // as the majority outcome of the resolved samples, the pixel's hypothesis before any):
      // first lanes whose slot needs no record (none, a miss, or a slot the chain has passed),
      // then lanes holding a hit beyond the frontier, whose outcome stays known (state 3) while
      // its record is given up (recomputed if the chain lands on it).
      const uint32_t sth = held < RRT_SLOTS ? lget(&gs.sst[gid][0], held) : 0u;
      const bool free_a = open && !on_chain && (held >= RRT_SLOTS || held < m || sth != 2);
      const bool free_b = open && !on_chain && !free_a;
      const uint64_t ba = __ballot(free_a), bb = __ballot(free_b);
      const uint32_t rank = free_a ? (uint32_t)__popcll(ba & lt) : (uint32_t)(__popcll(ba & gmask) + __popcll(bb & lt));
      if (free_a || free_b) {
        const uint32_t guess = (k > 0 ? 2 * kh >= k : lget(gs.hyp, gid) != 0) ? S1 : 1u;
        uint32_t mm = m, j = 0;
        for (int kk = k; kk < left && mm < RRT_SLOTS; ++kk) {
          const uint32_t st = lget(&gs.sst[gid][0], mm);
          if (st == 0) {
            if (j == rank) { my = mm; break; }
            ++j;
          }
          mm += st == 0 ? guess : st >= 2 ? S1 : 1u;
        }
        if (my < RRT_SLOTS && free_b) lput(&gs.sst[gid][0], held, (uint8_t)3);
      }
      RRT_ACC(t_chain, tw0);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const bool act = have && (int)gl < n_step;
    const bool hit = act && hk;
    const uint32_t off = O0 + mk * Dm;
    {  // move each hit sample's record into its own lane's ShadeLds slot (recompute a given-up one)
      const bool lost = hit && lget(&gs.sst[gid][0], mk) == 3;
      const uint32_t src = (t - gl) + lget(&gs.sown[gid][0], mk);
      const bool move = hit && !lost && src != t;
      Isect is0 = {};
      if (move) {
        is0.hit_p = V(lget(cl.hp[0], src), lget(cl.hp[1], src), lget(cl.hp[2], src));
        is0.n = V(lget(cl.nn[0], src), lget(cl.nn[1], src), lget(cl.nn[2], src));
        is0.w_out = V(lget(cl.wo[0], src), lget(cl.wo[1], src), lget(cl.wo[2], src));
        is0.bsdf = (int)lget(cl.bsdf, src);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lost) slot_query(mk, &is0);  // the same ray: the same hit
      if (move || lost) park_hit(cl, t, is0);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const uint64_t hits = __ballot(hit);

    // ---- shading (est_radiance_global_illumination, :103-123), all samples in parallel
    RRT_T0(ts0);
    spec s = S(0, 0, 0);
    if (!is_lean(LEAN) && act && !hit && kp.env.w) {  // miss: envLight->sample_dir of the unbent camera ray
      Rng g; g.key = lget(gs.key, gid); g.ctr = off;  // re-derive the ray from its jitter draws
      double jx, jy; g.grid(jx, jy);
      const double sx = (double)lget(gs.px, gid) + jx, sy = (double)lget(gs.py, gid) + jy;
      const double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
      const double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
      const v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
      s = env_dir(kp.env, unit(w));
    }
    if (act && hit) {
      Rng g; g.key = lget(gs.key, gid); g.ctr = off + Dm;
      const spec e = emission(kp.bsdfs[lget(cl.bsdf, t)]);
      if (kp.max_ray_depth == 0) s = e;
      else if (is_lean(LEAN)) s = e + direct_importance_parked<false, LEAN, RRT_OCC_TAG(LEAN, WAVES)>(kp, g, cl, t, cn);
      else if (kp.direct_hemisphere) s = e + direct_hemisphere_parked<false, LEAN>(kp, g, cl, t, cn);
      else s = e + direct_importance_parked<false, LEAN, RRT_OCC_TAG(LEAN, WAVES)>(kp, g, cl, t, cn);
    }
    if (act) { lput(fr, t, s.r); lput(fg, t, s.g); lput(fb, t, s.b); }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    RRT_ACC(t_shade, ts0);
    // ---- ordered fold by the group leader (raytrace_pixel's loop body, :136-158)
    RRT_T0(tf0);
    uint32_t stop = 0;
#if RRT_PROFILE
    ++px_steps;
#endif
    // Adding a zero sample is an identity on the sums (ret, s1, s2 are never -0), and a step
    // ends at the next adaptive check or at ns_aa, so its only possible stop is its last sample:
    // the leader adds the nonzero samples in sample order and tests the stop once.
    const uint64_t nonzero = __ballot(act && (s.r != 0.0f || s.g != 0.0f || s.b != 0.0f));
    if (have && gl == 0) {
      const int n = n_step;
      spec ret = S(lget(gs.rr, gid), lget(gs.rg, gid), lget(gs.rb, gid));
      double s1 = lget(gs.s1, gid), s2 = lget(gs.s2, gid);
      int i = (int)lget(gs.i, gid) + n;
      uint64_t nz = (nonzero >> gbase) & (n >= 64 ? ~0ull : ((1ull << n) - 1ull));
      while (nz) {
        const int k = (int)__builtin_ctzll(nz);
        nz &= nz - 1;
        const spec sk = S(lget(fr, t + k), lget(fg, t + k), lget(fb, t + k));
        ret = ret + sk;
        const double il = illum(sk);
        s1 += il;
        s2 += il * il;
      }
      const uint64_t hm = (hits >> gbase) & (n >= 64 ? ~0ull : ((1ull << n) - 1ull));
      const uint32_t nh = (uint32_t)__popcll(hm);
      const uint32_t O = lget(gs.O, gid) + nh * Dh + ((uint32_t)n - nh) * Dm;
      const uint32_t hyp = n > 0 ? (uint32_t)((hm >> (n - 1)) & 1ull) : lget(gs.hyp, gid);
      bool st = i >= (int)kp.ns_aa;
      if ((uint32_t)i % kp.samples_per_batch == 0) {  // ADAPTIVE == 1 (:147-158)
        const double avg = s1 / i, sd = sqrt((s2 - avg * s1) / (i - 1));
        if (1.96 * sd / sqrt((double)i) <= (double)kp.max_tolerance * avg) st = true;
      }
      if (st) stop = 1;
      else if (kp.cont && (uint32_t)((int)kp.ns_aa - i) >= kp.cont_min_left &&
               cont_push(kp, lget(gs.px, gid), lget(gs.py, gid), lget(gs.slot, gid), (uint32_t)i, O, ret, s1, s2))
        stop = 2;  // handed over: the heavy block writes the result
      if (stop == 1) {
        const uint32_t slot = lget(gs.slot, gid);
#if RRT_PROFILE
        {  // elapsed wall ticks (26 bits) | rounds (7) | steps (7) | pixel slot (24)
          const unsigned long long el = min(wall_clock64() - t_claim, (uint64_t)0x3ffffff);
          atomicMax(&rrt_prof_slow[slot & 63u], (el << 38) | ((unsigned long long)min(px_rounds, 127u) << 31) |
                                                    ((unsigned long long)min(px_steps, 127u) << 24) |
                                                    (unsigned long long)(slot & 0xffffffu));
          if (slot < (1u << 21)) {
            rrt_prof_px[slot] = ((uint32_t)min(el, (uint64_t)0xffffff) << 8) | min(px_rounds, 255u);
            rrt_prof_px_end[slot] = (uint32_t)wall_clock64();
          }
        }
#endif
        const spec r = ret / (float)i;
        kp.rgb[3 * slot] = r.r; kp.rgb[3 * slot + 1] = r.g; kp.rgb[3 * slot + 2] = r.b;
        kp.count[slot] = i;
        if (kp.draws) kp.draws[slot] = O;
      } else if (stop == 0) {
        lput(gs.rr, gid, ret.r); lput(gs.rg, gid, ret.g); lput(gs.rb, gid, ret.b);
        lput(gs.s1, gid, s1); lput(gs.s2, gid, s2);
        lput(gs.i, gid, (uint32_t)i); lput(gs.O, gid, O); lput(gs.hyp, gid, hyp);
      }
    }
    stop = __shfl(stop, (int)gbase);
    if (stop) have = false;
    RRT_ACC(t_fold, tf0);
  }
  cont_wave_done(kp, lane);
#if RRT_PROFILE
  if (wd && lane == 0) wd[3] = 0xdeadu;  // exited
#endif
#if RRT_PROFILE
  const uint64_t t_end = clock64(), w_end = wall_clock64();
  uint64_t v[12] = {t_end - t_start, cn.t_query, cn.t_micro, cn.t_trav, cn.t_proof, cn.t_squery, cn.t_strav, 0,
                    cn.t_claim, cn.t_chain, cn.t_shade, cn.t_fold};
  {  // lane sums of the phases (slot 12 + i): a phase's lane use = lane sum / (64 x busiest lane)
    const int ks[8] = {0, 1, 2, 3, 4, 5, 6, 10};
    const int slot[8] = {15, 12, 23, 21, 14, 13, 22, 20};
    for (int i = 0; i < 8; ++i) {
      uint64_t sm = v[ks[i]];
      for (int off2 = 32; off2 > 0; off2 >>= 1) sm += __shfl_xor(sm, off2);
      if (lane == 0) atomicAdd(&rrt_prof[slot[i]], (unsigned long long)sm);
    }
  }
  for (int k = 0; k < 12; ++k) {
    for (int off2 = 32; off2 > 0; off2 >>= 1) {
      const uint64_t o2 = __shfl_xor(v[k], off2);
      v[k] = v[k] > o2 ? v[k] : o2;
    }
    if (lane == 0) atomicAdd(&rrt_prof[k < 8 ? k : k + 8], (unsigned long long)v[k]);
  }
  uint32_t nb = gl == 0 ? prof_blocks : 0;
  for (int off2 = 32; off2 > 0; off2 >>= 1) nb += __shfl_xor(nb, off2);
  if (lane == 0) {
    atomicMin(&rrt_prof[8], (unsigned long long)w_start);
    atomicMax(&rrt_prof[9], (unsigned long long)w_end);
    const unsigned long long w = atomicAdd(&rrt_prof[10], 1ull) & 16383;
    rrt_prof_ends[w] = w_end;
    rrt_prof_starts[w] = w_start;
    rrt_prof_work[w] = ((unsigned long long)nb << 32) | prof_samples;
  }
#endif
}

// Pixel miss proof pass (rrt_device.h pixel_miss_proof), one lane per claim index
// in the batch kernel's order: a pixel whose every camera ray is a proven miss renders to black
// (no environment map in these builds): its samples are all zero, so it stops at the first
// adaptive check (raytrace_pixel, part1_code.cpp:147-158) with count = min(ns_aa,
// samples_per_batch) and count * draws_miss draws -- written here.  The others go to the claim
// list, appended per wave (one atomic) so claims keep their order within each wave's run.
// Claim index ix of the pass (a whole wave calls it together: ballots and one atomic per wave).
__device__ __forceinline__ void pixel_pass_one(const KParams& kp, uint32_t ix, uint32_t lane) {
  using namespace rrt;
  const uint32_t ts = kp.tile_size, tpix = ts * ts;
  bool listed = false, heavy = false;
  if (ix < kp.n_pixels) {
    const uint32_t tl = kp.tile_order[ix / tpix], r = claim_r(ix % tpix, ts);
    const uint32_t x = kp.tiles[2 * tl] + r % ts, y = kp.tiles[2 * tl + 1] + r / ts;
    if (x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 && y < kp.clip_y1) {
      if (pixel_miss_proof(kp, x, y)) {
        const uint32_t slot = tl * tpix + r, n = min(kp.ns_aa, kp.samples_per_batch);
        kp.rgb[3 * slot] = 0.0f; kp.rgb[3 * slot + 1] = 0.0f; kp.rgb[3 * slot + 2] = 0.0f;
        kp.count[slot] = (int32_t)n;
        if (kp.draws) kp.draws[slot] = n * kp.draws_miss;
      } else {
        listed = true;
        heavy = kp.heavy_list && pixel_heavy(kp, x, y);
      }
    }
  }
  // heavy pixels go to the slot kernel's list while it has room (the rest to the claim list)
  const uint64_t hb = __ballot(heavy);
  if (hb) {
    uint32_t hbase = 0;
    if (lane == 0) hbase = atomicAdd(kp.heavy_count, (uint32_t)__popcll(hb));
    hbase = __shfl(hbase, 0);
    const uint32_t k = hbase + (uint32_t)__popcll(hb & ((1ull << lane) - 1ull));
    if (heavy && k < kp.heavy_cap) {
      kp.heavy_list[k] = ix;
      listed = false;
    }
  }
  // a listed pixel's hint bit (31) = its central camera ray is no proven miss (the batch kernel's
  // first hypothesis for the pixel)
  uint32_t hint = 0u;
  if (listed) {
    const uint32_t tl = kp.tile_order[ix / tpix], r = claim_r(ix % tpix, ts);
    const uint32_t x = kp.tiles[2 * tl] + r % ts, y = kp.tiles[2 * tl + 1] + r / ts;
    Counters cn = {};
    hint = camera_miss_proof<false>(kp, ld3(kp.cam.pos), pixel_ray_dir(kp, x + 0.5, y + 0.5), cn) ? 0u : 1u;
  }
  const uint64_t b = __ballot(listed), lt = (1ull << lane) - 1ull;
  if (kp.claim_back) {
    // hit-first claim order: hinted pixels (their central ray reaches the scene: shading and
    // shadow rays, the costliest) from the list's front, the others from its back, so the
    // cheap ones are claimed last and the launch ends on short pixels
    const uint64_t bf = __ballot(listed && hint), bb = b & ~bf;
    uint32_t basef = 0, baseb = 0;
    if (lane == 0) {
      if (bf) basef = atomicAdd(kp.claim_count, (uint32_t)__popcll(bf));
      if (bb) baseb = atomicAdd(kp.claim_count + 1, (uint32_t)__popcll(bb));
    }
    basef = __shfl(basef, 0); baseb = __shfl(baseb, 0);
    if (listed && hint) kp.claim_list[basef + (uint32_t)__popcll(bf & lt)] = ix | (1u << 31);
    else if (listed) kp.claim_list[kp.n_pixels - 1u - (baseb + (uint32_t)__popcll(bb & lt))] = ix;
    return;
  }
  uint32_t base = 0;
  if (lane == 0 && b) base = atomicAdd(kp.claim_count, (uint32_t)__popcll(b));
  base = __shfl(base, 0);
  if (listed) kp.claim_list[base + (uint32_t)__popcll(b & lt)] = ix | (hint << 31);
}
// The per-pixel pass: every claim index (one lane each); behind the strip pass, the wave of a
// proven strip (its 64 claim indices) leaves at once.  Waves run in claim-index order, so the
// claim list keeps the batch kernel's centre-first order.
__global__ __launch_bounds__(256) void rrt_pixel_proof_kernel(const KParams* __restrict__ kpp) {
  const KParams& kp = *kpp;
  const uint32_t ix = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u;
  if (kp.strip_list && ix / 64u < kp.n_pixels / 64u && kp.strip_list[ix / 64u]) return;  // wave-uniform
  pixel_pass_one(kp, ix, lane);
}
// First level of the pixel pass: one lane per strip of 64 consecutive claim indices
// -- an 8x8 block (claim_r; with row-major claims, 64 / ts full rows of a tile for ts <= 64 or 64
// pixels of one row for ts >= 64) -- proven as a
// whole by rect_miss_proof; a proven strip's pixels get the pass's result for a proven pixel and
// its flag (kp.strip_list[s] = 1) sends the per-pixel pass's wave away; the others (and strips
// that leave the clip region) stay with the per-pixel pass.
__global__ __launch_bounds__(256) void rrt_strip_proof_kernel(const KParams* __restrict__ kpp) {
  const KParams& kp = *kpp;
  using namespace rrt;
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  const uint32_t ts = kp.tile_size, tpix = ts * ts;
  if (s < kp.n_pixels / 64u) {
    const uint32_t ix0 = s * 64u, tl = kp.tile_order[ix0 / tpix], r0 = claim_r(ix0 % tpix, ts);
    const uint32_t w = 8u, hh = 8u;
    const uint32_t x = kp.tiles[2 * tl] + r0 % ts, y = kp.tiles[2 * tl + 1] + r0 / ts;
    const bool inside = x >= kp.clip_x0 && y >= kp.clip_y0 && x + w <= kp.clip_x1 && y + hh <= kp.clip_y1;
    if (inside && rect_miss_proof(kp, (double)x, (double)y, (double)w, (double)hh)) {
      const uint32_t n = min(kp.ns_aa, kp.samples_per_batch);
      for (uint32_t k = 0; k < 64u; ++k) {
        const uint32_t slot = tl * tpix + claim_r(ix0 % tpix + k, ts);
        kp.rgb[3 * slot] = 0.0f; kp.rgb[3 * slot + 1] = 0.0f; kp.rgb[3 * slot + 2] = 0.0f;
        kp.count[slot] = (int32_t)n;
        if (kp.draws) kp.draws[slot] = n * kp.draws_miss;
      }
      kp.strip_list[s] = 1u;
    } else {
      kp.strip_list[s] = 0u;
    }
  }
}
// strips: the two-level pass (kp.strip_list set: the strip flags)
hipError_t rrt_launch_pixel_proof(const KParams* d_kp, uint32_t n_pixels, bool strips, hipStream_t stream) {
  if (strips)
    hipLaunchKernelGGL(rrt_strip_proof_kernel, dim3((n_pixels / 64u + 255) / 256), dim3(256), 0, stream, d_kp);
  hipLaunchKernelGGL(rrt_pixel_proof_kernel, dim3((n_pixels + 255) / 256), dim3(256), 0, stream, d_kp);
  return hipGetLastError();
}


// Sample 0 of every pixel, one lane per pixel (tile-list order, so a wave covers two rows of a
// tile).  Its draw offset is always 0, so it needs no speculation; its hit status then seeds the
// batch kernel's hypothesis for the pixel's other samples (all-hit and all-miss pixels -- 99.9%
// of cfg3 -- then need a single round), and its radiance is the first term of the pixel's sums.
template <int LEAN, int WAVES>
__global__ __launch_bounds__(256, WAVES) void rrt_first_kernel(const KParams* __restrict__ kpp) {
  const KParams& kp = *kpp;
  using namespace rrt;
  __shared__ ShadeLds cl;
  const uint32_t t = threadIdx.x;
  const uint32_t ts = kp.tile_size, tpix = ts * ts;
  const DCamera& cam = kp.cam;
  Counters cn = {};
  for (uint32_t p = blockIdx.x * blockDim.x + t; p < kp.n_pixels; p += gridDim.x * blockDim.x) {
    const uint32_t tl = p / tpix, r = p % tpix, lx = r % ts, ly = r / ts;
    const uint32_t x = kp.tiles[2 * tl] + lx, y = kp.tiles[2 * tl + 1] + ly;
    if (!(x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 && y < kp.clip_y1)) continue;
    Rng g; g.key = rrt_pixel_key(kp.seed, x, y); g.ctr = 0;
    double jx, jy; g.grid(jx, jy);
    const double sx = (double)x + jx, sy = (double)y + jy;
    const double cx = sx / kp.frame_w, cy = sy / kp.frame_h;  // Camera::generate_ray (:182-187)
    const double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
    const v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
    Isect is;
    const v3 wd = unit(w);
    const bool hit = !camera_proven_miss<false, LEAN == V_KERR>(kp, ld3(cam.pos), wd, cn) &&
                     query<false, false, LEAN == V_KERR, is_lean(LEAN)>(kp, ld3(cam.pos), wd, &is, cn);
    spec s = S(0, 0, 0);
    if (!hit && !is_lean(LEAN) && kp.env.w) s = env_dir(kp.env, unit(w));
    if (hit) {
      park_hit(cl, t, is);
      g.ctr = kp.draws_miss;
      const spec e = emission(kp.bsdfs[is.bsdf]);
      if (kp.max_ray_depth == 0) s = e;
      else if (is_lean(LEAN)) s = e + direct_importance_parked<false, LEAN>(kp, g, cl, t, cn);
      else if (kp.direct_hemisphere) s = e + direct_hemisphere_parked<false, LEAN>(kp, g, cl, t, cn);
      else s = e + direct_importance_parked<false, LEAN>(kp, g, cl, t, cn);
    }
    KParams::FirstSample f0;
    f0.r = s.r; f0.g = s.g; f0.b = s.b; f0.hit = hit ? 1u : 0u;
    kp.first[p] = f0;
  }
}

hipError_t rrt_launch_first(const KParams& kp, const KParams* d_kp, int lean, int waves, uint32_t grid, hipStream_t stream) {
  // waves/SIMD: 3 by default; the LEAN area-light build also at 4 / 5 (A/B)
  if (lean == 1 && waves == 4) hipLaunchKernelGGL((rrt_first_kernel<1, 4>), dim3(grid), dim3(256), 0, stream, d_kp);
  else if (lean == 1 && waves == 5) hipLaunchKernelGGL((rrt_first_kernel<1, 5>), dim3(grid), dim3(256), 0, stream, d_kp);
  else if (lean == 1) hipLaunchKernelGGL((rrt_first_kernel<1, 3>), dim3(grid), dim3(256), 0, stream, d_kp);
  else if (lean == 2) hipLaunchKernelGGL((rrt_first_kernel<2, 3>), dim3(grid), dim3(256), 0, stream, d_kp);
  else if (lean == rrt::V_KERR) hipLaunchKernelGGL((rrt_first_kernel<rrt::V_KERR, 3>), dim3(grid), dim3(256), 0, stream, d_kp);
  else hipLaunchKernelGGL((rrt_first_kernel<0, 3>), dim3(grid), dim3(256), 0, stream, d_kp);
  return hipGetLastError();
}

hipError_t rrt_launch_batch(const KParams& kp, const KParams* d_kp, int lean, int waves, uint32_t grid, hipStream_t stream) {
#define RRT_LAUNCH_B(L, W) hipLaunchKernelGGL((rrt_batch_kernel<L, W>), dim3(grid), dim3(256), 0, stream, d_kp)
  if (lean == 1) {
    switch (waves) {
      case 2: RRT_LAUNCH_B(1, 2); break;
      case 3: RRT_LAUNCH_B(1, 3); break;
      case 4: RRT_LAUNCH_B(1, 4); break;
      case 5: RRT_LAUNCH_B(1, 5); break;
      default: RRT_LAUNCH_B(1, 5); break;
    }
  } else if (lean == 2) {
    switch (waves) {
      case 3: RRT_LAUNCH_B(2, 3); break;
      case 4: RRT_LAUNCH_B(2, 4); break;
      default: RRT_LAUNCH_B(2, 5); break;
    }
  } else if (lean == rrt::V_KERR) {  // general builds: waves/SIMD as an A/B knob
    switch (waves) {
      case 2: RRT_LAUNCH_B(rrt::V_KERR, 2); break;
      case 4: RRT_LAUNCH_B(rrt::V_KERR, 4); break;
      case 5: RRT_LAUNCH_B(rrt::V_KERR, 5); break;
      default: RRT_LAUNCH_B(rrt::V_KERR, 3); break;
    }
  } else {
    switch (waves) {
      case 2: RRT_LAUNCH_B(0, 2); break;
      case 4: RRT_LAUNCH_B(0, 4); break;
      case 5: RRT_LAUNCH_B(0, 5); break;
      default: RRT_LAUNCH_B(0, 3); break;
    }
  }
#undef RRT_LAUNCH_B
  return hipGetLastError();
}

hipError_t rrt_launch_sample(const KParams& kp, const KParams* d_kp, int count, int lean, int waves, uint32_t grid, hipStream_t stream) {
#define RRT_LAUNCH(C, L, W) hipLaunchKernelGGL((rrt_sample_kernel<C, L, W>), dim3(grid), dim3(256), 0, stream, d_kp)
#define RRT_LAUNCH_DEEP(W) hipLaunchKernelGGL((rrt_sample_kernel<false, 0, W, true>), dim3(grid), dim3(256), 0, stream, d_kp)
  if (!count && kp.max_ray_depth >= 2 && lean != rrt::V_KERR) {  // bounce paths, general build
    switch (waves) {
      case 2: RRT_LAUNCH_DEEP(2); break;
      case 4: RRT_LAUNCH_DEEP(4); break;
      default: RRT_LAUNCH_DEEP(3); break;
    }
  } else if (count) {
    if (lean == rrt::V_KERR) RRT_LAUNCH(true, rrt::V_KERR, 1); else RRT_LAUNCH(true, 0, 1);
  } else if (lean == rrt::V_KERR) {
    RRT_LAUNCH(false, rrt::V_KERR, 2);
  } else if (lean == 1) {
    switch (waves) {
      case 2: RRT_LAUNCH(false, 1, 2); break;
      case 4: RRT_LAUNCH(false, 1, 4); break;
      case 5: RRT_LAUNCH(false, 1, 5); break;
      default: RRT_LAUNCH(false, 1, 3); break;
    }
  } else if (lean == 2) {
    RRT_LAUNCH(false, 2, 3);
  } else {
    RRT_LAUNCH(false, false, 2);
  }
#undef RRT_LAUNCH
#undef RRT_LAUNCH_DEEP
  return hipGetLastError();
}
