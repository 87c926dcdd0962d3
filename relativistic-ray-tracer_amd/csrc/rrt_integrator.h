// rrt_integrator.h -- the reference's integrator (part1_code.cpp:15-101): direct lighting by
// importance or hemisphere sampling and at_least_one_bounce_radiance's recursion as a loop, over
// the geodesic-marched query.  Shared by the per-pixel-loop kernel (rrt_kernel.hip) and the
// per-sample refill kernel (rrt_sample.hip) for max_ray_depth >= 2.
#pragma once
#include "rrt_device.h"

namespace rrt {

// ------------------------------------------------------------------ integrator (part1_code.cpp)
// `trace` = the geodesic-marched BVH query; DEEP (bounce) builds and depth <= 1 builds share it.
template <bool ANY, bool COUNT, bool DEEP, int LEAN>
__device__ __forceinline__ bool trace(const KParams& kp, v3 o, v3 d, Isect* is, Counters& cn) {
  return query<ANY, COUNT, LEAN == V_KERR, is_lean(LEAN)>(kp, o, d, is, cn);
}

// LEAN: area/point lights only, no microfacet BSDF.  The shading frame is rebuilt per light sample
// (same values: make_coord_space is a pure function of the normal) instead of being kept live
// across the shadow query, which keeps 12 VGPRs out of the traversal loop.
template <bool COUNT, int LEAN, bool DEEP>
__device__ spec direct_importance(const KParams& kp, Rng& g, const Isect& is, Counters& cn) {  // :33-57
  const DBsdf b = kp.bsdfs[is.bsdf];
  spec L = S(0, 0, 0);
  int total = 0;
  for (uint32_t li = 0; li < kp.n_lights; ++li) {
    const DLight& l = kp.lights[li];
    int num = l.is_delta ? 1 : (int)kp.ns_area_light;
    total += num;
    for (int i = 0; i < num; ++i) {
      v3 wi_world; float dist, pdf;
      spec sample = light_sample_L<LEAN>(kp.env, l, g, is.hit_p, wi_world, dist, pdf,
                                         LEAN == V_SW && (kp.sw & SW_ENV_HEMI));
      const Frame f = coord_space(is.n);
      v3 w_in = to_local(f, wi_world);
      if (w_in.z < 0) continue;
      spec contrib = ((sample * bsdf_f<LEAN>(b, to_local(f, is.w_out), w_in)) * (float)w_in.z) / pdf;
      if (!trace<true, COUNT, DEEP, LEAN>(kp, is.hit_p + smul(EPS_D, wi_world), wi_world, nullptr, cn)) L = L + contrib;
    }
  }
  return L / (float)total;
}

template <bool COUNT, int LEAN, bool DEEP>
__device__ spec direct_hemisphere(const KParams& kp, Rng& g, const Isect& is, Counters& cn) {  // :15-31
  Frame f = coord_space(is.n);
  v3 w_out = to_local(f, is.w_out);
  const DBsdf b = kp.bsdfs[is.bsdf];
  int num = (int)(kp.n_lights * kp.ns_area_light);
  spec L = S(0, 0, 0);
  for (int i = 0; i < num; ++i) {
    v3 w_in = hemisphere_sample(g);
    v3 wi_world = to_world(f, w_in);
    Isect is2;
    if (trace<false, COUNT, DEEP, LEAN>(kp, is.hit_p + smul(EPS_D, wi_world), wi_world, &is2, cn))
      L = L + (emission(kp.bsdfs[is2.bsdf]) * bsdf_f(b, w_out, w_in)) * (float)w_in.z;
  }
  return ((L * 2.0f) * (float)PI_D) / (float)num;
}

template <bool COUNT, int LEAN, bool DEEP>
__device__ __forceinline__ spec one_bounce(const KParams& kp, Rng& g, const Isect& is, Counters& cn) {
  if (is_lean(LEAN)) return direct_importance<COUNT, LEAN, DEEP>(kp, g, is, cn);
  return kp.direct_hemisphere ? direct_hemisphere<COUNT, general_of(LEAN), DEEP>(kp, g, is, cn)
                              : direct_importance<COUNT, general_of(LEAN), DEEP>(kp, g, is, cn);
}

// The per-level terms of at_least_one_bounce (the recursion's pending values): the level's direct
// light Ld, its flags (child: the bounce ray hit, so the level folds the child's radiance in; dl: the
// BSDF is a delta), and for a child the BSDF sample, |cos|, pdf and the hit's emission.
// LevelsPriv: private arrays, any depth <= RRT_MAX_DEPTH (they live in scratch: dynamic indices).
struct LevelsPriv {
  static constexpr int D = RRT_MAX_DEPTH;
  spec Ld[D], smp[D], cem[D];
  float cs[D], pd[D];
  bool child[D], dl[D];
  __device__ __forceinline__ void level(int k, spec ld, bool d) { Ld[k] = ld; child[k] = false; dl[k] = d; }
  __device__ __forceinline__ void bounce(int k, spec sm, float c, float p, spec em) {
    child[k] = true; smp[k] = sm; cs[k] = c; pd[k] = p; cem[k] = em;
  }
  __device__ __forceinline__ spec fold(int k) const {
    spec L = S(0, 0, 0);
    for (int j = k; j >= 0; --j) {
      spec Lj = Ld[j];
      if (child[j]) {
        spec Lc = L;
        if (dl[j]) Lc = Lc + cem[j];
        Lj = Lj + (((Lc * smp[j]) * cs[j]) / pd[j]) / (float)0.7;
      }
      L = Lj;
    }
    return L;
  }
};
// LevelsLds: the same terms in LDS, one column per thread of a 256-thread block, for frames of
// max_ray_depth <= D (the loop then never reaches RRT_MAX_DEPTH's cap): the bounce kernel's levels
// left scratch, whose writes were most of its HBM traffic (bounce paths).
template <int D_>
struct LevelLds {
  float v[11][D_][256];  // Ld rgb, smp rgb, cem rgb, cs, pd
  uint8_t fl[D_][256];   // 1: child, 2: dl
};
template <int D_>
struct LevelsLds {
  static constexpr int D = D_;
  LevelLds<D_>* p;
  uint32_t t;
  __device__ __forceinline__ void level(int k, spec ld, bool d) {
    p->v[0][k][t] = ld.r; p->v[1][k][t] = ld.g; p->v[2][k][t] = ld.b;
    p->fl[k][t] = d ? 2 : 0;
  }
  __device__ __forceinline__ void bounce(int k, spec sm, float c, float pp, spec em) {
    p->v[3][k][t] = sm.r; p->v[4][k][t] = sm.g; p->v[5][k][t] = sm.b;
    p->v[6][k][t] = em.r; p->v[7][k][t] = em.g; p->v[8][k][t] = em.b;
    p->v[9][k][t] = c; p->v[10][k][t] = pp;
    p->fl[k][t] |= 1;
  }
  __device__ __forceinline__ spec fold(int k) const {
    spec L = S(0, 0, 0);
    for (int j = k; j >= 0; --j) {
      spec Lj = S(p->v[0][j][t], p->v[1][j][t], p->v[2][j][t]);
      const uint8_t f = p->fl[j][t];
      if (f & 1) {
        spec Lc = L;
        if (f & 2) Lc = Lc + S(p->v[6][j][t], p->v[7][j][t], p->v[8][j][t]);
        Lj = Lj + (((Lc * S(p->v[3][j][t], p->v[4][j][t], p->v[5][j][t])) * p->v[9][j][t]) / p->v[10][j][t]) / (float)0.7;
      }
      L = Lj;
    }
    return L;
  }
};

// at_least_one_bounce_radiance (:69-101) unrolled into a loop: the recursion is walked down
// storing each level's terms, then folded back up in the reference's evaluation order.
template <bool COUNT, int LEAN, class LV = LevelsPriv>
__device__ __forceinline__ spec at_least_one_bounce(const KParams& kp, Rng& g, Isect cur, Counters& cn, LV lv = LV()) {
  uint32_t depth = kp.max_ray_depth;
  int k = 0;
  for (;; ++k) {
    Frame f = coord_space(cur.n);
    v3 w_out = to_local(f, cur.w_out);
    const DBsdf b = kp.bsdfs[cur.bsdf];
    spec L_out = S(0, 0, 0);
    if (!is_delta(b)) L_out = L_out + one_bounce<COUNT, general_of(LEAN), true>(kp, g, cur, cn);
    if (LEAN == V_SW && sw_illum(kp) == 3u && depth == kp.max_ray_depth) L_out = S(0, 0, 0);  // ILLUM 3 (:78-81)
    lv.level(k, L_out, is_delta(b));
    if (depth == kp.max_ray_depth || (depth > 1 && g.coin(0.7))) {
      v3 w_in; float pdf;
      spec sample = bsdf_sample_f(b, g, w_out, w_in, pdf, LEAN == V_SW && (kp.sw & SW_MF_HEMI));
      if (pdf == 0.0f) break;
      v3 wi_world = to_world(f, w_in);
      Isect is2;
      if (trace<false, COUNT, true, LEAN>(kp, cur.hit_p + smul(EPS_D, wi_world), wi_world, &is2, cn) && k + 1 < LV::D) {
        lv.bounce(k, sample, (float)fabs(w_in.z), pdf, emission(kp.bsdfs[is2.bsdf]));
        cur = is2;
        depth -= 1;
        continue;
      }
    }
    break;
  }
  return lv.fold(k);
}

}  // namespace rrt
