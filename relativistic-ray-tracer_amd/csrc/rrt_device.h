// rrt_device.h -- device-side restatement of the reference's math, geometry, BSDFs, lights and
// the geodesic-marched BVH query, shared by the kernels (rrt_kernel.hip, rrt_sample.hip).
//
// Numerics follow the reference exactly: double geometry (CGL Vector3D), float Spectrum with
// the reference's narrowing points, the same operation order, no FMA contraction (the pragma
// below plus -ffp-contract=off), IEEE division / sqrt.  Transcendentals whose arguments are
// per-run constants (tan of the half FOV, cos/sin of delta_theta) come from the host libm, i.e.
// the values the reference uses; per-sample sin, cos, acos, atan2, sinf and cosf are the host C
// library's own routines restated in rrt_glibm.h (bit-identical); the microfacet BSDF's tan, exp,
// log, atan and erf still use the device libm.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rrt_internal.h"
#include "../../include/rrt.h"  // RRT_AUDIT_* proof kinds
#include "rrt_rng.h"
#include "rrt_glibm.h"

#pragma clang fp contract(off)

#define PI_D 3.14159265358979323
#define EPS_D 0.00000000001

namespace rrt {

// ------------------------------------------------------------------ Vector3D (double)
struct v3 { double x, y, z; };
__device__ __forceinline__ v3 V(double x, double y, double z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 operator-(v3 a) { return V(-a.x, -a.y, -a.z); }
__device__ __forceinline__ v3 vmul(v3 a, double c) { return V(a.x * c, a.y * c, a.z * c); }
__device__ __forceinline__ v3 smul(double c, v3 a) { return V(c * a.x, c * a.y, c * a.z); }
__device__ __forceinline__ double dot(v3 u, v3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
__device__ __forceinline__ v3 cross(v3 u, v3 v) {
  return V(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
// Correctly rounded f64 sqrt / division, in-range fast path.  hipcc lowers sqrt and `/` to
// range-scaling wrappers (v_cmp + v_ldexp / v_div_scale, v_div_fmas, v_div_fixup, class
// checks) around a core of v_rsq / v_rcp + FMA refinements.  For operands of magnitude in
// [2^-300, 2^300] the scaling is never triggered and the fix-ups are identities, so the bare
// core below returns the same bits (checked bit for bit by tests/test_gpu_parity.py); other
// operands take the library path.
__device__ __forceinline__ bool in_core_range(double v) {
  const double a = fabs(v);
  return a >= 0x1p-300 && a <= 0x1p300;
}
__device__ __forceinline__ double sqrt_core(double x) {  // = llvm f64 sqrt expansion, scale 0
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  double d = fma(-g, g, x);
  h = fma(h, r, h);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
}
__device__ __forceinline__ double div_core(double a, double b) {  // = llvm f64 fdiv, no scaling
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  const double q = a * y;
  const double r = fma(-b, q, a);
  return fma(r, y, q);
}
__device__ __forceinline__ double xsqrt(double x) {
  if (__builtin_expect(!in_core_range(x), 0)) return sqrt(x);
  return sqrt_core(x);
}
__device__ __forceinline__ double xdiv(double a, double b) {
  if (__builtin_expect(!(in_core_range(a) && in_core_range(b)), 0)) return a / b;
  return div_core(a, b);
}
__device__ __forceinline__ double norm(v3 a) { return xsqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ double norm2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ v3 unit(v3 a) {
  double r = xdiv(1., xsqrt(a.x * a.x + a.y * a.y + a.z * a.z));
  return V(r * a.x, r * a.y, r * a.z);
}
__device__ __forceinline__ v3 normalize(v3 a) { double c = xdiv(1., norm(a)); return V(a.x * c, a.y * c, a.z * c); }
__device__ __forceinline__ v3 divd(v3 a, double c) { double rc = xdiv(1.0, c); return V(rc * a.x, rc * a.y, rc * a.z); }
__device__ __forceinline__ double std_min(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double std_max(double a, double b) { return (a < b) ? b : a; }
__device__ __forceinline__ v3 ld3(const double* p) { return V(p[0], p[1], p[2]); }

// ------------------------------------------------------------------ Spectrum (float)
struct spec { float r, g, b; };
__device__ __forceinline__ spec S(float r, float g, float b) { spec s; s.r = r; s.g = g; s.b = b; return s; }
__device__ __forceinline__ spec operator+(spec a, spec b) { return S(a.r + b.r, a.g + b.g, a.b + b.b); }
__device__ __forceinline__ spec operator-(spec a, spec b) { return S(a.r - b.r, a.g - b.g, a.b - b.b); }
__device__ __forceinline__ spec operator*(spec a, spec b) { return S(a.r * b.r, a.g * b.g, a.b * b.b); }
__device__ __forceinline__ spec operator/(spec a, spec b) { return S(a.r / b.r, a.g / b.g, a.b / b.b); }
__device__ __forceinline__ spec operator*(spec a, float s) { return S(a.r * s, a.g * s, a.b * s); }
__device__ __forceinline__ spec operator/(spec a, float s) { return S(a.r / s, a.g / s, a.b / s); }
__device__ __forceinline__ spec operator+(spec a, float s) { return S(a.r + s, a.g + s, a.b + s); }
__device__ __forceinline__ float illum(spec s) { return 0.2126f * s.r + 0.7152f * s.g + 0.0722f * s.b; }

// ------------------------------------------------------------------ RNG + samplers
struct Rng {
  uint64_t key;
  uint32_t ctr;
  __device__ __forceinline__ double uniform() { return ((double)rrt_keyed_rand(key, ctr++)) / 2147483647.0; }
  __device__ __forceinline__ bool coin(double p) { return uniform() < p; }
  // UniformGridSampler2D (sampler.cpp:7-11): g++ evaluates Vector2D(ru(), ru()) right to left
  __device__ __forceinline__ void grid(double& x, double& y) { y = uniform(); x = uniform(); }
};
__device__ __forceinline__ v3 cosine_sample(Rng& g, float* pdf) {  // sampler.cpp:47-56
  double Xi1 = g.uniform();
  double Xi2 = g.uniform();
  double r = sqrt(Xi1);
  double theta = 2. * PI_D * Xi2;
  *pdf = (float)(sqrt(1 - Xi1) / PI_D);
  return V(r * rrt_glibm_cos(theta), r * rrt_glibm_sin(theta), sqrt(1 - Xi1));
}
__device__ __forceinline__ v3 hemisphere_sample(Rng& g) {  // sampler.cpp:15-29 (float trig)
  double Xi1 = g.uniform();
  double Xi2 = g.uniform();
  double theta = rrt_glibm_acos(Xi1);
  double phi = 2.0 * PI_D * Xi2;
  double xs = rrt_glibm_sinf((float)theta) * rrt_glibm_cosf((float)phi);
  double ys = rrt_glibm_sinf((float)theta) * rrt_glibm_sinf((float)phi);
  double zs = rrt_glibm_cosf((float)theta);
  return V(xs, ys, zs);
}

#ifndef RRT_PROFILE
#define RRT_PROFILE 0  // 1: diagnostic build with per-phase cycle counters (tools/phase_profile.py)
#endif
struct Counters {
  uint32_t bbox, micro, prim, query;
#if RRT_PROFILE
  uint64_t t_micro, t_trav, t_query, t_proof, t_squery, t_strav;
  uint64_t t_claim, t_chain, t_shade, t_fold;  // batch kernel phases
#endif
};
#if RRT_PROFILE
#define RRT_T0(v) const uint64_t v = clock64()
#define RRT_ACC(field, v) cn.field += clock64() - v
#else
#define RRT_T0(v)
#define RRT_ACC(field, v)
#endif

// ------------------------------------------------------------------ geometry
// Correctly rounded a / b given y = RN(1/b): two Markstein correction steps (residuals exact by
// FMA).  Equals IEEE a / b whenever nothing under/overflows (Markstein's theorem); callers only
// use it in ranges where that is guaranteed (see in_fast_range / rrt_host.cpp fast_div).
__device__ __forceinline__ double qdiv(double a, double b, double y) {
  double q0 = a * y;
  double r0 = fma(-q0, b, a);
  double q1 = fma(r0, y, q0);
  double r1 = fma(-q1, b, a);
  return fma(r1, y, q1);
}
__device__ __forceinline__ bool in_fast_range(double v) {
  const double a = fabs(v);
  return v == 0.0 || (a >= 0x1p-800 && a <= 0x1p20);
}
// BBox::intersect (bbox.cpp:10-25), dividing by the segment direction; min_t is 0 for every
// micro segment.  EXACT: IEEE division; else qdiv with the per-segment reciprocals y.
template <bool EXACT>
__device__ __forceinline__ bool slab(const double* mn, const double* mx, v3 o, v3 d, v3 y, double max_t) {
  double tx0, tx1, ty0, ty1, tz0, tz1;
  if (EXACT) {
    tx0 = (mn[0] - o.x) / d.x; tx1 = (mx[0] - o.x) / d.x;
    ty0 = (mn[1] - o.y) / d.y; ty1 = (mx[1] - o.y) / d.y;
    tz0 = (mn[2] - o.z) / d.z; tz1 = (mx[2] - o.z) / d.z;
  } else {
    const double nx0 = mn[0] - o.x, nx1 = mx[0] - o.x, ny0 = mn[1] - o.y, ny1 = mx[1] - o.y,
                 nz0 = mn[2] - o.z, nz1 = mx[2] - o.z;
    {  // approximate-then-verify: the products n * y are within 2^-50 (relative to the result of
       // the min / max chains) of the exact RN(n / d) on a fast segment, so a decision that
       // holds with a 2^-45 relative margin is the exact test's decision; the rest go exact.
      const double ax0 = nx0 * y.x, ax1 = nx1 * y.x, ay0 = ny0 * y.y, ay1 = ny1 * y.y, az0 = nz0 * y.z,
                   az1 = nz1 * y.z;
      const double amin = fmax(fmax(fmin(ax0, ax1), fmin(ay0, ay1)), fmin(az0, az1)),
                   amax = fmin(fmin(fmax(ax0, ax1), fmax(ay0, ay1)), fmax(az0, az1));
      const double e = 0x1p-45, m1 = e * (fabs(amin) + fabs(amax)), m2 = e * (fabs(amin) + max_t),
                   m3 = e * fabs(amax);
      if (amin > amax + m1 || amin > max_t + m2 || amax < -m3) return false;
      if (amin <= amax - m1 && amin <= max_t - m2 && amax >= m3) return true;
    }
    tx0 = qdiv(nx0, d.x, y.x); tx1 = qdiv(nx1, d.x, y.x);
    ty0 = qdiv(ny0, d.y, y.y); ty1 = qdiv(ny1, d.y, y.y);
    tz0 = qdiv(nz0, d.z, y.z); tz1 = qdiv(nz1, d.z, y.z);
    // On a fast segment every quotient is finite (|d| >= 2^-800, |n - o| <= 2^21), so
    // std::min/max (NaN -> first argument) and the hardware v_min/max_f64 agree except on the
    // sign of a zero, which no comparison below can see.
    const double tmin = fmax(fmax(fmin(tx0, tx1), fmin(ty0, ty1)), fmin(tz0, tz1)),
                 tmax = fmin(fmin(fmax(tx0, tx1), fmax(ty0, ty1)), fmax(tz0, tz1));
    return tmin <= tmax && tmin <= max_t && tmax >= 0.0;
  }
  double tmin = std_max(std_max(std_min(tx0, tx1), std_min(ty0, ty1)), std_min(tz0, tz1)),
         tmax = std_min(std_min(std_max(tx0, tx1), std_max(ty0, ty1)), std_max(tz0, tz1));
  return tmin <= tmax && tmin <= max_t && tmax >= 0.0;
}
template <bool EXACT>
__device__ __forceinline__ bool slab(const DNode& n, v3 o, v3 d, v3 y, double max_t) {
  return slab<EXACT>(n.mn, n.mx, o, d, y, max_t);
}
// exact chosen per segment at run time (one copy of the walk; non-fast segments are rare)
__device__ __forceinline__ bool slab_rt(const double* mn, const double* mx, v3 o, v3 d, v3 y, double max_t,
                                        bool exact) {
  if (__builtin_expect(exact, 0)) return slab<true>(mn, mx, o, d, y, max_t);
  return slab<false>(mn, mx, o, d, y, max_t);
}
// May the segment (o, d) use qdiv?  Quotients (n - o) / d then stay in [2^-852, 2^820] or 0.
__device__ __forceinline__ bool segment_fast(const KParams& kp, v3 o, v3 d) {
  return kp.fast_div && in_fast_range(o.x) && in_fast_range(o.y) && in_fast_range(o.z) &&
         fabs(d.x) >= 0x1p-800 && fabs(d.y) >= 0x1p-800 && fabs(d.z) >= 0x1p-800;
}
// Is the micro segment [o, o + d max_t] provably clear of every BVH leaf box (DGrid)?  Then the
// reference's traversal of it tests no primitive and returns "no hit"; skipping it is
// result-identical.  Points outside the grid answer "not provably clear".
// The grid cell of point o, or -1 (no grid, or o outside it).
__device__ __forceinline__ int grid_cell(const DGrid& g, v3 o) {
  if (!g.k) return -1;
  const double fx = (o.x - g.g0[0]) * g.inv_h, fy = (o.y - g.g0[1]) * g.inv_h, fz = (o.z - g.g0[2]) * g.inv_h;
  if (!(fx >= 0.0 && fy >= 0.0 && fz >= 0.0 && fx < (double)g.n[0] && fy < (double)g.n[1] && fz < (double)g.n[2]))
    return -1;
  const int ix = (int)fx, iy = (int)fy, iz = (int)fz;
  return (iz * g.n[1] + iy) * g.n[0] + ix;
}
__device__ __forceinline__ bool cell_clear(const DGrid& g, int cell, double max_t) {
  return cell >= 0 && (double)((int)g.k[cell] - 2) * g.h_free > max_t;
}
__device__ __forceinline__ bool segment_clear(const DGrid& g, v3 o, double max_t) {
  return cell_clear(g, grid_cell(g, o), max_t);
}
// Does the segment [o, e] keep, along some axis, more than plane_eps (~1e6 ulps of the scene
// scale) outside the root box?  Then the reference's first test -- the root box slab test --
// fails: on that axis both quotients (bound - o) / d have the sign and size of a point outside
// [0, max_t] by far more than rounding (d = 0: both are the same infinity), so tmin > max_t or
// tmax < 0.  Nothing else of the walk runs, so skipping it (and the reciprocals it needs) is
// result-identical.
__device__ __forceinline__ bool segment_outside_root(const KParams& kp, v3 o, v3 e) {
  return fmax(o.x, e.x) < kp.root_lo[0] || fmin(o.x, e.x) > kp.root_hi[0] || fmax(o.y, e.y) < kp.root_lo[1] ||
         fmin(o.y, e.y) > kp.root_hi[1] || fmax(o.z, e.z) < kp.root_lo[2] || fmin(o.z, e.z) > kp.root_hi[2];
}
// Sphere::test + the range checks of Sphere::intersect (sphere.cpp:10-53), min_t = 0
__device__ __forceinline__ bool sphere_t(v3 c, double r2, v3 o, v3 d, double max_t, double& t) {
  v3 tmp = o - c;
  double b = 2 * dot(tmp, d), cc = norm2(tmp) - r2, disc = b * b - 4 * cc;
  if (disc < 0) return false;
  double t1 = (-b - sqrt(disc)) / 2, t2 = (-b + sqrt(disc)) / 2;
  if (0.0 <= t1 && t1 <= max_t) { t = t1; return true; }
  if (0.0 <= t2 && t2 <= max_t) { t = t2; return true; }
  return false;
}
// sphere_t with tmp = o - c and |tmp|^2 already known (the hole's capture test, query())
__device__ __forceinline__ bool sphere_t_rel(v3 tmp, double tmp2, double r2, v3 d, double max_t) {
  double b = 2 * dot(tmp, d), cc = tmp2 - r2, disc = b * b - 4 * cc;
  if (disc < 0) return false;
  double t1 = (-b - sqrt(disc)) / 2, t2 = (-b + sqrt(disc)) / 2;
  return (0.0 <= t1 && t1 <= max_t) || (0.0 <= t2 && t2 <= max_t);
}
// Triangle::intersect (triangle.cpp:25-55) with e1, e2 precomputed (bit-identical values)
__device__ __forceinline__ bool tri_t(const DPrimGeo& gp, v3 o, v3 d, double max_t, double& t, double& b1o,
                                      double& b2o) {
  v3 p0 = V(gp.v[0], gp.v[1], gp.v[2]), e1 = V(gp.v[3], gp.v[4], gp.v[5]), e2 = V(gp.v[6], gp.v[7], gp.v[8]);
  v3 s = o - p0, s1 = cross(d, e2), s2 = cross(s, e1);
  double inv = xdiv(1., dot(s1, e1));
  double tt = dot(s2, e2) * inv, b1 = dot(s1, s) * inv, b2 = dot(s2, d) * inv, b0 = 1 - b1 - b2;
  if (0.0 <= tt && tt <= max_t && b0 >= 0 && b1 >= 0 && b2 >= 0) { t = tt; b1o = b1; b2o = b2; return true; }
  return false;
}

struct Isect { v3 hit_p, w_out, n; int bsdf; };

// BVHAccel::intersect_micro (bvh.cpp:115-138) for one micro segment.  ANY: shadow query, stop
// at the first accepted primitive (only the boolean is used; result-identical).
template <bool ANY, bool COUNT, bool EXACT>
__device__ __forceinline__ bool traverse(const KParams& kp, v3 o, v3 d, v3 y, double& max_t, int& hit_slot,
                                         double& hb1, double& hb2, Counters& cn) {
  bool hit = false;
  int node = 0;
  while (node >= 0) {
    const DNode n = kp.nodes[node];
    if (COUNT) cn.bbox++;
    if (!slab<EXACT>(n, o, d, y, max_t)) { node = n.skip; continue; }
    if (n.count == 0) { node = node + 1; continue; }
    for (int i = 0; i < n.count; ++i) {
      const int slot = n.first + i;
      const DPrimMeta meta = kp.meta[slot];
      const DPrimGeo gp = kp.geo[slot];
      if (COUNT) cn.prim++;
      double t, b1 = 0, b2 = 0;
      bool ok = (meta & 1u) ? sphere_t(V(gp.v[0], gp.v[1], gp.v[2]), gp.v[3], o, d, max_t, t)
                            : tri_t(gp, o, d, max_t, t, b1, b2);
      if (ok) {
        max_t = t; hit = true; hit_slot = slot; hb1 = b1; hb2 = b2;
        if (ANY) return true;
      }
    }
    node = n.skip;
  }
  return hit;
}

// Test the primitives of an accepted leaf (slots [first, first + count)), as intersect_micro's
// leaf loop: every accepted hit shrinks max_t (t <= max_t: a later equal t wins).
template <bool ANY>
__device__ __forceinline__ bool leaf_prims(const KParams& kp, int first, int count, v3 o, v3 d, double& max_t,
                                           int& hit_slot, double& hb1, double& hb2) {
  bool hit = false;
  for (int i = 0; i < count; ++i) {
    const int slot = first + i;
    const DPrimMeta meta = kp.meta[slot];
    const DPrimGeo gp = kp.geo[slot];
    double t, b1 = 0, b2 = 0;
    const bool ok = (meta & 1u) ? sphere_t(V(gp.v[0], gp.v[1], gp.v[2]), gp.v[3], o, d, max_t, t)
                                : tri_t(gp, o, d, max_t, t, b1, b2);
    if (ok) {
      max_t = t; hit = true; hit_slot = slot; hb1 = b1; hb2 = b2;
      if (ANY) return true;
    }
  }
  return hit;
}

// Plane cull: may primitive `slot` accept a segment whose end points lie at signed distances
// a, b from its supporting plane?  Triangle::intersect accepts only if the segment meets the
// plane at some t in [0, max_t]; with both ends farther than plane_eps on one side it cannot
// -- its t is then out of range by far more than rounding (the margin is ~1e6 ulps of the
// scene scale, and sliver triangles, whose rounding is unbounded, carry n = 0: never culled).
// max_t only shrinks along the walk, so the segment's first end point b stays valid.
__device__ __forceinline__ bool plane_may_hit(const DPlane& pl, v3 o, v3 e, double eps) {
  const double a = (pl.n[0] * o.x + pl.n[1] * o.y + pl.n[2] * o.z) - pl.c;
  const double b = (pl.n[0] * e.x + pl.n[1] * e.y + pl.n[2] * e.z) - pl.c;
  return !((a > eps && b > eps) || (a < -eps && b < -eps));
}
// leaf_prims with the plane cull in front of every primitive test (skipped primitives are ones
// the reference tests and rejects, so the answer is the same)
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool leaf_prims_cull(const KParams& kp, int first, int count, v3 o, v3 d, v3 e,
                                                double& max_t, int& hit_slot, double& hb1, double& hb2,
                                                Counters& cn) {
  bool hit = false;
  for (int i = 0; i < count; ++i) {
    const int slot = first + i;
    if (COUNT) cn.query++;  // plane tests (executed-work counting)
    if (!plane_may_hit(kp.planes[slot], o, e, kp.plane_eps)) continue;
    if (COUNT) cn.prim++;
    const DPrimMeta meta = kp.meta[slot];
    const DPrimGeo gp = kp.geo[slot];
    double t, b1 = 0, b2 = 0;
    const bool ok = (meta & 1u) ? sphere_t(V(gp.v[0], gp.v[1], gp.v[2]), gp.v[3], o, d, max_t, t)
                                : tri_t(gp, o, d, max_t, t, b1, b2);
    if (ok) {
      max_t = t; hit = true; hit_slot = slot; hb1 = b1; hb2 = b2;
      if (ANY) return true;
    }
  }
  return hit;
}
// Does any primitive of the leaf survive the plane cull?
template <bool COUNT>
__device__ __forceinline__ bool leaf_may_hit(const KParams& kp, int first, int count, v3 o, v3 e, Counters& cn) {
  bool any = false;
  for (int i = 0; i < count; ++i) any |= plane_may_hit(kp.planes[first + i], o, e, kp.plane_eps);
  if (COUNT) cn.query += (uint32_t)count;
  return any;
}

// next set bit >= from of the oversized-leaf mask (bit i = kp.big[i]), or nb
__device__ __forceinline__ int next_big_in(uint64_t m, int from, int nb) {
  const uint64_t r = from < 64 ? (m >> from) : 0ull;
  return r ? min(from + (int)__builtin_ctzll(r), nb) : nb;
}
// BVHAccel::intersect_micro's result (bvh.cpp:115-138) from the search tree (rrt_host.cpp
// build_free_tree): an SAH hierarchy over the reference tree's leaves -- their boxes and slot runs
// are the reference's own -- without the oversized ones (the room's walls and lights, kp.big,
// tested from a short list).  Why only leaf boxes matter: the slab test is monotone under box
// inclusion (every quotient RN((m - o) / d) is monotone in m), so a passing leaf passes the
// inner boxes above it, in any hierarchy; inner boxes only prune.
// 1. Walk the search tree at the segment's full max_t L, in its own order, testing every leaf
//    whose box passes (plus the oversized leaves): exactly the leaves whose boxes pass at L, the
//    only ones the reference can test (max_t only shrinks and the slab test is monotone in it).
//    No primitive accepted at L  <=>  the reference finds no hit (order plays no part): done.
//    A shadow query (ANY) stops at the first accepted primitive, as before.
// 2. A closest-hit query keeps the slots of the primitives accepted at L (4 per window; more take
//    further windows above the last kept slot) with their leaves, and replays the reference on
//    them in slot order --
//    slots are laid out in left-first leaf order, so slot order is the reference's visiting order:
//    a leaf's box is tested once, with the max_t the reference would hold on reaching it, and its
//    accepted primitives re-tested with that max_t.  Every other primitive the reference tests is
//    rejected at L, hence at any max_t <= L (acceptance is t in [0, max_t] plus tests that do not
//    depend on max_t; a sphere returns the same t whenever it accepts), so it changes nothing.
//    Leaves without an accepted primitive do not change max_t, so the replay's max_t at each
//    accepted leaf is the reference's: the result (slot, t, barycentrics) is the reference's.
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool traverse_free(const KParams& kp, v3 o, v3 d, v3 y, double& max_t, int& hit_slot,
                                              double& hb1, double& hb2, Counters& cn, bool exact,
                                              uint64_t bmask = ~0ull, bool any_rt = false) {
  if (COUNT) cn.bbox++;
  if (!slab_rt(kp.nodes[0].mn, kp.nodes[0].mx, o, d, y, max_t, exact)) return false;
  bmask &= kp.free_big_mask;  // the local oversized leaves sit in the search tree
  const double L = max_t;
  const v3 e = o + vmul(d, L);
  const int nb = (int)kp.n_big;
  bool hit = false;
  double m = L;  // the reference's max_t as the replay goes
  // Windows of the accepted primitives in slot order: each collect pass keeps the 4 smallest
  // accepted slots above `after` (more than 4 on one segment take another pass); a leaf cut by
  // the window edge keeps its box outcome for the next window
  int32_t after = -1, leaf_cut = 0x7fffffff;
  bool cut_pass = false;
#pragma unroll 1
  for (;;) {
    int32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    int na = 0;
    bool more = false;
    // ---- collect: every leaf whose box passes at L -- the oversized leaves (the room's walls
    // and lights: plane cull first, their boxes pass for almost every segment), then the search
    // tree -- one item per iteration, so both kinds share one box test and one primitive loop
    int bi = next_big_in(bmask, 0, nb), node = 0;
#pragma unroll 1
    for (;;) {
      const bool big = bi < nb;
      if (!big && node < 0) break;
      const DNode* n = big ? nullptr : &kp.free_nodes[node];
      const double* mn = big ? kp.big[bi].mn : n->mn;
      const double* mx = big ? kp.big[bi].mx : n->mx;
      const int first = big ? kp.big[bi].first : n->first;
      const int count = big ? kp.big[bi].count : n->count;
      bool pass = !big || leaf_may_hit<COUNT>(kp, first, count, o, e, cn);
      if (pass) {
        if (COUNT) cn.bbox++;
        pass = slab_rt(mn, mx, o, d, y, L, exact);
      }
      if (pass && count != 0) {
        const int32_t ref = big ? -1 - bi : node;
#pragma unroll 1
        for (int i = 0; i < count; ++i) {
          const int32_t slot = first + i;
          if (slot <= after) continue;
          if (COUNT) cn.query++;
          if (!plane_may_hit(kp.planes[slot], o, e, kp.plane_eps)) continue;
          if (COUNT) cn.prim++;
          const DPrimMeta meta = kp.meta[slot];
          const DPrimGeo gp = kp.geo[slot];
          double t, b1 = 0, b2 = 0;
          const bool ok = (meta & 1u) ? sphere_t(V(gp.v[0], gp.v[1], gp.v[2]), gp.v[3], o, d, L, t)
                                      : tri_t(gp, o, d, L, t, b1, b2);
          if (!ok) continue;
          if (ANY || any_rt) return true;
          if (na == 4) {  // keep the 4 smallest
            more = true;
            if (slot > s3) continue;
            --na;
          }
          // insert keeping s0 < s1 < s2 < s3 (slots are distinct): shift the larger ones up
          bool placed = false;
          if (na >= 3) { if (s2 > slot) { s3 = s2; r3 = r2; } else { s3 = slot; r3 = ref; placed = true; } }
          if (!placed && na >= 2) { if (s1 > slot) { s2 = s1; r2 = r1; } else { s2 = slot; r2 = ref; placed = true; } }
          if (!placed && na >= 1) { if (s0 > slot) { s1 = s0; r1 = r0; } else { s1 = slot; r1 = ref; placed = true; } }
          if (!placed) { s0 = slot; r0 = ref; }
          ++na;
        }
      }
      if (big) bi = next_big_in(bmask, bi + 1, nb);
      else node = (pass && count == 0) ? node + 1 : n->skip;
    }
    if (ANY || na == 0) break;
    // ---- replay the reference on this window, in slot (= its visiting) order: a leaf's box is
    // tested once, with the max_t held on reaching it
    bool pass = false;
    int32_t cur = 0x7fffffff;
#pragma unroll 1
    for (int k = 0; k < na; ++k) {
      const int32_t slot = k == 0 ? s0 : k == 1 ? s1 : k == 2 ? s2 : s3;
      const int32_t ref = k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : r3;
      if (ref != cur) {
        cur = ref;
        const double* mn = ref >= 0 ? kp.free_nodes[ref].mn : kp.big[-1 - ref].mn;
        const double* mx = ref >= 0 ? kp.free_nodes[ref].mx : kp.big[-1 - ref].mx;
        pass = ref == leaf_cut ? cut_pass : slab_rt(mn, mx, o, d, y, m, exact);
      }
      if (!pass) continue;
      const DPrimMeta meta = kp.meta[slot];
      const DPrimGeo gp = kp.geo[slot];
      double t, b1 = 0, b2 = 0;
      const bool ok = (meta & 1u) ? sphere_t(V(gp.v[0], gp.v[1], gp.v[2]), gp.v[3], o, d, m, t)
                                  : tri_t(gp, o, d, m, t, b1, b2);
      if (ok) { m = t; hit = true; hit_slot = slot; hb1 = b1; hb2 = b2; }
    }
    if (!more) break;
    after = s3; leaf_cut = r3; cut_pass = pass;
  }
  max_t = m;
  return hit;
}

// traverse_free over the 4-wide search tree (kp.free4, rrt_host.cpp build_free4): the same leaves,
// each tested with the same slab test at L, but four child boxes per node load -- a walk of a slow
// pixel's micro segment is a chain of ~40 dependent box tests on the binary tree, ~10 node loads
// here.  The collect order differs, which the collect pass allows (it keeps every
// primitive accepted at L; the replay below is traverse_free's).  DFS stack: up to 8 node indices
// of 16 bits in two registers; returns 2 when it would overflow (no result: the caller walks the
// binary tree), else hit (1) or not (0).
template <bool ANY, bool COUNT>
__device__ __forceinline__ int traverse_free4(const KParams& kp, v3 o, v3 d, v3 y, double& max_t, int& hit_slot,
                                              double& hb1, double& hb2, Counters& cn, bool exact,
                                              uint64_t bmask = ~0ull, bool any_rt = false) {
  // the f32 pre-test's range: origins within free4_omax (else the binary walk)
  if (!(fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z)) <= kp.free4_omax)) return 2;
  if (COUNT) cn.bbox++;
  if (!slab_rt(kp.nodes[0].mn, kp.nodes[0].mx, o, d, y, max_t, exact)) return 0;
  bmask &= kp.free_big_mask;
  const double L = max_t;
  const v3 e = o + vmul(d, L);
  const int nb = (int)kp.n_big;
  bool hit = false;
  double m = L;
  int32_t after = -1, leaf_cut = 0x7fffffff;
  bool cut_pass = false;
  // the segment in f32 for the pre-test: origin rounded to nearest, reciprocals clamped finite,
  // the length rounded up
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  const float ix = (float)fmin(fmax(y.x, -1e30), 1e30), iy = (float)fmin(fmax(y.y, -1e30), 1e30),
              iz = (float)fmin(fmax(y.z, -1e30), 1e30);
  const float Lf = (float)(L * (1.0 + 1e-6)) * 1.000001f;
#pragma unroll 1
  for (;;) {
    int32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    int na = 0;
    bool more = false;
    // a leaf whose box passed at L: its primitives accepted at L into the window (traverse_free)
    auto take = [&](int32_t first, int32_t count, int32_t ref) -> bool {  // true: a shadow query's hit
#pragma unroll 1
      for (int i = 0; i < count; ++i) {
        const int32_t slot = first + i;
        if (slot <= after) continue;
        if (COUNT) cn.query++;
        if (!plane_may_hit(kp.planes[slot], o, e, kp.plane_eps)) continue;
        if (COUNT) cn.prim++;
        const DPrimMeta meta = kp.meta[slot];
        const DPrimGeo gp = kp.geo[slot];
        double t, b1 = 0, b2 = 0;
        const bool ok = (meta & 1u) ? sphere_t(V(gp.v[0], gp.v[1], gp.v[2]), gp.v[3], o, d, L, t)
                                    : tri_t(gp, o, d, L, t, b1, b2);
        if (!ok) continue;
        if (ANY || any_rt) return true;
        if (na == 4) {
          more = true;
          if (slot > s3) continue;
          --na;
        }
        bool placed = false;
        if (na >= 3) { if (s2 > slot) { s3 = s2; r3 = r2; } else { s3 = slot; r3 = ref; placed = true; } }
        if (!placed && na >= 2) { if (s1 > slot) { s2 = s1; r2 = r1; } else { s2 = slot; r2 = ref; placed = true; } }
        if (!placed && na >= 1) { if (s0 > slot) { s1 = s0; r1 = r0; } else { s1 = slot; r1 = ref; placed = true; } }
        if (!placed) { s0 = slot; r0 = ref; }
        ++na;
      }
      return false;
    };
    // the room-spanning oversized leaves (plane cull first)
#pragma unroll 1
    for (int bi = next_big_in(bmask, 0, nb); bi < nb; bi = next_big_in(bmask, bi + 1, nb)) {
      const DBig& B = kp.big[bi];
      if (!leaf_may_hit<COUNT>(kp, B.first, B.count, o, e, cn)) continue;
      if (COUNT) cn.bbox++;
      if (!slab_rt(B.mn, B.mx, o, d, y, L, exact)) continue;
      if (take(B.first, B.count, -1 - bi)) return 1;
    }
    // the tree: the search tree's root box, then its nodes four children at a time
    if (COUNT) cn.bbox++;
    if (slab_rt(kp.free_nodes[0].mn, kp.free_nodes[0].mx, o, d, y, L, exact)) {
      uint64_t st0 = 0, st1 = 0;
      int sp = 0;
      uint32_t cur = 0;
#pragma unroll 1
      for (;;) {
        const DNode4& N = kp.free4[cur];
        uint32_t pass = 0;
        // the conservative f32 pre-test of the four children (widened boxes: never fails a box the
        // exact test passes)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a0 = (N.mnx[i] - ox) * ix, a1 = (N.mxx[i] - ox) * ix;
          const float b0 = (N.mny[i] - oy) * iy, b1 = (N.mxy[i] - oy) * iy;
          const float c0 = (N.mnz[i] - oz) * iz, c1 = (N.mxz[i] - oz) * iz;
          const float tmin = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fminf(c0, c1));
          const float tmax = fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fmaxf(c0, c1));
          if (N.count[i] >= 0 && !(tmin > tmax || tmin > Lf || tmax < 0.0f)) pass |= 1u << i;
        }
#pragma unroll 1
        while (pass) {
          const int i = (int)__builtin_ctz(pass);
          pass &= pass - 1;
          if (N.count[i] > 0) {
            // a leaf: the exact test on its own box (traverse_free's), then its primitives
            const DNode& F = kp.free_nodes[N.child[i]];
            if (COUNT) cn.bbox++;
            if (!slab_rt(F.mn, F.mx, o, d, y, L, exact)) continue;
            if (take(N.first[i], N.count[i], N.child[i])) return 1;
          } else {
            if (sp == 8) return 2;  // the stack is full: the caller walks the binary tree
            st1 = (st1 << 16) | (st0 >> 48);
            st0 = (st0 << 16) | (uint64_t)(uint32_t)N.child[i];
            ++sp;
          }
        }
        if (sp == 0) break;
        cur = (uint32_t)(st0 & 0xffffull);
        st0 = (st0 >> 16) | (st1 << 48);
        st1 >>= 16;
        --sp;
      }
    }
    if (ANY || na == 0) break;
    // ---- replay the reference on this window, in slot (= its visiting) order (traverse_free)
    bool pass = false;
    int32_t curr = 0x7fffffff;
#pragma unroll 1
    for (int k = 0; k < na; ++k) {
      const int32_t slot = k == 0 ? s0 : k == 1 ? s1 : k == 2 ? s2 : s3;
      const int32_t ref = k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : r3;
      if (ref != curr) {
        curr = ref;
        const double* mn = ref >= 0 ? kp.free_nodes[ref].mn : kp.big[-1 - ref].mn;
        const double* mx = ref >= 0 ? kp.free_nodes[ref].mx : kp.big[-1 - ref].mx;
        pass = ref == leaf_cut ? cut_pass : slab_rt(mn, mx, o, d, y, m, exact);
      }
      if (!pass) continue;
      const DPrimMeta meta = kp.meta[slot];
      const DPrimGeo gp = kp.geo[slot];
      double t, b1 = 0, b2 = 0;
      const bool ok = (meta & 1u) ? sphere_t(V(gp.v[0], gp.v[1], gp.v[2]), gp.v[3], o, d, m, t)
                                  : tri_t(gp, o, d, m, t, b1, b2);
      if (ok) { m = t; hit = true; hit_slot = slot; hb1 = b1; hb2 = b2; }
    }
    if (!more) break;
    after = s3; leaf_cut = r3; cut_pass = pass;
  }
  max_t = m;
  return hit ? 1 : 0;
}

// BlackHole::next_micro_ray (blackhole.cpp:17-40); f4 is computed but unused there.  Each norm
// is computed once and its reciprocal shared: normalize(v) = v * (1 / norm(v)) (vector3D.h), and
// u = 1 / |x| is that same reciprocal -- the same values as evaluating them separately, at half
// the sqrt / division work.  FAST: every sqrt / division takes the bare core (sqrt_core,
// div_core, qdiv) and `ok` collects whether all operands were in the core's exact range; the
// caller re-runs the step with IEEE operations when one was not (rare: zero / tiny / huge
// operands), so the result is always the IEEE one without a range branch per operation.
// The step's planar state (the camera-ray miss proof starts from step 0's): orbital-plane basis
// x_axis, y_axis, u and u' before the update, and the updated u (v).
struct MicroOut { v3 x, y; double u, up, v; };
template <bool FAST>
__device__ __forceinline__ void next_micro_impl(const DHole& h, v3 no, v3& o, v3& d, double& max_t, v3& rel,
                                                double& rel2, bool& ok, MicroOut* mo = nullptr) {
  auto SQ = [&](double x) -> double {
    if (!FAST) return sqrt(x);
    ok = ok && in_core_range(x);
    return sqrt_core(x);
  };
  auto DV = [&](double a, double b) -> double {
    if (!FAST) return a / b;
    ok = ok && in_core_range(a) && in_core_range(b);
    return div_core(a, b);
  };
  auto RC = [&](double b) -> double {  // 1 / b
    if (!FAST) return 1.0 / b;
    ok = ok && in_core_range(b);
    return div_core(1.0, b);
  };
  auto D6 = [&](double x) -> double {  // x / 6
    if (!FAST) return x / 6.0;
    ok = ok && in_core_range(x);
    return qdiv(x, 6.0, 1.0 / 6.0);
  };
  v3 x_axis = no - V(h.c[0], h.c[1], h.c[2]);
  rel = x_axis;
  rel2 = norm2(x_axis);
  const double dist = SQ(rel2);
  double u = RC(dist);
  x_axis = V(x_axis.x * u, x_axis.y * u, x_axis.z * u);  // normalize: *= 1. / norm()
  double dx = dot(d, x_axis);
  v3 y_axis = d - smul(dx, x_axis);
  double dy = SQ(norm2(y_axis));
  const double idy = RC(dy);
  y_axis = V(y_axis.x * idy, y_axis.y * idy, y_axis.z * idy);
  double up = DV(-u * dx, dy);
  const double dt = h.dt, k = 3.0 * h.r;
  double f1 = -u + k * u * u / 2.0;
  double u2 = u + up * dt / 2.0;
  double f2 = -u2 + k * u2 * u2 / 2.0;
  double u3 = u + up * dt / 2.0 + f1 * dt * dt / 4.0;
  double f3 = -u3 + k * u3 * u3 / 2.0;
  if (mo) { mo->x = x_axis; mo->y = y_axis; mo->u = u; mo->up = up; }
  u += up * dt + D6((f1 + f2 + f3) * dt * dt);
  if (mo) mo->v = u;
  double dd = RC(u);
  double next_x = dd * h.cos_dt, next_y = dd * h.sin_dt;
  v3 nd = ((V(h.c[0], h.c[1], h.c[2]) + smul(next_x, x_axis)) + smul(next_y, y_axis)) - no;
  max_t = SQ(norm2(nd));
  const double inv = RC(max_t);
  d = V(nd.x * inv, nd.y * inv, nd.z * inv);
  o = no;
}
// The step from the previous segment's end point no = o + d * max_t (the caller keeps it: the
// same value the reference computes at blackhole.cpp:18); rel = no - c and rel2 = |rel|^2 are
// also the capture test's o - c and |o - c|^2 (sphere.cpp:12-14 on the new segment).
__device__ __forceinline__ void next_micro_at(const DHole& h, v3 no, v3& o, v3& d, double& max_t, v3& rel,
                                              double& rel2, MicroOut* mo = nullptr) {
  bool ok = true;
  const v3 d0 = d;
  next_micro_impl<true>(h, no, o, d, max_t, rel, rel2, ok, mo);
  if (__builtin_expect(!ok, 0)) {  // some operand outside the core's range: the IEEE step
    d = d0;
    next_micro_impl<false>(h, no, o, d, max_t, rel, rel2, ok, mo);
  }
}
__device__ __forceinline__ void next_micro(const DHole& h, v3& o, v3& d, double& max_t) {
  v3 rel;
  double rel2;
  next_micro_at(h, o + vmul(d, max_t), o, d, max_t, rel, rel2);
}

// One micro segment (o, d, max_t) against the scene -- BVHAccel::intersect_micro (bvh.cpp:115-138)
// behind the result-identical skips -- filling *is on a hit.  Shared by the
// Schwarzschild march below and the Kerr march (query_kerr).
// any_rt: a shadow query chosen at run time (the path pool kernel's rays share one query call)
// The walk of a segment that passed the skips (segment_query); cell: its start's grid cell or -1.
// W4: the 4-wide walk may run (query's W4; the Kerr march walks the binary tree only)
template <bool ANY, bool COUNT, bool W4 = true>
__device__ __forceinline__ bool segment_walk(const KParams& kp, v3 o, v3 d, double max_t, v3 e, int cell,
                                             Isect* is, Counters& cn, bool any_rt = false) {
  // oversized leaves with no primitive within reach of a short segment are not offered
  const uint64_t bmask = (kp.big_mask && cell >= 0 && max_t < kp.big_reach) ? (uint64_t)kp.big_mask[cell] : ~0ull;
  if (!COUNT && kp.diag) {  // diagnostics: skip all / interior-start / exterior-start walks
    const bool in = o.x >= kp.nodes[0].mn[0] && o.x <= kp.nodes[0].mx[0] && o.y >= kp.nodes[0].mn[1] &&
                    o.y <= kp.nodes[0].mx[1] && o.z >= kp.nodes[0].mn[2] && o.z <= kp.nodes[0].mx[2];
    if ((kp.diag & 1) || ((kp.diag & 4) && in) || ((kp.diag & 8) && !in)) return false;
  }
  bool clear_diag = false;
  if (COUNT && (kp.diag & 2)) {  // diagnostic: query slot = clear segments, prim = AABB tests left
    clear_diag = segment_clear(kp.grid, o, max_t);
    if (clear_diag) cn.query++;
  }
  const uint32_t bbox_before = cn.bbox, prim_before = cn.prim;
  int slot = -1;
  double b1 = 0, b2 = 0, seg_t = max_t;
  const v3 y = V(xdiv(1.0, d.x), xdiv(1.0, d.y), xdiv(1.0, d.z));
  const bool fast = segment_fast(kp, o, d);
  RRT_T0(tt0);
  bool hit;
  if (!COUNT) {  // the search tree (4 wide, else binary; or, for A/B, the clean tree or the reference tree)
    const int r4 = (W4 && kp.free4) ? traverse_free4<ANY, false>(kp, o, d, y, seg_t, slot, b1, b2, cn, !fast, bmask, any_rt) : 2;
    hit = r4 == 2 ? traverse_free<ANY, false>(kp, o, d, y, seg_t, slot, b1, b2, cn, !fast, bmask, any_rt) : r4 == 1;
  } else if (kp.count_exec) {
    const int r4 = (W4 && kp.free4) ? traverse_free4<ANY, true>(kp, o, d, y, seg_t, slot, b1, b2, cn, !fast, bmask) : 2;
    hit = r4 == 2 ? traverse_free<ANY, true>(kp, o, d, y, seg_t, slot, b1, b2, cn, !fast, bmask) : r4 == 1;
  }
  else
    hit = fast ? traverse<ANY, COUNT, false>(kp, o, d, y, seg_t, slot, b1, b2, cn)
               : traverse<ANY, COUNT, true>(kp, o, d, y, seg_t, slot, b1, b2, cn);
#if RRT_PROFILE
  if (ANY) cn.t_strav += clock64() - tt0; else cn.t_trav += clock64() - tt0;
#endif
  if (COUNT && (kp.diag & 2)) cn.prim = prim_before + (clear_diag ? 0u : cn.bbox - bbox_before);
  if (!hit) return false;
  if (!ANY && !any_rt) {
    const DPrimMeta meta = kp.meta[slot];
    is->bsdf = (int)((meta >> 8) & 0xffu);
    is->hit_p = o + vmul(d, seg_t);
    is->w_out = -d;
    if (meta & 1u) {  // sphere: normal((o + d t) - c).unit()  (sphere.h:71-73)
      const DPrimGeo gp = kp.geo[slot];
      is->n = unit((o + vmul(d, seg_t)) - V(gp.v[0], gp.v[1], gp.v[2]));
    } else {          // unnormalised interpolated normal (triangle.cpp:47)
      const DPrimNrm nn = kp.nrm[slot];
      double b0 = 1 - b1 - b2;
      is->n = (smul(b0, V(nn.n[0], nn.n[1], nn.n[2])) + smul(b1, V(nn.n[3], nn.n[4], nn.n[5]))) +
              smul(b2, V(nn.n[6], nn.n[7], nn.n[8]));
    }
  }
  return true;
}
template <bool ANY, bool COUNT, bool W4 = true>
__device__ __forceinline__ bool segment_query(const KParams& kp, v3 o, v3 d, double max_t, v3 e, Isect* is,
                                              Counters& cn, bool any_rt = false) {
  // e = o + d * max_t.  COUNT && kp.count_exec: count the work this path executes (grid / root
  // skips, clean walk, plane tests in the query slot) instead of the reference's
  const bool opt = !COUNT || kp.count_exec;
  if (opt && segment_outside_root(kp, o, e)) return false;  // root test fails
  const int cell = opt ? grid_cell(kp.grid, o) : -1;
  if (cell_clear(kp.grid, cell, max_t)) return false;  // no primitive within reach
  return segment_walk<ANY, COUNT, W4>(kp, o, d, max_t, e, cell, is, cn, any_rt);
}

// ------------------------------------------------------------------ kernel variants
// The integrator templates take an int variant V (named LEAN at the use sites):
//   0 general, Schwarzschild;  1 LEAN: area lights only, no microfacet BSDF, importance-sampled
//   direct light;  2 LEAN with point lights too;  V_KERR general with the Kerr march.
// Each variant is its own kernel build, so no build carries code (and registers) it never runs.
constexpr int V_KERR = 3;
// V_SW: the general Schwarzschild build with the reference's compile-time switches as run-time
// flags (KParams::sw; include/rrt.h RRT_RENDER_THIN_LENS .. RRT_RENDER_ILLUM_MASK)
constexpr int V_SW = 4;
enum { SW_THIN_LENS = 1u, SW_NO_ADAPTIVE = 2u, SW_ENV_HEMI = 4u, SW_MF_HEMI = 8u };
__device__ __forceinline__ uint32_t sw_illum(const KParams& kp) { return ((kp.sw >> 4) & 3u) ^ 2u; }  // ILLUM
__host__ __device__ constexpr bool is_lean(int v) { return v == 1 || v == 2; }
__host__ __device__ constexpr int general_of(int v) { return v == V_KERR || v == V_SW ? v : 0; }  // non-LEAN build

// ------------------------------------------------------------------ Kerr (build-defined)
// The reference has no Kerr metric; this integrator is this build's design
//  and oracle/restate/rrt_oracle.c restates it operation for operation.
//
// Kerr-Schild Cartesian coordinates about the hole (local frame ex, ey, ez = spin axis):
//   g_mn = eta_mn + f l_m l_n,  f = 2 M r^3 / (r^4 + a^2 z^2),
//   l_m = (1, (r x + a y) / (r^2 + a^2), (r y - a x) / (r^2 + a^2), z / r),
//   r^2 = (rho^2 - a^2) / 2 + sqrt((rho^2 - a^2)^2 / 4 + a^2 z^2)   (Boyer-Lindquist r).
// Photons follow H = (eta^mn p_m p_n - f (l^m p_m)^2) / 2 = 0 with p_t = -1 (E = 1):
//   dx_i/dl = p_i - f L l_i,   dp_i/dl = (1/2) d_i (f L^2),   L = 1 + l . p.
// The gradient d_i(f L^2) is evaluated in closed form (kerr_rhs).  At a = 0 the spatial
// coordinates are r times the unit direction, so the spatial path is the Schwarzschild photon
// orbit u'' + u = 3 M u^2 that BlackHole::next_micro_ray steps.
// Arithmetic of one Kerr step (next_micro_impl's scheme): FAST takes the bare sqrt / division
// cores and records in `ok` whether every operand lay in their exact range (a +0 numerator is
// exact too); the caller re-runs the step IEEE (FAST = false) when one did not.
template <bool FAST>
struct KArith {
  bool ok = true;
  __device__ __forceinline__ double sq(double x) {
    if (!FAST) return sqrt(x);
    ok = ok && in_core_range(x);
    return sqrt_core(x);
  }
  __device__ __forceinline__ double dv(double a, double b) {
    if (!FAST) return a / b;
    ok = ok && (in_core_range(a) || (a == 0.0 && !signbit(a))) && in_core_range(b);
    return div_core(a, b);
  }
};
// Field quantities at local point q (values only: the capture test and the initial covector):
// r (Boyer-Lindquist), f and l_i
template <class A>
__device__ __forceinline__ void kerr_fl(const DHole& h, v3 q, double& f, v3& l, double& r_out, A& ar) {
  const double zz = q.z * q.z;
  const double w = ((q.x * q.x + q.y * q.y) + zz) - h.a2;
  const double r2 = 0.5 * w + ar.sq(0.25 * (w * w) + h.a2 * zz);
  const double r = ar.sq(r2);
  const double iw = ar.dv(1.0, r2 + h.a2);
  l = V((r * q.x + h.a * q.y) * iw, (r * q.y - h.a * q.x) * iw, ar.dv(q.z, r));
  f = ar.dv((2.0 * h.m) * (r * r2), r2 * r2 + h.a2 * zz);
  r_out = r;
}
// r^2 (Boyer-Lindquist) at local point q (capture test)
__device__ __forceinline__ double kerr_r2(const DHole& h, v3 q) {
  const double w = ((q.x * q.x + q.y * q.y) + q.z * q.z) - h.a2;
  return 0.5 * w + xsqrt(0.25 * (w * w) + h.a2 * (q.z * q.z));
}
// Hamilton's equations at (q, p): dq = p - f L l, dp = (1/2) grad(f L^2) = L ((L/2) grad f + f grad L),
// grad L = sum_i p_i grad l_i, with the gradients in closed form.  From the quartic
// r^4 - (rho^2 - a^2) r^2 - a^2 z^2 = 0, with Sigma = r^4 + a^2 z^2 and W = r^2 + a^2:
//   grad r = (x r^3, y r^3, z r W) / Sigma,
//   grad f = f (3 grad r / r - (4 r^3 grad r + 2 a^2 z e_z) / Sigma)          (f = 2 M r^3 / Sigma),
//   grad l_x = (r e_x + a e_y) / W + (x - 2 r l_x) grad r / W,
//   grad l_y = (r e_y - a e_x) / W + (y - 2 r l_y) grad r / W,
//   grad l_z = e_z / r - z grad r / r^2.
// Three reciprocals and two square roots per evaluation; r out.
template <class A>
__device__ __forceinline__ void kerr_rhs(const DHole& h, v3 q, v3 p, v3& dq, v3& dp, double& r_out, A& ar) {
  const double zz = q.z * q.z;
  const double w = ((q.x * q.x + q.y * q.y) + zz) - h.a2;
  const double r2 = 0.5 * w + ar.sq(0.25 * (w * w) + h.a2 * zz);
  const double r = ar.sq(r2);
  const double W = r2 + h.a2;
  const double isg = ar.dv(1.0, r2 * r2 + h.a2 * zz), iw = ar.dv(1.0, W), ir = ar.dv(1.0, r);
  const double r3 = r * r2, gk = r3 * isg;
  const v3 g = V(q.x * gk, q.y * gk, (q.z * r) * (W * isg));  // grad r
  const double lx = (r * q.x + h.a * q.y) * iw, ly = (r * q.y - h.a * q.x) * iw, lz = q.z * ir;
  const double f = (2.0 * h.m) * gk;
  const double cf = 3.0 * ir - (4.0 * r3) * isg;
  const v3 gf = V(f * (cf * g.x), f * (cf * g.y), f * (cf * g.z - ((2.0 * h.a2) * q.z) * isg));
  const double L = ((1.0 + p.x * lx) + p.y * ly) + p.z * lz;
  const double c = (p.x * (q.x - (2.0 * r) * lx) + p.y * (q.y - (2.0 * r) * ly)) * iw - (p.z * q.z) * (ir * ir);
  const v3 gL = V((r * p.x - h.a * p.y) * iw + c * g.x, (h.a * p.x + r * p.y) * iw + c * g.y, p.z * ir + c * g.z);
  const double hL = 0.5 * L, fL = f * L;
  dq = V(p.x - fL * lx, p.y - fL * ly, p.z - fL * lz);
  dp = V(L * (hL * gf.x + f * gL.x), L * (hL * gf.y + f * gL.y), L * (hL * gf.z + f * gL.z));
  r_out = r;
}
__device__ __forceinline__ v3 kerr_local(const DHole& h, v3 v) {
  return V(dot(v, ld3(h.ex)), dot(v, ld3(h.ey)), dot(v, ld3(h.ez)));
}
__device__ __forceinline__ v3 kerr_world(const DHole& h, v3 q) {
  return V(h.c[0] + ((h.ex[0] * q.x + h.ey[0] * q.y) + h.ez[0] * q.z),
           h.c[1] + ((h.ex[1] * q.x + h.ey[1] * q.y) + h.ez[1] * q.z),
           h.c[2] + ((h.ex[2] * q.x + h.ey[2] * q.y) + h.ez[2] * q.z));
}
// Initial covector of a photon at world point o moving along world direction d: coordinate
// velocity k = (k^t, d_local) made null (g_mn k^m k^n = 0, future root), p_m = g_mn k^n,
// scaled to p_t = -1.  Once per query: IEEE arithmetic.
__device__ __forceinline__ void kerr_init(const DHole& h, v3 o, v3 d, v3& q, v3& p) {
  KArith<false> ar;
  q = kerr_local(h, o - ld3(h.c));
  const v3 k = kerr_local(h, d);
  double f, r;
  v3 l;
  kerr_fl(h, q, f, l, r, ar);
  const double ld = (l.x * k.x + l.y * k.y) + l.z * k.z;
  const double A = f - 1.0, B = 2.0 * f * ld, C = 1.0 + f * (ld * ld);
  double disc = B * B - 4.0 * A * C;
  if (!(disc > 0.0)) disc = 0.0;
  const double kt = (2.0 * C) / (sqrt(disc) - B);
  const double pt = A * kt + f * ld;
  const double s = f * (kt + ld);
  p = V(k.x + s * l.x, k.y + s * l.y, k.z + s * l.z);
  if (pt < 0.0) p = vmul(p, -1.0 / pt);
}
// One march step: the first RK4 stage at (q, p); escape test (outgoing beyond r_esc: returns
// true); h = delta_theta * r / |dq/dl| (the path advances delta_theta * r); the polar angle
// swept; then the classical RK4 update.
// st: step stretch (1: the march; the occlusion proof's coarse march takes kp.kproof.stretch)
template <class A>
__device__ __forceinline__ bool kerr_advance(const DHole& h, v3& q, v3& p, double& swept, A& ar, double st = 1.0) {
  v3 dq1, dp1;
  double r, rr;
  kerr_rhs(h, q, p, dq1, dp1, r, ar);
  const double rho2 = norm2(q);
  if (rho2 > h.r_esc2 && dot(q, dq1) > 0.0) return true;  // outgoing beyond the scene
  const double hh = ar.dv((h.dt * r) * st, ar.sq(norm2(dq1)));  // (dt r) * 1 = dt r exactly
  swept += ar.dv(hh * ar.sq(norm2(cross(q, dq1))), rho2);  // polar angle of this step
  const double half = 0.5 * hh;
  // stages 2-4 folded into running sums as they come: ((k1 + 2 k2) + 2 k3) + k4, the same
  // operations in the same order as summing at the end, with one stage live at a time
  v3 aq = dq1, ap = dp1, dq, dp;
  kerr_rhs(h, q + vmul(dq1, half), p + vmul(dp1, half), dq, dp, rr, ar);
  aq = aq + vmul(dq, 2.0); ap = ap + vmul(dp, 2.0);
  kerr_rhs(h, q + vmul(dq, half), p + vmul(dp, half), dq, dp, rr, ar);
  aq = aq + vmul(dq, 2.0); ap = ap + vmul(dp, 2.0);
  kerr_rhs(h, q + vmul(dq, hh), p + vmul(dp, hh), dq, dp, rr, ar);
  aq = aq + dq; ap = ap + dp;
  const double c6 = ar.dv(hh, 6.0);
  q = q + vmul(aq, c6);
  p = p + vmul(ap, c6);
  return false;
}
// BVHAccel::intersect with the Kerr march.  Like the reference's march it
// follows the photon for one revolution about the hole (it stops once the swept polar angle
// reaches 2 pi; the reference takes ceil(2 pi / delta_theta) fixed-angle steps), the first
// segment with a hit wins and capture means "no hit"; captured = the segment ends inside the
// outer horizon.  Steps are sized by distance (accurate for radial motion too), so the sweep is
// budgeted by angle, not by count (at most kerr_max_steps), and a photon moving outward beyond
// every primitive (|q|^2 > r_esc2 >= (4M)^2, outside all photon orbits) has escaped: no hit.
// ------------------------------------------------------------------ run-time proof audit
// The proofs (camera miss, shadow occlusion, pixel and strip miss, Kerr occlusion) write a result
// without marching; their margins were validated by sweeps.  A counting launch with kp.audit set
// (rrt_set_proof_audit; bench.py's executed-work pass) re-marches every 2^audit_shift-th proven ray
// exactly and tallies disagreements: kp.audit[2 k] rays checked, [2 k + 1] violations.
// (proof kinds k: include/rrt.h RRT_AUDIT_*)
__device__ __forceinline__ bool audit_pick(const KParams& kp, v3 o, v3 d) {
  const uint64_t h = rrt_mix64((uint64_t)__double_as_longlong(d.x) ^
                               rrt_mix64((uint64_t)__double_as_longlong(d.y) ^ ((uint64_t)__double_as_longlong(d.z) << 1)) ^
                               ((uint64_t)__double_as_longlong(o.x) >> 2));
  return (h & ((1ull << kp.audit_shift) - 1ull)) == 0ull;
}
__device__ __forceinline__ void audit_note(const KParams& kp, int k, bool violated) {
  atomicAdd(kp.audit + 2 * k, 1ull);
  if (violated) atomicAdd(kp.audit + 2 * k + 1, 1ull);
}
__device__ __forceinline__ bool kerr_occluded_proof(const KParams& kp, v3 o, v3 d);
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool kerr_march(const KParams& kp, v3 o, v3 d, Isect* is, Counters& cn);
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool query_kerr(const KParams& kp, v3 o, v3 d, Isect* is, Counters& cn) {
  // shadow rays: the occlusion proof first (never in the reference-work counts)
  if (ANY && kp.kproof.on && !(COUNT && !kp.count_exec) && kerr_occluded_proof(kp, o, d)) {
    if (COUNT && kp.audit && audit_pick(kp, o, d)) {
      Counters c2 = {};
      audit_note(kp, RRT_AUDIT_KERR, !kerr_march<true, false>(kp, o, d, nullptr, c2));
    }
    return true;
  }
  return kerr_march<ANY, COUNT>(kp, o, d, is, cn);
}
// the march of query_kerr (no proof)
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool kerr_march(const KParams& kp, v3 o, v3 d, Isect* is, Counters& cn) {
  const DHole& h = kp.hole;
  v3 q, p;
  kerr_init(h, o, d, q, p);
  v3 a = o;
  const double rh2 = h.r_hor * h.r_hor;
  double swept = 0.0;
  for (int j = 0; j < h.kerr_max_steps && swept < 2.0 * PI_D; ++j) {
    v3 q1 = q, p1 = p;
    double sw1 = swept;
    KArith<true> fast;
    bool escaped = kerr_advance(h, q1, p1, sw1, fast);
    if (__builtin_expect(!fast.ok, 0)) {  // an operand outside the cores' range: the IEEE step
      KArith<false> ieee;
      q1 = q; p1 = p; sw1 = swept;
      escaped = kerr_advance(h, q1, p1, sw1, ieee);
    }
    if (escaped) return false;
    q = q1; p = p1; swept = sw1;
    if (COUNT) cn.micro++;
    if (kerr_r2(h, q) <= rh2) return false;  // captured
    const v3 b = kerr_world(h, q);
    const v3 seg = b - a;
    const double max_t = norm(seg);
    const double inv = xdiv(1., max_t);
    const v3 sd = V(seg.x * inv, seg.y * inv, seg.z * inv);  // normalize(seg), norm shared
    if (segment_query<ANY, COUNT, false>(kp, a, sd, max_t, a + vmul(sd, max_t), is, cn)) return true;
    a = b;
  }
  return false;
}

// ------------------------------------------------------------------ shadow-ray occlusion proof
// (DESIGN.md §5).  The reference's shadow query (bvh.cpp:103-113; the caller uses only the
// boolean) is true iff some micro segment before the capture hits a primitive.  Most shadow rays
// of a closed room end on a wall, after ~15-30 exact steps and walks.  The proof marches the
// camera proof's recurrence from the shadow ray itself: every segment must clear the
// capture sphere by the margin m, and once a segment end leaves the trigger box (the root box
// shrunk past the wall triangles kept by rrt_host.cpp build_occluders) the segment must cross one
// of those triangles with margin -- end points m beyond its plane on either side, the crossing
// point mq inside every edge.  The reference's segment then crosses it too, its triangle test
// accepts (triangle.cpp:25-55) and the leaf boxes on the way pass, so the query returns true.
// Anything else (an end point near a wall, a face without triangles, a cancelling step, the
// march ending) is no proof: the caller marches exactly.
// A certain crossing of a triangle of face f by the segment a -> b: end points more than m on
// either side of its plane (either way), the crossing point mq inside every edge.
__device__ __forceinline__ bool occ_face(const DShadowProof& sp, int f, v3 a, v3 b, double m) {
#pragma clang fp contract(fast)
#pragma unroll 1
  for (uint32_t i = 0; i < sp.n[f]; ++i) {
    const DOccluder& t = sp.tri[f][i];
    const double da = t.n[0] * a.x + t.n[1] * a.y + t.n[2] * a.z - t.d;
    const double db = t.n[0] * b.x + t.n[1] * b.y + t.n[2] * b.z - t.d;
    if (!((da > m && db < -m) || (da < -m && db > m))) continue;
    const double tq = da / (da - db);
    const v3 q = V(a.x + (b.x - a.x) * tq, a.y + (b.y - a.y) * tq, a.z + (b.z - a.z) * tq);
    // end points within m of the reference's move the crossing by <= m (2 + |b - a| / |da - db|)
    const double mq = m * (2.0 + (fabs(b.x - a.x) + fabs(b.y - a.y) + fabs(b.z - a.z)) / fabs(da - db));
    bool in = true;
    for (int k = 0; k < 3; ++k) in = in && t.en[k][0] * q.x + t.en[k][1] * q.y + t.en[k][2] * q.z - t.eo[k] >= mq;
    if (in) return true;
  }
  return false;
}
// The segment a -> b with an end outside the trigger box: 1 = a certain crossing of a triangle of
// a face that an end is past; -1 = no proof and b has left the root box (the ray leaves the room:
// give up); 0 = go on.  Loops kept rolled: this runs once or twice per shadow ray.
__device__ __forceinline__ int occ_exit(const KParams& kp, v3 a, v3 b, double m) {
  const DShadowProof& sp = kp.occ;
  bool out = false;
#pragma unroll 1
  for (int f = 0; f < 6; ++f) {
    const int k = f < 3 ? f : f - 3;
    const double ak = k == 0 ? a.x : k == 1 ? a.y : a.z, bk = k == 0 ? b.x : k == 1 ? b.y : b.z;
    const bool past = f < 3 ? !(bk >= sp.in_lo[k] && ak >= sp.in_lo[k]) : !(bk <= sp.in_hi[k] && ak <= sp.in_hi[k]);
    if (past && occ_face(sp, f, a, b, m)) return 1;
    out = out || !(f < 3 ? bk >= kp.miss.lo[k] : bk <= kp.miss.hi[k]);  // NaN: out
  }
  return out ? -1 : 0;
}
// occ_exit out of line, one copy per kernel build W (inline or the whole proof out of
// line measured slower)
template <int W>
__device__ __noinline__ int occ_exit_call(const KParams& kp, v3 a, v3 b, double m) { return occ_exit(kp, a, b, m); }
__device__ __forceinline__ bool occ_inside(const DShadowProof& sp, v3 b) {
  return b.x >= sp.in_lo[0] && b.x <= sp.in_hi[0] && b.y >= sp.in_lo[1] && b.y <= sp.in_hi[1] && b.z >= sp.in_lo[2] &&
         b.z <= sp.in_hi[2];
}
// Kerr shadow rays ("Kerr occlusion proof").  A shadow query is true iff some
// segment of the march before the capture hits a primitive; from inside a closed room most end on
// a wall after 20-60 RK4 steps, each step four Hamiltonian evaluations plus a walk.  The proof
// marches the same Hamiltonian with steps kp.kproof.stretch times longer and accepts "occluded"
// when one of its chords crosses a wall piece (build_occluders: kp.occ's triangles, coplanar pairs
// merged into convex quads, kp.kproof.quad) with margin delta:
// end points more than delta on either side of the plane, the crossing point inside every edge by
// occ_face's mq.  The exact march's chords stay within delta of the coarse chords while the coarse
// march keeps sqrt(r_near2) from the hole (tools/kerr_proof_sweep.py: the largest deviation seen
// over the envelope rrt_host.cpp allows is under a third of delta), so they cross that triangle
// too, uncaptured (the coarse path, and so the exact one, stays far outside the horizon) and
// within the exact march's budget (max_steps coarse steps, swept angle below swept_max); the
// triangle test accepts and the leaf boxes on the way contain the crossing, so the query is true.
// Anything else -- near the hole, the ray leaving the room, an operand outside the fast cores'
// range, the budget -- is no proof: the exact march runs.
// occ_face / occ_exit on the Kerr proof's wall pieces (DOccQuad: a convex quad or a triangle)
__device__ __forceinline__ bool occ_face_quad(const DKerrProof& kq, int f, v3 a, v3 b, double m) {
#pragma clang fp contract(fast)
#pragma unroll 1
  for (uint32_t i = 0; i < kq.nq[f]; ++i) {
    const DOccQuad& t = kq.quad[f][i];
    const double da = t.n[0] * a.x + t.n[1] * a.y + t.n[2] * a.z - t.d;
    const double db = t.n[0] * b.x + t.n[1] * b.y + t.n[2] * b.z - t.d;
    if (!((da > m && db < -m) || (da < -m && db > m))) continue;
    const double tq = da / (da - db);
    const v3 q = V(a.x + (b.x - a.x) * tq, a.y + (b.y - a.y) * tq, a.z + (b.z - a.z) * tq);
    const double mq = m * (2.0 + (fabs(b.x - a.x) + fabs(b.y - a.y) + fabs(b.z - a.z)) / fabs(da - db));
    bool in = true;
    for (int k = 0; k < 4; ++k) in = in && t.en[k][0] * q.x + t.en[k][1] * q.y + t.en[k][2] * q.z - t.eo[k] >= mq;
    if (in) return true;
  }
  return false;
}
__device__ __forceinline__ int occ_exit_quad(const KParams& kp, v3 a, v3 b, double m) {
  const DShadowProof& sp = kp.occ;
  bool out = false;
#pragma unroll 1
  for (int f = 0; f < 6; ++f) {
    const int k = f < 3 ? f : f - 3;
    const double ak = k == 0 ? a.x : k == 1 ? a.y : a.z, bk = k == 0 ? b.x : k == 1 ? b.y : b.z;
    const bool past = f < 3 ? !(bk >= sp.in_lo[k] && ak >= sp.in_lo[k]) : !(bk <= sp.in_hi[k] && ak <= sp.in_hi[k]);
    if (past && occ_face_quad(kp.kproof, f, a, b, m)) return 1;
    out = out || !(f < 3 ? bk >= kp.miss.lo[k] : bk <= kp.miss.hi[k]);  // NaN: out
  }
  return out ? -1 : 0;
}
// A ray whose straight line leaves the room through a face without wall pieces (the open side of a
// Cornell box) almost never ends on a wall: spare it the coarse march (false: no proof)
__device__ __forceinline__ bool kerr_proof_worth(const KParams& kp, v3 o, v3 d) {
  double te = 1e300;
  int fe = -1;
  for (int k = 0; k < 3; ++k) {
    const double dk = k == 0 ? d.x : k == 1 ? d.y : d.z, ok = k == 0 ? o.x : k == 1 ? o.y : o.z;
    if (dk == 0.0) continue;
    const double t = ((dk > 0.0 ? kp.miss.hi[k] : kp.miss.lo[k]) - ok) / dk;
    if (t < te) { te = t; fe = dk > 0.0 ? k + 3 : k; }
  }
  return !(fe >= 0 && kp.kproof.nq[fe] == 0);
}
__device__ __forceinline__ bool kerr_occluded_proof(const KParams& kp, v3 o, v3 d) {
  const DHole& h = kp.hole;
  const DKerrProof& kq = kp.kproof;
  if (!kerr_proof_worth(kp, o, d)) return false;
  v3 q, p;
  kerr_init(h, o, d, q, p);
  if (!(norm2(q) > kq.r_near2)) return false;  // starting near the hole
  const v3 c = ld3(h.c);
  v3 a = o, a0 = o;  // the chord's start, and the previous chord's
  bool a_in = occ_inside(kp.occ, a);
  double swept = 0.0;
#pragma unroll 1
  for (int j = 0; j < kq.max_steps; ++j) {
    KArith<true> ar;
    const bool escaped = kerr_advance(h, q, p, swept, ar, kq.stretch);
    if (!ar.ok || escaped || !(swept < kq.swept_max) || !(norm2(q) > kq.r_near2)) return false;
    const v3 b = kerr_world(h, q);
    {  // the chord keeps sqrt(r_near2) from the hole too
      const v3 u = b - a, w = c - a;
      const double uu = norm2(u), t = uu > 0.0 ? fmin(fmax(dot(u, w) / uu, 0.0), 1.0) : 0.0;
      if (!(norm2(w - vmul(u, t)) > kq.r_near2)) return false;
    }
    const bool b_in = occ_inside(kp.occ, b);
    if (!b_in || !a_in) {
      int res = occ_exit_quad(kp, a, b, kq.delta);
      if (res <= 0 && j > 0) {
        // a wall crossed across two chords (one of their common point's sides within delta of the
        // plane): the chord a0 -> b, with the margin grown by a's distance from it
        const v3 u = b - a0, w = a - a0;
        const double uu = norm2(u), uw = dot(u, w);
        const double beta = sqrt(fmax(norm2(w) - uw * uw / uu, 0.0)) * (1.0 + 1e-6);
        if (uu > 0.0 && occ_exit_quad(kp, a0, b, kq.delta + beta) > 0) res = 1;
      }
      if (res) return res > 0;
    }
    a_in = b_in;
    a0 = a;
    a = b;
  }
  return false;
}
// The whole march by the recurrence, step 0 included: the ray (o, d) is the state of a step from
// the point A = o itself (|A - c| = 1 / u, so v_prev = rho u, E_prev = x, s_prev chosen so the
// update yields s = u and the reference's u' = -u (d . x) / |d - (d . x) x|).
template <int W = 0>
__device__ __forceinline__ bool shadow_occluded_proof(const KParams& kp, v3 o, v3 d, int steps) {
#pragma clang fp contract(fast)
  const DMissProof& mp = kp.miss;
  const DShadowProof& sp = kp.occ;
  const DHole& h = kp.hole;
  const v3 c = V(h.c[0], h.c[1], h.c[2]);
  const v3 x0 = o - c;
  const double r0 = sqrt(norm2(x0)), u0 = 1.0 / r0;
  const v3 X = vmul(x0, u0);
  const double dx = dot(d, X);
  v3 Y = d - smul(dx, X);
  const double dy = sqrt(norm2(Y));
  Y = vmul(Y, 1.0 / dy);
  const double up0 = -u0 * dx / dy;
  double vprev = mp.rho * u0, s = u0 * mp.co1 - up0 * h.sin_dt * mp.inv_rho;
  double ea = 1.0, eb = 0.0, sig = 1.0, rp = r0;
  bool a_in = occ_inside(sp, o);
  const double si2 = h.sin_dt * h.sin_dt, rc = h.r * (1.0 + 1e-9);
#pragma unroll 1
  for (int j = 0; j < steps; ++j) {
    const double sg = vprev < 0.0 ? -1.0 : 1.0;
    const double up = (vprev * mp.co1 - mp.rho * s) * mp.inv_si;
    s = fabs(vprev) * mp.inv_rho;
    const double f1 = -s + mp.k15 * s * s;
    const double u2 = s + up * (h.dt * 0.5);
    const double f2 = -u2 + mp.k15 * u2 * u2;
    const double u3 = u2 + f1 * mp.dt2_4;
    const double f3 = -u3 + mp.k15 * u3 * u3;
    const double v = s + up * h.dt + (f1 + f2 + f3) * mp.dt2_6;
    if (!(fabs(v) >= mp.kappa * (s + fabs(up) * h.dt))) return false;  // cancelling step (or NaN)
    const double a = sg * mp.co1, b = sig * mp.si1;
    const double na = a * ea - b * eb, nb = a * eb + b * ea;
    sig *= sg;
    const double av = fabs(v), avp = fabs(vprev);
    const double r = mp.rho * __builtin_amdgcn_rcp(av) * (1.0 + 1e-6);  // |B - c| (upper bound)
    const double m = mp.eta * (fmax(rp, r) + mp.scale);
    // the segment must clear the capture sphere: its distance from the hole > r_s + m (the
    // camera proof's scalar distance: foot of the perpendicular inside, else the nearer end)
    const double rb = rc + m;
    const double D = v * v + vprev * vprev - 2.0 * mp.co1 * avp * v;
    const bool inside = v * (mp.co1 * avp - v) < 0.0 && avp * (avp - mp.co1 * v) > 0.0;
    const bool clear = inside ? si2 > rb * rb * D : mp.rho * mp.rho > rb * rb * fmax(v * v, vprev * vprev);
    if (!clear) return false;
    const double ib = mp.rho / v;
    const v3 pb = V(c.x + (na * ib) * X.x + (nb * ib) * Y.x, c.y + (na * ib) * X.y + (nb * ib) * Y.y,
                    c.z + (na * ib) * X.z + (nb * ib) * Y.z);
    const bool b_in = occ_inside(sp, pb);
    if (!b_in || !a_in) {
      const double ia = mp.rho / vprev;
      const v3 pa = V(c.x + (ea * ia) * X.x + (eb * ia) * Y.x, c.y + (ea * ia) * X.y + (eb * ia) * Y.y,
                      c.z + (ea * ia) * X.z + (eb * ia) * Y.z);
      const int res = occ_exit_call<W>(kp, pa, pb, m);
      if (res) return res > 0;
    }
    a_in = b_in;
    rp = r; vprev = v; ea = na; eb = nb;
  }
  return false;
}

// BVHAccel::intersect (bvh.cpp:103-113): march the geodesic as straight micro segments; the
// incoming ray's min_t / max_t are dropped (camera clip planes and shadow-ray distance are
// ignored, as in the reference).  Capture by the hole returns "no hit".  KERR: the Kerr build
// of the kernel (kernel variant V_KERR, chosen by rrt_host.cpp launch() for a Kerr spacetime).
#if RRT_PROFILE
#define RRT_QACC(v) do { if (ANY) cn.t_squery += clock64() - v; else cn.t_query += clock64() - v; } while (0)
#else
#define RRT_QACC(v)
#endif
#ifndef RRT_QUERY_ATTR  // inline into every kernel build: a query shared out of line by builds of
                        // different waves-per-SIMD budgets takes the loosest budget's registers, and
                        // every caller inherits them (occupancy 4 -> 1 when the 4-wide walk made the
                        // query too large for the inliner)
#define RRT_QUERY_ATTR __device__ __forceinline__
#endif
// W4: walks may take the 4-wide search tree -- the LEAN builds' choice; the general and Kerr builds
// walk the binary tree (with the 4-wide walk inlined their scratch grew 2.5-3x: general batch kernel
// 592 -> 1488 B/lane, Kerr 720 -> 2304 and cfg5 1.41 -> 3.76 s per frame, profiles/r05_ab_kerr_bvh4.txt)
template <bool ANY, bool COUNT, bool KERR = false, bool W4 = true>
RRT_QUERY_ATTR bool query(const KParams& kp, v3 o, v3 d, Isect* is, Counters& cn, bool any_rt = false) {
  if (KERR) return query_kerr<ANY, COUNT>(kp, o, d, is, cn);
  if (COUNT && !kp.count_exec && !(kp.diag & 2)) cn.query++;
  RRT_T0(tq0);
  double max_t = 0.0;
  v3 e = o + vmul(d, max_t);  // the next segment's start (micro = Ray(o, d, max_t = 0), bvh.cpp:104)
  for (int j = 0; j < kp.hole.steps; ++j) {
    RRT_T0(tm0);
    v3 rel;
    double rel2;
    next_micro_at(kp.hole, e, o, d, max_t, rel, rel2);
    RRT_ACC(t_micro, tm0);
    if (COUNT) cn.micro++;
    if (sphere_t_rel(rel, rel2, kp.hole.r2, d, max_t)) {  // captured
      RRT_QACC(tq0);
      return false;
    }
    e = o + vmul(d, max_t);
    if (segment_query<ANY, COUNT, W4>(kp, o, d, max_t, e, is, cn, any_rt)) {
      RRT_QACC(tq0);
      return true;
    }
  }
  RRT_QACC(tq0);
  return false;
}

// ------------------------------------------------------------------ camera-ray miss proof
// (DESIGN.md §5 "Miss proof").  In exact arithmetic the reference's march (next_micro_ray) is
// planar about the hole and reduces to a scalar recurrence: with s = u at a step's start, u' its
// derivative and v the updated u, the step places the next point at c + (cos dt x + sin dt y) / v
// (flipped through the hole when v < 0), and the next step starts from
//   s' = |v| / rho,   u'' = (v cos dt / rho - rho s) / sin dt,   rho = |(cos dt, sin dt)|,
// its x axis = sign(v) E and its y axis = E rotated a quarter turn the same way as y from x,
// E = (cos dt x + sin dt y) / rho.  The reference's floating-point march stays within a relative
// 1e-12 / kappa of that recurrence while no step cancels (|v| >= kappa (|s| + |u' dt|)) --
// measured over 3e5 rays per BASELINE scene (tools/miss_proof_check.py) and on the GPU
// (tests/test_gpu_parity.py) -- so a segment of the recurrence that misses the root box widened
// by eta (|P - c| + scale), eta >= 1e3 x that bound, is a reference segment whose root slab test
// fails.  If every segment misses, the reference's query returns "no hit" (captured or not), so
// the camera ray is a miss without the exact march.  Step 0 is the reference's own step (bit
// exact) and its segment takes the reference's root test.  Any doubt (a cancelling step, a
// segment near the box, NaN) returns false: the caller marches the ray exactly.
__device__ __forceinline__ bool seg_clear_of_box(v3 a, v3 b, const double* lo, const double* hi, double m) {
#pragma clang fp contract(fast)
  const double l0 = lo[0] - m, l1 = lo[1] - m, l2 = lo[2] - m, h0 = hi[0] + m, h1 = hi[1] + m, h2 = hi[2] + m;
  if (fmax(a.x, b.x) < l0 || fmin(a.x, b.x) > h0 || fmax(a.y, b.y) < l1 || fmin(a.y, b.y) > h1 ||
      fmax(a.z, b.z) < l2 || fmin(a.z, b.z) > h2)
    return true;
  // slab test of the segment a + t (b - a), t in [0, 1]; every axis overlaps the widened box here,
  // so an axis with no extent along the segment constrains nothing
  const double dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
  double tmin = 0.0, tmax = 1.0;
  if (dx != 0.0) { const double i = 1.0 / dx, t0 = (l0 - a.x) * i, t1 = (h0 - a.x) * i; tmin = fmax(tmin, fmin(t0, t1)); tmax = fmin(tmax, fmax(t0, t1)); }
  if (dy != 0.0) { const double i = 1.0 / dy, t0 = (l1 - a.y) * i, t1 = (h1 - a.y) * i; tmin = fmax(tmin, fmin(t0, t1)); tmax = fmin(tmax, fmax(t0, t1)); }
  if (dz != 0.0) { const double i = 1.0 / dz, t0 = (l2 - a.z) * i, t1 = (h2 - a.z) * i; tmin = fmax(tmin, fmin(t0, t1)); tmax = fmin(tmax, fmax(t0, t1)); }
  return tmin > tmax + 1e-9;  // NaN: not clear
}
template <bool COUNT = false>
__device__ __forceinline__ bool camera_miss_proof(const KParams& kp, v3 o, v3 d, Counters& cn) {
  const DMissProof& mp = kp.miss;
  const DHole& h = kp.hole;
  // step 0: the reference's own step from the camera ray (bit exact) and its root slab test
  MicroOut m0;
  v3 rel;
  double rel2, max_t = 0.0;
  next_micro_at(h, o + vmul(d, max_t), o, d, max_t, rel, rel2, &m0);
  const v3 e = o + vmul(d, max_t);
  if (!segment_outside_root(kp, o, e)) {
    const v3 y = V(xdiv(1.0, d.x), xdiv(1.0, d.y), xdiv(1.0, d.z));
    if (COUNT) cn.bbox++;
    if (slab_rt(kp.nodes[0].mn, kp.nodes[0].mx, o, d, y, max_t, !segment_fast(kp, o, d))) return false;
  }
  {
#pragma clang fp contract(fast)
    const v3 c = V(h.c[0], h.c[1], h.c[2]);
    const v3 X = m0.x, Y = m0.y;
    double s = m0.u, up = m0.up, vprev = m0.v;
    double ea = mp.co1, eb = mp.si1, sig = 1.0;  // E of the point just placed, in (X, Y); sense of y from x
    double rp = mp.rho / fabs(vprev);             // its distance from the hole
    const double si2 = h.sin_dt * h.sin_dt;
    for (int j = 1; j < h.steps; ++j) {
      // the next step's start: s, u', and its frame (x = sg E, y = E turned by sig)
      const double sg = vprev < 0.0 ? -1.0 : 1.0;
      up = (vprev * mp.co1 - mp.rho * s) * mp.inv_si;
      s = fabs(vprev) * mp.inv_rho;
      // blackhole.cpp:23-32 on (s, u')
      const double f1 = -s + mp.k15 * s * s;
      const double u2 = s + up * (h.dt * 0.5);
      const double f2 = -u2 + mp.k15 * u2 * u2;
      const double u3 = u2 + f1 * mp.dt2_4;
      const double f3 = -u3 + mp.k15 * u3 * u3;
      const double v = s + up * h.dt + (f1 + f2 + f3) * mp.dt2_6;
      if (!(fabs(v) >= mp.kappa * (s + fabs(up) * h.dt))) return false;  // cancelling step (or NaN)
      // E of the new point: cos dt x + sin dt y over rho, with x = sg E_prev, y = sig-turned E_prev
      const double a = sg * mp.co1, b = sig * mp.si1;
      const double na = a * ea - b * eb, nb = a * eb + b * ea;
      sig *= sg;
      // The segment A -> B, A = rho E_prev / vprev, B = rho E / v about the hole, with
      // E_prev . E = sg co1 and |E_prev x E| = si1: its distance from the hole from scalars alone
      // (foot of the perpendicular inside: line distance^2 = sin^2 dt / D, else the nearer end).
      const double av = fabs(v), avp = fabs(vprev);
      const double r = mp.rho * __builtin_amdgcn_rcp(av) * (1.0 + 1e-6);  // |B| (upper bound)
      const double rb = mp.r_ball + mp.eta * (fmax(rp, r) + mp.scale);
      const double D = v * v + vprev * vprev - 2.0 * mp.co1 * avp * v;
      const bool inside = v * (mp.co1 * avp - v) < 0.0 && avp * (avp - mp.co1 * v) > 0.0;
      const bool far = inside ? si2 > rb * rb * D : mp.rho * mp.rho > rb * rb * fmax(v * v, vprev * vprev);
      if (!far) {  // within reach of the root box: the segment itself against the widened box
        const double ia = mp.rho / vprev, ib = mp.rho / v;
        const v3 pa = V(c.x + (ea * ia) * X.x + (eb * ia) * Y.x, c.y + (ea * ia) * X.y + (eb * ia) * Y.y,
                        c.z + (ea * ia) * X.z + (eb * ia) * Y.z);
        const v3 pb = V(c.x + (na * ib) * X.x + (nb * ib) * Y.x, c.y + (na * ib) * X.y + (nb * ib) * Y.y,
                        c.z + (na * ib) * X.z + (nb * ib) * Y.z);
        if (!seg_clear_of_box(pa, pb, mp.lo, mp.hi, mp.eta * (fmax(rp, r) + mp.scale))) return false;
      }
      rp = r; vprev = v; ea = na; eb = nb;
    }
  }
  return true;
}
// Is the camera ray (o, d) a proven miss?  Schwarzschild builds only; the reference-work
// counting passes (COUNT without count_exec) always march exactly.
// W: the calling kernel build's tag -- one copy per build, since a callee shared by builds of
// different waves-per-SIMD budgets takes the smallest budget's registers for all of them
template <bool COUNT, int W>
__device__ __noinline__ bool camera_miss_proof_call(const KParams& kp, v3 o, v3 d, Counters& cn) {
  return camera_miss_proof<COUNT>(kp, o, d, cn);
}
// NI: out of line (the register-heavy per-pixel-loop builds keep their occupancy), W its build tag
template <bool COUNT, bool KERR, bool NI = false, int W = 0>
__device__ __forceinline__ bool camera_proven_miss(const KParams& kp, v3 o, v3 d, Counters& cn) {
  if (KERR || !kp.miss.on || (COUNT && !kp.count_exec)) return false;
  RRT_T0(tp0);
  const bool r = NI ? camera_miss_proof_call<COUNT, W>(kp, o, d, cn) : camera_miss_proof<COUNT>(kp, o, d, cn);
  RRT_ACC(t_proof, tp0);
  if (COUNT && r && kp.audit && audit_pick(kp, o, d)) {
    Counters c2 = {};
    Isect i2;
    audit_note(kp, RRT_AUDIT_CAMERA, query<false, false, false>(kp, o, d, &i2, c2));
  }
  return r;
}

// ------------------------------------------------------------------ pixel miss proof
// (DESIGN.md §5).  Every camera ray of pixel (px, py) -- jitter anywhere in the pixel's square,
// part1_code.cpp:182-187 -- is a proven miss.  All the rays start at the camera position O, so
// they share x = (O - c) / |O - c| and u = 1 / |O - c|; a ray's planar march depends on its
// direction only through dx = d . x (u' = -u dx / sqrt(1 - dx^2)), and its plane only through
// y.  The proof runs the recurrence for the pixel's least, central and largest dx (from its
// corners and centre, widened for curvature) and, while the three agree in the sign of every v
// and vary little, bounds every ray's points around the central ray's: with the frame (ea, eb)
// the same for all, |P - P_c| <= rho |1/v - 1/v_c| + (rho / |v|) |eb| |y - y_c|.  Each segment
// of the central ray must then clear the root box by the camera proof's margin plus that bound.
// Launch constants are the camera proof's (KParams::miss) and the camera's.
__device__ __forceinline__ v3 pixel_ray_dir(const KParams& kp, double sx, double sy) {
  const DCamera& cam = kp.cam;
  const double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
  const double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
  const v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
  return unit(w);
}
// A rectangle of pixels (the strip pass, rrt_strip_proof_kernel): jitter positions [px, px + w] x
// [py, py + h]; the same argument with the rectangle's corners and centre (the curvature term
// uses its half-diagonal, so it holds for any small rectangle; w = h = 1 is pixel_miss_proof).
__device__ __forceinline__ bool rect_miss_proof(const KParams& kp, double px, double py, double w, double hgt) {
#pragma clang fp contract(fast)
  const DMissProof& mp = kp.miss;
  const DHole& h = kp.hole;
  const v3 O = ld3(kp.cam.pos), c = ld3(h.c);
  const v3 x0 = O - c;
  const double r0 = sqrt(norm2(x0)), u0 = 1.0 / r0;
  const v3 X = vmul(x0, u0);
  // the pixel's directions: dx range, the centre's plane axis y_c and the spread of y
  const v3 dc = pixel_ray_dir(kp, px + 0.5 * w, py + 0.5 * hgt);
  const double dxc = dot(dc, X);
  v3 Yc = dc - smul(dxc, X);
  const double dyc = sqrt(norm2(Yc));
  if (!(dyc > 1e-3)) return false;  // towards the hole: no stable plane
  Yc = vmul(Yc, 1.0 / dyc);
  double dlo = dxc, dhi = dxc, dY = 0.0, dd = 0.0, dymin = dyc;
#pragma unroll 1
  for (int k = 0; k < 4; ++k) {
    const v3 d = pixel_ray_dir(kp, px + (k & 1) * w, py + (k >> 1) * hgt);
    const double dx = dot(d, X);
    dlo = fmin(dlo, dx);
    dhi = fmax(dhi, dx);
    const v3 yv = d - smul(dx, X);
    const double dy = sqrt(norm2(yv));
    if (!(dy > 1e-3)) return false;
    dymin = fmin(dymin, dy);
    dY = fmax(dY, sqrt(norm2(vmul(yv, 1.0 / dy) - Yc)));
    dd = fmax(dd, sqrt(norm2(d - dc)));
  }
  // Every direction of the rectangle lies within dd of dc (the farthest point of a convex spherical
  // polygon from an inner point is a vertex), so the directions +-X -- where the plane axis y turns
  // round -- stay outside it when dd is well below the sine of dc's angle from them, and y then
  // varies smoothly over the rectangle, its spread set by the corners.  A rectangle subtending a
  // large angle near +-X (small frames, wide fields of view) is left to the pixel level.
  if (!(dd <= 0.25 * dymin)) return false;
  // a smooth function over the small square: extremes within the corners' values plus a
  // curvature term of the square's angular radius squared
  const double slack = 2.0 * dd * dd + 1e-12, wdx = dhi - dlo;
  dlo -= 0.05 * wdx + slack;
  dhi += 0.05 * wdx + slack;
  dY = 1.25 * dY + slack;
  if (!(dlo > -1.0 && dhi < 1.0)) return false;
  // three planar recurrences (least, central, largest dx), started at A = O as the shadow proof
  double s[3], vp[3];
  {
    const double dxs[3] = {dlo, dxc, dhi};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double up0 = -u0 * dxs[i] / sqrt(1.0 - dxs[i] * dxs[i]);
      vp[i] = mp.rho * u0;
      s[i] = u0 * mp.co1 - up0 * h.sin_dt * mp.inv_rho;
    }
  }
  double ea = 1.0, eb = 0.0, sig = 1.0, rp = r0, dpa = 0.0, dvp = 0.0;  // A = O: the same for all rays
  const double si2 = h.sin_dt * h.sin_dt;
#pragma unroll 1
  for (int j = 0; j < h.steps; ++j) {
    double v[3];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double up = (vp[i] * mp.co1 - mp.rho * s[i]) * mp.inv_si;
      s[i] = fabs(vp[i]) * mp.inv_rho;
      const double f1 = -s[i] + mp.k15 * s[i] * s[i];
      const double u2 = s[i] + up * (h.dt * 0.5);
      const double f2 = -u2 + mp.k15 * u2 * u2;
      const double u3 = u2 + f1 * mp.dt2_4;
      const double f3 = -u3 + mp.k15 * u3 * u3;
      v[i] = s[i] + up * h.dt + (f1 + f2 + f3) * mp.dt2_6;
      ok = ok && fabs(v[i]) >= mp.kappa * (s[i] + fabs(up) * h.dt);  // NaN: false
    }
    // one sign history for the whole pixel, and v far from 0 compared with its spread
    const double dv = 1.5 * fmax(fabs(v[0] - v[1]), fabs(v[2] - v[1]));
    const double av = fabs(v[1]);
    if (!(ok && (v[0] < 0.0) == (v[1] < 0.0) && (v[2] < 0.0) == (v[1] < 0.0) && av > 2.0 * dv)) return false;
    const double sg = vp[1] < 0.0 ? -1.0 : 1.0;
    const double a = sg * mp.co1, b = sig * mp.si1;
    const double na = a * ea - b * eb, nb = a * eb + b * ea;
    sig *= sg;
    const double r = mp.rho / (av - dv) * (1.0 + 1e-6);  // |B - c| over the pixel (upper bound)
    const double dpb = mp.rho * dv / (av * (av - dv)) * (1.0 + 1e-6) + r * fabs(nb) * dY;
    const double m0 = mp.eta * (fmax(rp, r) + mp.scale);
    const double m = m0 + fmax(dpa, dpb);
    // Distance from the hole: a ray's segment depends only on its (v_prev, v) -- turning the
    // plane about x keeps it -- and the pixel's pairs lie in [v_prev +- dvp] x [v +- dv], a box
    // on which neither coordinate changes sign (checked above, and for v_prev one step earlier).
    // A segment is never nearer the hole than its line, at distance^2 sin^2 dt / D, and D is a
    // positive definite quadratic form on that box (convex: its maximum, the nearest line, at a
    // corner), so the line test at the four corners covers every ray of the pixel, whichever
    // side of its segment the foot of the perpendicular falls on.
    const double rb = mp.r_ball + m0;
    bool far = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double w = v[1] + ((k & 1) ? dv : -dv), wp = vp[1] + ((k & 2) ? dvp : -dvp);
      const double D = w * w + wp * wp - 2.0 * mp.co1 * fabs(wp) * w;
      far = far && si2 > rb * rb * D;
    }
    if (!far) {
      const double ia = mp.rho / vp[1], ib = mp.rho / v[1];
      const v3 pa = j == 0 ? O : V(c.x + (ea * ia) * X.x + (eb * ia) * Yc.x, c.y + (ea * ia) * X.y + (eb * ia) * Yc.y,
                                   c.z + (ea * ia) * X.z + (eb * ia) * Yc.z);
      const v3 pb = V(c.x + (na * ib) * X.x + (nb * ib) * Yc.x, c.y + (na * ib) * X.y + (nb * ib) * Yc.y,
                      c.z + (na * ib) * X.z + (nb * ib) * Yc.z);
      if (!seg_clear_of_box(pa, pb, mp.lo, mp.hi, m)) return false;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) vp[i] = v[i];
    rp = r; dpa = dpb; dvp = dv; ea = na; eb = nb;
  }
  return true;
}
__device__ __forceinline__ bool pixel_miss_proof(const KParams& kp, uint32_t px, uint32_t py) {
  return rect_miss_proof(kp, (double)px, (double)py, 1.0, 1.0);
}

// Heavy pixel (slot-parallel heavy pixels): some of the pixel's rays are captured
// by the hole and some not, or its rays pass within sqrt(kp.heavy_r2) of the hole.  Such pixels
// orbit the hole before they reach the geometry (the costliest queries of a frame) and mix hits
// with misses (several speculation rounds per step in the batch kernel), so their slots are
// rendered in parallel by whole batch-kernel waves (rrt_sample.hip heavy_pixel_wave).  A routing
// heuristic only -- the pixel's result is the same on either path.  The planar recurrence
// (camera_miss_proof) for the least and largest dx of the pixel's corners; a segment's distance
// from the hole follows from (v_prev, v) alone.
__device__ __forceinline__ bool pixel_heavy(const KParams& kp, uint32_t px, uint32_t py) {
#pragma clang fp contract(fast)
  const DMissProof& mp = kp.miss;
  const DHole& h = kp.hole;
  const v3 O = ld3(kp.cam.pos), c = ld3(h.c);
  const v3 x0 = O - c;
  const double r0 = sqrt(norm2(x0)), u0 = 1.0 / r0;
  const v3 X = vmul(x0, u0);
  double dlo = 2.0, dhi = -2.0;
#pragma unroll 1
  for (int k = 0; k < 4; ++k) {
    const double dx = dot(pixel_ray_dir(kp, (double)px + (k & 1), (double)py + (k >> 1)), X);
    dlo = fmin(dlo, dx);
    dhi = fmax(dhi, dx);
  }
  if (!(dlo > -1.0 && dhi < 1.0)) return true;  // looking at the hole
  const double r2 = h.r2, near2 = kp.heavy_r2, si2 = h.sin_dt * h.sin_dt, rho2 = mp.rho * mp.rho;
  bool cap[2] = {false, false}, close = false;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double dx = i ? dhi : dlo;
    const double up0 = -u0 * dx / sqrt(1.0 - dx * dx);
    double vp = mp.rho * u0, s = u0 * mp.co1 - up0 * h.sin_dt * mp.inv_rho;
#pragma unroll 1
    for (int j = 0; j < h.steps; ++j) {
      const double up = (vp * mp.co1 - mp.rho * s) * mp.inv_si;
      s = fabs(vp) * mp.inv_rho;
      const double f1 = -s + mp.k15 * s * s;
      const double u2 = s + up * (h.dt * 0.5);
      const double f2 = -u2 + mp.k15 * u2 * u2;
      const double u3 = u2 + f1 * mp.dt2_4;
      const double f3 = -u3 + mp.k15 * u3 * u3;
      const double v = s + up * h.dt + (f1 + f2 + f3) * mp.dt2_6;
      const double av = fabs(v), avp = fabs(vp);
      const double D = v * v + vp * vp - 2.0 * mp.co1 * avp * v;
      const bool inside = v * (mp.co1 * avp - v) < 0.0 && avp * (avp - mp.co1 * v) > 0.0;
      // distance^2 from the hole below d2  <=>  inside ? si2 / D : rho^2 / max(v, vp)^2 below d2
      const double m2 = fmax(v * v, vp * vp);
      const bool in_r = inside ? si2 < r2 * D : rho2 < r2 * m2;
      const bool in_n = inside ? si2 < near2 * D : rho2 < near2 * m2;
      close = close || in_n;
      if (in_r) { cap[i] = true; break; }
      if (!(av > 0.0)) break;  // NaN or a degenerate step
      vp = v;
    }
  }
  return cap[0] != cap[1] || (close && !(cap[0] && cap[1]));
}

// W: the occlusion proof's build tag (0: no proof in this build).  Its out-of-line part (the face
// test, occ_exit_call) gets one copy per calling kernel build: a callee shared by kernels of
// different waves-per-SIMD budgets gets the smallest budget's registers, and every caller then
// allocates the callee's count.  Measured on cfg3 (profiles/r02_ab_log.md): inline 31.5 ms, face
// test out of line 31.3, whole proof out of line 37.6 (the call's frame and SGPR saves), no proof
// 35.3.
template <bool ANY, bool COUNT, bool KERR = false, int W = 0, bool W4 = true>
__device__ __forceinline__ bool query_nx(const KParams& kp, v3 o, v3 d, Isect* is, Counters& cn) {
  // shadow rays: the occlusion proof first (Schwarzschild; never in the reference-work counts)
  if (W && ANY && !KERR && kp.occ.on && !(COUNT && !kp.count_exec)) {
    RRT_T0(tp0);
    const bool occluded = shadow_occluded_proof<W>(kp, o, d, kp.hole.steps);
    RRT_ACC(t_squery, tp0);
    if (occluded) {
      if (COUNT && kp.audit && audit_pick(kp, o, d)) {
        Counters c2 = {};
        audit_note(kp, RRT_AUDIT_SHADOW, !query<true, false, false>(kp, o, d, nullptr, c2));
      }
      return true;
    }
  }
  return query<ANY, COUNT, KERR, W4>(kp, o, d, is, cn);
}

// ------------------------------------------------------------------ BSDFs (bsdf.cpp / bsdf.h)
struct Frame { v3 X, Y, Z; };
__device__ __forceinline__ Frame coord_space(v3 n) {  // make_coord_space, bsdf.cpp:13-29
  v3 z = n, h = z;
  if (fabs(h.x) <= fabs(h.y) && fabs(h.x) <= fabs(h.z)) h.x = 1.0;
  else if (fabs(h.y) <= fabs(h.x) && fabs(h.y) <= fabs(h.z)) h.y = 1.0;
  else h.z = 1.0;
  z = normalize(z);
  v3 y = normalize(cross(h, z));
  v3 x = normalize(cross(z, y));
  Frame f; f.X = x; f.Y = y; f.Z = z;
  return f;
}
__device__ __forceinline__ v3 to_local(const Frame& f, v3 v) { return V(dot(v, f.X), dot(v, f.Y), dot(v, f.Z)); }
__device__ __forceinline__ v3 to_world(const Frame& f, v3 v) { return (smul(v.x, f.X) + smul(v.y, f.Y)) + smul(v.z, f.Z); }

enum { B_DIFFUSE = 0, B_EMISSION = 1, B_MIRROR = 2, B_GLASS = 3, B_MICROFACET = 4, B_REFRACTION = 5 };
__device__ __forceinline__ bool is_delta(const DBsdf& b) {
  return b.type == B_MIRROR || b.type == B_GLASS || b.type == B_REFRACTION;
}
__device__ __forceinline__ spec emission(const DBsdf& b) {
  return b.type == B_EMISSION ? S(b.p[0], b.p[1], b.p[2]) : S(0, 0, 0);
}
__device__ __forceinline__ double clamp_b(double n, double lo, double hi) { return std_max(lo, std_min(n, hi)); }
// The microfacet BSDF's exp/log/erf/atan/tan (bsdf.cpp:45-96, bsdf.h:159-191): glibc's own,
// restated in rrt_glibm.h (bit-exact against the library on the CPU and, through rrt_libm_eval, on
// the GPU), so the microfacet scenes are bit-exact too.  (Round 5 had to keep the device libm here:
// with the restatements inlined into bsdf_f the inliner stopped inlining the direct-lighting
// functions, and the general kernels' out-of-line calls to them faulted -- DESIGN.md §3.  Those
// functions are __forceinline__ now, so every build has the same call structure with or without
// the restatements.)
#define RRT_MF_TAN rrt_glibm_tan
#define RRT_MF_ERF rrt_glibm_erf
#define RRT_MF_EXP rrt_glibm_exp
#define RRT_MF_ATAN rrt_glibm_atan
#define RRT_MF_LOG rrt_glibm_log
__device__ __forceinline__ double mf_theta(v3 w) { return rrt_glibm_acos(clamp_b(w.z, -1.0 + 1e-5, 1.0 - 1e-5)); }
__device__ __forceinline__ double mf_lambda(float alpha, v3 w) {
  double theta = mf_theta(w);
  double a = 1.0 / (alpha * RRT_MF_TAN(theta));
  return 0.5 * (RRT_MF_ERF(a) - 1.0 + RRT_MF_EXP(-a * a) / (a * PI_D));
}
__device__ __forceinline__ spec mf_F(const DBsdf& b, v3 wi) {
  spec eta = S(b.p[0], b.p[1], b.p[2]), k = S(b.p[3], b.p[4], b.p[5]);
  spec eta2pk2 = eta * eta + k * k;
  double cti = wi.z, cti2 = cti * cti;
  spec tc = (eta * 2.0f) * (float)cti;
  spec Rs = ((eta2pk2 - tc) + (float)cti2) / ((eta2pk2 + tc) + (float)cti2);
  spec Rp = ((eta2pk2 * (float)cti2 - tc) + 1.0f) / ((eta2pk2 * (float)cti2 + tc) + 1.0f);
  return (Rs + Rp) / 2.0f;
}
__device__ __forceinline__ double mf_D(float alpha, v3 h) {
  double theta_h = mf_theta(h), tan_h = RRT_MF_TAN(theta_h), cos_h = h.z, cos_h2 = cos_h * cos_h;
  double alpha2 = alpha * alpha;  // float product, as the reference
  return RRT_MF_EXP(-tan_h * tan_h / alpha2) / (PI_D * alpha2 * cos_h2 * cos_h2);
}
__device__ __forceinline__ spec mf_f(const DBsdf& b, v3 wo, v3 wi) {
  if (wo.z <= 0 || wi.z <= 0) return S(0, 0, 0);
  float alpha = b.p[6];
  double G = 1.0 / (1.0 + mf_lambda(alpha, wi) + mf_lambda(alpha, wo));
  double D = mf_D(alpha, unit(wo + wi));
  return ((mf_F(b, wi) * (float)G) * (float)D) / (float)(4 * wo.z * wi.z);
}
// LEAN: the scene has no microfacet BSDF (only diffuse / emission / delta BSDFs reach f)
template <int LEAN = 0>
__device__ __forceinline__ spec bsdf_f(const DBsdf& b, v3 wo, v3 wi) {
  if (b.type == B_DIFFUSE) return S(b.p[0], b.p[1], b.p[2]) / (float)PI_D;
  if (!is_lean(LEAN) && b.type == B_MICROFACET) return mf_f(b, wo, wi);
  return S(0, 0, 0);
}
__device__ __forceinline__ bool refract(v3 wo, v3& wi, float ior) {  // bsdf.cpp:146-159
  double eta;
  if (wo.z > 0) eta = 1 / ior; else eta = ior;
  double wi_z2 = 1 - eta * eta * (1 - wo.z * wo.z);
  if (wi_z2 < 0) return false;
  wi = V(-eta * wo.x, -eta * wo.y, sqrt(wi_z2));
  if (wo.z > 0) wi.z = -wi.z;
  return true;
}
__device__ __forceinline__ spec bsdf_sample_f(const DBsdf& b, Rng& g, v3 wo, v3& wi, float& pdf, bool mf_hemi = false) {
  switch (b.type) {
    case B_DIFFUSE:
      wi = cosine_sample(g, &pdf);
      return bsdf_f(b, wo, wi);
    case B_MIRROR:
      wi = V(-wo.x, -wo.y, wo.z); pdf = 1.0f;
      return S(b.p[0], b.p[1], b.p[2]) / (float)fabs(wi.z);
    case B_GLASS: {
      float ior = b.p[7];
      spec tr = S(b.p[0], b.p[1], b.p[2]), rf = S(b.p[3], b.p[4], b.p[5]);
      if (refract(wo, wi, ior)) {
        double R0 = (1 - ior) / (1 + ior);
        R0 *= R0;
        double t = (1 - fabs(wi.z)), t2 = t * t, t4 = t2 * t2, R = R0 + (1 - R0) * t4 * t;
        if (g.coin(R)) {
          wi = V(-wo.x, -wo.y, wo.z); pdf = (float)R;
          return (rf * (float)R) / (float)fabs(wi.z);
        }
        double eta;
        if (wo.z > 0) eta = 1 / ior; else eta = ior;
        pdf = (float)(1 - R);
        return (tr * (float)(1 - R)) / (float)(fabs(wi.z) * eta * eta);
      }
      wi = V(-wo.x, -wo.y, wo.z); pdf = 1.0f;
      return rf / (float)fabs(wi.z);
    }
    case B_MICROFACET: {
      if (mf_hemi) {  // MICROFACET_HEMI 1 (bsdf.cpp:93-94): f(wo, *wi = cosine hemisphere sample)
        wi = cosine_sample(g, &pdf);
        return mf_f(b, wo, wi);
      }
      double ux, uy;
      g.grid(ux, uy);
      float alpha = b.p[6];
      double alpha2 = alpha * alpha,
             theta_h = RRT_MF_ATAN(sqrt(-alpha2 * RRT_MF_LOG(1 - ux))),
             phi_h = 2 * PI_D * uy,
             sin_h = rrt_glibm_sin(theta_h), cos_h = rrt_glibm_cos(theta_h), tan_h = RRT_MF_TAN(theta_h),
             p_theta = 2 * sin_h * RRT_MF_EXP(-tan_h * tan_h / alpha2) / (alpha2 * cos_h * cos_h * cos_h),
             p_phi = 0.5 / PI_D;
      v3 h = V(sin_h * rrt_glibm_cos(phi_h), sin_h * rrt_glibm_sin(phi_h), cos_h);
      wi = smul(2 * dot(wo, h), h) - wo;
      if (wi.z <= 0) { pdf = 0; return S(0, 0, 0); }
      pdf = (float)(p_theta * p_phi / (sin_h * 4 * dot(wi, h)));
      return mf_f(b, wo, wi);
    }
    case B_EMISSION:
      pdf = (float)(1.0 / PI_D);
      wi = cosine_sample(g, &pdf);
      return S(0, 0, 0);
    default:
      pdf = 0.0f;
      return S(0, 0, 0);
  }
}

// ------------------------------------------------------------------ environment light
// environment_light.cpp:89-148.  Texel arithmetic in float (Spectrum * double narrows the
// weight to float, as Spectrum::operator*(float) does).
__device__ __forceinline__ spec env_texel(const DEnv& e, size_t i) {
  return S(e.tex[3 * i], e.tex[3 * i + 1], e.tex[3 * i + 2]);
}
__device__ spec env_bilerp(const DEnv& e, double xx, double yy) {  // :112-127
  long right = lround(xx), left, v = lround(yy);
  double u1 = right - xx + .5, v1;
  if (right == 0 || right == (long)e.w) { left = (long)e.w - 1; right = 0; }
  else left = right - 1;
  if (v == 0) { v = 1; v1 = 1; }
  else if (v == (long)e.h) { v = (long)e.h - 1; v1 = 0; }
  else v1 = v - yy + .5;
  const size_t bottom = (size_t)e.w * (size_t)v, top = bottom - e.w;
  const double u0 = 1 - u1;
  const float fu1 = (float)u1, fu0 = (float)u0, fv1 = (float)v1, fv0 = (float)(1 - v1);
  return ((env_texel(e, top + left) * fu1) + (env_texel(e, top + right) * fu0)) * fv1 +
         ((env_texel(e, bottom + left) * fu1) + (env_texel(e, bottom + right) * fu0)) * fv0;
}
// sample_dir (:146-148): radiance seen along direction d (the unbent camera ray on a miss)
__device__ __forceinline__ spec env_dir(const DEnv& e, v3 d) {
  const v3 u = unit(d);
  const double theta = rrt_glibm_acos(u.y), phi = rrt_glibm_atan2(-u.z, u.x) + PI_D;  // dir_to_theta_phi (:89-94)
  const double x = phi / 2. / PI_D * e.w, y = theta / PI_D * e.h;  // theta_phi_to_xy (:71-77)
  return env_bilerp(e, x, y);
}
// std::upper_bound over a double array (libstdc++'s halving loop, value < *it)
__device__ __forceinline__ uint32_t upper_bound_d(const double* a, uint32_t n, double value) {
  uint32_t first = 0, count = n;
  while (count > 0) {
    const uint32_t step = count >> 1, it = first + step;
    if (!(value < a[it])) { first = it + 1; count -= step + 1; }
    else count = step;
  }
  return first;
}
// sample_L (:130-144, ENV_HEMI == 0): row by the marginal CDF, column by the row's conditional CDF
__device__ __forceinline__ spec env_sample(const DEnv& e, Rng& g, v3& wi, float& dist, float& pdf) {
  dist = INFINITY;
  double sx, sy;
  g.grid(sx, sy);
  uint32_t y = upper_bound_d(e.marg, e.h, sy);
  if (y >= e.h) y = e.h - 1;  // (the reference reads one row past the table when sy == 1)
  uint32_t x = upper_bound_d(e.conds + (size_t)e.w * y, e.w, sx);
  if (x >= e.w) x = e.w - 1;
  const double phi = (double)x / e.w * 2.0 * PI_D, theta = (double)y / e.h * PI_D;  // xy_to_theta_phi
  wi = V(rrt_glibm_cos(phi - PI_D) * rrt_glibm_sin(theta), rrt_glibm_cos(theta),
         -rrt_glibm_sin(phi - PI_D) * rrt_glibm_sin(theta));  // theta_phi_to_dir
  pdf = (float)(e.pdf[(size_t)e.w * y + x] * e.w * e.h / (2 * PI_D * PI_D * rrt_glibm_sin(theta)));
  return env_bilerp(e, (double)x, (double)y);
}

// ------------------------------------------------------------------ lights (light.cpp)
// LEAN: every light is an area or a point light
template <int LEAN = 0>
__device__ __forceinline__ spec light_sample_L(const DEnv& env, const DLight& l, Rng& g, v3 p, v3& wi, float& dist, float& pdf,
                               bool env_hemi = false) {
  spec rad = S(l.rad[0], l.rad[1], l.rad[2]);
  switch (LEAN == 1 ? 0u : LEAN == 2 ? (l.type == 1u ? 1u : 0u) : l.type) {
    case 0: {  // AreaLight::sample_L (light.cpp:80-92): float sqDist, sqrtf, float pdf
      double sx, sy;
      g.grid(sx, sy);
      sx = sx - 0.5f; sy = sy - 0.5f;
      v3 d = ((ld3(l.v[0]) + smul(sx, ld3(l.v[2]))) + smul(sy, ld3(l.v[3]))) - p;
      float sqDist = (float)norm2(d);
      float dd = sqrtf(sqDist);
      wi = divd(d, dd);
      float cosTheta = (float)dot(wi, ld3(l.v[1]));
      dist = dd;
      pdf = sqDist / (l.area * fabsf(cosTheta));
      return cosTheta < 0 ? rad : S(0, 0, 0);
    }
    case 1: {  // PointLight
      v3 d = ld3(l.v[0]) - p;
      wi = unit(d); dist = (float)norm(d); pdf = 1.0f;
      return rad;
    }
    case 2:  // DirectionalLight
      wi = ld3(l.v[0]); dist = INFINITY; pdf = 1.0f;
      return rad;
    case 5:  // EnvironmentLight (appended by PathTracer::set_scene, pathtracer.cpp:106-108)
      if (LEAN == V_SW && env_hemi) {  // ENV_HEMI 1 (environment_light.cpp:139-142)
        dist = INFINITY;
        // UniformSphereSampler3D::get_sample (sampler.cpp:33-40)
        const double z = g.uniform() * 2 - 1;
        const double q = 1.0 - z * z, sin_t = sqrt((0.0 < q) ? q : 0.0);  // std::max(0.0, 1.0f - z * z)
        const double phi = 2.0 * PI_D * g.uniform();
        wi = V(rrt_glibm_cos(phi) * sin_t, rrt_glibm_sin(phi) * sin_t, z);
        pdf = (float)(0.25 / PI_D);
        return env_dir(env, wi);  // sample_dir(Ray(p, wi))
      }
      return env_sample(env, g, wi, dist, pdf);
    default: {  // InfiniteHemisphereLight
      v3 dir = hemisphere_sample(g);
      Frame f; f.X = ld3(l.v[0]); f.Y = ld3(l.v[1]); f.Z = ld3(l.v[2]);
      wi = to_world(f, dir);
      dist = INFINITY; pdf = (float)(1.0 / (2.0 * PI_D));
      return rad;
    }
  }
}

}  // namespace rrt
