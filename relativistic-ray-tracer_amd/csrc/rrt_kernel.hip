// rrt_kernel.hip -- the hot path on gfx950: per-pixel radiance loop with geodesic-marched BVH
// queries (reference: part1_code.cpp:15-187, bvh.cpp:103-138, blackhole.cpp:17-40).
//
// Numerics follow the reference exactly: double geometry, float Spectrum with the reference's
// narrowing points, the same operation order, no FMA contraction (-ffp-contract=off and the
// pragma below), IEEE division / sqrt.  Transcendentals whose arguments are per-run constants
// (tan of the half FOV, cos/sin of delta_theta) are computed once on the host with its libm,
// i.e. with the same values the reference uses; per-sample transcendentals (only on the
// bounce / hemisphere / microfacet paths) use the device libm and may differ by an ulp.
//
// Work decomposition: persistent grid; each wave pulls 8x8 pixel blocks (one lane = one pixel,
// the whole adaptive sample loop) from a device atomic over the caller's tile list, so a
// partition of any shape (one GPU's block-cyclic share of the frame) load-balances inside the
// device.  BVH traversal is stackless over skip pointers (rrt_internal.h DNode), which visits
// exactly the reference's left-then-right recursion order.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rrt_internal.h"
#include "rrt_rng.h"

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
__device__ __forceinline__ double norm(v3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ double norm2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ v3 unit(v3 a) {
  double r = 1. / sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return V(r * a.x, r * a.y, r * a.z);
}
__device__ __forceinline__ v3 normalize(v3 a) { double c = 1. / norm(a); return V(a.x * c, a.y * c, a.z * c); }
__device__ __forceinline__ v3 divd(v3 a, double c) { double rc = 1.0 / c; return V(rc * a.x, rc * a.y, rc * a.z); }
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
  return V(r * cos(theta), r * sin(theta), sqrt(1 - Xi1));
}
__device__ __forceinline__ v3 hemisphere_sample(Rng& g) {  // sampler.cpp:15-29 (float trig)
  double Xi1 = g.uniform();
  double Xi2 = g.uniform();
  double theta = acos(Xi1);
  double phi = 2.0 * PI_D * Xi2;
  double xs = sinf((float)theta) * cosf((float)phi);
  double ys = sinf((float)theta) * sinf((float)phi);
  double zs = cosf((float)theta);
  return V(xs, ys, zs);
}

struct Counters { uint32_t bbox, micro, prim, query; };

// ------------------------------------------------------------------ geometry
// BBox::intersect (bbox.cpp:10-25); min_t is 0 for every micro segment
__device__ __forceinline__ bool bbox_hit(const DNode& n, v3 o, v3 d, double max_t) {
  double tx0 = (n.mn[0] - o.x) / d.x, tx1 = (n.mx[0] - o.x) / d.x,
         ty0 = (n.mn[1] - o.y) / d.y, ty1 = (n.mx[1] - o.y) / d.y,
         tz0 = (n.mn[2] - o.z) / d.z, tz1 = (n.mx[2] - o.z) / d.z,
         tmin = std_max(std_max(std_min(tx0, tx1), std_min(ty0, ty1)), std_min(tz0, tz1)),
         tmax = std_min(std_min(std_max(tx0, tx1), std_max(ty0, ty1)), std_max(tz0, tz1));
  return tmin <= tmax && tmin <= max_t && tmax >= 0.0;
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
// Triangle::intersect (triangle.cpp:25-55) with e1, e2 precomputed (bit-identical values)
__device__ __forceinline__ bool tri_t(const DPrimGeo& gp, v3 o, v3 d, double max_t, double& t, double& b1o,
                                      double& b2o) {
  v3 p0 = V(gp.v[0], gp.v[1], gp.v[2]), e1 = V(gp.v[3], gp.v[4], gp.v[5]), e2 = V(gp.v[6], gp.v[7], gp.v[8]);
  v3 s = o - p0, s1 = cross(d, e2), s2 = cross(s, e1);
  double inv = 1. / dot(s1, e1);
  double tt = dot(s2, e2) * inv, b1 = dot(s1, s) * inv, b2 = dot(s2, d) * inv, b0 = 1 - b1 - b2;
  if (0.0 <= tt && tt <= max_t && b0 >= 0 && b1 >= 0 && b2 >= 0) { t = tt; b1o = b1; b2o = b2; return true; }
  return false;
}

struct Isect { v3 hit_p, w_out, n; int bsdf; };

// BVHAccel::intersect_micro (bvh.cpp:115-138) for one micro segment.  ANY: shadow query, stop
// at the first accepted primitive (only the boolean is used; result-identical).
template <bool ANY, bool COUNT>
__device__ __forceinline__ bool traverse(const KParams& kp, v3 o, v3 d, double& max_t, int& hit_slot,
                                         double& hb1, double& hb2, Counters& cn) {
  bool hit = false;
  int node = 0;
  while (node >= 0) {
    const DNode n = kp.nodes[node];
    if (COUNT) cn.bbox++;
    if (!bbox_hit(n, o, d, max_t)) { node = n.skip; continue; }
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

// BlackHole::next_micro_ray (blackhole.cpp:17-40); f4 is computed but unused there
__device__ __forceinline__ void next_micro(const DHole& h, v3& o, v3& d, double& max_t) {
  v3 no = o + vmul(d, max_t);
  v3 x_axis = no - V(h.c[0], h.c[1], h.c[2]);
  double dist = norm(x_axis);
  x_axis = normalize(x_axis);
  double u = 1 / dist;
  double dx = dot(d, x_axis);
  v3 y_axis = d - smul(dx, x_axis);
  double dy = norm(y_axis);
  y_axis = normalize(y_axis);
  double up = -u * dx / dy;
  const double dt = h.dt, k = 3.0 * h.r;
  double f1 = -u + k * u * u / 2.0;
  double u2 = u + up * dt / 2.0;
  double f2 = -u2 + k * u2 * u2 / 2.0;
  double u3 = u + up * dt / 2.0 + f1 * dt * dt / 4.0;
  double f3 = -u3 + k * u3 * u3 / 2.0;
  u += up * dt + (f1 + f2 + f3) * dt * dt / 6.0;
  double dd = 1 / u;
  double next_x = dd * h.cos_dt, next_y = dd * h.sin_dt;
  v3 nd = ((V(h.c[0], h.c[1], h.c[2]) + smul(next_x, x_axis)) + smul(next_y, y_axis)) - no;
  max_t = norm(nd);
  d = normalize(nd);
  o = no;
}

// BVHAccel::intersect (bvh.cpp:103-113): march the geodesic as straight micro segments; the
// incoming ray's min_t / max_t are dropped (camera clip planes and shadow-ray distance are
// ignored, as in the reference).  Capture by the hole returns "no hit".
template <bool ANY, bool COUNT>
__device__ bool query(const KParams& kp, v3 o, v3 d, Isect* is, Counters& cn) {
  if (COUNT) cn.query++;
  double max_t = 0.0;
  const v3 hc = V(kp.hole.c[0], kp.hole.c[1], kp.hole.c[2]);
  for (int j = 0; j < kp.hole.steps; ++j) {
    next_micro(kp.hole, o, d, max_t);
    if (COUNT) cn.micro++;
    double tc;
    if (sphere_t(hc, kp.hole.r2, o, d, max_t, tc)) return false;  // captured
    int slot = -1;
    double b1 = 0, b2 = 0, seg_t = max_t;
    if (traverse<ANY, COUNT>(kp, o, d, seg_t, slot, b1, b2, cn)) {
      if (!ANY) {
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
  }
  return false;
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
__device__ __forceinline__ double mf_theta(v3 w) { return acos(clamp_b(w.z, -1.0 + 1e-5, 1.0 - 1e-5)); }
__device__ __forceinline__ double mf_lambda(float alpha, v3 w) {
  double theta = mf_theta(w);
  double a = 1.0 / (alpha * tan(theta));
  return 0.5 * (erf(a) - 1.0 + exp(-a * a) / (a * PI_D));
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
  double theta_h = mf_theta(h), tan_h = tan(theta_h), cos_h = h.z, cos_h2 = cos_h * cos_h;
  double alpha2 = alpha * alpha;  // float product, as the reference
  return exp(-tan_h * tan_h / alpha2) / (PI_D * alpha2 * cos_h2 * cos_h2);
}
__device__ __forceinline__ spec mf_f(const DBsdf& b, v3 wo, v3 wi) {
  if (wo.z <= 0 || wi.z <= 0) return S(0, 0, 0);
  float alpha = b.p[6];
  double G = 1.0 / (1.0 + mf_lambda(alpha, wi) + mf_lambda(alpha, wo));
  double D = mf_D(alpha, unit(wo + wi));
  return ((mf_F(b, wi) * (float)G) * (float)D) / (float)(4 * wo.z * wi.z);
}
__device__ __forceinline__ spec bsdf_f(const DBsdf& b, v3 wo, v3 wi) {
  if (b.type == B_DIFFUSE) return S(b.p[0], b.p[1], b.p[2]) / (float)PI_D;
  if (b.type == B_MICROFACET) return mf_f(b, wo, wi);
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
__device__ spec bsdf_sample_f(const DBsdf& b, Rng& g, v3 wo, v3& wi, float& pdf) {
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
      double ux, uy;
      g.grid(ux, uy);
      float alpha = b.p[6];
      double alpha2 = alpha * alpha,
             theta_h = atan(sqrt(-alpha2 * log(1 - ux))),
             phi_h = 2 * PI_D * uy,
             sin_h = sin(theta_h), cos_h = cos(theta_h), tan_h = tan(theta_h),
             p_theta = 2 * sin_h * exp(-tan_h * tan_h / alpha2) / (alpha2 * cos_h * cos_h * cos_h),
             p_phi = 0.5 / PI_D;
      v3 h = V(sin_h * cos(phi_h), sin_h * sin(phi_h), cos_h);
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

// ------------------------------------------------------------------ lights (light.cpp)
__device__ spec light_sample_L(const DLight& l, Rng& g, v3 p, v3& wi, float& dist, float& pdf) {
  spec rad = S(l.rad[0], l.rad[1], l.rad[2]);
  switch (l.type) {
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
    default: {  // InfiniteHemisphereLight
      v3 dir = hemisphere_sample(g);
      Frame f; f.X = ld3(l.v[0]); f.Y = ld3(l.v[1]); f.Z = ld3(l.v[2]);
      wi = to_world(f, dir);
      dist = INFINITY; pdf = (float)(1.0 / (2.0 * PI_D));
      return rad;
    }
  }
}

// ------------------------------------------------------------------ integrator (part1_code.cpp)
template <bool COUNT>
__device__ spec direct_importance(const KParams& kp, Rng& g, const Isect& is, Counters& cn) {  // :33-57
  Frame f = coord_space(is.n);
  v3 w_out = to_local(f, is.w_out);
  const DBsdf b = kp.bsdfs[is.bsdf];
  spec L = S(0, 0, 0);
  int total = 0;
  for (uint32_t li = 0; li < kp.n_lights; ++li) {
    const DLight& l = kp.lights[li];
    int num = l.is_delta ? 1 : (int)kp.ns_area_light;
    total += num;
    for (int i = 0; i < num; ++i) {
      v3 wi_world; float dist, pdf;
      spec sample = light_sample_L(l, g, is.hit_p, wi_world, dist, pdf);
      v3 w_in = to_local(f, wi_world);
      if (w_in.z < 0) continue;
      if (!query<true, COUNT>(kp, is.hit_p + smul(EPS_D, wi_world), wi_world, nullptr, cn))
        L = L + ((sample * bsdf_f(b, w_out, w_in)) * (float)w_in.z) / pdf;
    }
  }
  return L / (float)total;
}

template <bool COUNT>
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
    if (query<false, COUNT>(kp, is.hit_p + smul(EPS_D, wi_world), wi_world, &is2, cn))
      L = L + (emission(kp.bsdfs[is2.bsdf]) * bsdf_f(b, w_out, w_in)) * (float)w_in.z;
  }
  return ((L * 2.0f) * (float)PI_D) / (float)num;
}

template <bool COUNT>
__device__ __forceinline__ spec one_bounce(const KParams& kp, Rng& g, const Isect& is, Counters& cn) {
  return kp.direct_hemisphere ? direct_hemisphere<COUNT>(kp, g, is, cn) : direct_importance<COUNT>(kp, g, is, cn);
}

// at_least_one_bounce_radiance (:69-101) unrolled into a loop: the recursion is walked down
// storing each level's terms, then folded back up in the reference's evaluation order.
template <bool COUNT>
__device__ spec at_least_one_bounce(const KParams& kp, Rng& g, Isect cur, Counters& cn) {
  spec Ld[RRT_MAX_DEPTH], smp[RRT_MAX_DEPTH], cem[RRT_MAX_DEPTH];
  float cs[RRT_MAX_DEPTH], pd[RRT_MAX_DEPTH];
  bool child[RRT_MAX_DEPTH], dl[RRT_MAX_DEPTH];
  uint32_t depth = kp.max_ray_depth;
  int k = 0;
  for (;; ++k) {
    Frame f = coord_space(cur.n);
    v3 w_out = to_local(f, cur.w_out);
    const DBsdf b = kp.bsdfs[cur.bsdf];
    spec L_out = S(0, 0, 0);
    if (!is_delta(b)) L_out = L_out + one_bounce<COUNT>(kp, g, cur, cn);
    Ld[k] = L_out;
    child[k] = false;
    dl[k] = is_delta(b);
    if (depth == kp.max_ray_depth || (depth > 1 && g.coin(0.7))) {
      v3 w_in; float pdf;
      spec sample = bsdf_sample_f(b, g, w_out, w_in, pdf);
      if (pdf == 0.0f) break;
      v3 wi_world = to_world(f, w_in);
      Isect is2;
      if (query<false, COUNT>(kp, cur.hit_p + smul(EPS_D, wi_world), wi_world, &is2, cn) && k + 1 < RRT_MAX_DEPTH) {
        child[k] = true;
        smp[k] = sample; cs[k] = (float)fabs(w_in.z); pd[k] = pdf;
        cem[k] = emission(kp.bsdfs[is2.bsdf]);
        cur = is2;
        depth -= 1;
        continue;
      }
    }
    break;
  }
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

template <bool DEEP, bool COUNT>
__device__ __forceinline__ spec est_radiance(const KParams& kp, Rng& g, v3 o, v3 d, Counters& cn) {  // :103-123
  Isect is;
  if (!query<false, COUNT>(kp, o, d, &is, cn)) return S(0, 0, 0);
  spec e = emission(kp.bsdfs[is.bsdf]);
  if (kp.max_ray_depth == 0) return e;
  if (!DEEP || kp.max_ray_depth == 1) return e + one_bounce<COUNT>(kp, g, is, cn);
  return e + at_least_one_bounce<COUNT>(kp, g, is, cn);
}

// PathTracer::raytrace_pixel (:125-163) with ADAPTIVE == 1, THIN_LENS == 0
template <bool DEEP, bool COUNT>
__device__ spec raytrace_pixel(const KParams& kp, uint32_t x, uint32_t y, int& count, Rng& g, Counters& cn) {
  spec ret = S(0, 0, 0);
  int i;
  double s1 = 0.0, s2 = 0.0;
  const DCamera& cam = kp.cam;
  for (i = 0; i < (int)kp.ns_aa; ++i) {
    double sx = (double)x, sy = (double)y;
    if (kp.ns_aa == 1) { sx += 0.5; sy += 0.5; }
    else { double jx, jy; g.grid(jx, jy); sx += jx; sy += jy; }
    // Camera::generate_ray (part1_code.cpp:182-187)
    double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
    double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
    v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
    spec s = est_radiance<DEEP, COUNT>(kp, g, ld3(cam.pos), unit(w), cn);
    ret = ret + s;
    double il = illum(s);
    s1 += il;
    s2 += il * il;
    if ((uint32_t)(i + 1) % kp.samples_per_batch == 0) {
      double avg = s1 / (i + 1), sd = sqrt((s2 - avg * s1) / i);
      if (1.96 * sd / sqrt((double)(i + 1)) <= (double)kp.max_tolerance * avg) { ++i; break; }
    }
  }
  count = i;
  return ret / (float)i;
}

}  // namespace rrt

// ------------------------------------------------------------------ kernels
template <bool DEEP, bool COUNT>
__global__ __launch_bounds__(256) void rrt_render_kernel(KParams kp) {
  using namespace rrt;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t bpt = kp.blocks_per_tile_side;
  const uint32_t tpix = kp.tile_size * kp.tile_size;
  for (;;) {
    uint32_t blk = 0;
    if (lane == 0) blk = atomicAdd(kp.block_counter, 1u);
    blk = __shfl(blk, 0);
    if (blk >= kp.n_blocks) break;
    const uint32_t t = blk / (bpt * bpt), b = blk % (bpt * bpt);
    const uint32_t lx = (b % bpt) * 8 + (lane & 7u), ly = (b / bpt) * 8 + (lane >> 3);
    const uint32_t x = kp.tiles[2 * t] + lx, y = kp.tiles[2 * t + 1] + ly;
    if (lx < kp.tile_size && ly < kp.tile_size && x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 &&
        y < kp.clip_y1) {
      Rng g; g.key = rrt_pixel_key(kp.seed, x, y); g.ctr = 0;
      Counters cn = {0, 0, 0, 0};
      int cnt;
      spec s = raytrace_pixel<DEEP, COUNT>(kp, x, y, cnt, g, cn);
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

// ------------------------------------------------------------------ launch shims (C++ linkage)
hipError_t rrt_launch_render(const KParams& kp, int deep, int count, uint32_t grid, hipStream_t stream) {
  if (deep && count) hipLaunchKernelGGL((rrt_render_kernel<true, true>), dim3(grid), dim3(256), 0, stream, kp);
  else if (deep) hipLaunchKernelGGL((rrt_render_kernel<true, false>), dim3(grid), dim3(256), 0, stream, kp);
  else if (count) hipLaunchKernelGGL((rrt_render_kernel<false, true>), dim3(grid), dim3(256), 0, stream, kp);
  else hipLaunchKernelGGL((rrt_render_kernel<false, false>), dim3(grid), dim3(256), 0, stream, kp);
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
hipError_t rrt_launch_tonemap(uint32_t n, const float* rgb, uint32_t* out, float exposure, float inv_gamma,
                              hipStream_t stream) {
  uint32_t grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(rrt_tonemap_kernel, dim3(grid), dim3(256), 0, stream, n, rgb, out, exposure, inv_gamma);
  return hipGetLastError();
}
