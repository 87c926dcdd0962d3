// oracle/ref/harness_kat.cpp -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/ref_kat).
//
// Function-level known-answer vectors taken from the reference's OWN compiled functions
// (objects built by Makefile from /root/reference).  Inputs come from a fixed splitmix64
// stream; rand() is scripted (harness_common.h RAND_SCRIPTED) so sampler/BSDF/light draws are
// known.  Each family is written as <outdir>/kat_<name>_{in,out}.npy (float64 / int32 rows).
//
// Families (reference file:line):
//   micro    BlackHole::next_micro_ray chains + capture test   blackhole.cpp:17-40, bvh.cpp:104-108
//   bbox     BBox::intersect                                   bbox.cpp:10-25
//   tri      Triangle::intersect (max_t shrink, hit, normal)   triangle.cpp:25-55
//   sphere   Sphere::intersect (max_t shrink)                  sphere.cpp:10-53
//   coord    make_coord_space                                  bsdf.cpp:13-29
//   sampler  UniformGrid / CosineWeighted / UniformHemisphere / UniformSphere  sampler.cpp:7-56
//   bsdf     Diffuse / Mirror / Glass / Microfacet sample_f    part1_code.cpp:167-173, bsdf.cpp:33-140
//   area     AreaLight::sample_L                               light.cpp:80-92
//   light    Point / Directional / InfiniteHemisphere sample_L  light.cpp:17-23, 34-42, 49-57
//   camray   Camera::generate_ray                              part1_code.cpp:182-187
#include <cmath>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "harness_common.h"

#define private public
#define protected public
#include "bbox.h"
#include "bsdf.h"
#include "camera.h"
#include "pathtracer.h"
#include "sampler.h"
#include "static_scene/blackhole.h"
#include "static_scene/light.h"
#include "static_scene/sphere.h"
#include "static_scene/triangle.h"
#include "static_scene/object.h"
#undef private
#undef protected

using namespace CGL;
using namespace CGL::StaticScene;

namespace harness { thread_local ThreadRng g_rng; }
using harness::g_rng;

extern "C" int __real_rand(void);
extern "C" int __wrap_rand(void) {
  if (g_rng.mode == harness::RAND_SCRIPTED) {
    if (g_rng.ctr >= g_rng.script_len) { std::fprintf(stderr, "script exhausted\n"); std::abort(); }
    return g_rng.script[g_rng.ctr++];
  }
  std::fprintf(stderr, "[kat] unscripted rand()\n");
  std::abort();
}
extern "C" bool __real__ZNK3CGL4BBox9intersectERKNS_3RayERdS4_(const BBox*, const Ray&, double&, double&);
extern "C" bool __wrap__ZNK3CGL4BBox9intersectERKNS_3RayERdS4_(const BBox* b, const Ray& r, double& t0, double& t1) {
  return __real__ZNK3CGL4BBox9intersectERKNS_3RayERdS4_(b, r, t0, t1);
}
extern "C" Ray __real__ZN3CGL11StaticScene9BlackHole14next_micro_rayERKNS_3RayE(BlackHole*, const Ray&);
extern "C" Ray __wrap__ZN3CGL11StaticScene9BlackHole14next_micro_rayERKNS_3RayE(BlackHole* bh, const Ray& r) {
  return __real__ZN3CGL11StaticScene9BlackHole14next_micro_rayERKNS_3RayE(bh, r);
}
extern "C" Spectrum __real__ZN3CGL10PathTracer14raytrace_pixelEmmb(PathTracer*, size_t, size_t, bool);
extern "C" Spectrum __wrap__ZN3CGL10PathTracer14raytrace_pixelEmmb(PathTracer* self, size_t x, size_t y, bool t) {
  return __real__ZN3CGL10PathTracer14raytrace_pixelEmmb(self, x, y, t);
}

// ---- deterministic input stream ----
static uint64_t g_state = 0x1234567ULL;
static double u01() { return (double)(harness::mix64(g_state++) >> 11) * (1.0 / 9007199254740992.0); }
static double urange(double a, double b) { return a + (b - a) * u01(); }
static int rint31() { return (int)(harness::mix64(g_state++) >> 33); }
static Vector3D uvec(double a, double b) { double x = urange(a, b), y = urange(a, b), z = urange(a, b); return Vector3D(x, y, z); }

static std::string g_out = ".";
struct Table {
  std::string name;
  size_t cols;
  std::vector<double> v;
  void row(std::initializer_list<double> r) { if (r.size() != cols) { std::fprintf(stderr, "%s: bad row\n", name.c_str()); std::abort(); } v.insert(v.end(), r); }
  void row(const std::vector<double>& r) { if (r.size() != cols) { std::fprintf(stderr, "%s: bad row\n", name.c_str()); std::abort(); } v.insert(v.end(), r.begin(), r.end()); }
  void save() { harness::write_npy(g_out + "/kat_" + name + ".npy", "<f8", {v.size() / cols, cols}, v.data(), v.size() * 8); }
};
static void script(std::vector<int>& s) { g_rng.mode = harness::RAND_SCRIPTED; g_rng.script = s.data(); g_rng.script_len = s.size(); g_rng.ctr = 0; }

int main(int argc, char** argv) {
  if (argc > 1) g_out = argv[1];

  // ---- micro: chains of next_micro_ray + capture test, for several hole settings ----
  // row: bh(cx,cy,cz,r,dtheta), ray0 (o3,d3), step j, out o3, d3, max_t, captured
  {
    Table t{"micro", 5 + 6 + 1 + 7 + 1};
    const double holes[][5] = {{0, 1, 0, 0.1, 0.1}, {0, 1, 0, 0.0, 0.1}, {0.1, 0.9, -0.2, 0.25, 0.05}, {0, 1, 0, 0.1, 0.3}};
    for (auto& hp : holes) {
      BlackHole bh(nullptr, Vector3D(hp[0], hp[1], hp[2]), hp[3], hp[4]);
      for (int k = 0; k < 16; ++k) {
        Vector3D o = uvec(-3, 3) + Vector3D(0, 1, 0);
        Vector3D aim = Vector3D(hp[0], hp[1], hp[2]) + uvec(-0.6, 0.6);
        if (k % 8 == 0) aim = Vector3D(hp[0], hp[1], hp[2]);  // radial-ish rays
        Vector3D d = (aim - o).unit();
        Ray micro(o, d, 0.0);
        for (int j = 0; j * bh.delta_theta < 2 * M_PI; ++j) {
          micro = bh.next_micro_ray(micro);
          Ray probe = micro;  // Sphere::intersect mutates max_t; record pre-test state
          bool cap = bh.intersect(probe);
          t.row({hp[0], hp[1], hp[2], hp[3], hp[4], o.x, o.y, o.z, d.x, d.y, d.z, (double)j,
                 micro.o.x, micro.o.y, micro.o.z, micro.d.x, micro.d.y, micro.d.z, micro.max_t, cap ? 1.0 : 0.0});
          if (cap) break;
        }
      }
    }
    t.save();
  }

  // ---- bbox: min3 max3 o3 d3 min_t max_t -> hit t0 t1 ----
  {
    Table t{"bbox", 14 + 3};
    for (int k = 0; k < 2048; ++k) {
      Vector3D a = uvec(-1, 1), b = uvec(-1, 1);
      Vector3D mn(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z));
      Vector3D mx(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z));
      if (k % 5 == 1) mx.x = mn.x;        // zero-thickness boxes (Cornell walls)
      if (k % 7 == 2) mx.y = mn.y;
      Vector3D o = uvec(-2, 2);
      Vector3D d = (k % 4 == 0) ? uvec(-1, 1).unit() : (((mn + mx) * 0.5 + uvec(-0.8, 0.8)) - o).unit();
      if (k % 11 == 3) d.x = 0;           // axis-parallel: inf / NaN slabs
      if (k % 13 == 4) { d.y = 0; o.y = mn.y; }  // 0/0 = NaN
      if (k % 17 == 5) d = -d;
      double min_t = 0, max_t = (k % 3 == 0) ? INF_D : urange(0, 3);
      Ray r(o, d, max_t);
      r.min_t = min_t;
      BBox bb(mn, mx);
      double t0 = -7, t1 = -7;
      bool hit = bb.intersect(r, t0, t1);
      t.row({mn.x, mn.y, mn.z, mx.x, mx.y, mx.z, o.x, o.y, o.z, d.x, d.y, d.z, min_t, max_t, hit ? 1.0 : 0.0, t0, t1});
    }
    t.save();
  }

  // ---- tri: p0 p1 p2 n0 n1 n2 o d max_t -> hit new_max_t hit_p3 n3 ----
  {
    Table t{"tri", 18 + 6 + 1 + 2 + 6};
    HalfedgeMesh empty;
    StaticScene::Mesh mesh(empty, nullptr);  // vertex arrays are re-pointed below
    Vector3D pos[3], nrm[3];
    mesh.positions = pos;
    mesh.normals = nrm;
    for (int k = 0; k < 2048; ++k) {
      for (int i = 0; i < 3; ++i) { pos[i] = uvec(-1, 1); nrm[i] = uvec(-1, 1); }
      if (k % 4 == 0) { pos[1].x = pos[0].x; pos[2].x = pos[0].x; }  // axis-aligned wall triangle
      Vector3D o = uvec(-2, 2);
      Vector3D target = pos[0] * 0.3 + pos[1] * 0.3 + pos[2] * 0.4 + uvec(-0.5, 0.5);
      Vector3D d = (target - o).unit();
      double max_t = (k % 3 == 0) ? INF_D : urange(0, 4);
      Ray r(o, d, max_t);
      Triangle tri(&mesh, 0, 1, 2);
      StaticScene::Intersection is;
      bool hit = tri.intersect(r, &is);
      std::vector<double> row;
      for (int i = 0; i < 3; ++i) { row.push_back(pos[i].x); row.push_back(pos[i].y); row.push_back(pos[i].z); }
      for (int i = 0; i < 3; ++i) { row.push_back(nrm[i].x); row.push_back(nrm[i].y); row.push_back(nrm[i].z); }
      row.insert(row.end(), {o.x, o.y, o.z, d.x, d.y, d.z, max_t, hit ? 1.0 : 0.0, r.max_t});
      if (hit) row.insert(row.end(), {is.hit_p.x, is.hit_p.y, is.hit_p.z, is.n.x, is.n.y, is.n.z});
      else row.insert(row.end(), {0, 0, 0, 0, 0, 0});
      t.row(row);
    }
    t.save();
  }

  // ---- sphere: c3 r o3 d3 max_t -> hit new_max_t hit_p3 n3 ----
  {
    Table t{"sphere", 11 + 2 + 6};
    for (int k = 0; k < 2048; ++k) {
      Vector3D c = uvec(-1, 1);
      double rad = urange(0.05, 0.8);
      Vector3D o = uvec(-2, 2);
      if (k % 5 == 0) o = c + uvec(-0.1, 0.1) * rad;  // inside
      Vector3D d = ((c + uvec(-1, 1) * rad) - o).unit();
      double max_t = (k % 3 == 0) ? INF_D : urange(0, 4);
      StaticScene::SphereObject so(c, rad, nullptr);
      StaticScene::Sphere sp(&so, c, rad);
      Ray r(o, d, max_t);
      StaticScene::Intersection is;
      bool hit = k % 2 ? sp.intersect(r) : sp.intersect(r, &is);
      std::vector<double> row = {c.x, c.y, c.z, rad, o.x, o.y, o.z, d.x, d.y, d.z, max_t, hit ? 1.0 : 0.0, r.max_t};
      if (hit && k % 2 == 0) row.insert(row.end(), {is.hit_p.x, is.hit_p.y, is.hit_p.z, is.n.x, is.n.y, is.n.z});
      else row.insert(row.end(), {0, 0, 0, 0, 0, 0});
      t.row(row);
    }
    t.save();
  }

  // ---- coord: n3 -> o2w columns x3 y3 z3, and w2o * v for a random v ----
  {
    Table t{"coord", 3 + 3 + 9 + 3 + 3};
    for (int k = 0; k < 1024; ++k) {
      Vector3D n = uvec(-1, 1);
      if (k % 6 == 0) n.x = 0;
      if (k % 9 == 0) n = Vector3D(0, 0, (k % 2) ? 1 : -1) * urange(0.5, 2);
      Vector3D v = uvec(-1, 1);
      Matrix3x3 o2w;
      make_coord_space(o2w, n);
      Matrix3x3 w2o = o2w.T();
      Vector3D a = w2o * v, b = o2w * v;
      t.row({n.x, n.y, n.z, v.x, v.y, v.z, o2w[0].x, o2w[0].y, o2w[0].z, o2w[1].x, o2w[1].y, o2w[1].z,
             o2w[2].x, o2w[2].y, o2w[2].z, a.x, a.y, a.z, b.x, b.y, b.z});
    }
    t.save();
  }

  // ---- sampler: kind, rand ints (2) -> sample3, pdf ----
  // kind 0 UniformGridSampler2D (x,y,0), 1 CosineWeighted (+pdf), 2 UniformHemisphere, 3 UniformSphere
  {
    Table t{"sampler", 3 + 4};
    UniformGridSampler2D g; CosineWeightedHemisphereSampler3D cw; UniformHemisphereSampler3D uh; UniformSphereSampler3D us;
    for (int k = 0; k < 4 * 512; ++k) {
      int kind = k % 4;
      std::vector<int> s = {rint31(), rint31()};
      if (k < 16) { s[0] = (k & 1) ? 2147483647 : 0; s[1] = (k & 2) ? 2147483647 : 0; }
      script(s);
      Vector3D out; float pdf = 0;
      if (kind == 0) { Vector2D v = g.get_sample(); out = Vector3D(v.x, v.y, 0); }
      else if (kind == 1) out = cw.get_sample(&pdf);
      else if (kind == 2) out = uh.get_sample();
      else out = us.get_sample();
      if (g_rng.ctr != 2) { std::fprintf(stderr, "sampler draw count\n"); return 6; }
      t.row({(double)kind, (double)s[0], (double)s[1], out.x, out.y, out.z, (double)pdf});
    }
    t.save();
  }

  // ---- bsdf: kind, params[8], wo3, rand ints (3) -> f3 (f(wo,wi) or sample), wi3, pdf, draws ----
  // kind 0 Diffuse, 1 Mirror, 2 Glass, 3 Microfacet, 4 Emission(sample_f)
  {
    Table t{"bsdf", 1 + 8 + 3 + 3 + 3 + 3 + 1 + 1 + 3};
    for (int k = 0; k < 5 * 400; ++k) {
      int kind = k % 5;
      double prm[8];
      for (double& p : prm) p = urange(0.05, 0.95);
      prm[7] = urange(1.1, 2.0);  // ior
      Vector3D wo = uvec(-1, 1).unit();
      if (kind != 2 && wo.z < 0 && (k % 3)) wo.z = -wo.z;
      std::vector<int> s = {rint31(), rint31(), rint31()};
      script(s);
      BSDF* b = nullptr;
      Spectrum sp1((float)prm[0], (float)prm[1], (float)prm[2]), sp2((float)prm[3], (float)prm[4], (float)prm[5]);
      if (kind == 0) b = new DiffuseBSDF(sp1);
      else if (kind == 1) b = new MirrorBSDF(sp1);
      else if (kind == 2) b = new GlassBSDF(sp1, sp2, (float)prm[6], (float)prm[7]);
      else if (kind == 3) b = new MicrofacetBSDF(sp1, sp2, (float)(prm[6] * 0.6));
      else b = new EmissionBSDF(sp1);
      Vector3D wi; float pdf = -1;
      Spectrum f = b->sample_f(wo, &wi, &pdf);
      Spectrum fe = (kind == 3 && pdf != 0) ? b->f(wo, wi) : Spectrum();
      t.row({(double)kind, prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], wo.x, wo.y, wo.z,
             (double)s[0], (double)s[1], (double)s[2], f.r, f.g, f.b, wi.x, wi.y, wi.z, (double)pdf, (double)g_rng.ctr,
             fe.r, fe.g, fe.b});
      delete b;
    }
    t.save();
  }

  // ---- area: rad3 pos3 dir3 dimx3 dimy3 p3 rand ints(2) -> L3 wi3 dist pdf ----
  {
    Table t{"area", 3 + 12 + 3 + 2 + 3 + 3 + 2};
    for (int k = 0; k < 1024; ++k) {
      Vector3D pos = uvec(-1, 1), dir = uvec(-1, 1).unit(), dx = uvec(-0.5, 0.5), dy = uvec(-0.5, 0.5);
      if (k % 2 == 0) { pos = Vector3D(0, 1.49, 0); dir = Vector3D(0, -1, 0); dx = Vector3D(0.47, 0, 0); dy = Vector3D(0, 0, 0.38); }
      Spectrum rad((float)urange(0, 20), (float)urange(0, 20), (float)urange(0, 20));
      Vector3D p = uvec(-1, 1);
      StaticScene::AreaLight al(rad, pos, dir, dx, dy);
      std::vector<int> s = {rint31(), rint31()};
      script(s);
      Vector3D wi; float dist = -1, pdf = -1;
      Spectrum L = al.sample_L(p, &wi, &dist, &pdf);
      t.row({rad.r, rad.g, rad.b, pos.x, pos.y, pos.z, dir.x, dir.y, dir.z, dx.x, dx.y, dx.z, dy.x, dy.y, dy.z,
             p.x, p.y, p.z, (double)s[0], (double)s[1], L.r, L.g, L.b, wi.x, wi.y, wi.z, (double)dist, (double)pdf});
    }
    t.save();
  }

  // ---- camray: hFov vFov pos3 c2w(9, column vectors) nClip fClip x y -> o3 d3 min_t max_t ----
  {
    Table t{"camray", 2 + 3 + 9 + 2 + 2 + 8};
    for (int k = 0; k < 512; ++k) {
      Camera cam;
      cam.hFov = urange(20, 100); cam.vFov = urange(15, 80);
      cam.pos = uvec(-5, 5);
      Vector3D dir = uvec(-1, 1).unit();
      cam.c2w[2] = dir;
      cam.c2w[0] = cross(Vector3D(0, 1, 0), dir).unit();
      cam.c2w[1] = cross(dir, cam.c2w[0]).unit();
      cam.nClip = 0.1; cam.fClip = 100;
      double x = u01(), y = u01();
      Ray r = cam.generate_ray(x, y);
      t.row({cam.hFov, cam.vFov, cam.pos.x, cam.pos.y, cam.pos.z,
             cam.c2w[0].x, cam.c2w[0].y, cam.c2w[0].z, cam.c2w[1].x, cam.c2w[1].y, cam.c2w[1].z,
             cam.c2w[2].x, cam.c2w[2].y, cam.c2w[2].z, cam.nClip, cam.fClip, x, y,
             r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, r.min_t, r.max_t});
    }
    t.save();
  }

  // ---- light: the other lights' sample_L (light.cpp:17-23 directional, :34-42 infinite
  // hemisphere, :49-57 point), scripted draws.  row: kind (1 point, 2 directional, 3 hemisphere),
  // rad3, ctor argument3 (point position / directional lightDir; unused for the hemisphere),
  // the light's own vector (PointLight::position / DirectionalLight::dirToLight), p3,
  // rand ints(2) -> L3 wi3 dist pdf draws
  {
    Table t{"light", 1 + 3 + 3 + 3 + 3 + 2 + 3 + 3 + 3};
    for (int k = 0; k < 768; ++k) {
      const int kind = 1 + k % 3;
      Spectrum rad((float)urange(0, 5), (float)urange(0, 5), (float)urange(0, 5));
      Vector3D arg = uvec(-2, 2), p = uvec(-1, 1);
      if (k % 24 == 2) arg = Vector3D(0, -1, 0);  // straight down, as the scenes' sun
      std::vector<int> s = {rint31(), rint31()};
      if (k % 48 == 5) s = {0, 0};
      if (k % 48 == 8) s = {2147483647, 2147483647};
      script(s);
      Vector3D wi, own;
      float dist = -1, pdf = -1;
      Spectrum L;
      if (kind == 1) {
        StaticScene::PointLight l(rad, arg);
        own = l.position;
        L = l.sample_L(p, &wi, &dist, &pdf);
      } else if (kind == 2) {
        StaticScene::DirectionalLight l(rad, arg);
        own = l.dirToLight;
        L = l.sample_L(p, &wi, &dist, &pdf);
      } else {
        StaticScene::InfiniteHemisphereLight l(rad);
        L = l.sample_L(p, &wi, &dist, &pdf);
      }
      t.row({(double)kind, rad.r, rad.g, rad.b, arg.x, arg.y, arg.z, own.x, own.y, own.z, p.x, p.y, p.z,
             (double)s[0], (double)s[1], L.r, L.g, L.b, wi.x, wi.y, wi.z, (double)dist, (double)pdf,
             (double)g_rng.ctr});
    }
    t.save();
  }
  return 0;
}
