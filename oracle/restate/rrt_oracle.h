/* rrt_oracle.h -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * It is the checker (and the timed CPU baseline), never the product: the product path
 * (include/rrt.h, relativistic-ray-tracer_amd/) has no dependency on it.
 *
 * Pinned against the reference itself: tests/golden/ holds known-answer vectors and per-pixel
 * outputs produced by the compiled reference (oracle/ref, tests/golden/make_golden.py), and
 * tests/test_oracle_*.py require this restatement to reproduce them bit for bit.
 */
#ifndef RRT_ORACLE_H
#define RRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double x, y, z; } ov3;

typedef struct ro_scene ro_scene;

/* Load a .rrts scene file (include/rrt_scene_format.h) and build the reference BVH
 * (bvh.cpp:49-96, max_leaf_size 4).  Returns NULL and fills err on failure. */
ro_scene* ro_scene_load(const char* path, char* err, int errlen);
void ro_scene_free(ro_scene* s);
int ro_scene_num_prims(const ro_scene* s);
int ro_scene_num_nodes(const ro_scene* s);
/* BVH in left-first pre-order: boxes [n][6] (min, max), nodes [n][4] (first, count, left,
 * right), prims [n_prims] (build-order primitive ids) -- same layout as the oracle dump. */
void ro_scene_bvh(const ro_scene* s, double* boxes, int32_t* nodes, uint32_t* prims);
/* Attach an environment map ([h][w][3] RGB, HDRImageBuffer layout): EnvironmentLight::init's
 * tables, and the light appended after the scene's lights (pathtracer.cpp:61-63, 106-108). */
int ro_scene_set_envmap(ro_scene* s, uint32_t w, uint32_t h, const float* texels);

typedef struct {
  double hFov, vFov, nClip, fClip;
  double pos[3];
  double c2w[9];  /* row-major c2w(i, j) as in the .rrtc record */
  double lensRadius, focalDistance;
} ro_camera;
int ro_camera_load(const char* path, ro_camera* cam, char* err, int errlen);

typedef struct {
  uint32_t ns_aa, max_ray_depth, ns_area_light, samples_per_batch;
  float max_tolerance;
  uint32_t direct_hemisphere;
  uint64_t seed;
  uint32_t frame_w, frame_h;
  double bh_center[3], bh_radius, bh_dtheta;  /* global_black_hole, blackhole.cpp:5 */
  /* Kerr (build-defined, no reference -- parity of the GPU against this restatement is the
   * build's own; physics pinned by tests/test_kerr_oracle.py): bh_kind 1 = Kerr, spin = a/M */
  uint32_t bh_kind, pad_;
  double bh_spin, bh_axis[3];
  /* the reference's compile-time switches, defaults as the reference build (pathtracer.h:4-6,
   * environment_light.h:4, bsdf.h:4) */
  uint32_t illum, adaptive, thin_lens, env_hemi, microfacet_hemi, pad2_;
} ro_params;
void ro_params_default(ro_params* p);

/* Render region [x0,x0+w) x [y0,y0+h) of the frame (y = 0 at the bottom, sampleBuffer rows).
 * Outputs are row-major over the region.  draws / counters may be NULL.
 * counters (per pixel): [0] AABB tests, [1] micro steps, [2] primitive tests, [3] queries.
 * Threads pull 32x32 tiles from a shared counter (pathtracer.cpp:251-255, 611-625). */
int ro_render(const ro_scene* s, const ro_camera* cam, const ro_params* p, uint32_t x0, uint32_t y0,
              uint32_t w, uint32_t h, float* rgb, int32_t* count, uint32_t* draws, uint32_t* counters,
              int nthreads);

/* ---- function-level entry points for the known-answer tests ---- */
/* keyed RNG (oracle/ref/harness_common.h) */
uint64_t ro_pixel_key(uint64_t seed, uint32_t x, uint32_t y);
int ro_keyed_rand(uint64_t key, uint32_t n);
/* next_micro_ray chain: writes per step (o3, d3, max_t, captured) until capture or n_steps */
int ro_micro_chain(const double* bh /*cx,cy,cz,r,dtheta*/, const double* o, const double* d, double* out, int max_rows);
/* Kerr geodesic chain: bh = cx,cy,cz,r_s,dtheta,spin,ax,ay,az.  Writes per step
 * (segment start o3, unit d3, max_t, captured, q3 local position, p3 local momentum) = 14 doubles,
 * until capture or max_rows steps (not capped at the renderer's ceil(2 pi / dtheta)); returns the
 * number of rows.  frame (9, may be NULL): ex, ey, ez. */
int ro_kerr_chain_st(const double* bh, const double* o, const double* d, double* out, int max_rows, double* frame,
                     double st, double* extra);
int ro_shadow_query(const ro_scene* s, const ro_params* p, const double* o, const double* d);
int ro_query(const ro_scene* s, const ro_params* p, const double* o, const double* d, double* out /*7*/);
int ro_kerr_chain(const double* bh, const double* o, const double* d, double* out, int max_rows, double* frame);
int ro_bbox_intersect(const double* mn, const double* mx, const double* o, const double* d, double min_t,
                      double max_t, double* t0, double* t1);
int ro_tri_intersect(const double* p /*9*/, const double* n /*9*/, const double* o, const double* d,
                     double* max_t, double* hit_p, double* nrm);
int ro_sphere_intersect(const double* c, double r, const double* o, const double* d, double* max_t,
                        double* hit_p, double* nrm, int want_isect);
void ro_coord_space(const double* n, const double* v, double* o2w /*9: cols x,y,z*/, double* w2o_v, double* o2w_v);
/* sampler kinds: 0 grid2D, 1 cosine hemisphere, 2 uniform hemisphere, 3 uniform sphere */
void ro_sampler(int kind, const int* rands, double* out3, float* pdf, int* used);
/* bsdf kinds: 0 Diffuse, 1 Mirror, 2 Glass, 3 Microfacet, 4 Emission */
void ro_bsdf_sample(int kind, const double* prm /*8*/, const double* wo, const int* rands, float* f3,
                    double* wi, float* pdf, int* used, float* feval3);
void ro_area_sample(const float* rad, const double* v /*12*/, const double* p, const int* rands, float* L,
                    double* wi, float* dist, float* pdf);
/* light types 1 point, 2 directional, 3 infinite hemisphere (v: the light's 4 vectors) */
void ro_light_sample(int type, const float* rad, const double* v /*12*/, const double* p, const int* rands, float* L,
                     double* wi, float* dist, float* pdf, int* used);
void ro_camera_ray(double hFov, double vFov, const double* pos, const double* c2w_cols /*9*/, double nClip,
                   double fClip, double x, double y, double* o, double* d, double* min_t, double* max_t);

#ifdef __cplusplus
}
#endif
/* the host C library's sin/cos/acos/atan2/sinf/cosf on n arguments (checker for rrt_libm_eval) */
void ro_libm_eval(int fn, const double* a, const double* b, double* out, long n);

#endif
