/* rrt_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * A line-by-line restatement, in C99, of what the reference computes per pixel
 * (part1_code.cpp:15-187, bvh.cpp:49-138, blackhole.cpp:13-40, bbox.cpp:10-25,
 * triangle.cpp:25-55, sphere.cpp:10-53, bsdf.cpp:13-171, bsdf.h:20-191, sampler.cpp:7-56,
 * light.cpp:11-92, CGL vector3D.h / spectrum.h / matrix3x3.cpp), keeping the reference's
 * types (double geometry, float Spectrum), operation order and float narrowing points so that
 * results are bit-identical with the compiled reference (x86-64 SSE2, no FMA: build with
 * -ffp-contract=off).  The only behavioural change is the RNG: glibc rand() is replaced by the
 * keyed per-pixel generator of oracle/ref/harness_common.h, exactly as in the oracle harness.
 *
 * Pinned by tests/test_oracle_*.py against tests/golden/ (reference-generated).
 * Used by: tests/ (checker), __graft_entry__.smoke() (checker), bench.py (cpu_baseline).
 */
#include "rrt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define PI_D 3.14159265358979323   /* CGL misc.h:11 */
#define EPS_D 0.00000000001        /* CGL misc.h:12 */
#define RAND_MAX_D 2147483647.0    /* glibc RAND_MAX */

/* ------------------------------------------------------------------ Vector3D (vector3D.h) */
typedef ov3 v3;
static inline v3 V(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline v3 vmul(v3 a, double c) { return V(a.x * c, a.y * c, a.z * c); }   /* v * c */
static inline v3 smul(double c, v3 a) { return V(c * a.x, c * a.y, c * a.z); }   /* c * v */
static inline double vdot(v3 u, v3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
static inline v3 vcross(v3 u, v3 v) {
  return V(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline double vnorm(v3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static inline double vnorm2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline v3 vunit(v3 a) {
  double r = 1. / sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return V(r * a.x, r * a.y, r * a.z);
}
static inline v3 vnormalize(v3 a) { /* (*this) /= norm()  ->  *= (1./c) */
  double c = 1. / vnorm(a);
  return V(a.x * c, a.y * c, a.z * c);
}
static inline v3 vdivd(v3 a, double c) { /* operator/(c): rc = 1.0/c; rc * x */
  double rc = 1.0 / c;
  return V(rc * a.x, rc * a.y, rc * a.z);
}
static inline double std_min(double a, double b) { return (b < a) ? b : a; }
static inline double std_max(double a, double b) { return (a < b) ? b : a; }

/* ------------------------------------------------------------------ Spectrum (spectrum.h) */
typedef struct { float r, g, b; } spec;
static inline spec S(float r, float g, float b) { spec s = {r, g, b}; return s; }
static inline spec sadd(spec a, spec b) { return S(a.r + b.r, a.g + b.g, a.b + b.b); }
static inline spec ssub(spec a, spec b) { return S(a.r - b.r, a.g - b.g, a.b - b.b); }
static inline spec smulS(spec a, spec b) { return S(a.r * b.r, a.g * b.g, a.b * b.b); }
static inline spec sdivS(spec a, spec b) { return S(a.r / b.r, a.g / b.g, a.b / b.b); }
static inline spec smulf(spec a, float s) { return S(a.r * s, a.g * s, a.b * s); }
static inline spec sdivf(spec a, float s) { return S(a.r / s, a.g / s, a.b / s); }
static inline spec saddf(spec a, float s) { return S(a.r + s, a.g + s, a.b + s); }
static inline float illum(spec s) { return 0.2126f * s.r + 0.7152f * s.g + 0.0722f * s.b; }

/* ------------------------------------------------------------------ keyed RNG */
static inline uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27; z *= 0x94D049BB133111EBULL;
  z ^= z >> 31; return z;
}
uint64_t ro_pixel_key(uint64_t seed, uint32_t x, uint32_t y) {
  return mix64((((uint64_t)y << 32) | (uint64_t)x) ^ mix64(seed + 0x9E3779B97F4A7C15ULL));
}
int ro_keyed_rand(uint64_t key, uint32_t n) {
  return (int)(mix64(key + (uint64_t)(n + 1) * 0x9E3779B97F4A7C15ULL) >> 33);
}

typedef struct {
  uint64_t key;
  uint32_t ctr;
  const int* script; /* function tests: scripted draws */
  int script_len;
  /* work counters (reference algorithm) */
  uint64_t bbox_tests, micro_steps, prim_tests, queries;
} rng_t;

static inline int next_rand(rng_t* g) {
  if (g->script) {
    if ((int)g->ctr >= g->script_len) { fprintf(stderr, "rrt_oracle: script exhausted\n"); abort(); }
    return g->script[g->ctr++];
  }
  return ro_keyed_rand(g->key, g->ctr++);
}
/* random_util.h:11-20 */
static inline double random_uniform(rng_t* g) { return ((double)next_rand(g)) / RAND_MAX_D; }
static inline int coin_flip(rng_t* g, double p) { return random_uniform(g) < p; }
/* UniformGridSampler2D::get_sample (sampler.cpp:7-11): Vector2D(random_uniform(),
 * random_uniform()) -- g++ evaluates the arguments right to left: y draws first. */
static inline void grid_sample(rng_t* g, double* x, double* y) {
  *y = random_uniform(g);
  *x = random_uniform(g);
}
/* CosineWeightedHemisphereSampler3D::get_sample(float*) (sampler.cpp:47-56) */
static inline v3 cosine_sample(rng_t* g, float* pdf) {
  double Xi1 = random_uniform(g);
  double Xi2 = random_uniform(g);
  double r = sqrt(Xi1);
  double theta = 2. * PI_D * Xi2;
  *pdf = (float)(sqrt(1 - Xi1) / PI_D);
  return V(r * cos(theta), r * sin(theta), sqrt(1 - Xi1));
}
/* UniformHemisphereSampler3D::get_sample (sampler.cpp:15-29): float trig */
static inline v3 hemisphere_sample(rng_t* g) {
  double Xi1 = random_uniform(g);
  double Xi2 = random_uniform(g);
  double theta = acos(Xi1);
  double phi = 2.0 * PI_D * Xi2;
  double xs = sinf((float)theta) * cosf((float)phi);
  double ys = sinf((float)theta) * sinf((float)phi);
  double zs = cosf((float)theta);
  return V(xs, ys, zs);
}
/* UniformSphereSampler3D::get_sample (sampler.cpp:33-40) */
static inline v3 sphere_sample(rng_t* g) {
  double z = random_uniform(g) * 2 - 1;
  double sinTheta = sqrt(std_max(0.0, 1.0f - z * z));
  double phi = 2.0f * PI_D * random_uniform(g);
  return V(cos(phi) * sinTheta, sin(phi) * sinTheta, z);
}

/* ------------------------------------------------------------------ scene */
enum { BSDF_DIFFUSE = 0, BSDF_EMISSION = 1, BSDF_MIRROR = 2, BSDF_GLASS = 3, BSDF_MICROFACET = 4,
       BSDF_REFRACTION = 5 };
typedef struct { uint32_t type; float p[14]; } bsdf_t;
typedef struct { uint32_t kind, bsdf, v0, v1, v2; v3 c; double r, r2; } prim_t;
typedef struct { uint32_t type, is_delta; float rad[3]; float area; v3 v[4]; } light_t;
typedef struct { v3 mn, mx; int32_t first, count, left, right; } node_t;

struct ro_scene {
  v3* pos; v3* nrm; uint32_t nverts;
  prim_t* prims; uint32_t nprims;
  bsdf_t* bsdfs; uint32_t nbsdfs;
  light_t* lights; uint32_t nlights;
  /* environment map (ro_scene_set_envmap): texels + EnvironmentLight::init tables */
  uint32_t env_w, env_h;
  float* env_tex; double* env_pdf; double* env_conds; double* env_marg;
  node_t* nodes; uint32_t nnodes, cap_nodes;
  uint32_t* leaf; uint32_t nleaf;
};

/* BBox helpers (bbox.h) */
typedef struct { v3 mx, mn, ext; } bbox_t;
static inline bbox_t bb_empty(void) {
  bbox_t b; b.mx = V(-INFINITY, -INFINITY, -INFINITY); b.mn = V(INFINITY, INFINITY, INFINITY);
  b.ext = vsub(b.mx, b.mn); return b;
}
static inline bbox_t bb_point(v3 p) { bbox_t b; b.mn = p; b.mx = p; b.ext = vsub(b.mx, b.mn); return b; }
static inline void bb_expand_pt(bbox_t* b, v3 p) {
  b->mn.x = std_min(b->mn.x, p.x); b->mn.y = std_min(b->mn.y, p.y); b->mn.z = std_min(b->mn.z, p.z);
  b->mx.x = std_max(b->mx.x, p.x); b->mx.y = std_max(b->mx.y, p.y); b->mx.z = std_max(b->mx.z, p.z);
  b->ext = vsub(b->mx, b->mn);
}
static inline void bb_expand(bbox_t* b, const bbox_t* o) {
  b->mn.x = std_min(b->mn.x, o->mn.x); b->mn.y = std_min(b->mn.y, o->mn.y); b->mn.z = std_min(b->mn.z, o->mn.z);
  b->mx.x = std_max(b->mx.x, o->mx.x); b->mx.y = std_max(b->mx.y, o->mx.y); b->mx.z = std_max(b->mx.z, o->mx.z);
  b->ext = vsub(b->mx, b->mn);
}
static inline v3 bb_centroid(const bbox_t* b) { return vdivd(vadd(b->mn, b->mx), 2); }
static bbox_t prim_bbox(const ro_scene* s, const prim_t* p) {
  if (p->kind == 0) { /* Triangle::get_bbox, triangle.cpp:11-19 */
    bbox_t b = bb_point(s->pos[p->v0]);
    bb_expand_pt(&b, s->pos[p->v1]);
    bb_expand_pt(&b, s->pos[p->v2]);
    return b;
  }
  bbox_t b; /* Sphere::get_bbox, sphere.h:30-32 */
  b.mn = vsub(p->c, V(p->r, p->r, p->r)); b.mx = vadd(p->c, V(p->r, p->r, p->r)); b.ext = vsub(b.mx, b.mn);
  return b;
}

/* BVHAccel::construct_bvh (bvh.cpp:49-96), flattened left-first pre-order */
static int build_node(ro_scene* s, const uint32_t* ids, uint32_t n, uint32_t* scratch) {
  bbox_t bb = bb_empty();
  for (uint32_t i = 0; i < n; ++i) { bbox_t pb = prim_bbox(s, &s->prims[ids[i]]); bb_expand(&bb, &pb); }
  if (s->nnodes == s->cap_nodes) {
    s->cap_nodes = s->cap_nodes ? 2 * s->cap_nodes : 64;
    s->nodes = (node_t*)realloc(s->nodes, s->cap_nodes * sizeof(node_t));
  }
  int id = (int)s->nnodes++;
  s->nodes[id].mn = bb.mn; s->nodes[id].mx = bb.mx;
  s->nodes[id].left = s->nodes[id].right = -1;
  if (n <= 4) {
    s->nodes[id].first = (int32_t)s->nleaf; s->nodes[id].count = (int32_t)n;
    for (uint32_t i = 0; i < n; ++i) s->leaf[s->nleaf++] = ids[i];
    return id;
  }
  s->nodes[id].first = 0; s->nodes[id].count = 0;
  uint32_t* L = scratch; uint32_t* R = scratch + n; uint32_t nl = 0, nr = 0;
  int axis = (bb.ext.x > bb.ext.y && bb.ext.x > bb.ext.z) ? 0 : (bb.ext.y > bb.ext.x && bb.ext.y > bb.ext.z) ? 1 : 2;
  v3 cc = bb_centroid(&bb);
  double c = axis == 0 ? cc.x : axis == 1 ? cc.y : cc.z;
  for (uint32_t i = 0; i < n; ++i) {
    bbox_t pb = prim_bbox(s, &s->prims[ids[i]]);
    v3 pc = bb_centroid(&pb);
    double v = axis == 0 ? pc.x : axis == 1 ? pc.y : pc.z;
    if (v < c) L[nl++] = ids[i]; else R[nr++] = ids[i];
  }
  if (nl == 0 || nr == 0) {
    nl = nr = 0;
    for (uint32_t i = 0; i < n / 2; ++i) L[nl++] = ids[i];
    for (uint32_t i = n / 2; i < n; ++i) R[nr++] = ids[i];
  }
  /* children need their own copies: the scratch below this level is reused */
  uint32_t* lc = (uint32_t*)malloc((size_t)(nl + nr) * sizeof(uint32_t));
  memcpy(lc, L, nl * sizeof(uint32_t)); memcpy(lc + nl, R, nr * sizeof(uint32_t));
  int l = build_node(s, lc, nl, scratch);
  int r = build_node(s, lc + nl, nr, scratch);
  free(lc);
  s->nodes[id].left = l; s->nodes[id].right = r;
  return id;
}

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

ro_scene* ro_scene_load(const char* path, char* err, int errlen) {
  FILE* f = fopen(path, "rb");
  if (!f) { snprintf(err, errlen, "cannot open %s", path); return NULL; }
  char magic[8]; uint32_t hdr[4];
  if (!rd(f, magic, 8) || memcmp(magic, "RRTSCN1", 8) != 0 || !rd(f, hdr, 16)) {
    snprintf(err, errlen, "bad scene header"); fclose(f); return NULL;
  }
  ro_scene* s = (ro_scene*)calloc(1, sizeof(ro_scene));
  s->nbsdfs = hdr[0]; s->nlights = hdr[2];
  uint32_t nobj = hdr[1];
  s->bsdfs = (bsdf_t*)calloc(s->nbsdfs ? s->nbsdfs : 1, sizeof(bsdf_t));
  for (uint32_t i = 0; i < s->nbsdfs; ++i) {
    uint32_t tp[2];
    if (!rd(f, tp, 8) || !rd(f, s->bsdfs[i].p, 56)) goto bad;
    s->bsdfs[i].type = tp[0];
  }
  for (uint32_t o = 0; o < nobj; ++o) {
    uint32_t oh[4];
    if (!rd(f, oh, 16)) goto bad;
    if (oh[0] == 0) {
      uint32_t nv = oh[2], nt = oh[3], base = s->nverts;
      s->pos = (v3*)realloc(s->pos, (size_t)(base + nv) * sizeof(v3));
      s->nrm = (v3*)realloc(s->nrm, (size_t)(base + nv) * sizeof(v3));
      if (!rd(f, s->pos + base, (size_t)nv * 24) || !rd(f, s->nrm + base, (size_t)nv * 24)) goto bad;
      s->nverts += nv;
      s->prims = (prim_t*)realloc(s->prims, (size_t)(s->nprims + nt) * sizeof(prim_t));
      for (uint32_t t = 0; t < nt; ++t) {
        uint32_t idx[3];
        if (!rd(f, idx, 12)) goto bad;
        prim_t* p = &s->prims[s->nprims++];
        memset(p, 0, sizeof(*p));
        p->kind = 0; p->bsdf = oh[1]; p->v0 = base + idx[0]; p->v1 = base + idx[1]; p->v2 = base + idx[2];
      }
    } else if (oh[0] == 1) {
      double sp[4];
      if (!rd(f, sp, 32)) goto bad;
      s->prims = (prim_t*)realloc(s->prims, (size_t)(s->nprims + 1) * sizeof(prim_t));
      prim_t* p = &s->prims[s->nprims++];
      memset(p, 0, sizeof(*p));
      p->kind = 1; p->bsdf = oh[1]; p->c = V(sp[0], sp[1], sp[2]); p->r = sp[3]; p->r2 = sp[3] * sp[3];
    } else goto bad;
  }
  s->lights = (light_t*)calloc(s->nlights ? s->nlights : 1, sizeof(light_t));
  for (uint32_t i = 0; i < s->nlights; ++i) {
    uint32_t th[2]; float fv[4]; double dv[12];
    if (!rd(f, th, 8) || !rd(f, fv, 16) || !rd(f, dv, 96)) goto bad;
    light_t* l = &s->lights[i];
    l->type = th[0]; l->is_delta = th[1];
    l->rad[0] = fv[0]; l->rad[1] = fv[1]; l->rad[2] = fv[2]; l->area = fv[3];
    for (int k = 0; k < 4; ++k) l->v[k] = V(dv[3 * k], dv[3 * k + 1], dv[3 * k + 2]);
    if (l->type > 3) { snprintf(err, errlen, "light type %u not supported by the restatement", l->type); goto fail; }
  }
  fclose(f);
  {
    uint32_t n = s->nprims;
    uint32_t* ids = (uint32_t*)malloc((size_t)(n ? n : 1) * sizeof(uint32_t));
    uint32_t* scratch = (uint32_t*)malloc((size_t)(2 * n + 2) * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; ++i) ids[i] = i;
    s->leaf = (uint32_t*)malloc((size_t)(n ? n : 1) * sizeof(uint32_t));
    build_node(s, ids, n, scratch);
    free(ids); free(scratch);
  }
  return s;
bad:
  snprintf(err, errlen, "truncated or malformed scene file");
fail:
  fclose(f);
  ro_scene_free(s);
  return NULL;
}

void ro_scene_free(ro_scene* s) {
  if (!s) return;
  free(s->pos); free(s->nrm); free(s->prims); free(s->bsdfs); free(s->lights); free(s->nodes); free(s->leaf);
  free(s->env_tex); free(s->env_pdf); free(s->env_conds); free(s->env_marg);
  free(s);
}
int ro_scene_num_prims(const ro_scene* s) { return (int)s->nprims; }
int ro_scene_num_nodes(const ro_scene* s) { return (int)s->nnodes; }
void ro_scene_bvh(const ro_scene* s, double* boxes, int32_t* nodes, uint32_t* prims) {
  for (uint32_t i = 0; i < s->nnodes; ++i) {
    const node_t* n = &s->nodes[i];
    double b[6] = {n->mn.x, n->mn.y, n->mn.z, n->mx.x, n->mx.y, n->mx.z};
    memcpy(boxes + 6 * i, b, sizeof(b));
    nodes[4 * i] = n->first; nodes[4 * i + 1] = n->count; nodes[4 * i + 2] = n->left; nodes[4 * i + 3] = n->right;
  }
  memcpy(prims, s->leaf, s->nleaf * sizeof(uint32_t));
}

int ro_camera_load(const char* path, ro_camera* cam, char* err, int errlen) {
  FILE* f = fopen(path, "rb");
  if (!f) { snprintf(err, errlen, "cannot open %s", path); return -1; }
  char magic[8]; double d[30];
  int ok = rd(f, magic, 8) && memcmp(magic, "RRTCAM1", 8) == 0 && rd(f, d, sizeof(d));
  fclose(f);
  if (!ok) { snprintf(err, errlen, "bad camera file"); return -1; }
  cam->hFov = d[0]; cam->vFov = d[1]; cam->nClip = d[3]; cam->fClip = d[4];
  cam->pos[0] = d[5]; cam->pos[1] = d[6]; cam->pos[2] = d[7];
  memcpy(cam->c2w, d + 16, 9 * sizeof(double));
  cam->focalDistance = d[28]; cam->lensRadius = d[29];
  return 0;
}

void ro_params_default(ro_params* p) {
  memset(p, 0, sizeof(*p));
  p->ns_aa = 1; p->max_ray_depth = 1; p->ns_area_light = 1; p->samples_per_batch = 32;
  p->max_tolerance = 0.05f; p->direct_hemisphere = 0; p->seed = 0;
  p->bh_center[0] = 0; p->bh_center[1] = 1; p->bh_center[2] = 0; p->bh_radius = 0.1; p->bh_dtheta = 0.1;
  p->illum = 2; p->adaptive = 1; p->thin_lens = 0; p->env_hemi = 0; p->microfacet_hemi = 0;  /* ILLUM, ADAPTIVE, ... */
}

/* ------------------------------------------------------------------ rays & geometry */
typedef struct { v3 o, d; double min_t, max_t; } ray_t;
typedef struct { v3 hit_p, w_out, n; int bsdf; } isect_t;
typedef struct {
  v3 c; double r, r2, dt, cos_dt, sin_dt; int steps;
  int kerr; double m, a, a2, r_hor; v3 ex, ey, ez;  /* Kerr (build-defined) */
  double r_esc2; int kerr_max_steps;
} hole_t;

static void hole_init(hole_t* h, const double* c, double r, double dt) {
  h->c = V(c[0], c[1], c[2]); h->r = r; h->r2 = r * r; h->dt = dt;
  h->cos_dt = cos(dt); h->sin_dt = sin(dt);
  int j = 0;
  while (j * dt < 2 * PI_D) ++j; /* bvh.cpp:105 */
  h->steps = j;
  h->kerr = 0;
}

/* Kerr local frame: ez = unit(axis); ex = unit(t x ez), t the world axis least aligned with ez
 * (z, or x when |ez.z| >= 0.9); ey = ez x ex.  (Restates rrt_kerr_frame, include/rrt.h.) */
static void kerr_frame(const double* axis, v3* ex, v3* ey, v3* ez) {
  const double n = sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
  v3 z = V(axis[0] / n, axis[1] / n, axis[2] / n);
  v3 t = V(0, 0, 1);
  if (fabs(z.z) >= 0.9) t = V(1, 0, 0);
  v3 x = V(t.y * z.z - t.z * z.y, t.z * z.x - t.x * z.z, t.x * z.y - t.y * z.x);
  const double xn = sqrt(x.x * x.x + x.y * x.y + x.z * x.z);
  x = V(x.x / xn, x.y / xn, x.z / xn);
  *ez = z; *ex = x;
  *ey = V(z.y * x.z - z.z * x.y, z.z * x.x - z.x * x.z, z.x * x.y - z.y * x.x);
}

static void hole_init_kerr(hole_t* h, const double* c, double r_s, double dt, double spin, const double* axis) {
  hole_init(h, c, r_s, dt);
  h->kerr = 1;
  double ax[3] = {axis[0], axis[1], axis[2]};
  if (ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2] == 0) { ax[0] = 0; ax[1] = 1; ax[2] = 0; }
  kerr_frame(ax, &h->ex, &h->ey, &h->ez);
  h->m = 0.5 * r_s;
  h->a = spin * h->m;
  h->a2 = h->a * h->a;
  h->r_hor = h->m + sqrt(h->m * h->m - h->a2);
  h->r_esc2 = INFINITY;  /* set from the scene's root box by kerr_set_escape */
  h->kerr_max_steps = 4 * h->steps;
}
/* escape radius: the farthest root-box corner from the hole, at least 4M (photon orbits) */
static void kerr_set_escape(hole_t* h, v3 lo, v3 hi) {
  const double l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z}, c3[3] = {h->c.x, h->c.y, h->c.z};
  double m3[3];
  for (int k = 0; k < 3; ++k) {
    const double dl = fabs(l3[k] - c3[k]), dh = fabs(h3[k] - c3[k]);
    m3[k] = dl > dh ? dl : dh;
  }
  const double e2 = (m3[0] * m3[0] + m3[1] * m3[1]) + m3[2] * m3[2], f2 = (4.0 * h->m) * (4.0 * h->m);
  h->r_esc2 = e2 > f2 ? e2 : f2;
}

/* BBox::intersect (bbox.cpp:10-25) */
static inline int bbox_hit(v3 mn, v3 mx, const ray_t* r, double* t0, double* t1) {
  double tx0 = (mn.x - r->o.x) / r->d.x, tx1 = (mx.x - r->o.x) / r->d.x,
         ty0 = (mn.y - r->o.y) / r->d.y, ty1 = (mx.y - r->o.y) / r->d.y,
         tz0 = (mn.z - r->o.z) / r->d.z, tz1 = (mx.z - r->o.z) / r->d.z,
         tmin = std_max(std_max(std_min(tx0, tx1), std_min(ty0, ty1)), std_min(tz0, tz1)),
         tmax = std_min(std_min(std_max(tx0, tx1), std_max(ty0, ty1)), std_max(tz0, tz1));
  int ret = tmin <= tmax && tmin <= r->max_t && tmax >= r->min_t;
  if (ret) { *t0 = tmin; *t1 = tmax; }
  return ret;
}

/* Sphere::test / intersect (sphere.cpp:10-53); mutates r->max_t like the reference */
static inline int sphere_hit(v3 c, double r2, ray_t* r, isect_t* is, int bsdf) {
  v3 tmp = vsub(r->o, c);
  double b = 2 * vdot(tmp, r->d), cc = vnorm2(tmp) - r2, d = b * b - 4 * cc;
  if (d < 0) return 0;
  double t1 = (-b - sqrt(d)) / 2, t2 = (-b + sqrt(d)) / 2, t;
  if (r->min_t <= t1 && t1 <= r->max_t) t = t1;
  else if (r->min_t <= t2 && t2 <= r->max_t) t = t2;
  else return 0;
  r->max_t = t;
  if (is) {
    is->hit_p = vadd(r->o, vmul(r->d, t));
    is->w_out = vneg(r->d);
    is->n = vunit(vsub(vadd(r->o, vmul(r->d, t)), c));
    is->bsdf = bsdf;
  }
  return 1;
}

/* Triangle::intersect (triangle.cpp:25-55) */
static inline int tri_hit(v3 p0, v3 p1, v3 p2, v3 n0, v3 n1, v3 n2, ray_t* r, isect_t* is, int bsdf) {
  v3 e1 = vsub(p1, p0), e2 = vsub(p2, p0), s = vsub(r->o, p0), s1 = vcross(r->d, e2), s2 = vcross(s, e1);
  v3 res = V(vdot(s2, e2), vdot(s1, s), vdot(s2, r->d));
  double inv = 1. / vdot(s1, e1);
  res = V(res.x * inv, res.y * inv, res.z * inv);
  double t = res.x, b1 = res.y, b2 = res.z, b0 = 1 - b1 - b2;
  int ret = r->min_t <= t && t <= r->max_t && b0 >= 0 && b1 >= 0 && b2 >= 0;
  if (ret) {
    r->max_t = t;
    if (is) {
      is->hit_p = vadd(r->o, vmul(r->d, t));
      is->w_out = vneg(r->d);
      is->n = vadd(vadd(smul(b0, n0), smul(b1, n1)), smul(b2, n2));
      is->bsdf = bsdf;
    }
  }
  return ret;
}

static inline int prim_hit(const ro_scene* s, const prim_t* p, ray_t* r, isect_t* is) {
  if (p->kind == 0)
    return tri_hit(s->pos[p->v0], s->pos[p->v1], s->pos[p->v2], s->nrm[p->v0], s->nrm[p->v1], s->nrm[p->v2], r,
                   is, (int)p->bsdf);
  return sphere_hit(p->c, p->r2, r, is, (int)p->bsdf);
}

/* BlackHole::next_micro_ray (blackhole.cpp:17-40) */
static inline ray_t next_micro_ray(const hole_t* h, const ray_t* ray) {
  ray_t ret;
  ret.o = vadd(ray->o, vmul(ray->d, ray->max_t));
  ret.min_t = 0.0;
  v3 x_axis = vsub(ret.o, h->c);
  double d = vnorm(x_axis);
  x_axis = vnormalize(x_axis);
  double u = 1 / d;
  double dx = vdot(ray->d, x_axis);
  v3 y_axis = vsub(ray->d, smul(dx, x_axis));
  double dy = vnorm(y_axis);
  y_axis = vnormalize(y_axis);
  double up = -u * dx / dy;
  const double dt = h->dt, k = 3.0 * h->r;
  double f1 = -u + k * u * u / 2.0;
  double u2 = u + up * dt / 2.0;
  double f2 = -u2 + k * u2 * u2 / 2.0;
  double u3 = u + up * dt / 2.0 + f1 * dt * dt / 4.0;
  double f3 = -u3 + k * u3 * u3 / 2.0;
  u += up * dt + (f1 + f2 + f3) * dt * dt / 6.0;
  d = 1 / u;
  double next_x = d * h->cos_dt, next_y = d * h->sin_dt;
  ret.d = vsub(vadd(vadd(h->c, smul(next_x, x_axis)), smul(next_y, y_axis)), ret.o);
  ret.max_t = vnorm(ret.d);
  ret.d = vnormalize(ret.d);
  return ret;
}

/* ---- Kerr null geodesics (build-defined; restates rrt_device.h kerr_* operation for operation).
 * Kerr-Schild Cartesian coordinates about the hole, spin along the local z:
 *   g = eta + f l l,  f = 2 M r^3 / (r^4 + a^2 z^2),
 *   l = (1, (r x + a y) / (r^2 + a^2), (r y - a x) / (r^2 + a^2), z / r),
 *   r^2 = (rho^2 - a^2) / 2 + sqrt((rho^2 - a^2)^2 / 4 + a^2 z^2).
 * H = (|p|^2 - f L^2) / 2 with p_t = -1, L = 1 + l . p:
 *   dq/dl = p - f L l,  dp/dl = (1/2) grad(f L^2) = L ((L/2) grad f + f grad L), the gradients in
 * closed form: with Sigma = r^4 + a^2 z^2 and W = r^2 + a^2 (from r^4 - (rho^2 - a^2) r^2 - a^2 z^2 = 0),
 *   grad r = (x r^3, y r^3, z r W) / Sigma,  grad f = f (3 grad r / r - (4 r^3 grad r + 2 a^2 z e_z) / Sigma),
 *   grad l_x = (r e_x + a e_y) / W + (x - 2 r l_x) grad r / W,  grad l_y = (r e_y - a e_x) / W + (y - 2 r l_y) grad r / W,
 *   grad l_z = e_z / r - z grad r / r^2. */
static inline double kerr_r2(const hole_t* h, v3 q) {
  const double w = ((q.x * q.x + q.y * q.y) + q.z * q.z) - h->a2;
  return 0.5 * w + sqrt(0.25 * (w * w) + h->a2 * (q.z * q.z));
}
/* values only: f, l, r at local point q */
static inline void kerr_fl(const hole_t* h, v3 q, double* f, v3* l, double* r_out) {
  const double zz = q.z * q.z;
  const double w = ((q.x * q.x + q.y * q.y) + zz) - h->a2;
  const double r2 = 0.5 * w + sqrt(0.25 * (w * w) + h->a2 * zz);
  const double r = sqrt(r2);
  const double iw = 1.0 / (r2 + h->a2);
  *l = V((r * q.x + h->a * q.y) * iw, (r * q.y - h->a * q.x) * iw, q.z / r);
  *f = ((2.0 * h->m) * (r * r2)) / (r2 * r2 + h->a2 * zz);
  *r_out = r;
}
static inline void kerr_rhs(const hole_t* h, v3 q, v3 p, v3* dq, v3* dp, double* r_out) {
  const double zz = q.z * q.z;
  const double w = ((q.x * q.x + q.y * q.y) + zz) - h->a2;
  const double r2 = 0.5 * w + sqrt(0.25 * (w * w) + h->a2 * zz);
  const double r = sqrt(r2);
  const double W = r2 + h->a2;
  const double isg = 1.0 / (r2 * r2 + h->a2 * zz), iw = 1.0 / W, ir = 1.0 / r;
  const double r3 = r * r2, gk = r3 * isg;
  const v3 g = V(q.x * gk, q.y * gk, (q.z * r) * (W * isg));
  const double lx = (r * q.x + h->a * q.y) * iw, ly = (r * q.y - h->a * q.x) * iw, lz = q.z * ir;
  const double f = (2.0 * h->m) * gk;
  const double cf = 3.0 * ir - (4.0 * r3) * isg;
  const v3 gf = V(f * (cf * g.x), f * (cf * g.y), f * (cf * g.z - ((2.0 * h->a2) * q.z) * isg));
  const double L = ((1.0 + p.x * lx) + p.y * ly) + p.z * lz;
  const double c = (p.x * (q.x - (2.0 * r) * lx) + p.y * (q.y - (2.0 * r) * ly)) * iw - (p.z * q.z) * (ir * ir);
  const v3 gL = V((r * p.x - h->a * p.y) * iw + c * g.x, (h->a * p.x + r * p.y) * iw + c * g.y, p.z * ir + c * g.z);
  const double hL = 0.5 * L, fL = f * L;
  *dq = V(p.x - fL * lx, p.y - fL * ly, p.z - fL * lz);
  *dp = V(L * (hL * gf.x + f * gL.x), L * (hL * gf.y + f * gL.y), L * (hL * gf.z + f * gL.z));
  *r_out = r;
}
static inline v3 kerr_local(const hole_t* h, v3 v) { return V(vdot(v, h->ex), vdot(v, h->ey), vdot(v, h->ez)); }
static inline v3 kerr_world(const hole_t* h, v3 q) {
  return V(h->c.x + ((h->ex.x * q.x + h->ey.x * q.y) + h->ez.x * q.z),
           h->c.y + ((h->ex.y * q.x + h->ey.y * q.y) + h->ez.y * q.z),
           h->c.z + ((h->ex.z * q.x + h->ey.z * q.y) + h->ez.z * q.z));
}
/* photon at world o along world d: k = (k^t, d) made null (future root), p = g k, scaled to p_t = -1 */
static inline void kerr_init(const hole_t* h, v3 o, v3 d, v3* q, v3* p) {
  *q = kerr_local(h, vsub(o, h->c));
  const v3 k = kerr_local(h, d);
  double f, r;
  v3 l;
  kerr_fl(h, *q, &f, &l, &r);
  const double ld = (l.x * k.x + l.y * k.y) + l.z * k.z;
  const double A = f - 1.0, B = 2.0 * f * ld, C = 1.0 + f * (ld * ld);
  double disc = B * B - 4.0 * A * C;
  if (!(disc > 0.0)) disc = 0.0;
  const double kt = (2.0 * C) / (sqrt(disc) - B);
  const double pt = A * kt + f * ld;
  const double s = f * (kt + ld);
  *p = V(k.x + s * l.x, k.y + s * l.y, k.z + s * l.z);
  if (pt < 0.0) *p = vmul(*p, -1.0 / pt);
}
/* classical RK4 in the affine parameter from (q, p) with its first stage given, h = dtheta * r / |dq/dl| */
static inline void kerr_step(const hole_t* h, v3* q, v3* p, v3 dq1, v3 dp1, double hh) {
  v3 dq, dp, aq = dq1, ap = dp1;  /* running sums ((k1 + 2 k2) + 2 k3) + k4 */
  double rr;
  const double half = 0.5 * hh;
  kerr_rhs(h, vadd(*q, vmul(dq1, half)), vadd(*p, vmul(dp1, half)), &dq, &dp, &rr);
  aq = vadd(aq, vmul(dq, 2.0)); ap = vadd(ap, vmul(dp, 2.0));
  kerr_rhs(h, vadd(*q, vmul(dq, half)), vadd(*p, vmul(dp, half)), &dq, &dp, &rr);
  aq = vadd(aq, vmul(dq, 2.0)); ap = vadd(ap, vmul(dp, 2.0));
  kerr_rhs(h, vadd(*q, vmul(dq, hh)), vadd(*p, vmul(dp, hh)), &dq, &dp, &rr);
  aq = vadd(aq, dq); ap = vadd(ap, dp);
  const double c6 = hh / 6.0;
  *q = vadd(*q, vmul(aq, c6));
  *p = vadd(*p, vmul(ap, c6));
}
/* one march step: 0 = stepped, 1 = escaped (outgoing beyond r_esc); *swept += polar angle.
 * st: step stretch (1 for the march; the coarse march of the Kerr occlusion proof's sweep, tests/
 * kerr_proof_sim.py, takes st > 1: h = st * dtheta * r / |dq/dl|) */
static inline int kerr_advance_st(const hole_t* h, v3* q, v3* p, double* swept, double st) {
  v3 dq1, dp1;
  double r;
  kerr_rhs(h, *q, *p, &dq1, &dp1, &r);
  const double rho2 = vnorm2(*q);
  if (rho2 > h->r_esc2 && vdot(*q, dq1) > 0.0) return 1;
  const double hh = ((h->dt * r) * st) / vnorm(dq1);
  *swept += (hh * vnorm(vcross(*q, dq1))) / rho2;
  kerr_step(h, q, p, dq1, dp1, hh);
  return 0;
}
static inline int kerr_advance(const hole_t* h, v3* q, v3* p, double* swept) {
  return kerr_advance_st(h, q, p, swept, 1.0);  /* (dt r) * 1 = dt r exactly */
}

typedef struct {
  const ro_scene* s;
  hole_t hole;
  rng_t* g;
} qctx;

/* BVHAccel::intersect_micro (bvh.cpp:115-138): recursive, left then right, no early exit */
static int intersect_micro(qctx* q, ray_t* r, isect_t* is, int node) {
  const node_t* n = &q->s->nodes[node];
  double t0, t1;
  q->g->bbox_tests++;
  if (!bbox_hit(n->mn, n->mx, r, &t0, &t1)) return 0;
  int hit = 0;
  if (n->count > 0) {
    for (int32_t i = 0; i < n->count; ++i) {
      q->g->prim_tests++;
      if (prim_hit(q->s, &q->s->prims[q->s->leaf[n->first + i]], r, is)) hit = 1;
    }
  } else {
    if (intersect_micro(q, r, is, n->left)) hit = 1;
    if (intersect_micro(q, r, is, n->right)) hit = 1;
  }
  return hit;
}

/* BVHAccel::intersect (bvh.cpp:103-113): geodesic march; ray.min_t / max_t are dropped */
static int bvh_intersect_kerr(qctx* q, v3 o, v3 d, isect_t* is) {
  const hole_t* h = &q->hole;
  v3 kq, kp;
  kerr_init(h, o, d, &kq, &kp);
  v3 a = o;
  const double rh2 = h->r_hor * h->r_hor;
  double swept = 0.0;
  q->g->queries++;
  for (int j = 0; j < h->kerr_max_steps && swept < 2.0 * PI_D; ++j) {
    if (kerr_advance(h, &kq, &kp, &swept)) return 0; /* escaped */
    q->g->micro_steps++;
    if (kerr_r2(h, kq) <= rh2) return 0; /* captured: inside the outer horizon */
    const v3 b = kerr_world(h, kq);
    ray_t micro;
    micro.o = a; micro.d = vsub(b, a); micro.min_t = 0.0;
    micro.max_t = vnorm(micro.d);
    micro.d = vnormalize(micro.d);
    if (intersect_micro(q, &micro, is, 0)) return 1;
    a = b;
  }
  return 0;
}

static int bvh_intersect(qctx* q, v3 o, v3 d, isect_t* is) {
  if (q->hole.kerr) return bvh_intersect_kerr(q, o, d, is);
  ray_t micro; micro.o = o; micro.d = d; micro.min_t = 0.0; micro.max_t = 0.0;
  q->g->queries++;
  for (int j = 0; j < q->hole.steps; ++j) {
    micro = next_micro_ray(&q->hole, &micro);
    q->g->micro_steps++;
    ray_t probe = micro;
    if (sphere_hit(q->hole.c, q->hole.r2, &probe, NULL, -1)) return 0; /* captured */
    if (intersect_micro(q, &micro, is, 0)) return 1;
  }
  return 0;
}

/* ------------------------------------------------------------------ BSDFs */
static inline void coord_space(v3 n, v3* X, v3* Y, v3* Z) { /* make_coord_space, bsdf.cpp:13-29 */
  v3 z = n, h = z;
  if (fabs(h.x) <= fabs(h.y) && fabs(h.x) <= fabs(h.z)) h.x = 1.0;
  else if (fabs(h.y) <= fabs(h.x) && fabs(h.y) <= fabs(h.z)) h.y = 1.0;
  else h.z = 1.0;
  z = vnormalize(z);
  v3 y = vnormalize(vcross(h, z));
  v3 x = vnormalize(vcross(z, y));
  *X = x; *Y = y; *Z = z;
}
static inline v3 to_local(v3 X, v3 Y, v3 Z, v3 v) { return V(vdot(v, X), vdot(v, Y), vdot(v, Z)); } /* w2o * v */
static inline v3 to_world(v3 X, v3 Y, v3 Z, v3 v) { /* o2w * v = v.x*X + v.y*Y + v.z*Z */
  return vadd(vadd(smul(v.x, X), smul(v.y, Y)), smul(v.z, Z));
}
static inline int bsdf_is_delta(const bsdf_t* b) {
  return b->type == BSDF_MIRROR || b->type == BSDF_GLASS || b->type == BSDF_REFRACTION;
}
static inline spec bsdf_emission(const bsdf_t* b) {
  return b->type == BSDF_EMISSION ? S(b->p[0], b->p[1], b->p[2]) : S(0, 0, 0);
}
static inline double clamp_b(double n, double lo, double hi) { return std_max(lo, std_min(n, hi)); } /* bsdf.h:20 */
static inline double mf_theta(v3 w) { return acos(clamp_b(w.z, -1.0 + 1e-5, 1.0 - 1e-5)); }
static inline double mf_lambda(float alpha, v3 w) {
  double theta = mf_theta(w);
  double a = 1.0 / (alpha * tan(theta));
  return 0.5 * (erf(a) - 1.0 + exp(-a * a) / (a * PI_D));
}
static inline spec mf_F(const bsdf_t* b, v3 wi) {
  spec eta = S(b->p[0], b->p[1], b->p[2]), k = S(b->p[3], b->p[4], b->p[5]);
  spec eta2pk2 = sadd(smulS(eta, eta), smulS(k, k));
  double cti = wi.z, cti2 = cti * cti;
  spec tc = smulf(smulf(eta, 2.0f), (float)cti);
  spec Rs = sdivS(saddf(ssub(eta2pk2, tc), (float)cti2), saddf(sadd(eta2pk2, tc), (float)cti2));
  spec Rp = sdivS(saddf(ssub(smulf(eta2pk2, (float)cti2), tc), 1.0f), saddf(sadd(smulf(eta2pk2, (float)cti2), tc), 1.0f));
  return sdivf(sadd(Rs, Rp), 2.0f);
}
static inline double mf_D(float alpha, v3 h) {
  double theta_h = mf_theta(h), tan_h = tan(theta_h), cos_h = h.z, cos_h2 = cos_h * cos_h;
  double alpha2 = alpha * alpha; /* float product */
  return exp(-tan_h * tan_h / alpha2) / (PI_D * alpha2 * cos_h2 * cos_h2);
}
static inline spec mf_f(const bsdf_t* b, v3 wo, v3 wi) {
  if (wo.z <= 0 || wi.z <= 0) return S(0, 0, 0);
  float alpha = b->p[6];
  double G = 1.0 / (1.0 + mf_lambda(alpha, wi) + mf_lambda(alpha, wo));
  double D = mf_D(alpha, vunit(vadd(wo, wi)));
  return sdivf(smulf(smulf(mf_F(b, wi), (float)G), (float)D), (float)(4 * wo.z * wi.z));
}
static inline spec bsdf_f(const bsdf_t* b, v3 wo, v3 wi) {
  if (b->type == BSDF_DIFFUSE) return sdivf(S(b->p[0], b->p[1], b->p[2]), (float)PI_D);
  if (b->type == BSDF_MICROFACET) return mf_f(b, wo, wi);
  return S(0, 0, 0);
}
static inline int refract(v3 wo, v3* wi, float ior) { /* bsdf.cpp:146-159 */
  double eta;
  if (wo.z > 0) eta = 1 / ior; else eta = ior;
  double wi_z2 = 1 - eta * eta * (1 - wo.z * wo.z);
  if (wi_z2 < 0) return 0;
  *wi = V(-eta * wo.x, -eta * wo.y, sqrt(wi_z2));
  if (wo.z > 0) wi->z = -wi->z;
  return 1;
}
static spec bsdf_sample_f_sw(const bsdf_t* b, rng_t* g, v3 wo, v3* wi, float* pdf, int mf_hemi);
static spec bsdf_sample_f(const bsdf_t* b, rng_t* g, v3 wo, v3* wi, float* pdf) {
  return bsdf_sample_f_sw(b, g, wo, wi, pdf, 0);
}
static spec bsdf_sample_f_sw(const bsdf_t* b, rng_t* g, v3 wo, v3* wi, float* pdf, int mf_hemi) {
  switch (b->type) {
    case BSDF_DIFFUSE: /* part1_code.cpp:171-173 */
      *wi = cosine_sample(g, pdf);
      return bsdf_f(b, wo, *wi);
    case BSDF_MIRROR: /* bsdf.cpp:37-41 */
      *wi = V(-wo.x, -wo.y, wo.z); *pdf = 1.0;
      return sdivf(S(b->p[0], b->p[1], b->p[2]), (float)fabs(wi->z));
    case BSDF_GLASS: { /* bsdf.cpp:114-140 */
      float ior = b->p[7];
      spec tr = S(b->p[0], b->p[1], b->p[2]), rf = S(b->p[3], b->p[4], b->p[5]);
      if (refract(wo, wi, ior)) {
        double R0 = (1 - ior) / (1 + ior);
        R0 *= R0;
        double t = (1 - fabs(wi->z)), t2 = t * t, t4 = t2 * t2, R = R0 + (1 - R0) * t4 * t;
        if (coin_flip(g, R)) {
          *wi = V(-wo.x, -wo.y, wo.z); *pdf = (float)R;
          return sdivf(smulf(rf, (float)R), (float)fabs(wi->z));
        } else {
          double eta;
          if (wo.z > 0) eta = 1 / ior; else eta = ior;
          *pdf = (float)(1 - R);
          return sdivf(smulf(tr, (float)(1 - R)), (float)(fabs(wi->z) * eta * eta));
        }
      } else {
        *wi = V(-wo.x, -wo.y, wo.z); *pdf = 1.0;
        return sdivf(rf, (float)fabs(wi->z));
      }
    }
    case BSDF_MICROFACET: { /* bsdf.cpp:74-92, MICROFACET_HEMI == 0 */
      if (mf_hemi) { /* MICROFACET_HEMI == 1 (bsdf.cpp:93-94) */
        *wi = cosine_sample(g, pdf);
        return mf_f(b, wo, *wi);
      }
      double ux, uy;
      grid_sample(g, &ux, &uy);
      float alpha = b->p[6];
      double alpha2 = alpha * alpha,
             theta_h = atan(sqrt(-alpha2 * log(1 - ux))),
             phi_h = 2 * PI_D * uy,
             sin_h = sin(theta_h), cos_h = cos(theta_h), tan_h = tan(theta_h),
             p_theta = 2 * sin_h * exp(-tan_h * tan_h / alpha2) / (alpha2 * cos_h * cos_h * cos_h),
             p_phi = 0.5 / PI_D;
      v3 h = V(sin_h * cos(phi_h), sin_h * sin(phi_h), cos_h);
      *wi = vsub(smul(2 * vdot(wo, h), h), wo);
      if (wi->z <= 0) { *pdf = 0; return S(0, 0, 0); }
      *pdf = (float)(p_theta * p_phi / (sin_h * 4 * vdot(*wi, h)));
      return mf_f(b, wo, *wi);
    }
    case BSDF_EMISSION: /* bsdf.cpp:167-171 */
      *pdf = (float)(1.0 / PI_D);
      *wi = cosine_sample(g, pdf);
      return S(0, 0, 0);
    default: /* RefractionBSDF stub (bsdf.cpp:104-106): wi, pdf untouched */
      return S(0, 0, 0);
  }
}

/* ------------------------------------------------------------------ environment light
 * environment_light.cpp:21-148 (ENV_HEMI == 0).  Spectrum * double narrows the weight to float. */
static spec env_texel(const ro_scene* s, size_t i) { return S(s->env_tex[3 * i], s->env_tex[3 * i + 1], s->env_tex[3 * i + 2]); }
static spec env_bilerp(const ro_scene* s, double xx, double yy) { /* :112-127 */
  long right = lround(xx), left, v = lround(yy);
  double u1 = right - xx + .5, v1;
  if (right == 0 || right == (long)s->env_w) { left = (long)s->env_w - 1; right = 0; }
  else left = right - 1;
  if (v == 0) { v = 1; v1 = 1; }
  else if (v == (long)s->env_h) { v = (long)s->env_h - 1; v1 = 0; }
  else v1 = v - yy + .5;
  size_t bottom = (size_t)s->env_w * (size_t)v, top = bottom - s->env_w;
  double u0 = 1 - u1;
  float fu1 = (float)u1, fu0 = (float)u0, fv1 = (float)v1, fv0 = (float)(1 - v1);
  spec a = sadd(smulf(env_texel(s, top + left), fu1), smulf(env_texel(s, top + right), fu0));
  spec b = sadd(smulf(env_texel(s, bottom + left), fu1), smulf(env_texel(s, bottom + right), fu0));
  return sadd(smulf(a, fv1), smulf(b, fv0));
}
static spec env_dir(const ro_scene* s, v3 d) { /* sample_dir :146-148 */
  v3 u = vunit(d);
  double theta = acos(u.y), phi = atan2(-u.z, u.x) + PI_D;
  double x = phi / 2. / PI_D * s->env_w, y = theta / PI_D * s->env_h;
  return env_bilerp(s, x, y);
}
static uint32_t upper_bound_d(const double* a, uint32_t n, double value) { /* std::upper_bound */
  uint32_t first = 0, count = n;
  while (count > 0) {
    uint32_t step = count >> 1, it = first + step;
    if (!(value < a[it])) { first = it + 1; count -= step + 1; }
    else count = step;
  }
  return first;
}
static spec env_sample(const ro_scene* s, rng_t* g, v3* wi, float* dist, float* pdf) { /* :130-144 */
  *dist = INFINITY;
  double sx, sy;
  grid_sample(g, &sx, &sy);
  uint32_t y = upper_bound_d(s->env_marg, s->env_h, sy);
  if (y >= s->env_h) y = s->env_h - 1;  /* (the reference reads one row past the table) */
  uint32_t x = upper_bound_d(s->env_conds + (size_t)s->env_w * y, s->env_w, sx);
  if (x >= s->env_w) x = s->env_w - 1;
  double phi = (double)x / s->env_w * 2.0 * PI_D, theta = (double)y / s->env_h * PI_D;
  *wi = V(cos(phi - PI_D) * sin(theta), cos(theta), -sin(phi - PI_D) * sin(theta));
  *pdf = (float)(s->env_pdf[(size_t)s->env_w * y + x] * s->env_w * s->env_h / (2 * M_PI * M_PI * sin(theta)));
  return env_bilerp(s, (double)x, (double)y);
}

int ro_scene_set_envmap(ro_scene* s, uint32_t w, uint32_t h, const float* texels) {
  if (!s || !texels || !w || !h || s->env_w) return -1;
  s->env_tex = (float*)malloc(sizeof(float) * 3 * (size_t)w * h);
  s->env_pdf = (double*)calloc((size_t)w * h, sizeof(double));
  s->env_conds = (double*)calloc((size_t)w * h, sizeof(double));
  s->env_marg = (double*)calloc(h, sizeof(double));
  memcpy(s->env_tex, texels, sizeof(float) * 3 * (size_t)w * h);
  double sum = 0;  /* EnvironmentLight::init :21-45 */
  for (uint32_t j = 0; j < h; ++j)
    for (uint32_t i = 0; i < w; ++i) {
      const float* t = &s->env_tex[3 * ((size_t)w * j + i)];
      float il = 0.2126f * t[0] + 0.7152f * t[1] + 0.0722f * t[2];
      s->env_pdf[(size_t)w * j + i] = il * sin(PI_D * (j + .5) / h);
      sum += s->env_pdf[(size_t)w * j + i];
    }
  for (uint32_t j = 0; j < h; ++j) {
    for (uint32_t i = 0; i < w; ++i) s->env_marg[j] += (s->env_pdf[(size_t)w * j + i] /= sum);
    for (uint32_t i = 0; i < w; ++i) {
      s->env_conds[(size_t)w * j + i] = s->env_pdf[(size_t)w * j + i] / s->env_marg[j];
      if (i > 0) s->env_conds[(size_t)w * j + i] += s->env_conds[(size_t)w * j + i - 1];
    }
    if (j > 0) s->env_marg[j] += s->env_marg[j - 1];
  }
  s->env_w = w; s->env_h = h;
  /* PathTracer::set_scene appends envLight after the scene's lights (pathtracer.cpp:106-108) */
  s->lights = (light_t*)realloc(s->lights, sizeof(light_t) * (s->nlights + 1));
  memset(&s->lights[s->nlights], 0, sizeof(light_t));
  s->lights[s->nlights].type = 5;
  s->lights[s->nlights].is_delta = 0;
  s->nlights++;
  return 0;
}

/* ------------------------------------------------------------------ lights (light.cpp) */
static spec light_sample_L_sw(const ro_scene* s, const light_t* l, rng_t* g, v3 p, v3* wi, float* dist, float* pdf,
                              int env_hemi);
static spec light_sample_L(const ro_scene* s, const light_t* l, rng_t* g, v3 p, v3* wi, float* dist, float* pdf) {
  return light_sample_L_sw(s, l, g, p, wi, dist, pdf, 0);
}
static spec light_sample_L_sw(const ro_scene* s, const light_t* l, rng_t* g, v3 p, v3* wi, float* dist, float* pdf,
                              int env_hemi) {
  spec rad = S(l->rad[0], l->rad[1], l->rad[2]);
  switch (l->type) {
    case 5: /* EnvironmentLight */
      if (env_hemi) { /* ENV_HEMI == 1 (environment_light.cpp:139-142): UniformSphereSampler3D (sampler.cpp:33-40) */
        *dist = INFINITY;
        double z = random_uniform(g) * 2 - 1;
        double q = 1.0f - z * z, sin_t = sqrt(0.0 < q ? q : 0.0);
        double phi = 2.0f * PI_D * random_uniform(g);
        *wi = V(cos(phi) * sin_t, sin(phi) * sin_t, z);
        *pdf = (float)(0.25 / M_PI);
        return env_dir(s, *wi); /* sample_dir(Ray(p, *wi)) */
      }
      return env_sample(s, g, wi, dist, pdf);
    case 0: { /* AreaLight::sample_L, light.cpp:80-92 */
      double sx, sy;
      grid_sample(g, &sx, &sy);
      sx = sx - 0.5f; sy = sy - 0.5f;
      v3 d = vsub(vadd(vadd(l->v[0], smul(sx, l->v[2])), smul(sy, l->v[3])), p);
      float sqDist = (float)vnorm2(d);
      float dd = sqrtf(sqDist);
      *wi = vdivd(d, dd);
      float cosTheta = (float)vdot(*wi, l->v[1]);
      *dist = dd;
      *pdf = sqDist / (l->area * fabsf(cosTheta));
      return cosTheta < 0 ? rad : S(0, 0, 0);
    }
    case 1: { /* PointLight, light.cpp:49-57 */
      v3 d = vsub(l->v[0], p);
      *wi = vunit(d); *dist = (float)vnorm(d); *pdf = 1.0;
      return rad;
    }
    case 2: /* DirectionalLight, light.cpp:17-23 */
      *wi = l->v[0]; *dist = INFINITY; *pdf = 1.0;
      return rad;
    default: { /* InfiniteHemisphereLight, light.cpp:34-42 */
      v3 dir = hemisphere_sample(g);
      *wi = to_world(l->v[0], l->v[1], l->v[2], dir);
      *dist = INFINITY; *pdf = (float)(1.0 / (2.0 * PI_D));
      return rad;
    }
  }
}

/* ------------------------------------------------------------------ integrator (part1_code.cpp) */
typedef struct {
  qctx q;
  const ro_params* p;
  v3 cam_pos, c2w0, c2w1, c2w2;
  double blx, bly;
  double lens_r, focal;  /* Camera::lensRadius / focalDistance (thin lens) */
} pctx;

static spec direct_hemisphere(pctx* c, const isect_t* is) { /* :15-31 */
  v3 X, Y, Z; coord_space(is->n, &X, &Y, &Z);
  v3 hit_p = is->hit_p, w_out = to_local(X, Y, Z, is->w_out);
  int num = (int)(c->q.s->nlights * c->p->ns_area_light);
  spec L = S(0, 0, 0);
  const bsdf_t* b = &c->q.s->bsdfs[is->bsdf];
  for (int i = 0; i < num; ++i) {
    v3 w_in = hemisphere_sample(c->q.g);
    v3 wi_world = to_world(X, Y, Z, w_in);
    isect_t is2;
    if (bvh_intersect(&c->q, vadd(hit_p, smul(EPS_D, wi_world)), wi_world, &is2))
      L = sadd(L, smulf(smulS(bsdf_emission(&c->q.s->bsdfs[is2.bsdf]), bsdf_f(b, w_out, w_in)), (float)w_in.z));
  }
  return sdivf(smulf(smulf(L, 2.0f), (float)M_PI), (float)num);
}

static spec direct_importance(pctx* c, const isect_t* is) { /* :33-57 */
  v3 X, Y, Z; coord_space(is->n, &X, &Y, &Z);
  v3 hit_p = is->hit_p, w_out = to_local(X, Y, Z, is->w_out);
  spec L = S(0, 0, 0);
  int total = 0;
  const bsdf_t* b = &c->q.s->bsdfs[is->bsdf];
  for (uint32_t li = 0; li < c->q.s->nlights; ++li) {
    const light_t* l = &c->q.s->lights[li];
    int num = l->is_delta ? 1 : (int)c->p->ns_area_light;
    total += num;
    for (int i = 0; i < num; ++i) {
      v3 wi_world; float dist, pdf;
      spec sample = light_sample_L_sw(c->q.s, l, c->q.g, hit_p, &wi_world, &dist, &pdf, (int)c->p->env_hemi);
      v3 w_in = to_local(X, Y, Z, wi_world);
      if (w_in.z < 0) continue;
      if (!bvh_intersect(&c->q, vadd(hit_p, smul(EPS_D, wi_world)), wi_world, NULL))
        L = sadd(L, sdivf(smulf(smulS(sample, bsdf_f(b, w_out, w_in)), (float)w_in.z), pdf));
    }
  }
  return sdivf(L, (float)total);
}

static spec one_bounce(pctx* c, const isect_t* is) { /* :63-67 */
  return c->p->direct_hemisphere ? direct_hemisphere(c, is) : direct_importance(c, is);
}

static spec at_least_one_bounce(pctx* c, uint32_t depth, const isect_t* is) { /* :69-101 */
  v3 X, Y, Z; coord_space(is->n, &X, &Y, &Z);
  v3 hit_p = is->hit_p, w_out = to_local(X, Y, Z, is->w_out);
  const bsdf_t* b = &c->q.s->bsdfs[is->bsdf];
  spec L_out = S(0, 0, 0);
  if (!bsdf_is_delta(b)) L_out = sadd(L_out, one_bounce(c, is));
  if (c->p->illum == 3 && depth == c->p->max_ray_depth) L_out = S(0, 0, 0); /* ILLUM == 3 (:78-81) */
  const double prob = 0.7;
  if (depth == c->p->max_ray_depth || (depth > 1 && coin_flip(c->q.g, prob))) {
    v3 w_in; float pdf;
    spec sample = bsdf_sample_f_sw(b, c->q.g, w_out, &w_in, &pdf, (int)c->p->microfacet_hemi);
    if (pdf == 0.0f) return L_out;
    v3 wi_world = to_world(X, Y, Z, w_in);
    isect_t is2;
    if (bvh_intersect(&c->q, vadd(hit_p, smul(EPS_D, wi_world)), wi_world, &is2)) {
      spec L = at_least_one_bounce(c, depth - 1, &is2);
      if (bsdf_is_delta(b)) L = sadd(L, bsdf_emission(&c->q.s->bsdfs[is2.bsdf]));
      L_out = sadd(L_out, sdivf(sdivf(smulf(smulS(L, sample), (float)fabs(w_in.z)), pdf), (float)prob));
    }
  }
  return L_out;
}

static spec est_radiance(pctx* c, v3 o, v3 d) { /* :103-123, ILLUM == 2 */
  isect_t is;
  if (!bvh_intersect(&c->q, o, d, &is)) /* miss: envLight->sample_dir(r), r unbent */
    return c->q.s->env_w ? env_dir(c->q.s, d) : S(0, 0, 0);
  if (c->p->illum == 0) /* normal_shading (pathtracer.h:199-201) */
    return sadd(smulf(S((float)is.n.x, (float)is.n.y, (float)is.n.z), (float).5), S(.5f, .5f, .5f));
  if (c->p->illum == 1) return one_bounce(c, &is);
  if (c->p->illum == 3) return at_least_one_bounce(c, c->p->max_ray_depth, &is);
  spec e = bsdf_emission(&c->q.s->bsdfs[is.bsdf]);
  if (c->p->max_ray_depth == 0) return e;
  if (c->p->max_ray_depth == 1) return sadd(e, one_bounce(c, &is));
  return sadd(e, at_least_one_bounce(c, c->p->max_ray_depth, &is));
}

static void gen_ray(const pctx* c, double x, double y, v3* o, v3* d) { /* Camera::generate_ray :182-187 */
  double vx = (1 - x) * c->blx + x * -c->blx, vy = (1 - y) * c->bly + y * -c->bly;
  v3 w = vadd(vadd(smul(vx, c->c2w0), smul(vy, c->c2w1)), smul(-1.0, c->c2w2));
  *o = c->cam_pos;
  *d = vunit(w);
}

static void gen_ray_thin_lens(const pctx* c, double x, double y, double rnd_r, double rnd_theta, v3* o, v3* d) {
  v3 pin = V((1 - x) * c->blx + x * -c->blx, (1 - y) * c->bly + y * -c->bly, -1);
  double lr = c->lens_r * sqrt(rnd_r);
  v3 pl = V(lr * cos(rnd_theta), lr * sin(rnd_theta), 0);
  /* Matrix3x3 * Vector3D = x[0]*col0 + x[1]*col1 + x[2]*col2 (matrix3x3.cpp:124-128) */
  *o = vadd(c->cam_pos, vadd(vadd(smul(pl.x, c->c2w0), smul(pl.y, c->c2w1)), smul(pl.z, c->c2w2)));
  v3 q = vsub(smul(c->focal, pin), pl);
  *d = vunit(vadd(vadd(smul(q.x, c->c2w0), smul(q.y, c->c2w1)), smul(q.z, c->c2w2)));
}

static spec raytrace_pixel(pctx* c, uint32_t x, uint32_t y, int32_t* count_out) { /* :125-163 */
  const ro_params* p = c->p;
  spec ret = S(0, 0, 0);
  int i;
  double s1 = 0.0, s2 = 0.0;
  for (i = 0; i < (int)p->ns_aa; ++i) {
    double sx = (double)x, sy = (double)y;
    if (p->ns_aa == 1) { sx += 0.5; sy += 0.5; }
    else { double jx, jy; grid_sample(c->q.g, &jx, &jy); sx += jx; sy += jy; }
    v3 o, d;
    if (p->thin_lens) { /* Camera::generate_ray_for_thin_lens (camera.cpp:176-184), part1_code.cpp:137-139 */
      double lx, ly;
      grid_sample(c->q.g, &lx, &ly);
      gen_ray_thin_lens(c, sx / (double)p->frame_w, sy / (double)p->frame_h, lx, ly * 2 * M_PI, &o, &d);
    } else {
      gen_ray(c, sx / (double)p->frame_w, sy / (double)p->frame_h, &o, &d);
    }
    spec s = est_radiance(c, o, d);
    ret = sadd(ret, s);
    if (!p->adaptive) continue; /* ADAPTIVE == 0 */
    double il = illum(s);
    s1 += il;
    s2 += il * il;
    if ((i + 1) % p->samples_per_batch == 0) {
      double avg = s1 / (i + 1), sd = sqrt((s2 - avg * s1) / i);
      if (1.96 * sd / sqrt(i + 1) <= (double)p->max_tolerance * avg) { ++i; break; }
    }
  }
  *count_out = i;
  return sdivf(ret, (float)i);
}

static void pctx_init(pctx* c, const ro_scene* s, const ro_camera* cam, const ro_params* p, rng_t* g) {
  c->q.s = s; c->q.g = g; c->p = p;
  if (p->bh_kind == 1) {
    hole_init_kerr(&c->q.hole, p->bh_center, p->bh_radius, p->bh_dtheta, p->bh_spin, p->bh_axis);
    kerr_set_escape(&c->q.hole, s->nodes[0].mn, s->nodes[0].mx);
  } else hole_init(&c->q.hole, p->bh_center, p->bh_radius, p->bh_dtheta);
  c->cam_pos = V(cam->pos[0], cam->pos[1], cam->pos[2]);
  c->c2w0 = V(cam->c2w[0], cam->c2w[3], cam->c2w[6]);
  c->c2w1 = V(cam->c2w[1], cam->c2w[4], cam->c2w[7]);
  c->c2w2 = V(cam->c2w[2], cam->c2w[5], cam->c2w[8]);
  /* radians(deg) = deg * (PI / 180) (misc.h:49-52) */
  c->blx = -tan(cam->hFov * (PI_D / 180) / 2);
  c->bly = -tan(cam->vFov * (PI_D / 180) / 2);
  c->lens_r = cam->lensRadius; c->focal = cam->focalDistance;
}

/* ------------------------------------------------------------------ tiled thread pool */
typedef struct {
  const ro_scene* s; const ro_camera* cam; const ro_params* p;
  uint32_t x0, y0, w, h, tiles_w, ntiles;
  float* rgb; int32_t* count; uint32_t* draws; uint32_t* counters;
  int next; pthread_mutex_t mu;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  rng_t g; memset(&g, 0, sizeof(g));
  pctx c; pctx_init(&c, j->s, j->cam, j->p, &g);
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int t = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (t >= (int)j->ntiles) break;
    uint32_t tx = (t % j->tiles_w) * 32, ty = (t / j->tiles_w) * 32;
    for (uint32_t yy = ty; yy < ty + 32 && yy < j->h; ++yy)
      for (uint32_t xx = tx; xx < tx + 32 && xx < j->w; ++xx) {
        uint32_t px = j->x0 + xx, py = j->y0 + yy;
        g.key = ro_pixel_key(j->p->seed, px, py); g.ctr = 0;
        g.bbox_tests = g.micro_steps = g.prim_tests = g.queries = 0;
        int32_t cnt;
        spec s = raytrace_pixel(&c, px, py, &cnt);
        size_t k = (size_t)yy * j->w + xx;
        j->rgb[3 * k] = s.r; j->rgb[3 * k + 1] = s.g; j->rgb[3 * k + 2] = s.b;
        j->count[k] = cnt;
        if (j->draws) j->draws[k] = g.ctr;
        if (j->counters) {
          j->counters[4 * k] = (uint32_t)g.bbox_tests; j->counters[4 * k + 1] = (uint32_t)g.micro_steps;
          j->counters[4 * k + 2] = (uint32_t)g.prim_tests; j->counters[4 * k + 3] = (uint32_t)g.queries;
        }
      }
  }
  return NULL;
}

int ro_render(const ro_scene* s, const ro_camera* cam, const ro_params* p, uint32_t x0, uint32_t y0, uint32_t w,
              uint32_t h, float* rgb, int32_t* count, uint32_t* draws, uint32_t* counters, int nthreads) {
  if (!s || !cam || !p || !rgb || !count || p->frame_w == 0 || p->frame_h == 0 || p->samples_per_batch == 0) return -1;
  job_t j;
  memset(&j, 0, sizeof(j));
  j.s = s; j.cam = cam; j.p = p; j.x0 = x0; j.y0 = y0; j.w = w; j.h = h;
  j.tiles_w = (w + 31) / 32; j.ntiles = j.tiles_w * ((h + 31) / 32);
  j.rgb = rgb; j.count = count; j.draws = draws; j.counters = counters;
  pthread_mutex_init(&j.mu, NULL);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, worker, &j);
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&j.mu);
  return 0;
}

/* ------------------------------------------------------------------ KAT entry points */
int ro_kerr_chain_st(const double* bh, const double* o, const double* d, double* out, int max_rows, double* frame,
                     double st, double* extra) {
  hole_t h; hole_init_kerr(&h, bh, bh[3], bh[4], bh[5], bh + 6);
  if (frame) {
    frame[0] = h.ex.x; frame[1] = h.ex.y; frame[2] = h.ex.z; frame[3] = h.ey.x; frame[4] = h.ey.y;
    frame[5] = h.ey.z; frame[6] = h.ez.x; frame[7] = h.ez.y; frame[8] = h.ez.z;
  }
  v3 q, p, a = V(o[0], o[1], o[2]);
  kerr_init(&h, a, V(d[0], d[1], d[2]), &q, &p);
  const double rh2 = h.r_hor * h.r_hor;
  int rows = 0;
  double swept = 0.0;
  while (rows < max_rows) {  /* physics checks: no escape cutoff, no sweep or step budget */
    kerr_advance_st(&h, &q, &p, &swept, st);
    const int cap = kerr_r2(&h, q) <= rh2;
    const v3 b = kerr_world(&h, q);
    v3 sd = vsub(b, a);
    const double mt = vnorm(sd);
    sd = vnormalize(sd);
    double* r = out + 14 * rows++;
    r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = sd.x; r[4] = sd.y; r[5] = sd.z; r[6] = mt; r[7] = cap;
    r[8] = q.x; r[9] = q.y; r[10] = q.z; r[11] = p.x; r[12] = p.y; r[13] = p.z;
    if (extra) {  /* the swept polar angle after the step and the segment's end point */
      double* x = extra + 4 * (rows - 1);
      x[0] = swept; x[1] = b.x; x[2] = b.y; x[3] = b.z;
    }
    if (cap) break;
    a = b;
  }
  return rows;
}

int ro_kerr_chain(const double* bh, const double* o, const double* d, double* out, int max_rows, double* frame) {
  return ro_kerr_chain_st(bh, o, d, out, max_rows, frame, 1.0, NULL);
}
/* The shadow query of the ray (o, d) -- BVHAccel::intersect's boolean (bvh.cpp:103-113) -- with the
 * spacetime of params p (Schwarzschild stepper or the Kerr march).  Sweep checks of the proofs. */
int ro_shadow_query(const ro_scene* s, const ro_params* p, const double* o, const double* d) {
  rng_t g; memset(&g, 0, sizeof(g));
  qctx q; q.s = s; q.g = &g;
  if (p->bh_kind == 1) {
    hole_init_kerr(&q.hole, p->bh_center, p->bh_radius, p->bh_dtheta, p->bh_spin, p->bh_axis);
    kerr_set_escape(&q.hole, s->nodes[0].mn, s->nodes[0].mx);
  } else hole_init(&q.hole, p->bh_center, p->bh_radius, p->bh_dtheta);
  isect_t is; memset(&is, 0, sizeof(is));
  return bvh_intersect(&q, V(o[0], o[1], o[2]), V(d[0], d[1], d[2]), &is);
}
/* The closest-hit query (BVHAccel::intersect with an Intersection, bvh.cpp:103-113) of one ray:
 * returns hit (0/1) and out[0..2] hit_p, out[3..5] n, out[6] bsdf (test infrastructure: the camera
 * hit proof's checks, tests/hit_proof_sim.py) */
int ro_query(const ro_scene* s, const ro_params* p, const double* o, const double* d, double* out) {
  rng_t g; memset(&g, 0, sizeof(g));
  qctx q; q.s = s; q.g = &g;
  if (p->bh_kind == 1) {
    hole_init_kerr(&q.hole, p->bh_center, p->bh_radius, p->bh_dtheta, p->bh_spin, p->bh_axis);
    kerr_set_escape(&q.hole, s->nodes[0].mn, s->nodes[0].mx);
  } else hole_init(&q.hole, p->bh_center, p->bh_radius, p->bh_dtheta);
  isect_t is; memset(&is, 0, sizeof(is));
  const int hit = bvh_intersect(&q, V(o[0], o[1], o[2]), V(d[0], d[1], d[2]), &is);
  out[0] = is.hit_p.x; out[1] = is.hit_p.y; out[2] = is.hit_p.z;
  out[3] = is.n.x; out[4] = is.n.y; out[5] = is.n.z; out[6] = is.bsdf;
  return hit;
}
int ro_micro_chain(const double* bh, const double* o, const double* d, double* out, int max_rows) {
  hole_t h; hole_init(&h, bh, bh[3], bh[4]);
  ray_t m; m.o = V(o[0], o[1], o[2]); m.d = V(d[0], d[1], d[2]); m.min_t = 0; m.max_t = 0;
  int rows = 0;
  for (int j = 0; j < h.steps && rows < max_rows; ++j) {
    m = next_micro_ray(&h, &m);
    ray_t probe = m;
    int cap = sphere_hit(h.c, h.r2, &probe, NULL, -1);
    double* r = out + 8 * rows++;
    r[0] = m.o.x; r[1] = m.o.y; r[2] = m.o.z; r[3] = m.d.x; r[4] = m.d.y; r[5] = m.d.z; r[6] = m.max_t; r[7] = cap;
    if (cap) break;
  }
  return rows;
}
int ro_bbox_intersect(const double* mn, const double* mx, const double* o, const double* d, double min_t,
                      double max_t, double* t0, double* t1) {
  ray_t r; r.o = V(o[0], o[1], o[2]); r.d = V(d[0], d[1], d[2]); r.min_t = min_t; r.max_t = max_t;
  return bbox_hit(V(mn[0], mn[1], mn[2]), V(mx[0], mx[1], mx[2]), &r, t0, t1);
}
int ro_tri_intersect(const double* p, const double* n, const double* o, const double* d, double* max_t,
                     double* hit_p, double* nrm) {
  ray_t r; r.o = V(o[0], o[1], o[2]); r.d = V(d[0], d[1], d[2]); r.min_t = 0; r.max_t = *max_t;
  isect_t is;
  int hit = tri_hit(V(p[0], p[1], p[2]), V(p[3], p[4], p[5]), V(p[6], p[7], p[8]), V(n[0], n[1], n[2]),
                    V(n[3], n[4], n[5]), V(n[6], n[7], n[8]), &r, &is, 0);
  *max_t = r.max_t;
  if (hit) {
    hit_p[0] = is.hit_p.x; hit_p[1] = is.hit_p.y; hit_p[2] = is.hit_p.z;
    nrm[0] = is.n.x; nrm[1] = is.n.y; nrm[2] = is.n.z;
  }
  return hit;
}
int ro_sphere_intersect(const double* c, double rad, const double* o, const double* d, double* max_t,
                        double* hit_p, double* nrm, int want_isect) {
  ray_t r; r.o = V(o[0], o[1], o[2]); r.d = V(d[0], d[1], d[2]); r.min_t = 0; r.max_t = *max_t;
  isect_t is;
  int hit = sphere_hit(V(c[0], c[1], c[2]), rad * rad, &r, want_isect ? &is : NULL, 0);
  *max_t = r.max_t;
  if (hit && want_isect) {
    hit_p[0] = is.hit_p.x; hit_p[1] = is.hit_p.y; hit_p[2] = is.hit_p.z;
    nrm[0] = is.n.x; nrm[1] = is.n.y; nrm[2] = is.n.z;
  }
  return hit;
}
void ro_coord_space(const double* n, const double* v, double* o2w, double* a, double* b) {
  v3 X, Y, Z; coord_space(V(n[0], n[1], n[2]), &X, &Y, &Z);
  double m[9] = {X.x, X.y, X.z, Y.x, Y.y, Y.z, Z.x, Z.y, Z.z};
  memcpy(o2w, m, sizeof(m));
  v3 vv = V(v[0], v[1], v[2]);
  v3 l = to_local(X, Y, Z, vv), w = to_world(X, Y, Z, vv);
  a[0] = l.x; a[1] = l.y; a[2] = l.z; b[0] = w.x; b[1] = w.y; b[2] = w.z;
}
void ro_sampler(int kind, const int* rands, double* out, float* pdf, int* used) {
  rng_t g; memset(&g, 0, sizeof(g)); g.script = rands; g.script_len = 2;
  v3 r = V(0, 0, 0); *pdf = 0;
  if (kind == 0) { double x, y; grid_sample(&g, &x, &y); r = V(x, y, 0); }
  else if (kind == 1) r = cosine_sample(&g, pdf);
  else if (kind == 2) r = hemisphere_sample(&g);
  else r = sphere_sample(&g);
  out[0] = r.x; out[1] = r.y; out[2] = r.z; *used = (int)g.ctr;
}
void ro_bsdf_sample(int kind, const double* prm, const double* wo, const int* rands, float* f3, double* wi,
                    float* pdf, int* used, float* fe3) {
  bsdf_t b; memset(&b, 0, sizeof(b));
  float s1[3] = {(float)prm[0], (float)prm[1], (float)prm[2]}, s2[3] = {(float)prm[3], (float)prm[4], (float)prm[5]};
  switch (kind) {
    case 0: b.type = BSDF_DIFFUSE; memcpy(b.p, s1, 12); break;
    case 1: b.type = BSDF_MIRROR; memcpy(b.p, s1, 12); break;
    case 2: b.type = BSDF_GLASS; memcpy(b.p, s1, 12); memcpy(b.p + 3, s2, 12); b.p[6] = (float)prm[6]; b.p[7] = (float)prm[7]; break;
    case 3: b.type = BSDF_MICROFACET; memcpy(b.p, s1, 12); memcpy(b.p + 3, s2, 12); b.p[6] = (float)(prm[6] * 0.6); break;
    default: b.type = BSDF_EMISSION; memcpy(b.p, s1, 12); break;
  }
  rng_t g; memset(&g, 0, sizeof(g)); g.script = rands; g.script_len = 3;
  v3 w = V(wo[0], wo[1], wo[2]), wiv = V(0, 0, 0);
  *pdf = -1;
  spec f = bsdf_sample_f(&b, &g, w, &wiv, pdf);
  f3[0] = f.r; f3[1] = f.g; f3[2] = f.b;
  wi[0] = wiv.x; wi[1] = wiv.y; wi[2] = wiv.z;
  *used = (int)g.ctr;
  spec fe = (kind == 3 && *pdf != 0) ? bsdf_f(&b, w, wiv) : S(0, 0, 0);
  fe3[0] = fe.r; fe3[1] = fe.g; fe3[2] = fe.b;
}
void ro_area_sample(const float* rad, const double* v, const double* p, const int* rands, float* L, double* wi,
                    float* dist, float* pdf) {
  light_t l; memset(&l, 0, sizeof(l));
  l.type = 0; l.rad[0] = rad[0]; l.rad[1] = rad[1]; l.rad[2] = rad[2];
  for (int k = 0; k < 4; ++k) l.v[k] = V(v[3 * k], v[3 * k + 1], v[3 * k + 2]);
  l.area = (float)(vnorm(l.v[2]) * vnorm(l.v[3])); /* light.cpp:78 */
  rng_t g; memset(&g, 0, sizeof(g)); g.script = rands; g.script_len = 2;
  v3 w;
  spec s = light_sample_L(NULL, &l, &g, V(p[0], p[1], p[2]), &w, dist, pdf);
  L[0] = s.r; L[1] = s.g; L[2] = s.b; wi[0] = w.x; wi[1] = w.y; wi[2] = w.z;
}
/* point (1) / directional (2) / infinite hemisphere (3) lights' sample_L (light.cpp:17-57) */
void ro_light_sample(int type, const float* rad, const double* v, const double* p, const int* rands, float* L,
                     double* wi, float* dist, float* pdf, int* used) {
  light_t l; memset(&l, 0, sizeof(l));
  l.type = (uint32_t)type; l.rad[0] = rad[0]; l.rad[1] = rad[1]; l.rad[2] = rad[2];
  for (int k = 0; k < 4; ++k) l.v[k] = V(v[3 * k], v[3 * k + 1], v[3 * k + 2]);
  rng_t g; memset(&g, 0, sizeof(g)); g.script = rands; g.script_len = 2;
  v3 w;
  spec s = light_sample_L(NULL, &l, &g, V(p[0], p[1], p[2]), &w, dist, pdf);
  L[0] = s.r; L[1] = s.g; L[2] = s.b; wi[0] = w.x; wi[1] = w.y; wi[2] = w.z;
  *used = (int)g.ctr;
}
void ro_camera_ray(double hFov, double vFov, const double* pos, const double* c2w, double nClip, double fClip,
                   double x, double y, double* o, double* d, double* min_t, double* max_t) {
  pctx c; memset(&c, 0, sizeof(c));
  c.cam_pos = V(pos[0], pos[1], pos[2]);
  c.c2w0 = V(c2w[0], c2w[1], c2w[2]); c.c2w1 = V(c2w[3], c2w[4], c2w[5]); c.c2w2 = V(c2w[6], c2w[7], c2w[8]);
  c.blx = -tan(hFov * (PI_D / 180) / 2);
  c.bly = -tan(vFov * (PI_D / 180) / 2);
  v3 oo, dd;
  gen_ray(&c, x, y, &oo, &dd);
  o[0] = oo.x; o[1] = oo.y; o[2] = oo.z; d[0] = dd.x; d[1] = dd.y; d[2] = dd.z;
  *min_t = nClip; *max_t = fClip;
}

/* ------------------------------------------------------------------ the host C library itself */
/* The reference's transcendentals as the reference gets them: straight from this machine's libm
 * (glibc).  tests/test_gpu_glibm.py compares the device restatement (rrt_libm_eval) with these.
 * fn: 0 sin, 1 cos, 2 acos, 3 atan2(a, b), 4 sinf((float)a), 5 cosf((float)a). */
void ro_libm_eval(int fn, const double* a, const double* b, double* out, long n) {
  for (long k = 0; k < n; ++k) {
    switch (fn) {
      case 0: out[k] = sin(a[k]); break;
      case 1: out[k] = cos(a[k]); break;
      case 2: out[k] = acos(a[k]); break;
      case 3: out[k] = atan2(a[k], b[k]); break;
      case 4: out[k] = sinf((float)a[k]); break;
      case 5: out[k] = cosf((float)a[k]); break;
      case 6: out[k] = exp(a[k]); break;
      case 7: out[k] = log(a[k]); break;
      case 8: out[k] = erf(a[k]); break;
      case 9: out[k] = atan(a[k]); break;
      default: out[k] = tan(a[k]); break;
    }
  }
}
