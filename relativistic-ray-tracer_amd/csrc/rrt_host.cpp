// rrt_host.cpp -- C ABI (include/rrt.h): scene flattening, the reference BVH build, camera and
// spacetime set-up, HBM residency and kernel launches.
//
// Host-side work the reference does once per frame (PathTracer::set_scene -> build_accel,
// pathtracer.cpp:95-117, 304-328; BVHAccel::construct_bvh, bvh.cpp:49-96) is reproduced in C++
// here with the reference's arithmetic (std::min/max, centroid = (min + max) * (1.0 / 2)), so the
// BVH is node-for-node the reference's; it is then laid out for the GPU (rrt_internal.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#if RRT_PROFILE
#include <chrono>
#include <cstdlib>
#include <thread>
#include <unistd.h>
#endif

#include "../../include/rrt.h"
#include "../../include/rrt_scene_format.h"
#include "rrt_internal.h"
#include "rrt_scene_file.h"

hipError_t rrt_launch_render(const KParams& kp, const KParams* d_kp, int deep, int count, int lean, int waves, uint32_t grid,
                             hipStream_t stream);
hipError_t rrt_launch_sample(const KParams& kp, const KParams* d_kp, int count, int lean, int waves, uint32_t grid, hipStream_t stream);
hipError_t rrt_launch_batch(const KParams& kp, const KParams* d_kp, int lean, int waves, uint32_t grid, hipStream_t stream);
hipError_t rrt_launch_first(const KParams& kp, const KParams* d_kp, int lean, int waves, uint32_t grid, hipStream_t stream);
hipError_t rrt_launch_pixel_proof(const KParams* d_kp, uint32_t n_pixels, bool strips, hipStream_t stream);
hipError_t rrt_launch_heavy(const KParams* d_kp, int lean, int waves, int nw, uint32_t grid, int drain, hipStream_t stream);
hipError_t rrt_launch_path(const KParams* d_kp, int waves, uint32_t grid, hipStream_t stream);
hipError_t rrt_launch_unpack(const uint32_t* tiles, uint32_t n_tiles, uint32_t ts, uint32_t fw, uint32_t fh,
                             const float* rgb_p, const int32_t* cnt_p, float* rgb, int32_t* cnt, hipStream_t stream);
hipError_t rrt_launch_libm(int fn, uint64_t n, const double* a, const double* b, double* out, hipStream_t stream);
hipError_t rrt_launch_tonemap(uint32_t n, const float* rgb, uint32_t* out, float exposure, float inv_gamma,
                              hipStream_t stream);

namespace {

constexpr double kPI = 3.14159265358979323;  // CGL misc.h:11
// claim counters + the pixel proof's list length + the heavy list's + the continuation queue's
constexpr size_t kCounterBytes = sizeof(uint32_t) * RRT_QUEUE_STRIDE * (RRT_MAX_QUEUES + 2 + RRT_CONT_WORDS);
// Heavy pixels (rrt_sample.hip heavy_pixel_block): rays passing within RRT_HEAVY_NEAR r_s of the hole (or straddling
// its capture boundary) make a pixel heavy (profiles/r03_heavy_ab.md)
#define RRT_HEAVY_NEAR 1.2
// Kerr occlusion proof (rrt_device.h kerr_occluded_proof): coarse steps RRT_KPROOF_STRETCH times the
// march's, no proof within RRT_KPROOF_NEAR_M M of the hole, crossing margin RRT_KPROOF_DELTA_M M;
// on for holes with delta_theta in [DT_MIN, DT_MAX], a/M <= SPIN_MAX and every root-box corner
// within REACH_M M -- the envelope tools/kerr_proof_sweep.py swept (tests/test_kerr_proof.py)
#define RRT_KPROOF_STRETCH 4.0
#define RRT_KPROOF_NEAR_M 6.0
#define RRT_KPROOF_DELTA_M 0.25
#define RRT_KPROOF_DT_MIN 0.02
#define RRT_KPROOF_DT_MAX 0.1
#define RRT_KPROOF_SPIN_MAX 0.99
#define RRT_KPROOF_REACH_M 40.0
#define RRT_KPROOF_CENTRE_LO 0.2
#define RRT_KPROOF_CENTRE_HI 0.8
#define RRT_KPROOF_RS_LO 0.04
#define RRT_KPROOF_RS_HI 0.15

struct V3 { double x, y, z; };
inline V3 mk(double x, double y, double z) { return V3{x, y, z}; }
inline V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline double get(V3 a, int k) { return k == 0 ? a.x : k == 1 ? a.y : a.z; }
inline double smin(double a, double b) { return (b < a) ? b : a; }  // std::min
inline double smax(double a, double b) { return (a < b) ? b : a; }  // std::max

struct Box {
  V3 mx, mn, ext;
  static Box empty() {
    Box b; b.mx = mk(-INFINITY, -INFINITY, -INFINITY); b.mn = mk(INFINITY, INFINITY, INFINITY); b.ext = sub(b.mx, b.mn);
    return b;
  }
  static Box point(V3 p) { Box b; b.mn = p; b.mx = p; b.ext = sub(b.mx, b.mn); return b; }
  void expand(V3 p) {
    mn.x = smin(mn.x, p.x); mn.y = smin(mn.y, p.y); mn.z = smin(mn.z, p.z);
    mx.x = smax(mx.x, p.x); mx.y = smax(mx.y, p.y); mx.z = smax(mx.z, p.z);
    ext = sub(mx, mn);
  }
  void expand(const Box& o) {
    mn.x = smin(mn.x, o.mn.x); mn.y = smin(mn.y, o.mn.y); mn.z = smin(mn.z, o.mn.z);
    mx.x = smax(mx.x, o.mx.x); mx.y = smax(mx.y, o.mx.y); mx.z = smax(mx.z, o.mx.z);
    ext = sub(mx, mn);
  }
  V3 centroid() const {  // (min + max) / 2 with Vector3D::operator/ (rc = 1.0 / c)
    const double rc = 1.0 / 2;
    V3 s = add(mn, mx);
    return mk(rc * s.x, rc * s.y, rc * s.z);
  }
};

struct Prim {  // build-order primitive
  uint32_t kind, bsdf;
  uint32_t v[3];       // triangle: global vertex indices
  V3 c; double r, r2;  // sphere
};

struct BNode { Box bb; int32_t first, count, left, right, skip; };

}  // namespace

struct rrt_ctx {
  int device = -1;
  std::string err;
  hipStream_t stream = nullptr;
  // per-launch timing ring: ev0 before the launch, ev_main before its main kernel (after any
  // pre-pass), ev1 after it; slot = launch number % kRing
  static constexpr uint32_t kRing = 32;
  hipEvent_t ev0[kRing] = {}, ev_main[kRing] = {}, ev1[kRing] = {};
  uint64_t n_launch = 0;
  // scratch fence: every launch and unpack rewrites the per-context workspace below (KParams,
  // claim counters, tile list/order, sample-0 slots) with async copies on the caller's stream;
  // a use on a different stream than the previous one first waits for this event
  hipEvent_t ev_fence = nullptr;
  hipStream_t fence_stream = nullptr;
  // heavy pixels (rrt_pixel_proof_kernel's heavy list, taken first by the batch kernel's waves)
  uint32_t* d_heavy_list = nullptr;
  uint32_t* d_strip_list = nullptr;  // the pixel pass's strips left to the per-pixel level
  unsigned long long* d_audit = nullptr;  // proof-audit tallies (rrt_set_proof_audit), 16 64-bit words
  uint32_t audit_shift = 0;          // 0: no audit; else re-check every 2^(audit_shift - 1)-th proven ray
  size_t strip_list_cap = 0;
  size_t heavy_list_cap = 0;
  ContRec* d_cont = nullptr;  // continuation records (rrt_sample.hip cont_push)
  size_t cont_cap = 0;
  uint32_t cont_seq = 0;      // the last launch's record tag (never 0)
  float* d_path_stack = nullptr;  // the path pool kernel's per-level terms (rrt_path.hip)
  size_t path_stack_cap = 0;      // bytes
  hipStream_t side = nullptr;  // the heavy pixels' kernel runs here, beside the batch kernel
  hipEvent_t ev_go = nullptr, ev_heavy = nullptr;
#if RRT_PROFILE
  uint32_t* h_wd = nullptr;  // watchdog progress records (host-coherent, RRT_WATCHDOG_MS)
  uint32_t* d_wd = nullptr;
#endif
  bool fenced = false;
  int n_cu = 256;
  // host scene
  std::vector<V3> pos, nrm;
  std::vector<Prim> prims;
  std::vector<BNode> nodes;
  std::vector<uint32_t> leaf;
  uint32_t max_depth = 0;
  bool fast_div = false;  // every BVH coordinate is 0 or in [2^-800, 2^20] (qdiv, rrt_device.h)
  int lean = 0;           // LEAN kernel builds: 1 area lights only, 2 area + point lights; no microfacet BSDF
  uint32_t grid_res = 128;  // empty-space grid cells along the longest root-box axis (<= 1: none)
  std::vector<uint8_t> grid;
  DGrid hgrid{};           // host copy (k = nullptr)
  std::vector<DBsdf> bsdfs;
  std::vector<DLight> lights;  // the scene's lights (the environment light is appended on upload)
  // environment map (rrt_set_envmap): texels and EnvironmentLight::init's tables, host + device
  uint32_t env_w = 0, env_h = 0;
  std::vector<float> env_tex;
  std::vector<double> env_pdf, env_conds, env_marg;
  float* d_env_tex = nullptr;
  double* d_env_pdf = nullptr;
  double* d_env_conds = nullptr;
  double* d_env_marg = nullptr;
  bool has_scene = false, has_camera = false;
  DCamera cam{};
  double lens_r = 0.0, focal = 0.0;  // Camera::lensRadius / focalDistance (thin lens, RRT_RENDER_THIN_LENS)
  DHole hole{};
  // device scene
  DNode* d_nodes = nullptr;
  DPrimGeo* d_geo = nullptr;
  DPrimNrm* d_nrm = nullptr;
  DPrimMeta* d_meta = nullptr;
  DBsdf* d_bsdfs = nullptr;
  DLight* d_lights = nullptr;
  uint8_t* d_grid = nullptr;
  DNode* d_clean = nullptr;
  DPlane* d_planes = nullptr;
  double plane_eps = 0;
  DBig* d_big = nullptr;
  int32_t clean_root = -1;
  uint32_t n_big = 0;
  bool has_clean = false;
  std::vector<DNode> clean;  // host copies (rrt_get_clean_tree)
  std::vector<DBig> big;
  std::vector<uint32_t> big_mask;   // build_big_masks (host copy; rrt_get_big_masks)
  std::vector<DNode> free_tree;     // build_free_tree: SAH hierarchy over the clean tree's leaves
  std::vector<DNode4> free4;        // build_free4: the same hierarchy 4 wide (empty: none)
  DNode4* d_free4 = nullptr;
  double free4_omax = 0.0;
  uint64_t free_big_mask = ~0ull;   // oversized leaves the search-tree walk still tests from its list
  DNode* d_free = nullptr;
  DShadowProof occ{};               // build_occluders (the root box's face triangles)
  DOccQuad occ_quad[6][RRT_OCC_PER_FACE]{};  // the same triangles, coplanar pairs merged (Kerr proof)
  uint32_t occ_nq[6]{};
  uint32_t* d_big_mask = nullptr;
  uint64_t device_bytes = 0;
  // per-launch workspace
  KParams* d_kp = nullptr;  // the launch's parameters (kernels take them by pointer)
  uint32_t* d_counter = nullptr;
  uint32_t* d_tiles = nullptr;
  size_t tiles_cap = 0;
  uint32_t* d_order = nullptr;  // batch kernel: tile claim order
  size_t order_cap = 0;
  std::vector<uint32_t> h_order;  // what d_order holds
  KParams::FirstSample* d_first = nullptr;  // batch kernel: sample 0 per pixel slot
  uint32_t* d_list = nullptr;  // batch kernel: the pixel proof's claim list
  size_t list_cap = 0;
  size_t first_cap = 0;
  float* d_rgb = nullptr; int32_t* d_cnt = nullptr; uint32_t* d_draws = nullptr; uint32_t* d_ctr = nullptr;
  size_t px_cap = 0;
  float last_ms = 0.f, last_main_ms = 0.f;
  bool timed = false;
  uint32_t last_grid = 0;
  uint32_t last_heavy = 0;  // the last launch's heavy-list capacity (0: no heavy path)
  uint32_t last_cont = 0;   // the last launch's continuation capacity (0: none)
  std::string last_kernel;
};

static int fail(rrt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(c, x)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(c, RRT_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

static void free_env_dev(rrt_ctx* c) {
  if (c->device < 0) return;
  hipFree(c->d_env_tex); hipFree(c->d_env_pdf); hipFree(c->d_env_conds); hipFree(c->d_env_marg);
  c->d_env_tex = nullptr; c->d_env_pdf = nullptr; c->d_env_conds = nullptr; c->d_env_marg = nullptr;
}

static void free_scene_dev(rrt_ctx* c) {
  if (c->device < 0) return;
  hipFree(c->d_nodes); hipFree(c->d_geo); hipFree(c->d_nrm); hipFree(c->d_meta); hipFree(c->d_bsdfs);
  hipFree(c->d_lights); hipFree(c->d_grid); hipFree(c->d_clean); hipFree(c->d_big); hipFree(c->d_planes);
  hipFree(c->d_big_mask);
  hipFree(c->d_free);
  c->d_free = nullptr;
  hipFree(c->d_free4);
  c->d_free4 = nullptr;
  c->d_grid = nullptr; c->d_clean = nullptr; c->d_big = nullptr; c->d_planes = nullptr; c->d_big_mask = nullptr;
  c->d_nodes = nullptr; c->d_geo = nullptr; c->d_nrm = nullptr; c->d_meta = nullptr; c->d_bsdfs = nullptr;
  c->d_lights = nullptr;
  c->device_bytes = 0;
}


// The heavy pixels' stream: a high-priority stream, on a hardware queue of its own, so its kernel
// runs beside the batch kernel (a CU-masked stream ran it behind the batch kernel: cfg3 23.9 ms
// against 19.4 ms for a plain or a high-priority stream).
static bool create_side_stream(rrt_ctx* c) {
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return false;
  return hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi) == hipSuccess;
}

static bool create_ring(rrt_ctx* c) {
  for (uint32_t i = 0; i < rrt_ctx::kRing; ++i)
    if (hipEventCreate(&c->ev0[i]) != hipSuccess || hipEventCreate(&c->ev_main[i]) != hipSuccess ||
        hipEventCreate(&c->ev1[i]) != hipSuccess)
      return false;
  return true;
}

extern "C" {

int rrt_abi_version(void) { return RRT_ABI_VERSION; }

int rrt_create(rrt_ctx** out, const rrt_device_cfg* cfg) {
  if (!out) return RRT_E_INVALID;
  std::unique_ptr<rrt_ctx> c(new rrt_ctx());
  c->device = cfg ? cfg->device : 0;
  if (cfg && cfg->free_grid_res) c->grid_res = std::min<uint32_t>(cfg->free_grid_res, 1024);
  // default spacetime: global_black_hole (blackhole.cpp:5)
  rrt_spacetime_desc st{};
  st.kind = RRT_METRIC_SCHWARZSCHILD; st.center[1] = 1.0; st.r_s = 0.1; st.delta_theta = 0.1;
  if (c->device >= 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= c->device) { *out = nullptr; return RRT_E_NO_DEVICE; }
    if (hipSetDevice(c->device) != hipSuccess) { *out = nullptr; return RRT_E_HIP; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        !create_ring(c.get()) ||
        hipEventCreateWithFlags(&c->ev_fence, hipEventDisableTiming) != hipSuccess ||
        !create_side_stream(c.get()) ||
        hipEventCreateWithFlags(&c->ev_go, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_heavy, hipEventDisableTiming) != hipSuccess ||

        hipMalloc(&c->d_counter, kCounterBytes) != hipSuccess || hipMalloc(&c->d_kp, sizeof(KParams)) != hipSuccess) {
      *out = nullptr;
      return RRT_E_HIP;
    }
  }
  rrt_set_spacetime(c.get(), &st);
  *out = c.release();
  return RRT_OK;
}

void rrt_destroy(rrt_ctx* c) {
  if (!c) return;
  if (c->device >= 0) {
    hipSetDevice(c->device);
    free_scene_dev(c);
    free_env_dev(c);
    hipFree(c->d_counter); hipFree(c->d_kp); hipFree(c->d_tiles); hipFree(c->d_order); hipFree(c->d_first); hipFree(c->d_list); hipFree(c->d_rgb); hipFree(c->d_cnt); hipFree(c->d_draws);
    hipFree(c->d_ctr);
    hipFree(c->d_heavy_list);
    hipFree(c->d_strip_list);
    hipFree(c->d_audit);
    hipFree(c->d_cont);
    hipFree(c->d_path_stack);
    for (uint32_t i = 0; i < rrt_ctx::kRing; ++i) {
      if (c->ev0[i]) hipEventDestroy(c->ev0[i]);
      if (c->ev_main[i]) hipEventDestroy(c->ev_main[i]);
      if (c->ev1[i]) hipEventDestroy(c->ev1[i]);
    }
    if (c->ev_fence) hipEventDestroy(c->ev_fence);
    if (c->ev_go) hipEventDestroy(c->ev_go);
    if (c->ev_heavy) hipEventDestroy(c->ev_heavy);
    if (c->side) hipStreamDestroy(c->side);

    if (c->stream) hipStreamDestroy(c->stream);
  }
  delete c;
}

const char* rrt_last_error(const rrt_ctx* c) { return c ? c->err.c_str() : "null context"; }

void rrt_render_params_default(rrt_render_params* p) {  // AppConfig defaults, application.h:45-62
  std::memset(p, 0, sizeof(*p));
  p->ns_aa = 1; p->max_ray_depth = 1; p->ns_area_light = 1; p->samples_per_batch = 32;
  p->max_tolerance = 0.05f; p->direct_hemisphere = 0; p->seed = 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------- BVH build
static Box prim_box(const rrt_ctx* c, const Prim& p) {
  if (p.kind == RRT_OBJ_MESH) {  // Triangle::get_bbox (triangle.cpp:11-19)
    Box b = Box::point(c->pos[p.v[0]]);
    b.expand(c->pos[p.v[1]]);
    b.expand(c->pos[p.v[2]]);
    return b;
  }
  Box b;  // Sphere::get_bbox (sphere.h:30-32)
  b.mn = sub(p.c, mk(p.r, p.r, p.r)); b.mx = add(p.c, mk(p.r, p.r, p.r)); b.ext = sub(b.mx, b.mn);
  return b;
}

// BVHAccel::construct_bvh (bvh.cpp:49-96): leaf if <= max_leaf_size (4); split at the bbox
// centroid of the strictly longest axis (ties -> z); centroid < c goes left; if one side is
// empty, split the list in halves.  Emitted in left-first pre-order.
static int build(rrt_ctx* c, const std::vector<uint32_t>& ids, uint32_t depth) {
  Box bb = Box::empty();
  for (uint32_t id : ids) bb.expand(prim_box(c, c->prims[id]));
  int me = (int)c->nodes.size();
  c->nodes.push_back(BNode{bb, 0, 0, -1, -1, -1});
  c->max_depth = std::max(c->max_depth, depth);
  if (ids.size() <= 4) {
    c->nodes[me].first = (int32_t)c->leaf.size();
    c->nodes[me].count = (int32_t)ids.size();
    c->leaf.insert(c->leaf.end(), ids.begin(), ids.end());
    return me;
  }
  std::vector<uint32_t> L, R;
  int axis = (bb.ext.x > bb.ext.y && bb.ext.x > bb.ext.z) ? 0 : (bb.ext.y > bb.ext.x && bb.ext.y > bb.ext.z) ? 1 : 2;
  V3 cc = bb.centroid();
  double cv = axis == 0 ? cc.x : axis == 1 ? cc.y : cc.z;
  for (uint32_t id : ids) {
    V3 pc = prim_box(c, c->prims[id]).centroid();
    double v = axis == 0 ? pc.x : axis == 1 ? pc.y : pc.z;
    (v < cv ? L : R).push_back(id);
  }
  if (L.empty() || R.empty()) {
    L.assign(ids.begin(), ids.begin() + ids.size() / 2);
    R.assign(ids.begin() + ids.size() / 2, ids.end());
  }
  int l = build(c, L, depth + 1);
  int r = build(c, R, depth + 1);
  c->nodes[me].left = l;
  c->nodes[me].right = r;
  return me;
}

// Empty-space grid (DGrid, rrt_internal.h).  Cubic cells of size h over the root box.  A cell is
// "occupied" if some primitive could report a hit for a segment passing through it:
//  * sphere: its bounding box;
//  * triangle: the part of its leaf's box within one cell of the triangle's plane.  In exact
//    arithmetic a hit lies on the triangle; in floating point Triangle::intersect can also
//    accept a segment that is parallel to the plane to within rounding (det, t and both
//    barycentric numerators all vanish), anywhere along the plane -- but only inside the leaf
//    box, because the leaf's slab test gates every primitive test;
//  * sliver triangle (|e1 x e2| < 1e-6 |e1| |e2|): its whole leaf box.
// Every range is widened by one cell per side.  A multi-source BFS over the 26-neighbourhood
// then gives each cell its Chebyshev distance k (in cells, capped at 255) to the nearest
// occupied cell.  A point p whose computed cell is c lies in a true cell c* with |c - c*| <= 1
// (rounding of (p - g0) / h); any point q of a hit region lies in an occupied cell c_q, so
// |c* - c_q|_inf >= k - 1 and |p - q| >= |p - q|_inf >= (k - 2) h.  A segment shorter than that
// stays about a cell (~1e13 ulps) away from every hit region, so no primitive accepts it.
// Mark the grid cells (geometry g0, h, n) holding a hit region of the leaf's primitives: for a
// sphere its box, for a triangle the cells of its leaf box (widened by one) whose centre lies
// within one cell of its plane (all of them for slivers).  False if a box is not finite.
template <class F>
static bool grid_mark_leaf(const rrt_ctx* c, const double g0[3], double h, const int32_t n[3], const Box& leaf_bb,
                           int first, int count, F&& mark) {
  const double inv_h = 1.0 / h;
  auto range = [&](const V3& mn, const V3& mx, int lo[3], int hi[3]) {  // widened by one cell
    const double a[3] = {mn.x, mn.y, mn.z}, b[3] = {mx.x, mx.y, mx.z};
    for (int i = 0; i < 3; ++i) {
      if (!std::isfinite(a[i]) || !std::isfinite(b[i])) return false;
      lo[i] = std::max(0, (int)std::floor((a[i] - g0[i]) * inv_h) - 1);
      hi[i] = std::min(n[i] - 1, (int)std::floor((b[i] - g0[i]) * inv_h) + 1);
    }
    return true;
  };
  const double reach = h * (std::sqrt(3.0) / 2 + 1.0);  // cell centre to plane: within one cell
  int llo[3], lhi[3];
  if (!range(leaf_bb.mn, leaf_bb.mx, llo, lhi)) return false;
  for (int j = 0; j < count; ++j) {
    const Prim& p = c->prims[c->leaf[first + j]];
    int lo[3], hi[3];
    if (p.kind == RRT_OBJ_SPHERE) {
      const Box b = prim_box(c, p);
      if (!range(b.mn, b.mx, lo, hi)) return false;
      for (int z = lo[2]; z <= hi[2]; ++z)
        for (int y = lo[1]; y <= hi[1]; ++y)
          for (int x = lo[0]; x <= hi[0]; ++x) mark(x, y, z);
      continue;
    }
    const V3 p0 = c->pos[p.v[0]], e1 = sub(c->pos[p.v[1]], p0), e2 = sub(c->pos[p.v[2]], p0);
    const V3 nn = mk(e1.y * e2.z - e1.z * e2.y, e1.z * e2.x - e1.x * e2.z, e1.x * e2.y - e1.y * e2.x);
    const double nl = std::sqrt(nn.x * nn.x + nn.y * nn.y + nn.z * nn.z);
    const double l1 = std::sqrt(e1.x * e1.x + e1.y * e1.y + e1.z * e1.z);
    const double l2 = std::sqrt(e2.x * e2.x + e2.y * e2.y + e2.z * e2.z);
    const bool sliver = !(nl >= 1e-6 * l1 * l2) || !std::isfinite(nl);
    for (int z = llo[2]; z <= lhi[2]; ++z)
      for (int y = llo[1]; y <= lhi[1]; ++y)
        for (int x = llo[0]; x <= lhi[0]; ++x) {
          if (!sliver) {
            const double cx = g0[0] + (x + 0.5) * h, cy = g0[1] + (y + 0.5) * h, cz = g0[2] + (z + 0.5) * h;
            const double dist = std::fabs(nn.x * (cx - p0.x) + nn.y * (cy - p0.y) + nn.z * (cz - p0.z)) / nl;
            if (dist > reach) continue;
          }
          mark(x, y, z);
        }
  }
  return true;
}

// Shadow-ray occlusion proof (rrt_device.h shadow_occluded_proof): the large triangles within 1%
// of the scene's extent of a root-box face and facing along its axis (walls; CBempty's back wall
// sits 0.2% inside the box), taken as the reference intersects them (p0, p0 + e1, p0 + e2),
// largest first, RRT_OCC_PER_FACE per face, none under 5% of the face's largest: plane (normal
// toward the box's inside) and in-plane edge normals.  Any triangle of the scene would do (a certain crossing of any of them is
// a reference hit); these are the ones a shadow ray leaving a closed room crosses last.
static void build_occluders(rrt_ctx* c) {
  DShadowProof& o = c->occ;
  o = DShadowProof{};
  std::memset(c->occ_nq, 0, sizeof(c->occ_nq));
  if (c->nodes.empty()) return;
  const Box& rb = c->nodes[0].bb;
  const double lo[3] = {rb.mn.x, rb.mn.y, rb.mn.z}, hi[3] = {rb.mx.x, rb.mx.y, rb.mx.z};
  double sc = 0.0;
  for (int k = 0; k < 3; ++k) sc = std::max(sc, hi[k] - lo[k]);
  if (!(sc > 0.0) || !std::isfinite(sc)) return;
  const double tol = 1e-2 * sc;
  struct Cand { double area, w; DOccluder t; V3 v[3]; uint32_t prim; };
  std::vector<Cand> cand[6];
  for (uint32_t pi = 0; pi < (uint32_t)c->prims.size(); ++pi) {
    const Prim& p = c->prims[pi];
    if (p.kind != RRT_OBJ_MESH) continue;
    const V3 p0 = c->pos[p.v[0]], e1 = sub(c->pos[p.v[1]], p0), e2 = sub(c->pos[p.v[2]], p0);
    const V3 q[3] = {p0, add(p0, e1), add(p0, e2)};
    const V3 nn = mk(e1.y * e2.z - e1.z * e2.y, e1.z * e2.x - e1.x * e2.z, e1.x * e2.y - e1.y * e2.x);
    const double nl = std::sqrt(nn.x * nn.x + nn.y * nn.y + nn.z * nn.z);
    if (!(nl > 0.0) || !std::isfinite(nl)) continue;
    for (int f = 0; f < 6; ++f) {
      const int k = f % 3;
      const double face = f < 3 ? lo[k] : hi[k];
      double w = 0.0;
      for (const V3& v : q) w = std::max(w, std::fabs(get(v, k) - face));
      if (!(w <= tol)) continue;
      DOccluder t{};
      // plane normal toward the inside of the box (+axis on a low face, -axis on a high face)
      double s = (get(nn, k) >= 0.0) == (f < 3) ? 1.0 / nl : -1.0 / nl;
      const V3 n = mk(nn.x * s, nn.y * s, nn.z * s);
      if (!(std::fabs(get(n, k)) > 0.5)) continue;  // not facing along the axis
      t.n[0] = n.x; t.n[1] = n.y; t.n[2] = n.z;
      t.d = n.x * p0.x + n.y * p0.y + n.z * p0.z;
      bool ok = true;
      for (int i = 0; i < 3 && ok; ++i) {
        const V3 a = q[i], b = q[(i + 1) % 3];
        const V3 e = sub(b, a);
        // inward in-plane normal of edge a -> b: (e1 x e2) x e for the counter-clockwise winding
        V3 m = mk(nn.y * e.z - nn.z * e.y, nn.z * e.x - nn.x * e.z, nn.x * e.y - nn.y * e.x);
        const double ml = std::sqrt(m.x * m.x + m.y * m.y + m.z * m.z);
        if (!(ml > 0.0) || !std::isfinite(ml)) { ok = false; break; }
        m = mk(m.x / ml, m.y / ml, m.z / ml);
        t.en[i][0] = m.x; t.en[i][1] = m.y; t.en[i][2] = m.z;
        t.eo[i] = m.x * a.x + m.y * a.y + m.z * a.z;
      }
      // the opposite vertex must be inside each edge (a proper, non-degenerate triangle)
      for (int i = 0; i < 3 && ok; ++i) {
        const V3 v = q[(i + 2) % 3];
        ok = t.en[i][0] * v.x + t.en[i][1] * v.y + t.en[i][2] * v.z - t.eo[i] > 0.0;
      }
      if (ok) cand[f].push_back({0.5 * nl, w, t, {q[0], q[1], q[2]}, pi});
    }
  }
  for (int f = 0; f < 6; ++f) {
    std::stable_sort(cand[f].begin(), cand[f].end(), [](const Cand& x, const Cand& y) { return x.area > y.area; });
    size_t keep = std::min<size_t>(cand[f].size(), RRT_OCC_PER_FACE);
    while (keep > 1 && cand[f][keep - 1].area < 0.05 * cand[f][0].area) --keep;
    o.n[f] = (uint32_t)keep;
    for (uint32_t i = 0; i < o.n[f]; ++i) {
      o.tri[f][i] = cand[f][i].t;
      o.w[f] = std::max(o.w[f], cand[f][i].w);
    }
    // The Kerr proof's wall pieces: two kept triangles that share an edge (vertices within 1e-9 of
    // the box's extent), lie in one plane and form a convex quad are one piece -- the crossing may
    // then land anywhere in the quad, not only inside one triangle -- else the triangle alone.
    // (The reference tests both triangles; a crossing on the shared edge itself is accepted by one
    // of them up to the rounding of triangle.cpp's barycentric signs there.)
    bool used[RRT_OCC_PER_FACE] = {};
    uint32_t nq = 0;
    auto edge_of = [](int a, int b) { return ((a + 1) % 3 == b) ? a : b; };  // edge k: q[k] -> q[k + 1]
    for (uint32_t i = 0; i < keep; ++i) {
      if (used[i]) continue;
      const Cand& A = cand[f][i];
      DOccQuad qd{};
      for (int k = 0; k < 3; ++k) qd.n[k] = A.t.n[k];
      qd.d = A.t.d;
      int ne = 0;
      for (uint32_t j = i + 1; j < keep && !ne; ++j) {
        if (used[j]) continue;
        const Cand& B = cand[f][j];
        int sa[2], sb[2], ns = 0;
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b) {
            const double dd = std::max(std::fabs(A.v[a].x - B.v[b].x),
                                       std::max(std::fabs(A.v[a].y - B.v[b].y), std::fabs(A.v[a].z - B.v[b].z)));
            if (dd <= 1e-9 * sc && ns < 2) { sa[ns] = a; sb[ns] = b; ++ns; }
          }
        if (ns != 2) continue;
        const double cosn = A.t.n[0] * B.t.n[0] + A.t.n[1] * B.t.n[1] + A.t.n[2] * B.t.n[2];
        if (!(cosn >= 1.0 - 1e-12) || !(std::fabs(A.t.d - B.t.d) <= 1e-9 * sc)) continue;
        const int ka = edge_of(sa[0], sa[1]), kb = edge_of(sb[0], sb[1]);
        const V3 fa = A.v[3 - sa[0] - sa[1]], fb = B.v[3 - sb[0] - sb[1]];  // the far vertices
        bool convex = true;
        for (int k = 0; k < 3 && convex; ++k) {
          if (k != ka) convex = A.t.en[k][0] * fb.x + A.t.en[k][1] * fb.y + A.t.en[k][2] * fb.z - A.t.eo[k] > 0.0;
          if (convex && k != kb)
            convex = B.t.en[k][0] * fa.x + B.t.en[k][1] * fa.y + B.t.en[k][2] * fa.z - B.t.eo[k] > 0.0;
        }
        if (!convex) continue;
        for (int k = 0; k < 3; ++k) {
          if (k != ka) { for (int x = 0; x < 3; ++x) qd.en[ne][x] = A.t.en[k][x]; qd.eo[ne++] = A.t.eo[k]; }
          if (k != kb) { for (int x = 0; x < 3; ++x) qd.en[ne][x] = B.t.en[k][x]; qd.eo[ne++] = B.t.eo[k]; }
        }
        used[j] = true;
      }
      if (!ne) {  // the triangle alone: its three edges, the first repeated
        for (int k = 0; k < 4; ++k) {
          for (int x = 0; x < 3; ++x) qd.en[k][x] = A.t.en[k % 3][x];
          qd.eo[k] = A.t.eo[k % 3];
        }
      }
      c->occ_quad[f][nq++] = qd;
    }
    c->occ_nq[f] = nq;
  }
}

static void build_free_grid(rrt_ctx* c) {
  c->grid.clear();
  c->hgrid = DGrid{};
  if (c->grid_res <= 1 || c->nodes.empty()) return;
  const Box& rb = c->nodes[0].bb;
  const double ext[3] = {rb.ext.x, rb.ext.y, rb.ext.z}, g0[3] = {rb.mn.x, rb.mn.y, rb.mn.z};
  const double emax = std::max(ext[0], std::max(ext[1], ext[2]));
  if (!(emax > 0) || !std::isfinite(emax)) return;
  for (double v : g0) if (!std::isfinite(v)) return;
  const double h = emax / c->grid_res, inv_h = 1.0 / h;
  int32_t n[3];
  for (int i = 0; i < 3; ++i) n[i] = (int32_t)std::floor(ext[i] * inv_h) + 2;
  const size_t total = (size_t)n[0] * n[1] * n[2];
  std::vector<uint8_t> k(total, 255);
  std::vector<uint32_t> q;
  q.reserve(total / 4);
  auto idx = [&](int x, int y, int z) { return ((size_t)z * n[1] + y) * n[0] + x; };
  auto mark = [&](int x, int y, int z) {
    const size_t i = idx(x, y, z);
    if (k[i] != 0) { k[i] = 0; q.push_back((uint32_t)i); }
  };
  for (const BNode& nd : c->nodes) {
    if (nd.count == 0) continue;
    if (!grid_mark_leaf(c, g0, h, n, nd.bb, nd.first, nd.count, mark)) { c->grid.clear(); return; }
  }
  for (size_t head = 0; head < q.size(); ++head) {  // BFS: Chebyshev distance transform
    const uint32_t i = q[head];
    const int x = (int)(i % n[0]), y = (int)((i / n[0]) % n[1]), z = (int)(i / ((size_t)n[0] * n[1]));
    const int nk = k[i] + 1;
    if (nk >= 255) continue;
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int xx = x + dx, yy = y + dy, zz = z + dz;
          if (xx < 0 || yy < 0 || zz < 0 || xx >= n[0] || yy >= n[1] || zz >= n[2]) continue;
          const size_t j = idx(xx, yy, zz);
          if (k[j] > nk) { k[j] = (uint8_t)nk; q.push_back((uint32_t)j); }
        }
  }
  c->grid.swap(k);
  DGrid& g = c->hgrid;
  for (int i = 0; i < 3; ++i) { g.g0[i] = g0[i]; g.n[i] = n[i]; }
  g.inv_h = inv_h;
  g.h_free = h * (1.0 - 0x1p-20);
}

// Per-cell masks of the oversized leaves (traverse_clean): bit b of cell c is set when leaf b
// has a primitive hit region within Chebyshev distance RRT_BIG_REACH cells of c (the free
// grid's marking, dilated).  A clear bit means every point of c lies at least
// (RRT_BIG_REACH - 1) * h_free from every primitive of leaf b (the free grid's argument with
// k = RRT_BIG_REACH + 1), so a segment starting in c and shorter than that cannot be accepted by
// any of them and the walk may skip the leaf without changing its answer.  Up to 32 leaves.
static void build_big_masks(rrt_ctx* c) {
  c->big_mask.clear();
  if (c->grid.empty() || c->big.empty() || c->big.size() > 32) return;
  const DGrid& g = c->hgrid;
  const int32_t n[3] = {g.n[0], g.n[1], g.n[2]};
  const size_t total = (size_t)n[0] * n[1] * n[2];
  const double h = 1.0 / g.inv_h;
  std::vector<uint32_t> mask(total, 0u);
  std::vector<uint8_t> a(total), b(total);
  auto idx = [&](int x, int y, int z) { return ((size_t)z * n[1] + y) * n[0] + x; };
  const int R = RRT_BIG_REACH;
  for (size_t bi = 0; bi < c->big.size(); ++bi) {
    const DBig& L = c->big[bi];
    std::fill(a.begin(), a.end(), 0);
    Box bb;
    bb.mn = mk(L.mn[0], L.mn[1], L.mn[2]);
    bb.mx = mk(L.mx[0], L.mx[1], L.mx[2]);
    if (!grid_mark_leaf(c, g.g0, h, n, bb, L.first, L.count, [&](int x, int y, int z) { a[idx(x, y, z)] = 1; })) {
      c->big_mask.clear();
      return;
    }
    // Chebyshev dilation by R: separable running max along x, y, z
    for (int axis = 0; axis < 3; ++axis) {
      const int len = n[axis];
      const size_t stride = axis == 0 ? 1 : axis == 1 ? (size_t)n[0] : (size_t)n[0] * n[1];
      const int o1 = axis == 0 ? 1 : 0, o2 = axis == 2 ? 1 : 2;  // the two other axes
      for (int u = 0; u < n[o1]; ++u)
        for (int v = 0; v < n[o2]; ++v) {
          int co[3] = {0, 0, 0};
          co[o1] = u; co[o2] = v;
          const size_t base = idx(co[0], co[1], co[2]);
          int cnt = 0;  // marked cells in the window [i - R, i + R]
          for (int i = 0; i < std::min(R, len); ++i) cnt += a[base + i * stride];
          for (int i = 0; i < len; ++i) {
            if (i + R < len) cnt += a[base + (size_t)(i + R) * stride];
            if (i - R - 1 >= 0) cnt -= a[base + (size_t)(i - R - 1) * stride];
            b[base + i * stride] = cnt > 0;
          }
        }
      a.swap(b);
    }
    for (size_t i = 0; i < total; ++i) if (a[i]) mask[i] |= 1u << bi;
  }
  c->big_mask.swap(mask);
}

// Clean tree for traverse_clean (rrt_device.h): the reference tree without its oversized leaves,
// inner boxes refit to the leaves left, in left-first pre-order with skip pointers; DNode.pad
// holds the left-first ordinal of the subtree's first leaf.  Oversized = box diagonal above
// 8x the median leaf diagonal (at most 64 leaves, the largest first; none if that would leave
// no tree).  Leaf boxes are the reference's own.
static void build_clean_tree(rrt_ctx* c, std::vector<DNode>& out, std::vector<DBig>& big) {
  out.clear(); big.clear();
  c->has_clean = false; c->clean_root = -1; c->n_big = 0;
  const size_t nn = c->nodes.size();
  if (nn == 0) return;
  std::vector<int32_t> ordinal(nn, -1);
  std::vector<double> diag;
  int32_t nl = 0;
  for (size_t i = 0; i < nn; ++i)
    if (c->nodes[i].count != 0) {
      ordinal[i] = nl++;
      const V3 e = c->nodes[i].bb.ext;
      diag.push_back(std::sqrt(e.x * e.x + e.y * e.y + e.z * e.z));
    }
  std::vector<double> sorted = diag;
  std::nth_element(sorted.begin(), sorted.begin() + sorted.size() / 2, sorted.end());
  const double thresh = 8.0 * sorted[sorted.size() / 2];
  std::vector<std::pair<double, int32_t>> cand;  // (diagonal, node)
  for (size_t i = 0; i < nn; ++i)
    if (c->nodes[i].count != 0 && diag[ordinal[i]] > thresh) cand.push_back({diag[ordinal[i]], (int32_t)i});
  std::sort(cand.begin(), cand.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  if (cand.size() > 64) cand.resize(64);
  if (cand.empty() || (int32_t)cand.size() >= nl) return;  // nothing to gain
  std::vector<char> is_big(nn, 0);
  for (const auto& pr : cand) is_big[pr.second] = 1;
  // rebuild: returns the new index of the subtree's clean root, or -1 if nothing is left
  struct T { Box bb; int32_t first, count, left, right, ord; };
  std::vector<T> tmp;
  std::function<int32_t(int32_t)> rec = [&](int32_t i) -> int32_t {
    const BNode& n = c->nodes[i];
    if (n.count != 0) {
      if (is_big[i]) return -1;
      tmp.push_back(T{n.bb, n.first, n.count, -1, -1, ordinal[i]});
      return (int32_t)tmp.size() - 1;
    }
    const int32_t l = rec(n.left), r = rec(n.right);
    if (l < 0) return r;
    if (r < 0) return l;
    Box b = tmp[l].bb;
    b.expand(tmp[r].bb);
    tmp.push_back(T{b, 0, 0, l, r, std::min(tmp[l].ord, tmp[r].ord)});
    return (int32_t)tmp.size() - 1;
  };
  const int32_t root = rec(0);
  if (root < 0) return;
  // linearise in pre-order (left first) with skip pointers
  std::vector<int32_t> order;
  std::function<void(int32_t)> pre = [&](int32_t i) {
    order.push_back(i);
    if (tmp[i].count == 0) { pre(tmp[i].left); pre(tmp[i].right); }
  };
  pre(root);
  std::vector<int32_t> pos(tmp.size());
  for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (int32_t)k;
  out.resize(order.size());
  std::vector<int32_t> skip(order.size(), -1);
  for (size_t k = 0; k < order.size(); ++k) {
    const T& t = tmp[order[k]];
    if (t.count == 0) {
      skip[pos[t.left]] = pos[t.right];
      skip[pos[t.right]] = skip[k];
    }
  }
  for (size_t k = 0; k < order.size(); ++k) {
    const T& t = tmp[order[k]];
    DNode& d = out[k];
    d.mn[0] = t.bb.mn.x; d.mn[1] = t.bb.mn.y; d.mn[2] = t.bb.mn.z;
    d.mx[0] = t.bb.mx.x; d.mx[1] = t.bb.mx.y; d.mx[2] = t.bb.mx.z;
    d.skip = skip[k]; d.first = t.first; d.count = t.count; d.pad = t.ord;
  }
  for (const auto& pr : cand) {
    const BNode& n = c->nodes[pr.second];
    DBig b{};
    b.mn[0] = n.bb.mn.x; b.mn[1] = n.bb.mn.y; b.mn[2] = n.bb.mn.z;
    b.mx[0] = n.bb.mx.x; b.mx[1] = n.bb.mx.y; b.mx[2] = n.bb.mx.z;
    b.first = n.first; b.count = n.count; b.dfs = ordinal[pr.second];
    big.push_back(b);
  }
  std::sort(big.begin(), big.end(), [](const DBig& a, const DBig& b) { return a.dfs < b.dfs; });
  c->has_clean = true; c->clean_root = 0; c->n_big = (uint32_t)big.size();
}

// Search tree for traverse_free (rrt_device.h): the clean tree's leaves -- the reference's own
// leaf boxes and slot runs -- under a new binary hierarchy chosen by the surface-area heuristic
// (full sweep over centroid-sorted leaves on each axis), in pre-order with skip pointers.  Inner
// boxes are exact unions of their leaves' boxes, so the slab test's monotonicity under box
// inclusion lets the walk prune with them; only the leaf boxes decide which primitives are
// tested, exactly as in the reference ("search tree").  DNode.pad of a leaf: its
// left-first ordinal.
static void build_free_tree(rrt_ctx* c) {
  c->free_tree.clear();
  struct Item { double mn[3], mx[3], cen[3]; int32_t first, count, ord; };
  std::vector<Item> items;
  c->free_big_mask = ~0ull;
  if (c->has_clean) {
    for (const DNode& n : c->clean)
      if (n.count != 0) {
        Item it;
        for (int k = 0; k < 3; ++k) { it.mn[k] = n.mn[k]; it.mx[k] = n.mx[k]; it.cen[k] = 0.5 * (n.mn[k] + n.mx[k]); }
        it.first = n.first; it.count = n.count; it.ord = n.pad;
        items.push_back(it);
      }
    // Oversized leaves that stay local (box diagonal at most a quarter of the root box's: CBbunny's
    // 9 bunny-region ones) join the hierarchy, where its inner boxes prune them; only the
    // room-spanning ones (walls, ceiling, light) stay on the walk's list (free_big_mask).  Any
    // hierarchy over the reference's own leaf boxes gives the same walk result (the monotonicity
    // argument above), so this only changes the work: 14 -> 5 listed leaves per segment on CBbunny.
    const Box& rb = c->nodes[0].bb;
    const double rd = std::sqrt(rb.ext.x * rb.ext.x + rb.ext.y * rb.ext.y + rb.ext.z * rb.ext.z);
    for (size_t bi = 0; bi < c->big.size() && bi < 64; ++bi) {
      const DBig& b = c->big[bi];
      const double ex = b.mx[0] - b.mn[0], ey = b.mx[1] - b.mn[1], ez = b.mx[2] - b.mn[2];
      if (!(std::sqrt(ex * ex + ey * ey + ez * ez) <= 0.25 * rd)) continue;
      Item it;
      for (int k = 0; k < 3; ++k) { it.mn[k] = b.mn[k]; it.mx[k] = b.mx[k]; it.cen[k] = 0.5 * (b.mn[k] + b.mx[k]); }
      it.first = b.first; it.count = b.count; it.ord = b.dfs;
      items.push_back(it);
      c->free_big_mask &= ~(1ull << bi);
    }
  } else {  // no oversized leaves: every reference leaf
    int32_t ord = 0;
    for (const BNode& n : c->nodes)
      if (n.count != 0) {
        Item it;
        const double mn[3] = {n.bb.mn.x, n.bb.mn.y, n.bb.mn.z}, mx[3] = {n.bb.mx.x, n.bb.mx.y, n.bb.mx.z};
        for (int k = 0; k < 3; ++k) { it.mn[k] = mn[k]; it.mx[k] = mx[k]; it.cen[k] = 0.5 * (mn[k] + mx[k]); }
        it.first = n.first; it.count = n.count; it.ord = ord++;
        items.push_back(it);
      }
  }
  if (items.size() < 2) return;
  auto area = [](const double* mn, const double* mx) {
    const double ex = std::max(mx[0] - mn[0], 0.0), ey = std::max(mx[1] - mn[1], 0.0), ez = std::max(mx[2] - mn[2], 0.0);
    return ex * ey + ey * ez + ez * ex;
  };
  std::vector<DNode>& out = c->free_tree;
  out.reserve(2 * items.size());
  std::vector<int32_t> idx(items.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
  std::vector<double> left_area;
  // returns the node index; children laid out in pre-order (left = me + 1)
  std::function<int32_t(int32_t*, int32_t)> rec = [&](int32_t* ids, int32_t n) -> int32_t {
    const int32_t me = (int32_t)out.size();
    out.push_back(DNode{});
    DNode box{};
    for (int k = 0; k < 3; ++k) { box.mn[k] = INFINITY; box.mx[k] = -INFINITY; }
    for (int32_t i = 0; i < n; ++i)
      for (int k = 0; k < 3; ++k) {
        box.mn[k] = std::min(box.mn[k], items[ids[i]].mn[k]);
        box.mx[k] = std::max(box.mx[k], items[ids[i]].mx[k]);
      }
    if (n == 1) {
      const Item& it = items[ids[0]];
      DNode& d = out[me];
      for (int k = 0; k < 3; ++k) { d.mn[k] = it.mn[k]; d.mx[k] = it.mx[k]; }
      d.first = it.first; d.count = it.count; d.pad = it.ord; d.skip = -1;
      return me;
    }
    int best_axis = 0, best_k = n / 2;
    double best = INFINITY;
    left_area.resize(n);
    for (int ax = 0; ax < 3; ++ax) {
      std::stable_sort(ids, ids + n, [&](int32_t a, int32_t b) { return items[a].cen[ax] < items[b].cen[ax]; });
      double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) { mn[k] = std::min(mn[k], items[ids[i]].mn[k]); mx[k] = std::max(mx[k], items[ids[i]].mx[k]); }
        left_area[i] = area(mn, mx);
      }
      for (int k = 0; k < 3; ++k) { mn[k] = INFINITY; mx[k] = -INFINITY; }
      for (int32_t i = n - 1; i >= 1; --i) {
        for (int k = 0; k < 3; ++k) { mn[k] = std::min(mn[k], items[ids[i]].mn[k]); mx[k] = std::max(mx[k], items[ids[i]].mx[k]); }
        const double cost = left_area[i - 1] * i + area(mn, mx) * (n - i);
        if (cost < best) { best = cost; best_axis = ax; best_k = i; }
      }
    }
    std::stable_sort(ids, ids + n, [&](int32_t a, int32_t b) { return items[a].cen[best_axis] < items[b].cen[best_axis]; });
    rec(ids, best_k);
    const int32_t r = rec(ids + best_k, n - best_k);
    DNode& d = out[me];
    d = box;
    d.count = 0; d.first = 0; d.pad = 0; d.skip = -1;
    (void)r;
    return me;
  };
  rec(idx.data(), (int32_t)idx.size());
  // skip pointers: the pre-order successor of each subtree
  std::vector<int32_t> end(out.size());
  std::function<int32_t(int32_t)> fill = [&](int32_t i) -> int32_t {
    if (out[i].count != 0) return end[i] = i + 1;
    const int32_t j = fill(i + 1);
    return end[i] = fill(j);
  };
  fill(0);
  for (size_t i = 0; i < out.size(); ++i) out[i].skip = end[i] < (int32_t)out.size() ? end[i] : -1;
}

// The search tree 4 wide: each node holds the boxes of a binary inner node's children, the inner
// ones opened (largest surface first) until there are four -- the search tree's nodes two levels
// down.  A walk then tests four boxes per dependent load instead of one (the slow pixels' walks
// are chains of ~40 dependent box tests per micro segment: tools/ notes in DESIGN.md §5).  Node
// indices fit 16 bits (the walk's register stack); larger trees keep the binary walk.
static void build_free4(rrt_ctx* c) {
  c->free4.clear();
  const std::vector<DNode>& t = c->free_tree;
  if (t.size() < 3 || t[0].count != 0) return;
  // f32 boxes: rounded outward, then widened by pad = 1e-4 of the scene's coordinate scale -- far
  // above the f32 pre-test's rounding for segment origins within free4_omax = 8 x that scale
  // (origin error <= 2^-24 x 8 scale, quotient error <= 2^-22 relative: both < 1e-6 of the scale)
  double sc = 1.0;
  for (int k = 0; k < 3; ++k) sc = std::max(sc, std::max(std::fabs(t[0].mn[k]), std::fabs(t[0].mx[k])));
  if (!std::isfinite(sc)) return;
  const double pad = 1e-4 * sc;
  c->free4_omax = 8.0 * sc;
  auto down = [&](double v) { float f = (float)(v - pad); while ((double)f > v - pad) f = std::nextafter(f, -INFINITY); return f; };
  auto up = [&](double v) { float f = (float)(v + pad); while ((double)f < v + pad) f = std::nextafter(f, INFINITY); return f; };
  auto area = [&](int32_t i) {
    const double ex = t[i].mx[0] - t[i].mn[0], ey = t[i].mx[1] - t[i].mn[1], ez = t[i].mx[2] - t[i].mn[2];
    return ex * ey + ey * ez + ez * ex;
  };
  // children of binary inner node b (pre-order: left = b + 1, right = the left subtree's successor)
  auto kids = [&](int32_t b, int32_t& l, int32_t& r) { l = b + 1; r = t[l].skip; };
  std::function<int32_t(int32_t)> rec = [&](int32_t b) -> int32_t {
    const int32_t me = (int32_t)c->free4.size();
    c->free4.push_back(DNode4{});
    int32_t ch[4], n = 0;
    kids(b, ch[0], ch[1]);
    n = 2;
    while (n < 4) {  // open the largest inner child
      int best = -1;
      for (int i = 0; i < n; ++i)
        if (t[ch[i]].count == 0 && (best < 0 || area(ch[i]) > area(ch[best]))) best = i;
      if (best < 0) break;
      int32_t l, r;
      kids(ch[best], l, r);
      ch[best] = l;
      ch[n++] = r;
    }
    int32_t sub[4];
    for (int i = 0; i < n; ++i) sub[i] = t[ch[i]].count == 0 ? rec(ch[i]) : -1;
    DNode4& d = c->free4[me];
    for (int i = 0; i < 4; ++i) {
      if (i >= n) {
        d.mnx[i] = d.mny[i] = d.mnz[i] = INFINITY;
        d.mxx[i] = d.mxy[i] = d.mxz[i] = -INFINITY;
        d.child[i] = -1; d.first[i] = 0; d.count[i] = -1;
        continue;
      }
      const DNode& s = t[ch[i]];
      d.mnx[i] = down(s.mn[0]); d.mny[i] = down(s.mn[1]); d.mnz[i] = down(s.mn[2]);
      d.mxx[i] = up(s.mx[0]); d.mxy[i] = up(s.mx[1]); d.mxz[i] = up(s.mx[2]);
      d.child[i] = s.count == 0 ? sub[i] : ch[i];
      d.first[i] = s.first; d.count[i] = s.count;
    }
    return me;
  };
  rec(0);
  if (c->free4.size() > 65535) c->free4.clear();
}

static int upload(rrt_ctx* c, void** dst, const void* src, size_t bytes) {
  if (bytes == 0) bytes = 16;
  HIPCHK(c, hipMalloc(dst, bytes));
  if (src) HIPCHK(c, hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  c->device_bytes += bytes;
  return RRT_OK;
}

// The light table the kernels see: the scene's lights, then the environment light if any
// (PathTracer::set_scene pushes envLight after the scene's lights, pathtracer.cpp:106-108).
static std::vector<DLight> all_lights(const rrt_ctx* c) {
  std::vector<DLight> l = c->lights;
  if (c->env_w) {
    DLight e{};
    e.type = 5; e.is_delta = 0;  // EnvironmentLight::is_delta_light() == false
    l.push_back(e);
  }
  return l;
}
static int upload_lights(rrt_ctx* c) {
  if (c->device < 0) return RRT_OK;
  hipFree(c->d_lights);
  c->d_lights = nullptr;
  const std::vector<DLight> l = all_lights(c);
  if (l.empty()) return RRT_OK;
  return upload(c, (void**)&c->d_lights, l.data(), l.size() * sizeof(DLight));
}

extern "C" int rrt_set_scene(rrt_ctx* c, const rrt_scene_desc* s) {
  if (!c || !s) return fail(c, RRT_E_INVALID, "null argument");
  if (s->n_bsdfs > RRT_MAX_BSDFS) return fail(c, RRT_E_INVALID, "too many BSDFs (max 64)");
  if (s->n_lights + 1 > RRT_MAX_LIGHTS) return fail(c, RRT_E_INVALID, "too many lights (max 15 + environment)");
  if (s->n_objects && !s->objects) return fail(c, RRT_E_INVALID, "objects missing");
  if (s->n_bsdfs && !s->bsdfs) return fail(c, RRT_E_INVALID, "bsdfs missing");
  if (s->n_lights && !s->lights) return fail(c, RRT_E_INVALID, "lights missing");
  // a failed set_scene leaves no scene: rrt_render then fails with RRT_E_INVALID instead of
  // reading the emptied host tables or the previous scene's device buffers
  c->has_scene = false;
  c->has_clean = false;
  c->pos.clear(); c->nrm.clear(); c->prims.clear(); c->nodes.clear(); c->leaf.clear(); c->max_depth = 0;
  c->bsdfs.assign(s->n_bsdfs, DBsdf{});
  for (uint32_t i = 0; i < s->n_bsdfs; ++i) {
    if (s->bsdfs[i].type > RRT_BSDF_REFRACTION) return fail(c, RRT_E_INVALID, "unknown BSDF type");
    c->bsdfs[i].type = s->bsdfs[i].type;
    std::memcpy(c->bsdfs[i].p, s->bsdfs[i].params, sizeof(float) * 14);
  }
  c->lights.assign(s->n_lights, DLight{});
  for (uint32_t i = 0; i < s->n_lights; ++i) {
    const rrt_light_desc& L = s->lights[i];
    if (L.type > RRT_LIGHT_HEMISPHERE)
      return fail(c, RRT_E_INVALID, "unsupported light type (spot/sphere/mesh lights are stubs in the reference; "
                                    "an environment map is given with rrt_set_envmap)");
    DLight& d = c->lights[i];
    d.type = L.type; d.is_delta = L.is_delta;
    std::memcpy(d.rad, L.radiance, sizeof(d.rad)); d.area = L.area;
    std::memcpy(d.v, L.v, sizeof(d.v));
  }
  for (uint32_t o = 0; o < s->n_objects; ++o) {
    const rrt_object_desc& ob = s->objects[o];
    if (ob.bsdf >= s->n_bsdfs) return fail(c, RRT_E_INVALID, "object bsdf index out of range");
    if (ob.kind == RRT_OBJ_MESH) {
      if ((ob.n_vertices && (!ob.positions || !ob.normals)) || (ob.n_triangles && !ob.indices))
        return fail(c, RRT_E_INVALID, "mesh arrays missing");
      uint32_t base = (uint32_t)c->pos.size();
      for (uint32_t v = 0; v < ob.n_vertices; ++v) {
        c->pos.push_back(mk(ob.positions[3 * v], ob.positions[3 * v + 1], ob.positions[3 * v + 2]));
        c->nrm.push_back(mk(ob.normals[3 * v], ob.normals[3 * v + 1], ob.normals[3 * v + 2]));
      }
      for (uint32_t t = 0; t < ob.n_triangles; ++t) {
        Prim p{};
        p.kind = RRT_OBJ_MESH; p.bsdf = ob.bsdf;
        for (int k = 0; k < 3; ++k) {
          uint32_t id = ob.indices[3 * t + k];
          if (id >= ob.n_vertices) return fail(c, RRT_E_INVALID, "triangle index out of range");
          p.v[k] = base + id;
        }
        c->prims.push_back(p);
      }
    } else if (ob.kind == RRT_OBJ_SPHERE) {
      Prim p{};
      p.kind = RRT_OBJ_SPHERE; p.bsdf = ob.bsdf;
      p.c = mk(ob.center[0], ob.center[1], ob.center[2]); p.r = ob.radius; p.r2 = ob.radius * ob.radius;
      c->prims.push_back(p);
    } else {
      return fail(c, RRT_E_INVALID, "unknown object kind");
    }
  }
  if (c->prims.empty()) return fail(c, RRT_E_INVALID, "scene has no primitives");
  std::vector<uint32_t> ids(c->prims.size());
  for (size_t i = 0; i < ids.size(); ++i) ids[i] = (uint32_t)i;
  build(c, ids, 0);
  // skip pointers: pre-order successor of each subtree
  c->nodes[0].skip = -1;
  for (size_t i = 0; i < c->nodes.size(); ++i) {
    BNode& n = c->nodes[i];
    if (n.count == 0) {
      c->nodes[n.left].skip = n.right;
      c->nodes[n.right].skip = n.skip;
    }
  }
  // Markstein-corrected slab quotients are exact when no quotient or residual can
  // under/overflow: require every BVH coordinate to be 0 or of magnitude in [2^-800, 2^20]
  c->fast_div = true;
  for (const BNode& n : c->nodes) {
    const double v[6] = {n.bb.mn.x, n.bb.mn.y, n.bb.mn.z, n.bb.mx.x, n.bb.mx.y, n.bb.mx.z};
    for (double x : v) {
      double a = std::fabs(x);
      if (!(x == 0.0 || (a >= 0x1p-800 && a <= 0x1p20))) c->fast_div = false;
    }
  }
  // first-leaf ordinal of every subtree (DNode.pad), for the walk's merge with the oversized list
  std::vector<int32_t> first_ord(c->nodes.size(), 0);
  {
    int32_t ord = 0;
    for (size_t i = 0; i < c->nodes.size(); ++i)  // pre-order: a subtree's first leaf comes first
      if (c->nodes[i].count != 0) first_ord[i] = ord++;
    for (size_t i = c->nodes.size(); i-- > 0;)
      if (c->nodes[i].count == 0) first_ord[i] = first_ord[c->nodes[i].left];
  }
  // device layout
  std::vector<DNode> dn(c->nodes.size());
  for (size_t i = 0; i < c->nodes.size(); ++i) {
    const BNode& n = c->nodes[i];
    DNode& d = dn[i];
    d.mn[0] = n.bb.mn.x; d.mn[1] = n.bb.mn.y; d.mn[2] = n.bb.mn.z;
    d.mx[0] = n.bb.mx.x; d.mx[1] = n.bb.mx.y; d.mx[2] = n.bb.mx.z;
    d.skip = n.skip; d.first = n.first; d.count = n.count; d.pad = first_ord[i];
  }
  std::vector<DPrimGeo> geo(c->leaf.size());
  std::vector<DPrimNrm> nrm(c->leaf.size());
  std::vector<DPrimMeta> meta(c->leaf.size());
  std::vector<DPlane> planes(c->leaf.size());
  for (size_t k = 0; k < c->leaf.size(); ++k) {
    const Prim& p = c->prims[c->leaf[k]];
    std::memset(&geo[k], 0, sizeof(DPrimGeo));
    std::memset(&nrm[k], 0, sizeof(DPrimNrm));
    if (p.kind == RRT_OBJ_MESH) {
      V3 p0 = c->pos[p.v[0]], e1 = sub(c->pos[p.v[1]], p0), e2 = sub(c->pos[p.v[2]], p0);
      double g[9] = {p0.x, p0.y, p0.z, e1.x, e1.y, e1.z, e2.x, e2.y, e2.z};
      std::memcpy(geo[k].v, g, sizeof(g));
      for (int j = 0; j < 3; ++j) {
        V3 n = c->nrm[p.v[j]];
        nrm[k].n[3 * j] = n.x; nrm[k].n[3 * j + 1] = n.y; nrm[k].n[3 * j + 2] = n.z;
      }
      meta[k] = (p.bsdf << 8);
      // supporting plane for the cull (rrt_device.h plane_may_hit); slivers never cull
      const V3 nn = mk(e1.y * e2.z - e1.z * e2.y, e1.z * e2.x - e1.x * e2.z, e1.x * e2.y - e1.y * e2.x);
      const double nl = std::sqrt(nn.x * nn.x + nn.y * nn.y + nn.z * nn.z);
      const double l1 = std::sqrt(e1.x * e1.x + e1.y * e1.y + e1.z * e1.z);
      const double l2 = std::sqrt(e2.x * e2.x + e2.y * e2.y + e2.z * e2.z);
      DPlane pl{};
      if (nl >= 1e-6 * l1 * l2 && std::isfinite(nl)) {
        pl.n[0] = nn.x / nl; pl.n[1] = nn.y / nl; pl.n[2] = nn.z / nl;
        pl.c = pl.n[0] * p0.x + pl.n[1] * p0.y + pl.n[2] * p0.z;
      }
      planes[k] = pl;
    } else {
      double g[9] = {p.c.x, p.c.y, p.c.z, p.r2, p.r, 0, 0, 0, 0};
      std::memcpy(geo[k].v, g, sizeof(g));
      meta[k] = (p.bsdf << 8) | 1u;
    }
  }
  build_free_grid(c);
  build_occluders(c);
  build_clean_tree(c, c->clean, c->big);
  build_free_tree(c);
  build_free4(c);
  build_big_masks(c);
  {  // plane-cull margin: 1e-9 of the scene's coordinate scale (rounding is ~1e-16 of it)
    const Box& rb = c->nodes[0].bb;
    double m = 1.0;
    for (double v : {rb.mn.x, rb.mn.y, rb.mn.z, rb.mx.x, rb.mx.y, rb.mx.z}) m = std::max(m, std::fabs(v));
    c->plane_eps = std::isfinite(m) ? 1e-9 * m : 0.0;
    if (c->plane_eps == 0.0) for (DPlane& pl : planes) pl = DPlane{};  // never cull
  }
  c->lean = 1;
  for (const DLight& l : c->lights) {
    if (l.type == RRT_LIGHT_POINT && c->lean == 1) c->lean = 2;
    if (l.type != RRT_LIGHT_AREA && l.type != RRT_LIGHT_POINT) c->lean = 0;
  }
  for (const DBsdf& b : c->bsdfs) if (b.type == RRT_BSDF_MICROFACET) c->lean = 0;
  if (c->device < 0) {
    c->has_scene = true;
    return RRT_OK;
  }
  HIPCHK(c, hipSetDevice(c->device));
  free_scene_dev(c);
  int rc;
  if ((rc = upload(c, (void**)&c->d_nodes, dn.data(), dn.size() * sizeof(DNode)))) return rc;
  if ((rc = upload(c, (void**)&c->d_geo, geo.data(), geo.size() * sizeof(DPrimGeo)))) return rc;
  if ((rc = upload(c, (void**)&c->d_nrm, nrm.data(), nrm.size() * sizeof(DPrimNrm)))) return rc;
  if ((rc = upload(c, (void**)&c->d_meta, meta.data(), meta.size() * sizeof(DPrimMeta)))) return rc;
  if ((rc = upload(c, (void**)&c->d_bsdfs, c->bsdfs.data(), c->bsdfs.size() * sizeof(DBsdf)))) return rc;
  if ((rc = upload_lights(c))) return rc;
  if (!c->grid.empty() && (rc = upload(c, (void**)&c->d_grid, c->grid.data(), c->grid.size()))) return rc;
  if ((rc = upload(c, (void**)&c->d_planes, planes.data(), planes.size() * sizeof(DPlane)))) return rc;
  if (!c->free_tree.empty() &&
      (rc = upload(c, (void**)&c->d_free, c->free_tree.data(), c->free_tree.size() * sizeof(DNode))))
    return rc;
  if (!c->free4.empty() &&
      (rc = upload(c, (void**)&c->d_free4, c->free4.data(), c->free4.size() * sizeof(DNode4))))
    return rc;
  if (c->has_clean) {
    if ((rc = upload(c, (void**)&c->d_clean, c->clean.data(), c->clean.size() * sizeof(DNode)))) return rc;
    if ((rc = upload(c, (void**)&c->d_big, c->big.data(), c->big.size() * sizeof(DBig)))) return rc;
    if (!c->big_mask.empty() &&
        (rc = upload(c, (void**)&c->d_big_mask, c->big_mask.data(), c->big_mask.size() * sizeof(uint32_t))))
      return rc;
  }
  c->has_scene = true;
  return RRT_OK;
}

extern "C" int rrt_set_camera(rrt_ctx* c, const rrt_camera_desc* cam) {
  if (!c || !cam) return fail(c, RRT_E_INVALID, "null argument");
  DCamera& d = c->cam;
  for (int i = 0; i < 3; ++i) {
    d.pos[i] = cam->pos[i];
    d.c2w0[i] = cam->c2w[3 * i + 0];  // column 0 = (c2w(0,0), c2w(1,0), c2w(2,0))
    d.c2w1[i] = cam->c2w[3 * i + 1];
    d.c2w2[i] = cam->c2w[3 * i + 2];
  }
  // Camera::generate_ray (part1_code.cpp:183): bl = (-tan(radians(hFov)/2), -tan(radians(vFov)/2)),
  // radians(deg) = deg * (PI / 180) (misc.h:49-52); host libm == the reference's values.
  d.blx = -std::tan(cam->hFov * (kPI / 180) / 2);
  d.bly = -std::tan(cam->vFov * (kPI / 180) / 2);
  c->lens_r = cam->lensRadius;
  c->focal = cam->focalDistance;
  c->has_camera = true;
  return RRT_OK;
}

// EnvironmentLight::init (environment_light.cpp:21-45): pdf = illum * sin(theta_j), normalised;
// per-row conditional CDFs; marginal CDF over rows (marginal_y starts at zero -- the reference
// reads an uninitialised array here).  Same loop and summation order, host libm.
extern "C" int rrt_set_envmap(rrt_ctx* c, const rrt_envmap_desc* env) {
  if (!c) return RRT_E_INVALID;
  free_env_dev(c);
  c->env_w = c->env_h = 0;
  c->env_tex.clear(); c->env_pdf.clear(); c->env_conds.clear(); c->env_marg.clear();
  if (env) {
    if (!env->texels || env->width == 0 || env->height == 0) return fail(c, RRT_E_INVALID, "empty environment map");
    if ((uint64_t)env->width * env->height > (1ull << 28)) return fail(c, RRT_E_INVALID, "environment map too large");
    const uint32_t w = env->width, h = env->height;
    c->env_tex.assign(env->texels, env->texels + (size_t)w * h * 3);
    c->env_pdf.assign((size_t)w * h, 0.0);
    c->env_conds.assign((size_t)w * h, 0.0);
    c->env_marg.assign(h, 0.0);
    double sum = 0;
    for (uint32_t j = 0; j < h; ++j)
      for (uint32_t i = 0; i < w; ++i) {
        const float* t = &c->env_tex[3 * ((size_t)w * j + i)];
        const float illum = 0.2126f * t[0] + 0.7152f * t[1] + 0.0722f * t[2];  // Spectrum::illum
        c->env_pdf[(size_t)w * j + i] = illum * std::sin(kPI * (j + .5) / h);
        sum += c->env_pdf[(size_t)w * j + i];
      }
    for (uint32_t j = 0; j < h; ++j) {
      for (uint32_t i = 0; i < w; ++i) c->env_marg[j] += (c->env_pdf[(size_t)w * j + i] /= sum);
      for (uint32_t i = 0; i < w; ++i) {
        c->env_conds[(size_t)w * j + i] = c->env_pdf[(size_t)w * j + i] / c->env_marg[j];
        if (i > 0) c->env_conds[(size_t)w * j + i] += c->env_conds[(size_t)w * j + i - 1];
      }
      if (j > 0) c->env_marg[j] += c->env_marg[j - 1];
    }
    c->env_w = w; c->env_h = h;
    if (c->device >= 0) {
      HIPCHK(c, hipSetDevice(c->device));
      int rc;
      if ((rc = upload(c, (void**)&c->d_env_tex, c->env_tex.data(), c->env_tex.size() * sizeof(float)))) return rc;
      if ((rc = upload(c, (void**)&c->d_env_pdf, c->env_pdf.data(), c->env_pdf.size() * sizeof(double)))) return rc;
      if ((rc = upload(c, (void**)&c->d_env_conds, c->env_conds.data(), c->env_conds.size() * sizeof(double)))) return rc;
      if ((rc = upload(c, (void**)&c->d_env_marg, c->env_marg.data(), c->env_marg.size() * sizeof(double)))) return rc;
    }
  }
  if (c->has_scene) {
    if (c->lights.size() + (c->env_w ? 1 : 0) > RRT_MAX_LIGHTS) return fail(c, RRT_E_INVALID, "too many lights");
    return upload_lights(c);
  }
  return RRT_OK;
}

extern "C" int rrt_set_spacetime(rrt_ctx* c, const rrt_spacetime_desc* st) {
  if (!c || !st) return fail(c, RRT_E_INVALID, "null argument");
  if (st->kind != RRT_METRIC_SCHWARZSCHILD && st->kind != RRT_METRIC_KERR)
    return fail(c, RRT_E_INVALID, "unknown metric kind");
  if (!(st->delta_theta > 0)) return fail(c, RRT_E_INVALID, "delta_theta must be > 0");
  DHole h{};
  for (int i = 0; i < 3; ++i) h.c[i] = st->center[i];
  h.r = st->r_s; h.r2 = st->r_s * st->r_s; h.dt = st->delta_theta;
  h.cos_dt = std::cos(h.dt); h.sin_dt = std::sin(h.dt);  // blackhole.cpp:36-37, host libm
  int j = 0;
  while (j * h.dt < 2 * M_PI) ++j;  // bvh.cpp:105
  h.steps = j;
  h.kind = (int32_t)st->kind;
  if (st->kind == RRT_METRIC_KERR) {
    // M = r_s / 2, a = spin * M, outer horizon r+ = M + sqrt(M^2 - a^2); the
    // local frame has ez along the spin axis (default: the scene's up, +y)
    if (!(st->r_s > 0)) return fail(c, RRT_E_INVALID, "Kerr needs r_s > 0");
    if (!(st->spin >= 0 && st->spin < 1)) return fail(c, RRT_E_INVALID, "Kerr spin a/M must be in [0, 1)");
    double ax[3] = {st->axis[0], st->axis[1], st->axis[2]};
    double n = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    if (n == 0) { ax[0] = 0; ax[1] = 1; ax[2] = 0; n = 1; }
    if (!std::isfinite(n)) return fail(c, RRT_E_INVALID, "Kerr spin axis must be finite");
    rrt_kerr_frame(ax, h.ex, h.ey, h.ez);
    h.m = 0.5 * st->r_s;
    h.a = st->spin * h.m;
    h.a2 = h.a * h.a;
    h.r_hor = h.m + std::sqrt(h.m * h.m - h.a2);
  }
  c->hole = h;
  return RRT_OK;
}

extern "C" void rrt_kerr_frame(const double* axis, double* ex, double* ey, double* ez) {
  // ez = unit(axis); ex = unit(t x ez) with t the world axis least aligned with ez; ey = ez x ex
  const double n = std::sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
  for (int i = 0; i < 3; ++i) ez[i] = axis[i] / n;
  double t[3] = {0, 0, 1};
  if (std::fabs(ez[2]) >= 0.9) { t[0] = 1; t[2] = 0; }
  double x[3] = {t[1] * ez[2] - t[2] * ez[1], t[2] * ez[0] - t[0] * ez[2], t[0] * ez[1] - t[1] * ez[0]};
  const double xn = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  for (int i = 0; i < 3; ++i) ex[i] = x[i] / xn;
  ey[0] = ez[1] * ex[2] - ez[2] * ex[1];
  ey[1] = ez[2] * ex[0] - ez[0] * ex[2];
  ey[2] = ez[0] * ex[1] - ez[1] * ex[0];
}

// The lattice deal of a region's tiles (origin x0, y0; w x h pixels) over `world` ranks: tile
// (tx, ty) goes to rank (tx + S ty) % world, S = rrt_deal_stride(world) -- every row dealt
// cyclically, each row shifted by S, so a rank's tiles form a sheared lattice: no rank owns whole
// columns (the serpentine order k % world did when the row length is a multiple of world: a 4K
// frame's 120 tiles a row), and a cluster of costly tiles spreads over every rank.  Measured, every
// rank's tiles timed on one MI355X, slowest of 8 ranks (profiles/r06_deal_w8.txt): cfg4 3.71 ->
// 3.26 ms, cfg3 3.24 -> 3.16 ms against the serpentine deal.
static uint32_t rrt_deal_stride(uint32_t world) {
  // the integer nearest 0.382 world that is prime to it (2 -> 1, 4 -> 1, 5 -> 2, 7 -> 3, 8 -> 3)
  uint32_t best = 1;
  double bd = 1e300;
  for (uint32_t s = 1; s < world; ++s) {
    uint32_t a = s, b = world;
    while (b) { const uint32_t t = a % b; a = b; b = t; }
    const double d = std::fabs((double)s - 0.382 * world);
    if (a == 1 && d < bd) { bd = d; best = s; }
  }
  return best;
}
extern "C" int rrt_region_tiles(uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t ts, uint32_t rank,
                                uint32_t world, uint32_t* out, uint32_t max_tiles) {
  if (ts == 0 || world == 0 || rank >= world) return RRT_E_INVALID;
  const uint32_t tw = (w + ts - 1) / ts, th = (h + ts - 1) / ts, S = rrt_deal_stride(world);
  uint32_t n = 0;
  for (uint32_t ty = 0; ty < th; ++ty) {
    for (uint32_t tx = 0; tx < tw; ++tx) {
      if ((uint32_t)(((uint64_t)tx + (uint64_t)S * ty) % world) != rank) continue;
      if (out && n < max_tiles) { out[2 * n] = x0 + tx * ts; out[2 * n + 1] = y0 + ty * ts; }
      ++n;
    }
  }
  return (int)n;
}
extern "C" int rrt_partition_tiles(uint32_t fw, uint32_t fh, uint32_t ts, uint32_t rank, uint32_t world,
                                   uint32_t* out, uint32_t max_tiles) {
  return rrt_region_tiles(0, 0, fw, fh, ts, rank, world, out, max_tiles);
}

static int ensure(rrt_ctx* c, void** p, size_t& cap, size_t need, size_t elem) {
  (void)cap;
  if (need == 0) need = 1;
  hipFree(*p);
  *p = nullptr;
  HIPCHK(c, hipMalloc(p, need * elem));
  return RRT_OK;
}

// Order this use of the context's workspace after the previous one when the streams differ
// (same-stream uses are ordered by the stream itself).
static int scratch_acquire(rrt_ctx* c, hipStream_t stream) {
  if (c->fenced && c->fence_stream != stream) HIPCHK(c, hipStreamWaitEvent(stream, c->ev_fence, 0));
  return RRT_OK;
}
static int scratch_release(rrt_ctx* c, hipStream_t stream) {
  HIPCHK(c, hipEventRecord(c->ev_fence, stream));
  c->fence_stream = stream;
  c->fenced = true;
  return RRT_OK;
}

// The envelope the three proofs were validated in (tools/proof_sweep.py, profiles/
// r03_proof_sweep.json: random holes inside and outside the room, cameras and resolutions, every
// Cornell-box scene; the recurrence's deviation from the reference's march stayed >= 1000x below
// the margins and no proven ray or pixel was contradicted): delta_theta in [0.04, 0.6] and r_s at
// most half the root box's largest extent.  Outside it every ray is marched exactly.
static bool in_proof_envelope(const rrt_ctx* c) {
  if (!c->has_scene || c->hole.kind != RRT_METRIC_SCHWARZSCHILD) return false;
  const Box& rb = c->nodes[0].bb;
  const double ext = std::max(std::max(rb.mx.x - rb.mn.x, rb.mx.y - rb.mn.y), rb.mx.z - rb.mn.z);
  return c->hole.dt >= RRT_PROOF_DT_MIN && c->hole.dt <= RRT_PROOF_DT_MAX && c->hole.r >= 0.0 &&
         c->hole.r <= RRT_PROOF_RS_OVER_EXTENT * ext && std::isfinite(ext);
}
extern "C" int rrt_proof_envelope(const rrt_ctx* c) {
  if (!c) return RRT_E_INVALID;
  return in_proof_envelope(c) ? 1 : 0;
}

static int launch(rrt_ctx* c, const rrt_render_params* p, const uint32_t* tiles, uint32_t n_tiles, uint32_t ts,
                  uint32_t cx0, uint32_t cy0, uint32_t cx1, uint32_t cy1, float* d_rgb, int32_t* d_cnt,
                  uint32_t* d_draws, uint32_t* d_ctr, hipStream_t stream) {
  if (!c->has_scene) return fail(c, RRT_E_INVALID, "no scene (rrt_set_scene)");
  if (!c->has_camera) return fail(c, RRT_E_INVALID, "no camera (rrt_set_camera)");
  if (c->device < 0) return fail(c, RRT_E_NO_DEVICE, "host-only context cannot render");
  if (p->frame_w == 0 || p->frame_h == 0) return fail(c, RRT_E_INVALID, "frame size is zero");
  if (p->samples_per_batch == 0) return fail(c, RRT_E_INVALID, "samples_per_batch must be > 0");
  if (p->max_ray_depth > RRT_MAX_DEPTH) return fail(c, RRT_E_INVALID, "max_ray_depth > 16 not supported");
  if (ts == 0 || ts % 8 != 0) return fail(c, RRT_E_INVALID, "tile_size must be a positive multiple of 8");
  if (n_tiles == 0) return RRT_OK;
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = scratch_acquire(c, stream)) return rc;
  // whatever path leaves this function, the work already enqueued on `stream` fences the
  // workspace for the next user on another stream
  struct FenceGuard {
    rrt_ctx* c; hipStream_t s;
    ~FenceGuard() { scratch_release(c, s); }
  } fence_guard{c, stream};
  // once the heavy pixels' kernel is forked onto the side stream, every path out of here joins it
  // into `stream` first (so the fence above covers its reads of d_kp / d_counter / the heavy list):
  // 1 = launched, 2 = its completion event recorded, 3 = joined
  struct JoinGuard {
    rrt_ctx* c; hipStream_t s; hipStream_t fork; hipEvent_t done; int state;
    ~JoinGuard() {
      if (state == 1) (void)hipStreamSynchronize(fork);
      else if (state == 2) (void)hipStreamWaitEvent(s, done, 0);
    }
  } join_guard{c, stream, c->side, c->ev_heavy, 0};
  if (c->tiles_cap < n_tiles) {
    // hipFree waits for the device, so no launch still reads the old list
    hipFree(c->d_tiles); c->d_tiles = nullptr;
    HIPCHK(c, hipMalloc(&c->d_tiles, sizeof(uint32_t) * 2 * n_tiles));
    c->tiles_cap = n_tiles;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_tiles, tiles, sizeof(uint32_t) * 2 * n_tiles, hipMemcpyHostToDevice, stream));
  HIPCHK(c, hipMemsetAsync(c->d_counter, 0, kCounterBytes, stream));
  KParams kp{};
  kp.nodes = c->d_nodes; kp.geo = c->d_geo; kp.nrm = c->d_nrm; kp.meta = c->d_meta;
  kp.bsdfs = c->d_bsdfs; kp.lights = c->d_lights; kp.n_lights = (uint32_t)c->lights.size() + (c->env_w ? 1u : 0u);
  kp.env.tex = c->d_env_tex; kp.env.pdf = c->d_env_pdf; kp.env.conds = c->d_env_conds; kp.env.marg = c->d_env_marg;
  kp.env.w = c->env_w; kp.env.h = c->env_h;
  kp.fast_div = (c->fast_div && !(p->flags & RRT_RENDER_EXACT_DIV)) ? 1u : 0u;
  kp.cam = c->cam; kp.hole = c->hole;
  kp.grid = c->hgrid;
  kp.grid.k = (p->flags & RRT_RENDER_NO_SKIP) ? nullptr : c->d_grid;
  // the walk always runs over a "clean" tree: the real one, or the reference tree (whose DNode
  // pad carries the first-leaf ordinals too) with an empty oversized-leaf list
  const bool use_clean = c->has_clean && !(p->flags & RRT_RENDER_NO_CLEAN);
  kp.clean_nodes = use_clean ? c->d_clean : c->d_nodes;
  kp.big = c->d_big; kp.clean_root = 0; kp.n_big = use_clean ? c->n_big : 0u;
  kp.big_mask = (use_clean && !(p->flags & RRT_RENDER_NO_SKIP)) ? c->d_big_mask : nullptr;
  kp.big_reach = (RRT_BIG_REACH - 1) * c->hgrid.h_free;
  kp.free_big_mask = ~0ull;
  // the walk's hierarchy (rrt_device.h traverse_free): the SAH search tree by default; for A/B
  // the clean tree (RRT_RENDER_NO_SEARCH_TREE) or the reference tree itself (RRT_RENDER_NO_CLEAN,
  // no oversized list) -- every one of them holds the reference's leaves, so results are equal
  {
    const bool no_search = (p->flags & RRT_RENDER_NO_SEARCH_TREE) || !c->d_free;
    if ((p->flags & RRT_RENDER_NO_CLEAN) || (!c->has_clean && no_search)) {
      kp.free_nodes = c->d_nodes; kp.n_big = 0;
    } else if (no_search) {
      kp.free_nodes = c->d_clean;
    } else {
      kp.free_nodes = c->d_free;  // over the clean tree's leaves (+ kp.big), or every leaf
      kp.free_big_mask = c->free_big_mask;
      // the 4-wide walk of the same tree (A/B: RRT_AB_NO_BVH4=1 in the environment)
      const char* nb4 = std::getenv("RRT_AB_NO_BVH4");
      kp.free4 = (nb4 && nb4[0] == '1') ? nullptr : c->d_free4;
      kp.free4_omax = c->free4_omax;
    }
  }
  kp.planes = c->d_planes; kp.plane_eps = c->plane_eps;
  {
    const Box& rb = c->nodes[0].bb;
    const double lo[3] = {rb.mn.x, rb.mn.y, rb.mn.z}, hi[3] = {rb.mx.x, rb.mx.y, rb.mx.z};
    const bool ok = c->plane_eps > 0 && !(p->flags & RRT_RENDER_NO_SKIP);
    for (int k = 0; k < 3; ++k) {  // no skip: an empty test range (-inf, +inf)
      kp.root_lo[k] = ok ? lo[k] - c->plane_eps : -INFINITY;
      kp.root_hi[k] = ok ? hi[k] + c->plane_eps : INFINITY;
    }
    // Kerr escape radius: the farthest root-box corner from the hole, >= 4M
    double m3[3];
    for (int k = 0; k < 3; ++k) {
      const double dl = std::fabs(lo[k] - kp.hole.c[k]), dh = std::fabs(hi[k] - kp.hole.c[k]);
      m3[k] = dl > dh ? dl : dh;
    }
    const double e2 = (m3[0] * m3[0] + m3[1] * m3[1]) + m3[2] * m3[2], f2 = (4.0 * kp.hole.m) * (4.0 * kp.hole.m);
    kp.hole.r_esc2 = e2 > f2 ? e2 : f2;
    kp.hole.kerr_max_steps = 4 * kp.hole.steps;
  }
  bool proofs_valid = false;
  {  // camera-ray miss proof constants (rrt_device.h camera_miss_proof)
    const DHole& h = kp.hole;
    DMissProof& mp = kp.miss;
    const Box& rb = c->nodes[0].bb;
    const double rho = std::sqrt(h.cos_dt * h.cos_dt + h.sin_dt * h.sin_dt);
    mp.rho = rho; mp.inv_rho = 1.0 / rho;
    mp.co1 = h.cos_dt / rho; mp.si1 = h.sin_dt / rho; mp.inv_si = 1.0 / h.sin_dt;
    mp.k15 = 1.5 * h.r;
    mp.dt2_4 = h.dt * h.dt / 4.0; mp.dt2_6 = h.dt * h.dt / 6.0;
    mp.kappa = 1e-3;
    mp.eta = 1e-5;
    const double lo[3] = {rb.mn.x, rb.mn.y, rb.mn.z}, hi[3] = {rb.mx.x, rb.mx.y, rb.mx.z};
    double sc = 1.0;
    for (int k = 0; k < 3; ++k) {
      mp.lo[k] = lo[k]; mp.hi[k] = hi[k];
      sc = std::max(sc, std::max(std::fabs(lo[k] - h.c[k]), std::fabs(hi[k] - h.c[k])));
    }
    mp.scale = 2.0 * sc;
    double rb2 = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double e = std::max(std::fabs(lo[k] - h.c[k]), std::fabs(hi[k] - h.c[k]));
      rb2 += e * e;
    }
    mp.r_ball = std::sqrt(rb2) * (1.0 + 1e-9);
    bool fin = std::isfinite(mp.scale) && std::isfinite(h.r) && h.r >= 0.0;
    for (int k = 0; k < 3; ++k) fin = fin && std::isfinite(h.c[k]);
    // the recurrence needs a proper turn per step (0 < dt < pi, sin dt > 0); the three proofs
    // share these constants, and each has its own switch below
    proofs_valid = h.kind == RRT_METRIC_SCHWARZSCHILD && fin && h.dt > 0.0 && h.dt < 3.0 && h.sin_dt > 0.0 &&
                   h.steps >= 1 && in_proof_envelope(c);
    mp.on = (proofs_valid && !(p->flags & RRT_RENDER_NO_MISS_PROOF)) ? 1u : 0u;
  }
  {  // shadow-ray occlusion proof: the same recurrence, against the root box's face triangles
    kp.occ = c->occ;
    uint32_t any = 0;
    for (int f = 0; f < 6; ++f) any += kp.occ.n[f];
    const bool fin = std::isfinite(kp.miss.scale) && std::isfinite(kp.hole.r) && kp.hole.r >= 0.0;
    // trigger box: the root box shrunk past every kept triangle by twice the largest margin
    // the proof uses inside the box, eta (r_ball + scale)
    const double m2 = 2.0 * kp.miss.eta * (kp.miss.r_ball + kp.miss.scale);
    for (int k = 0; k < 3; ++k) {
      kp.occ.in_lo[k] = kp.miss.lo[k] + kp.occ.w[k] + m2;
      kp.occ.in_hi[k] = kp.miss.hi[k] - kp.occ.w[k + 3] - m2;
    }
    // the point-light scenes' builds carry no proof (rrt_sample.hip RRT_OCC_TAG); off for them in
    // every kernel, so the counting passes count what their batch kernel executes
    kp.occ.on = (proofs_valid && any && fin && c->lean != 2 && !(p->flags & RRT_RENDER_NO_SHADOW_PROOF)) ? 1u : 0u;
    // Kerr shadow rays (rrt_device.h kerr_occluded_proof): the same face triangles
    // against a coarse march, inside the envelope its margin was swept over
    // (tools/kerr_proof_sweep.py -> profiles/r04_kerr_proof_sweep.json)
    DKerrProof& kq = kp.kproof;
    kq = DKerrProof{};
    const DHole& h = kp.hole;
    // the swept region only: the hole's centre within the middle 60% of the root box on every axis
    // and r_s within [0.04, 0.15] of its largest extent (the sweep's holes: 0.2 .. 0.8 of each axis,
    // r_s 0.08 .. 0.3 in rooms 2 units across)
    bool kin = true;
    double kext = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double e = kp.miss.hi[k] - kp.miss.lo[k];
      kext = std::max(kext, e);
      kin = kin && h.c[k] >= kp.miss.lo[k] + RRT_KPROOF_CENTRE_LO * e && h.c[k] <= kp.miss.lo[k] + RRT_KPROOF_CENTRE_HI * e;
    }
    kin = kin && h.r >= RRT_KPROOF_RS_LO * kext && h.r <= RRT_KPROOF_RS_HI * kext;
    const bool kenv = h.kind == RRT_METRIC_KERR && any && fin && kin && h.m > 0.0 && h.dt >= RRT_KPROOF_DT_MIN &&
                      h.dt <= RRT_KPROOF_DT_MAX && h.a <= RRT_KPROOF_SPIN_MAX * h.m &&
                      h.r_esc2 <= (RRT_KPROOF_REACH_M * h.m) * (RRT_KPROOF_REACH_M * h.m);
    if (kenv && !(p->flags & RRT_RENDER_NO_SHADOW_PROOF)) {
      kq.stretch = RRT_KPROOF_STRETCH;
      kq.r_near2 = (RRT_KPROOF_NEAR_M * h.m) * (RRT_KPROOF_NEAR_M * h.m);
      kq.delta = RRT_KPROOF_DELTA_M * h.m;
      kq.swept_max = 2.0 * M_PI - 0.5;
      // the exact march takes about stretch steps per coarse step: a quarter to spare
      kq.max_steps = (int32_t)((h.kerr_max_steps - 2) / (1.25 * kq.stretch));
      kq.on = 1u;
      std::memcpy(kq.quad, c->occ_quad, sizeof(kq.quad));
      std::memcpy(kq.nq, c->occ_nq, sizeof(kq.nq));
      for (int k = 0; k < 3; ++k) {  // trigger box: shrunk past every kept triangle by 2 delta
        kp.occ.in_lo[k] = kp.miss.lo[k] + kp.occ.w[k] + 2.0 * kq.delta;
        kp.occ.in_hi[k] = kp.miss.hi[k] - kp.occ.w[k + 3] - 2.0 * kq.delta;
      }
    }
  }
  kp.ns_aa = p->ns_aa; kp.max_ray_depth = p->max_ray_depth; kp.ns_area_light = p->ns_area_light;
  kp.samples_per_batch = p->samples_per_batch; kp.max_tolerance = p->max_tolerance;
  kp.direct_hemisphere = p->direct_hemisphere; kp.seed = p->seed;
  kp.diag = (p->flags >> 30) | ((p->flags >> 26) & 12u);
  kp.count_exec = (p->flags & RRT_RENDER_COUNT_EXECUTED) ? 1u : 0u;
  kp.frame_w = (double)p->frame_w; kp.frame_h = (double)p->frame_h;
  kp.frame_wi = p->frame_w; kp.frame_hi = p->frame_h;
  kp.tiles = c->d_tiles; kp.n_tiles = n_tiles; kp.tile_size = ts;
  kp.blocks_per_tile_side = ts / 8;
  kp.n_blocks = n_tiles * (ts / 8) * (ts / 8);
  kp.block_counter = c->d_counter;
  kp.clip_x0 = cx0; kp.clip_y0 = cy0; kp.clip_x1 = cx1; kp.clip_y1 = cy1;
  kp.rgb = d_rgb; kp.count = d_cnt; kp.draws = d_draws; kp.counters = d_ctr;
  // Kernel choice (depth <= 1): the per-sample kernel (rrt_sample.hip) by default;
  // RRT_RENDER_PIXEL_LOOP selects the general per-pixel-loop kernel (rrt_kernel.hip, also used
  // for depth >= 2).  LEAN
  // builds when the scene allows them; variant = register budget in waves per SIMD.
  const int deep = p->max_ray_depth >= 2 ? 1 : 0;
  const int count = (p->flags & RRT_RENDER_COUNTERS) && d_ctr ? 1 : 0;
  // kernel variant (rrt_device.h): the Kerr builds for a Kerr spacetime; else LEAN builds when
  // the scene allows (no environment map, importance-sampled direct light), else general
  const bool kerr = c->hole.kind == RRT_METRIC_KERR;
  // the reference's compile-time switches (RRT_RENDER_THIN_LENS .. RRT_RENDER_ILLUM_MASK): the
  // general per-pixel-loop build V_SW (rrt_kernel.hip), every ray marched exactly
  kp.sw = (p->flags >> 22) & 63u;
  kp.lens_r = c->lens_r; kp.focal = c->focal;
  const bool sw = kp.sw != 0;
  if (sw && kerr) return fail(c, RRT_E_INVALID, "the reference's switches (THIN_LENS, ADAPTIVE, ILLUM, ENV_HEMI, "
                                                "MICROFACET_HEMI) are built for the Schwarzschild stepper only");
  if (sw && ((kp.sw >> 4) ^ 2u) == 3u && p->max_ray_depth == 0)
    return fail(c, RRT_E_INVALID, "ILLUM 3 with max_ray_depth 0: the reference's recursion depth is unbounded there "
                                  "(Ray::depth is size_t and wraps below 0; only Russian roulette ends it), beyond "
                                  "RRT_MAX_DEPTH");
  if (sw) { kp.miss.on = 0u; kp.occ.on = 0u; }
  // bounce paths (depth >= 2): the per-pixel-loop kernel by default; RRT_RENDER_DEEP_SAMPLE selects
  // the per-sample refill kernel (rrt_sample.hip, one lane per pixel, a lane whose pixel is done
  // takes the next at the next sample boundary) -- m3 A/B, profiles/r03_ab_deep.jsonl: 177 ms
  // pixel loop vs 236 ms refill at 3 waves/SIMD, identical outputs
  const bool deep_sample = deep && !count && !kerr && !sw && (p->flags & RRT_RENDER_DEEP_SAMPLE) &&
                           !(p->flags & RRT_RENDER_PIXEL_LOOP);
  // RRT_RENDER_WAVEFRONT: the bounce paths (depth >= 2, Schwarzschild) in the path pool kernel
  // (rrt_path.hip: one ray per lane per round, the paths' integrator state between rays in LDS),
  // an A/B variant: m3 269 ms at 3 waves/SIMD vs 172 ms for the per-pixel loop.
  // Its light-sample cursor holds 11 bits: n_lights x ns_area_light < 2048.
  const bool path_pool = (p->flags & RRT_RENDER_WAVEFRONT) != 0;
  // its path records pack the pixel as x | y << 16
  if (path_pool && (p->frame_w > 65535u || p->frame_h > 65535u))
    return fail(c, RRT_E_INVALID, "RRT_RENDER_WAVEFRONT (the path pool kernel) renders frames of at most 65535 pixels a side");
  if (path_pool && !(deep && !count && !kerr && !sw && p->ns_aa >= 1 &&
                     (uint64_t)all_lights(c).size() * std::max<uint32_t>(1u, p->ns_area_light) < 2048u))
    return fail(c, RRT_E_INVALID, "RRT_RENDER_WAVEFRONT (the path pool kernel) renders max_ray_depth >= 2 "
                                  "Schwarzschild frames without counters or switches, n_lights x ns_area_light < 2048");
  const bool pixel_loop = !path_pool && ((deep && !deep_sample) || (p->flags & RRT_RENDER_PIXEL_LOOP) || sw);
  const int lean = kerr ? 3 /* V_KERR */
                 : sw ? 4 /* V_SW */
                 : (!deep && !count && !c->env_w && !p->direct_hemisphere) ? c->lean : 0;
  const uint32_t wv = p->variant & 0xffu;
  // bounce builds: 3 waves/SIMD (m3 A/B, profiles/r03_ab_deep.jsonl: 363 / 263 / 180 / 180 ms at 1 / 2 / 3 / 4)
  const int waves = (wv >= 1 && wv <= 6) ? (int)wv : path_pool ? RRT_PATH_WAVES : deep ? 3 : (pixel_loop ? 2 : 3);
  // persistent grid, 4 waves per block, up to 8 blocks per CU (the 32-wave limit): as many
  // blocks as the kernel's registers allow become resident; any others start when a resident
  // block exits and find the atomic work counter exhausted
  // Sample-parallel kernel (rrt_sample.hip rrt_batch_kernel) whenever a pixel takes more than
  // one sample: it needs each camera sample's RNG draw count to depend only on whether its query
  // hit, which holds at depth <= 1 (jitter + the direct-lighting samplers).
  const bool batch = !deep && !count && !pixel_loop && std::min(p->ns_aa, p->samples_per_batch) >= 5 &&
                     !(p->flags & RRT_RENDER_PER_PIXEL);
  // Continuations (rrt_sample.hip cont_push): the records, their control words and
  // the heavy blocks' waiting policy.  A/B in the environment: RRT_AB_CONT_MIN=samples left;
  // RRT_AB_CONT_ROOM=batch blocks of room; RRT_AB_CONT_WAITERS=heavy blocks that wait.  false: HIP error
  auto setup_cont = [&](bool part) -> bool {
    const uint32_t ccap = std::min<uint32_t>(kp.n_pixels, std::max<uint32_t>(4096u, kp.n_pixels / 256u));
    if (c->cont_cap < ccap) {
      hipFree(c->d_cont); c->d_cont = nullptr; c->cont_cap = 0;
      if (hipMalloc(&c->d_cont, sizeof(ContRec) * ccap) != hipSuccess ||
          hipMemset(c->d_cont, 0, sizeof(ContRec) * ccap) != hipSuccess) {
        fail(c, RRT_E_HIP, "continuation records: allocation failed");
        return false;
      }
      c->cont_cap = ccap;
    }
    kp.cont = c->d_cont;
    kp.cont_ctl = c->d_counter + RRT_QUEUE_STRIDE * (RRT_MAX_QUEUES + 2);
    kp.cont_cap = (uint32_t)c->cont_cap;
    const char* cm = std::getenv("RRT_AB_CONT_MIN");
    kp.cont_min_left = cm ? (uint32_t)std::strtoul(cm, nullptr, 10) : 2u * p->samples_per_batch;
    if (++c->cont_seq == 0) c->cont_seq = 1;
    kp.cont_seq = c->cont_seq;
    // room for 32 heavy blocks from the launch's start (a rank's first pixels are its centre's,
    // the costliest: their first checks come early)
    const char* cr = std::getenv("RRT_AB_CONT_ROOM");
    kp.cont_room = cr ? (uint32_t)std::strtoul(cr, nullptr, 10) : (part ? 32u : 0u);
    kp.cont_ticks = 5000000u;  // 50 ms of wall clock (100 MHz)
    const char* cw = std::getenv("RRT_AB_CONT_WAITERS");
    kp.cont_waiters = cw ? (uint32_t)std::strtoul(cw, nullptr, 10) : ~0u;
    return true;
  };
  if (batch) {
    kp.draws_miss = 2;
    uint32_t dh = 2;
    if (p->max_ray_depth >= 1) {
      if (p->direct_hemisphere) {
        dh += 2u * (uint32_t)all_lights(c).size() * p->ns_area_light;
      } else {
        for (const DLight& l : all_lights(c)) {
          const uint32_t num = l.is_delta ? 1u : p->ns_area_light;
          // area, hemisphere and environment samplers draw 2 each; point / directional none
          const bool sampled = l.type == RRT_LIGHT_AREA || l.type == RRT_LIGHT_HEMISPHERE || l.type == 5u;
          dh += sampled ? 2u * num : 0u;
        }
      }
    }
    kp.draws_hit = dh;
    uint32_t gsz = 8;  // groups of 8..32 lanes (GroupLds holds 32 groups per block)
    const uint32_t want_g = std::min<uint32_t>(std::min<uint32_t>(p->ns_aa, p->samples_per_batch), 32u);
    while (gsz < want_g) gsz <<= 1;
    kp.group = gsz;
    kp.n_pixels = n_tiles * ts * ts;
    // Claim order: tiles nearest the frame centre first (where the geometry and the black hole's
    // ring usually are), so the launch ends on cheap border tiles rather than on a costly
    // region; consecutive claims stay spatially adjacent (coherent waves, warm caches).
    // One queue per XCD (workgroups are dealt to the 8 XCDs round-robin, so block b starts on
    // queue b % 8): queue q holds the tiles of the q-th 45-degree sector about the frame centre,
    // centre-first.  Each XCD's L2 then serves a coherent wedge of the frame (a narrower slice
    // of the BVH), every wedge gets its share of the costly centre, and a block whose queue is
    // empty moves on to the next queue, so the load still balances at pixel granularity.
    std::vector<uint32_t> order(n_tiles);
    for (uint32_t k = 0; k < n_tiles; ++k) order[k] = k;
    const bool ordered = p->flags & RRT_RENDER_ORDERED;
    // A/B (profiles/r01_queues_ab.md): per-XCD queues cost the LEAN cfg3 build 6% and save the
    // Kerr cfg5 build 2%, so they are the default for the general / Kerr builds only
    const bool xcd_q = (p->flags & RRT_RENDER_XCD_QUEUES) || ((lean == 0 || lean == 3) && !(p->flags & RRT_RENDER_ONE_QUEUE) &&
                                                             !(p->flags & RRT_RENDER_STRIPED_QUEUES));
    // Striped queues (the LEAN default): the centre-first order dealt round-robin over one
    // counter per XCD, so the claim atomics spread over 8 addresses while the order stays global
    const bool striped = !ordered && !(p->flags & RRT_RENDER_ONE_QUEUE) && !(p->flags & RRT_RENDER_XCD_QUEUES) &&
                         ((p->flags & RRT_RENDER_STRIPED_QUEUES) || lean == 1 || lean == 2);
    const uint32_t nq = (ordered || !(xcd_q || striped)) ? 1u : RRT_MAX_QUEUES;
    kp.q_stripe = striped ? 1u : 0u;
    std::vector<uint32_t> sector(n_tiles, 0);
    if (!ordered) {
      const double cx = 0.5 * p->frame_w, cy = 0.5 * p->frame_h;
      std::vector<double> key(n_tiles);
      for (uint32_t k = 0; k < n_tiles; ++k) {
        const double dx = tiles[2 * k] + 0.5 * ts - cx, dy = tiles[2 * k + 1] + 0.5 * ts - cy;
        key[k] = dx * dx + dy * dy;
        if (nq > 1 && !striped) {
          const double a = std::atan2(dy, dx) + kPI;  // [0, 2 pi]
          sector[k] = std::min<uint32_t>((uint32_t)(a * (nq / (2 * kPI))), nq - 1);
        }
      }
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return sector[a] != sector[b] ? sector[a] < sector[b] : key[a] < key[b];
      });
    }
    kp.n_queues = nq;
    for (uint32_t q = 0, k = 0; q < RRT_MAX_QUEUES; ++q) {
      while (k < n_tiles && sector[order[k]] == q) ++k;
      kp.q_end[q] = q < nq ? k * ts * ts : kp.n_pixels;
    }
    kp.q_end[nq - 1] = kp.n_pixels;
    if (c->order_cap < n_tiles) {
      hipFree(c->d_order); c->d_order = nullptr;
      HIPCHK(c, hipMalloc(&c->d_order, sizeof(uint32_t) * n_tiles));
      c->order_cap = n_tiles;
      c->h_order.clear();
    }
    if (order != c->h_order) {  // re-upload only when the tile list or its order changed
      c->h_order = order;
      HIPCHK(c, hipMemcpyAsync(c->d_order, c->h_order.data(), sizeof(uint32_t) * n_tiles, hipMemcpyHostToDevice,
                               stream));
    }
    kp.tile_order = c->d_order;
    kp.first = nullptr;
    kp.claim_list = nullptr; kp.claim_count = nullptr;
    // sample-0 pre-pass: off by default (with the slot speculation a wrong first hypothesis
    // costs one round, less than the extra pass; tools/ab_kernels.py cfg3 46.4 vs 47.8 ms)
    if ((p->flags & RRT_RENDER_PREPASS) && !(p->flags & RRT_RENDER_NO_FIRST)) {
      if (c->first_cap < kp.n_pixels) {
        hipFree(c->d_first); c->d_first = nullptr;
        HIPCHK(c, hipMalloc(&c->d_first, sizeof(KParams::FirstSample) * kp.n_pixels));
        c->first_cap = kp.n_pixels;
      }
      kp.first = c->d_first;
    }
    // pixel miss proof pass (rrt_pixel_proof_kernel): the area/point-light builds, whose misses
    // are black, with a claim order it can compact (striped or one queue); list entries keep bit
    // 31 for the first-hypothesis hint
    // The pass writes a proven pixel's result as the first adaptive check's stop on all-zero
    // samples, which holds only when 1.96 * 0 <= max_tolerance * 0 (a finite tolerance; with an
    // infinite or NaN one the reference runs all ns_aa samples, part1_code.cpp:147-158)
    const bool zero_stops = 0.0 <= (double)p->max_tolerance * 0.0 && p->samples_per_batch >= 2;
    if ((lean == 1 || lean == 2) && proofs_valid && zero_stops && !c->env_w && !kp.first && (striped || nq == 1) &&
        kp.n_pixels < 0x80000000u && !(p->flags & RRT_RENDER_NO_PIXEL_PROOF)) {
      if (c->list_cap < kp.n_pixels) {
        hipFree(c->d_list); c->d_list = nullptr;
        HIPCHK(c, hipMalloc(&c->d_list, sizeof(uint32_t) * kp.n_pixels));
        c->list_cap = kp.n_pixels;
      }
      kp.claim_list = c->d_list;
      kp.claim_count = c->d_counter + RRT_QUEUE_STRIDE * RRT_MAX_QUEUES;
      // hit-first claim order (rrt_pixel_proof_kernel); variant bit 22: the pass's order (A/B)
      kp.claim_back = ((p->variant >> 22) & 1u) ? 0u : 1u;
      // Heavy pixels (rrt_device.h pixel_heavy): the pass lists them apart and rrt_heavy_kernel
      // renders them slot-parallel, a block of waves per pixel (rrt_sample.hip
      // heavy_pixel_block); needs a hit to take a whole number of slots (Dh = k Dm)
      // Where the heavy pixels' latency bounds the launch: launches covering at most 60% of the
      // frame (one rank's tiles of a multi-GPU frame, the regions of the host path; cfg3 split 8
      // ways, slowest rank 8.1 -> 4.4 ms), and pixels of 4 or more adaptive steps, whose chains of
      // rounds outlast the frame (cfg4, 256 spp: 16.5 -> 15.0 ms).  A whole cfg3 frame (2 steps a
      // pixel) is bound by its throughput, and the heavy kernel's room in the batch grid costs more
      // than it saves (18.3 -> 19.0 ms).
      const uint64_t frame_px = (uint64_t)p->frame_w * p->frame_h;
      const bool share_ok = (p->flags & RRT_RENDER_HEAVY) || (uint64_t)kp.n_pixels * 5u <= frame_px * 3u ||
                            p->ns_aa >= 4u * p->samples_per_batch;
      if (!(p->flags & RRT_RENDER_NO_HEAVY) && share_ok && c->hole.r > 0.0 && kp.draws_hit % kp.draws_miss == 0) {
        // at most 1/256 of the pixels (4096 at least): a frame mostly near the hole stays with
        // the batch kernel, whose rounds cost less than 64 slots a step for unmixed pixels
        const uint32_t cap = std::min<uint32_t>(kp.n_pixels, std::max<uint32_t>(4096u, kp.n_pixels / 256u));
        if (c->heavy_list_cap < cap) {
          hipFree(c->d_heavy_list); c->d_heavy_list = nullptr;
          HIPCHK(c, hipMalloc(&c->d_heavy_list, sizeof(uint32_t) * cap));
          c->heavy_list_cap = cap;
        }
        kp.heavy_list = c->d_heavy_list;
        kp.heavy_count = c->d_counter + RRT_QUEUE_STRIDE * (RRT_MAX_QUEUES + 1);
        kp.heavy_cap = cap;

        // A/B (variant bits 16..19): 1: capture-boundary pixels only, 2 .. 6: near 1.1 / 1.5 / 2.0 / 3.0 / 5.0
        const uint32_t nv = (p->variant >> 16) & 0xfu;
        const double near = nv == 1 ? 0.0 : nv == 2 ? 1.1 : nv == 3 ? 1.5 : nv == 4 ? 2.0 : nv == 5 ? 3.0 : nv == 6 ? 5.0 : RRT_HEAVY_NEAR;
        kp.heavy_r2 = (near * c->hole.r) * (near * c->hole.r);
        // Continuations (rrt_sample.hip cont_push): in launches of at most 60% of the
        // frame (a rank's share), pixels of three or more adaptive steps go to waiting heavy blocks
        // after a check with two or more steps to go (cfg4, 256 spp: the 8-way split's ranks ended
        // on a few 8-step pixels, one step a round on the group path; profiles/r06_cont_w8_cfg4.txt).
        // A whole frame keeps them on the group path (its waiting heavy blocks cost ~2%).
        // A/B in the environment: RRT_AB_CONT=0 off / 1 on for any launch; RRT_AB_CONT_MIN=samples
        // left; RRT_AB_CONT_ROOM=batch blocks of room; RRT_AB_CONT_WAITERS=heavy blocks that wait
        const char* ce = std::getenv("RRT_AB_CONT");
        const bool part = (uint64_t)kp.n_pixels * 5u <= frame_px * 3u;
        const bool cont_on = p->ns_aa >= 3u * p->samples_per_batch && (ce ? ce[0] == '1' : part);
        if (cont_on && !setup_cont(part)) return RRT_E_HIP;
      }
    }
  }
  // The bounce (depth >= 2) per-pixel-loop kernel behind the pixel miss proof pass: a proven
  // pixel's samples all miss at any depth (est_radiance returns the black miss, 2 draws each), so
  // the pass writes it and the kernel claims only the listed pixels, 64 per wave, in a
  // centre-first order
  // The path pool kernel claims from the same centre-first order, listed or not.
  const bool deep_list = deep && !count && !sw && proofs_valid && !c->env_w && !kerr && kp.miss.on &&
                         0.0 <= (double)p->max_tolerance * 0.0 && p->samples_per_batch >= 2 &&
                         !(p->flags & RRT_RENDER_NO_PIXEL_PROOF);
  if (deep_list || path_pool) {
    kp.draws_miss = 2;
    kp.n_pixels = n_tiles * ts * ts;
    std::vector<uint32_t> order(n_tiles);
    for (uint32_t k = 0; k < n_tiles; ++k) order[k] = k;
    if (!(p->flags & RRT_RENDER_ORDERED)) {
      const double cx = 0.5 * p->frame_w, cy = 0.5 * p->frame_h;
      std::vector<double> key(n_tiles);
      for (uint32_t k = 0; k < n_tiles; ++k) {
        const double dx = tiles[2 * k] + 0.5 * ts - cx, dy = tiles[2 * k + 1] + 0.5 * ts - cy;
        key[k] = dx * dx + dy * dy;
      }
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
    }
    if (c->order_cap < n_tiles) {
      hipFree(c->d_order); c->d_order = nullptr;
      HIPCHK(c, hipMalloc(&c->d_order, sizeof(uint32_t) * n_tiles));
      c->order_cap = n_tiles;
      c->h_order.clear();
    }
    if (order != c->h_order) {
      c->h_order = order;
      HIPCHK(c, hipMemcpyAsync(c->d_order, c->h_order.data(), sizeof(uint32_t) * n_tiles, hipMemcpyHostToDevice, stream));
    }
    kp.tile_order = c->d_order;
    if (deep_list) {
      if (c->list_cap < kp.n_pixels) {
        hipFree(c->d_list); c->d_list = nullptr;
        HIPCHK(c, hipMalloc(&c->d_list, sizeof(uint32_t) * kp.n_pixels));
        c->list_cap = kp.n_pixels;
      }
      kp.claim_list = c->d_list;
      kp.claim_count = c->d_counter + RRT_QUEUE_STRIDE * RRT_MAX_QUEUES;
    }
  }
  // the pass's strip level: tiles whose rows split into strips of 64 claim indices (ts | 64 or 64 | ts)
  if (kp.claim_list && kp.n_pixels >= 64u) {
    const size_t ns = kp.n_pixels / 64u;
    if (c->strip_list_cap < ns) {
      hipFree(c->d_strip_list); c->d_strip_list = nullptr;
      HIPCHK(c, hipMalloc(&c->d_strip_list, sizeof(uint32_t) * ns));
      c->strip_list_cap = ns;
    }
    kp.strip_list = c->d_strip_list;
  }
  // run-time proof audit: counting launches that run the proofs (executed-work counts)
  if (count && kp.count_exec && c->audit_shift && c->d_audit) {
    kp.audit = c->d_audit;
    kp.audit_shift = c->audit_shift - 1u;
  }
  uint32_t want = batch ? (uint32_t)(((uint64_t)kp.n_pixels * kp.group + 255) / 256) : (kp.n_blocks + 3) / 4;
  uint32_t grid = std::min<uint32_t>(want, (uint32_t)c->n_cu * 8u);
  if (path_pool) {  // 256 paths a block, the resident blocks only (each path holds a stack slot)
    const uint32_t pw = (waves >= 2 && waves <= 4) ? (uint32_t)waves : (uint32_t)RRT_PATH_WAVES;
    grid = std::min<uint32_t>((kp.n_pixels + 255u) / 256u, (uint32_t)c->n_cu * pw);
    if (grid == 0) grid = 1;
    // levels 0 .. max_ray_depth - 1 of the recursion, then each path's pixel record
    const size_t bytes = sizeof(float) * RRT_PATH_FIELDS * ((size_t)p->max_ray_depth + 1u) * grid * 256u;
    if (c->path_stack_cap < bytes) {
      hipFree(c->d_path_stack); c->d_path_stack = nullptr; c->path_stack_cap = 0;
      HIPCHK(c, hipMalloc(&c->d_path_stack, bytes));
      c->path_stack_cap = bytes;
    }
    kp.path_stack = c->d_path_stack;
  }
  if (grid == 0) grid = 1;
  c->last_grid = grid;
#if RRT_PROFILE
  // diagnostic build: RRT_WATCHDOG_MS=<ms> gives every batch wave and heavy block a progress record
  // in host-coherent memory and waits for the launch at most that long; on a stall it prints the
  // records of the waves that have not exited and ends the process (the hang)
  const char* wd_env = std::getenv("RRT_WATCHDOG_MS");
  const long wd_ms = wd_env ? std::atol(wd_env) : 0;
  if (wd_ms > 0) {
    if (!c->h_wd) {
      HIPCHK(c, hipHostMalloc((void**)&c->h_wd, sizeof(uint32_t) * RRT_WD_WORDS, hipHostMallocCoherent | hipHostMallocMapped));
      HIPCHK(c, hipHostGetDevicePointer((void**)&c->d_wd, c->h_wd, 0));
    }
    HIPCHK(c, hipStreamSynchronize(stream));
    std::memset(c->h_wd, 0, sizeof(uint32_t) * RRT_WD_WORDS);
    kp.wd = c->d_wd;
  }
#endif
  // the heavy pixels' kernel (batch launches with a heavy list): its waves per pixel and grid, and
  // whether the batch kernel sizes its room for it on the device (variant bits 22 / 23: A/B)
  const uint32_t hgv = (p->variant >> 28) & 0xfu, nwv = (p->variant >> 20) & 3u;
  // waves per heavy pixel: 2 (a 64-sample pixel's two steps in one round), 4 with continuations
  // (256 slots a round: the rest of a 256-sample pixel); A/B: variant bits 20..21 = 1 / 2 / 3:
  // 1 (2 for the point-light build) / 4 / 2
  const int heavy_nw = nwv == 0 ? (kp.cont ? 4 : 2) : nwv == 1 ? (lean == 2 ? 2 : 1) : nwv == 2 ? 4 : 2;
  // heavy waves: hgv x the CU count (default 2), in blocks of heavy_nw waves
  const uint32_t heavy_waves = std::min<uint32_t>((uint32_t)c->n_cu * (hgv ? hgv : 2u), (uint32_t)c->n_cu * 4u);
  const uint32_t heavy_grid = std::max<uint32_t>(1u, heavy_waves / (uint32_t)heavy_nw);
  const bool no_room = (p->variant >> 23) & 1u;      // A/B: leave the batch grid as it is
  // A/B: round 3's fixed room, of (variant bits 12..15) - 1 blocks per CU beyond the heavy waves
  const bool static_room = ((p->variant >> 12) & 0xfu) != 0u;
  if (batch && kp.heavy_list && !no_room && !static_room) {
    kp.heavy_grid = heavy_grid;
    kp.heavy_nw = (uint32_t)heavy_nw;
  }
  // the batch kernel's waves/SIMD and grid (known before the upload: the heavy kernel's
  // continuation wait ends when all kp.batch_waves batch waves have exited)
  // waves/SIMD: the area-light build at 4 (cfg3 15.71 -> 15.33 ms, cfg2 10.33 -> 10.01 ms against
  // 5, since the search tree took the local oversized leaves), the point-light build at 5 (cfg4
  // 14.15 ms against 14.65 at 4) -- profiles/r03_heavy_ab.md
  const int bw = (wv >= 2 && wv <= 5) ? (int)wv : 4;
  // general / Kerr builds: 3 waves/SIMD by default (cfg5: 4.56 s at 2 waves, 3.37 s at 3)
  const int gw = (wv >= 2 && wv <= 5) ? (int)wv : 3;
  const int batch_w = lean == 1 ? bw : lean == 2 ? (wv >= 3 && wv <= 5 ? (int)wv : 5) : gw;
  uint32_t bgrid = grid;
  if (batch && kp.heavy_list) {
    // the batch grid leaves room for the heavy kernel's blocks (one per CU at most, <= 128 VGPRs
    // and 25 KB of LDS next to four batch blocks), whichever kernel the hardware dispatches first
    const uint32_t resident = (uint32_t)c->n_cu * (uint32_t)batch_w;  // blocks of 4 waves
    const uint32_t spare = (static_room ? ((p->variant >> 12) & 0xfu) - 1u : 0u) * (uint32_t)c->n_cu +
                           (heavy_waves + 3u) / 4u;  // room, in batch blocks
    if (static_room) {
      if (!no_room && bgrid + spare > resident) bgrid = resident > spare ? resident - spare : 1u;
    } else if (!no_room) {
      // room sized on the device to the heavy pixels the pass found (rrt_batch_kernel prologue,
      // kp.heavy_grid / heavy_nw): the grid is exactly the resident blocks, so a block that
      // leaves frees a slot no pending batch block can take
      bgrid = std::min(bgrid, resident);
    }
  }
  kp.batch_waves = bgrid * 4u;

  // tail priority threshold (A/B: RRT_AB_PRIO_TICKS in the environment)
  kp.prio_ticks = 50000u;
  if (const char* pt = std::getenv("RRT_AB_PRIO_TICKS")) kp.prio_ticks = (uint32_t)std::strtoul(pt, nullptr, 10);
  HIPCHK(c, hipMemcpyAsync(c->d_kp, &kp, sizeof(KParams), hipMemcpyHostToDevice, stream));
  const uint32_t ring = (uint32_t)(c->n_launch % rrt_ctx::kRing);
  HIPCHK(c, hipEventRecord(c->ev0[ring], stream));
  const char* tf[2] = {"false", "true"};
  char name[96];
  if (batch) {
    const int w = batch_w;
    char first[32] = "";
    const uint32_t fwv = (p->variant >> 8) & 0xfu;  // pre-pass waves/SIMD (A/B), default 3
    const int fw = (lean == 1 && (fwv == 4 || fwv == 5)) ? (int)fwv : 3;
    if (kp.first) std::snprintf(first, sizeof(first), "rrt_first_kernel<%d, %d> + ", lean, fw);
    if (kp.claim_list) std::snprintf(first, sizeof(first), "rrt_pixel_proof_kernel + ");
    std::snprintf(name, sizeof(name), "%srrt_batch_kernel<%d, %d>", first, lean, w);
    if (kp.first)
      HIPCHK(c, rrt_launch_first(kp, c->d_kp, lean, fw, std::min<uint32_t>((kp.n_pixels + 255) / 256, (uint32_t)c->n_cu * 8u),
                                 stream));
    if (kp.claim_list) HIPCHK(c, rrt_launch_pixel_proof(c->d_kp, kp.n_pixels, kp.strip_list != nullptr, stream));
    HIPCHK(c, hipEventRecord(c->ev_main[ring], stream));
    const uint32_t hwv = (p->variant >> 24) & 0xfu;
    const int hw = hwv == 5 ? 5 : 4;  // the heavy kernel's waves/SIMD budget
    if (kp.heavy_list) {
      // the heavy pixels' kernel (rrt_sample.hip rrt_heavy_kernel) on the side stream (its own
      // hardware queue), after the pass, beside the batch kernel
      HIPCHK(c, hipEventRecord(c->ev_go, stream));
      HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_go, 0));
      join_guard.state = 1;
      HIPCHK(c, rrt_launch_heavy(c->d_kp, lean, hw, heavy_nw, heavy_grid, RRT_HEAVY_LIST, c->side));
      HIPCHK(c, hipEventRecord(c->ev_heavy, c->side));
      join_guard.state = 2;
    }
    HIPCHK(c, rrt_launch_batch(kp, c->d_kp, lean, w, bgrid, stream));
    if (kp.heavy_list) {
      HIPCHK(c, hipStreamWaitEvent(stream, c->ev_heavy, 0));
      join_guard.state = 3;
      // continuations no block took (every waiter stopped first): rendered behind the kernels
      if (kp.cont) HIPCHK(c, rrt_launch_heavy(c->d_kp, lean, hw, heavy_nw, 16u, RRT_HEAVY_DRAIN, stream));
    }
  } else if (path_pool) {
    std::snprintf(name, sizeof(name), "%srrt_path_kernel<%d>", deep_list ? "rrt_pixel_proof_kernel + " : "",
                  (waves >= 2 && waves <= 4) ? waves : RRT_PATH_WAVES);
    if (deep_list) HIPCHK(c, rrt_launch_pixel_proof(c->d_kp, kp.n_pixels, kp.strip_list != nullptr, stream));
    HIPCHK(c, hipEventRecord(c->ev_main[ring], stream));
    HIPCHK(c, rrt_launch_path(c->d_kp, waves, grid, stream));
  } else if (pixel_loop) {
    std::snprintf(name, sizeof(name), "%srrt_render_kernel<%s, %s, %d, ...>", deep_list ? "rrt_pixel_proof_kernel + " : "",
                  tf[deep || sw], tf[count], lean == 2 ? 0 : lean);
    if (deep_list) HIPCHK(c, rrt_launch_pixel_proof(c->d_kp, kp.n_pixels, kp.strip_list != nullptr, stream));
    HIPCHK(c, hipEventRecord(c->ev_main[ring], stream));
    HIPCHK(c, rrt_launch_render(kp, c->d_kp, deep, count, lean, waves, grid, stream));
  } else {
    std::snprintf(name, sizeof(name), "%srrt_sample_kernel<%s, %d, %d, %s>", deep_list ? "rrt_pixel_proof_kernel + " : "",
                  tf[count], lean, deep_sample ? (waves == 2 || waves == 4 ? waves : 3) : waves, tf[deep_sample]);
    if (deep_list) HIPCHK(c, rrt_launch_pixel_proof(c->d_kp, kp.n_pixels, kp.strip_list != nullptr, stream));
    HIPCHK(c, hipEventRecord(c->ev_main[ring], stream));
    HIPCHK(c, rrt_launch_sample(kp, c->d_kp, count, lean, waves, grid, stream));
  }
  c->last_kernel = name;
  c->last_heavy = kp.heavy_list ? kp.heavy_cap : 0u;
  c->last_cont = kp.cont ? kp.cont_cap : 0u;
  HIPCHK(c, hipEventRecord(c->ev1[ring], stream));
#if RRT_PROFILE
  if (wd_ms > 0) {
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(wd_ms);
    hipError_t q;
    while ((q = hipEventQuery(c->ev1[ring])) == hipErrorNotReady && std::chrono::steady_clock::now() < t_end)
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (q == hipErrorNotReady) {
      std::fprintf(stderr, "WATCHDOG: launch '%s' not done after %ld ms (grid %u, heavy list %s); live records:\n",
                   name, wd_ms, c->last_grid, kp.heavy_list ? "on" : "off");
      int shown = 0, live_b = 0, live_h = 0;
      for (uint32_t w = 0; w < RRT_WD_WORDS / 4; ++w) {
        const volatile uint32_t* r = c->h_wd + 4 * w;
        if (r[3] == 0 || r[3] == 0xdeadu) continue;
        if (w < RRT_WD_HEAVY / 4) ++live_b; else ++live_h;
        if (shown++ < 64)
          std::fprintf(stderr, "  %s %u: it %u state 0x%x pixel %u marker 0x%x\n", w < RRT_WD_HEAVY / 4 ? "wave" : "heavy",
                       w < RRT_WD_HEAVY / 4 ? w : w - RRT_WD_HEAVY / 4, r[0], r[1], r[2], r[3]);
      }
      std::fprintf(stderr, "WATCHDOG: %d batch waves and %d heavy blocks not exited\n", live_b, live_h);
      std::fflush(stderr);
      _exit(3);
    }
  }
#endif
  c->timed = true;
  ++c->n_launch;
  return RRT_OK;
}

extern "C" int rrt_render_tiles_device(rrt_ctx* c, const rrt_render_params* p, const uint32_t* tiles,
                                       uint32_t n_tiles, uint32_t ts, float* d_rgb, int32_t* d_count,
                                       uint32_t* d_counters, void* stream) {
  if (!c || !p || (n_tiles && (!tiles || !d_rgb || !d_count))) return fail(c, RRT_E_INVALID, "null argument");
  hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t)0;
  return launch(c, p, tiles, n_tiles, ts, 0, 0, p->frame_w, p->frame_h, d_rgb, d_count, nullptr, d_counters, s);
}

extern "C" int rrt_unpack_tiles_device(rrt_ctx* c, const uint32_t* tiles, uint32_t n_tiles, uint32_t ts,
                                       uint32_t fw, uint32_t fh, const float* rgb_p, const int32_t* cnt_p,
                                       float* rgb, int32_t* cnt, void* stream) {
  if (!c || c->device < 0) return fail(c, RRT_E_NO_DEVICE, "no device");
  if (n_tiles == 0) return RRT_OK;
  hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t)0;
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = scratch_acquire(c, s)) return rc;
  struct FenceGuard {
    rrt_ctx* c; hipStream_t s;
    ~FenceGuard() { scratch_release(c, s); }
  } fence_guard{c, s};
  if (c->tiles_cap < n_tiles) {
    hipFree(c->d_tiles); c->d_tiles = nullptr;
    HIPCHK(c, hipMalloc(&c->d_tiles, sizeof(uint32_t) * 2 * n_tiles));
    c->tiles_cap = n_tiles;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_tiles, tiles, sizeof(uint32_t) * 2 * n_tiles, hipMemcpyHostToDevice, s));
  HIPCHK(c, rrt_launch_unpack(c->d_tiles, n_tiles, ts, fw, fh, rgb_p, cnt_p, rgb, cnt, s));
  return RRT_OK;
}

extern "C" int rrt_tonemap_device(rrt_ctx* c, uint32_t n, const float* rgb, uint32_t* rgba, void* stream) {
  if (!c || c->device < 0) return fail(c, RRT_E_NO_DEVICE, "no device");
  hipStream_t s = stream ? (hipStream_t)stream : (hipStream_t)0;
  // HDRImageBuffer::toColor: gamma 2.2f, level 1.0f, exposure = sqrt(pow(2, level))
  const float inv_gamma = 1.0f / 2.2f;
  const float exposure = (float)std::sqrt(std::pow(2, 1.0f));
  HIPCHK(c, rrt_launch_tonemap(n, rgb, rgba, exposure, inv_gamma, s));
  return RRT_OK;
}

extern "C" int rrt_libm_eval(rrt_ctx* c, int fn, const double* a, const double* b, double* out, uint64_t n) {
  if (!c || !a || !out || fn < 0 || fn > 10 || (fn == 3 && !b)) return fail(c, RRT_E_INVALID, "bad argument");
  if (c->device < 0) return fail(c, RRT_E_NO_DEVICE, "no device");
  if (n == 0) return RRT_OK;
  HIPCHK(c, hipSetDevice(c->device));
  double *da = nullptr, *db = nullptr, *dout = nullptr;
  struct Free {
    double** p[3];
    ~Free() { for (double** q : p) if (*q) (void)hipFree(*q); }
  } guard{{&da, &db, &dout}};
  const size_t bytes = sizeof(double) * n;
  HIPCHK(c, hipMalloc(&da, bytes));
  HIPCHK(c, hipMalloc(&dout, bytes));
  HIPCHK(c, hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
  if (fn == 3) {
    HIPCHK(c, hipMalloc(&db, bytes));
    HIPCHK(c, hipMemcpy(db, b, bytes, hipMemcpyHostToDevice));
  }
  HIPCHK(c, rrt_launch_libm(fn, n, da, db, dout, (hipStream_t)0));
  HIPCHK(c, hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost));
  return RRT_OK;
}

extern "C" int rrt_render(rrt_ctx* c, const rrt_render_params* p, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                          float* rgb_out, int32_t* count_out, uint32_t* draws_out, uint32_t* counters_out,
                          const volatile int* cancel) {
  if (!c || !p || !rgb_out || !count_out) return fail(c, RRT_E_INVALID, "null argument");
  if (w == 0 || h == 0) return RRT_OK;
  if ((uint64_t)x0 + w > p->frame_w || (uint64_t)y0 + h > p->frame_h) return fail(c, RRT_E_INVALID, "region outside frame");
  if (c->device < 0) return fail(c, RRT_E_NO_DEVICE, "host-only context cannot render");
  if (cancel && *cancel) return fail(c, RRT_E_CANCELLED, "cancelled");
  HIPCHK(c, hipSetDevice(c->device));
  const uint32_t ts = 32;
  std::vector<uint32_t> tiles;
  for (uint32_t ty = y0; ty < y0 + h; ty += ts)
    for (uint32_t tx = x0; tx < x0 + w; tx += ts) { tiles.push_back(tx); tiles.push_back(ty); }
  const uint32_t nt = (uint32_t)(tiles.size() / 2);
  const size_t npx = (size_t)nt * ts * ts;
  if (c->px_cap < npx) {
    size_t dummy = 0;
    int rc;
    if ((rc = ensure(c, (void**)&c->d_rgb, dummy, npx, 3 * sizeof(float)))) return rc;
    if ((rc = ensure(c, (void**)&c->d_cnt, dummy, npx, sizeof(int32_t)))) return rc;
    if ((rc = ensure(c, (void**)&c->d_draws, dummy, npx, sizeof(uint32_t)))) return rc;
    if ((rc = ensure(c, (void**)&c->d_ctr, dummy, npx, 4 * sizeof(uint32_t)))) return rc;
    c->px_cap = npx;
  }
  rrt_render_params q = *p;
  if (counters_out) q.flags |= RRT_RENDER_COUNTERS;
  int rc = launch(c, &q, tiles.data(), nt, ts, x0, y0, x0 + w, y0 + h, c->d_rgb, c->d_cnt,
                  draws_out ? c->d_draws : nullptr, counters_out ? c->d_ctr : nullptr, c->stream);
  if (rc) return rc;
  std::vector<float> rgb(npx * 3);
  std::vector<int32_t> cnt(npx);
  std::vector<uint32_t> drw(draws_out ? npx : 0), ctr(counters_out ? npx * 4 : 0);
  HIPCHK(c, hipMemcpyAsync(rgb.data(), c->d_rgb, npx * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(cnt.data(), c->d_cnt, npx * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  if (draws_out) HIPCHK(c, hipMemcpyAsync(drw.data(), c->d_draws, npx * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  if (counters_out)
    HIPCHK(c, hipMemcpyAsync(ctr.data(), c->d_ctr, npx * 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint32_t t = 0; t < nt; ++t) {
    for (uint32_t j = 0; j < ts; ++j) {
      for (uint32_t i = 0; i < ts; ++i) {
        uint32_t x = tiles[2 * t] + i, y = tiles[2 * t + 1] + j;
        if (x >= x0 + w || y >= y0 + h) continue;
        size_t k = (size_t)t * ts * ts + (size_t)j * ts + i;
        size_t o = (size_t)(y - y0) * w + (x - x0);
        rgb_out[3 * o] = rgb[3 * k]; rgb_out[3 * o + 1] = rgb[3 * k + 1]; rgb_out[3 * o + 2] = rgb[3 * k + 2];
        count_out[o] = cnt[k];
        if (draws_out) draws_out[o] = drw[k];
        if (counters_out) std::memcpy(counters_out + 4 * o, &ctr[4 * k], 4 * sizeof(uint32_t));
      }
    }
  }
  return RRT_OK;
}

extern "C" int rrt_get_stats(const rrt_ctx* cc, rrt_stats* out) {
  rrt_ctx* c = const_cast<rrt_ctx*>(cc);
  if (!c || !out) return RRT_E_INVALID;
  std::memset(out, 0, sizeof(*out));
  out->n_prims = (uint32_t)c->prims.size();
  out->n_nodes = (uint32_t)c->nodes.size();
  out->n_leaf_refs = (uint32_t)c->leaf.size();
  out->max_depth = c->max_depth;
  out->device_bytes = c->device_bytes;
  out->grid_blocks = c->last_grid;
  std::snprintf(out->kernel, sizeof(out->kernel), "%s", c->last_kernel.c_str());
  out->n_clean = c->has_clean ? (uint32_t)c->clean.size() : 0u;
  out->n_big = c->has_clean ? (uint32_t)c->big.size() : 0u;
  if (!c->grid.empty()) {
    for (int i = 0; i < 3; ++i) out->grid_n[i] = (uint32_t)c->hgrid.n[i];
    size_t free_cells = 0;
    for (uint8_t v : c->grid) free_cells += v > 2;
    out->grid_free_frac = (float)((double)free_cells / (double)c->grid.size());
  }
  out->block_threads = 256;
  if (c->device >= 0 && c->timed) {
    hipSetDevice(c->device);
    const uint32_t last = (uint32_t)((c->n_launch + rrt_ctx::kRing - 1) % rrt_ctx::kRing);
    if (hipEventSynchronize(c->ev1[last]) == hipSuccess) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, c->ev0[last], c->ev1[last]) == hipSuccess) c->last_ms = ms;
      if (hipEventElapsedTime(&ms, c->ev_main[last], c->ev1[last]) == hipSuccess) c->last_main_ms = ms;
    }
  }
  out->last_kernel_ms = c->last_ms;
  out->last_main_kernel_ms = c->last_main_ms;
  if (c->device >= 0 && c->timed && c->last_heavy) {  // the pass's heavy-list length (counters persist until the next launch)
    uint32_t n = 0;
    if (hipMemcpy(&n, c->d_counter + RRT_QUEUE_STRIDE * (RRT_MAX_QUEUES + 1), sizeof(n), hipMemcpyDeviceToHost) == hipSuccess)
      out->last_heavy_pixels = std::min<uint32_t>(n, c->last_heavy);
  }
  if (c->device >= 0 && c->timed && c->last_cont) {  // continuation records reserved (capped)
    uint32_t n = 0;
    if (hipMemcpy(&n, c->d_counter + RRT_QUEUE_STRIDE * (RRT_MAX_QUEUES + 2 + RRT_CONT_TAIL), sizeof(n),
                  hipMemcpyDeviceToHost) == hipSuccess)
      out->last_cont_pixels = std::min<uint32_t>(n, c->last_cont);
  }
  return RRT_OK;
}

// Per-launch HIP-event times of the context's last n launches (n <= 32), oldest first: the whole
// launch and its main kernel alone.  Synchronises on the last of them.  Returns the count filled.
extern "C" int rrt_set_proof_audit(rrt_ctx* c, int every_log2) {
  if (!c || every_log2 > 30) return c ? fail(c, RRT_E_INVALID, "every_log2 > 30") : RRT_E_INVALID;
  if (every_log2 < 0) {  // off
    c->audit_shift = 0;
    return RRT_OK;
  }
  if (c->device < 0) return fail(c, RRT_E_NO_DEVICE, "host-only context cannot render");
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->d_audit) {
    HIPCHK(c, hipMalloc(&c->d_audit, sizeof(unsigned long long) * 16));
    HIPCHK(c, hipMemset(c->d_audit, 0, sizeof(unsigned long long) * 16));
  }
  c->audit_shift = (uint32_t)every_log2 + 1u;
  return RRT_OK;
}
extern "C" int rrt_get_proof_audit(rrt_ctx* c, uint64_t* out) {
  if (!c || !out) return RRT_E_INVALID;
  for (int k = 0; k < 2 * RRT_AUDIT_KINDS; ++k) out[k] = 0;
  if (!c->d_audit) return RRT_OK;
  HIPCHK(c, hipSetDevice(c->device));
  unsigned long long h[16];
  HIPCHK(c, hipDeviceSynchronize());
  HIPCHK(c, hipMemcpy(h, c->d_audit, sizeof(h), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemset(c->d_audit, 0, sizeof(h)));
  for (int k = 0; k < 2 * RRT_AUDIT_KINDS; ++k) out[k] = h[k];
  return RRT_OK;
}

extern "C" int rrt_get_launch_times(const rrt_ctx* cc, uint32_t n, float* total_ms, float* main_ms) {
  rrt_ctx* c = const_cast<rrt_ctx*>(cc);
  if (!c || (n && (!total_ms || !main_ms))) return RRT_E_INVALID;
  if (c->device < 0) return fail(c, RRT_E_NO_DEVICE, "no device");
  const uint64_t have = std::min<uint64_t>(c->n_launch, rrt_ctx::kRing);
  const uint32_t k = (uint32_t)std::min<uint64_t>(n, have);
  HIPCHK(c, hipSetDevice(c->device));
  for (uint32_t i = 0; i < k; ++i) {
    const uint32_t slot = (uint32_t)((c->n_launch - k + i) % rrt_ctx::kRing);
    HIPCHK(c, hipEventSynchronize(c->ev1[slot]));
    HIPCHK(c, hipEventElapsedTime(&total_ms[i], c->ev0[slot], c->ev1[slot]));
    HIPCHK(c, hipEventElapsedTime(&main_ms[i], c->ev_main[slot], c->ev1[slot]));
  }
  return (int)k;
}

extern "C" int rrt_get_free_grid(const rrt_ctx* c, uint8_t* k, double* geom, int32_t* n) {
  if (!c || !c->has_scene) return RRT_E_INVALID;
  if (c->grid.empty()) return 0;
  if (k) std::memcpy(k, c->grid.data(), c->grid.size());
  if (geom) {
    for (int i = 0; i < 3; ++i) geom[i] = c->hgrid.g0[i];
    geom[3] = c->hgrid.inv_h; geom[4] = c->hgrid.h_free;
  }
  if (n) for (int i = 0; i < 3; ++i) n[i] = c->hgrid.n[i];
  return (int)std::min<size_t>(c->grid.size(), 0x7fffffff);
}

extern "C" int rrt_get_occluders(const rrt_ctx* c, double* tris, uint32_t* counts) {
  if (!c || !c->has_scene) return RRT_E_INVALID;
  int total = 0;
  for (int f = 0; f < 6; ++f) {
    if (counts) counts[f] = c->occ.n[f];
    if (tris) std::memcpy(tris + 16 * RRT_OCC_PER_FACE * f, c->occ.tri[f], sizeof(c->occ.tri[f]));
    total += (int)c->occ.n[f];
  }
  return total;
}

extern "C" int rrt_get_big_masks(const rrt_ctx* c, uint32_t* mask, double* reach) {
  if (!c || !c->has_scene) return RRT_E_INVALID;
  if (mask && !c->big_mask.empty()) std::memcpy(mask, c->big_mask.data(), c->big_mask.size() * sizeof(uint32_t));
  if (reach) *reach = (RRT_BIG_REACH - 1) * c->hgrid.h_free;
  return (int)std::min<size_t>(c->big_mask.size(), 0x7fffffff);
}

extern "C" int rrt_get_search_tree(const rrt_ctx* c, double* boxes, int32_t* nodes) {
  if (!c || !c->has_scene) return RRT_E_INVALID;
  for (size_t i = 0; i < c->free_tree.size(); ++i) {
    const DNode& n = c->free_tree[i];
    if (boxes) for (int k = 0; k < 3; ++k) { boxes[6 * i + k] = n.mn[k]; boxes[6 * i + 3 + k] = n.mx[k]; }
    if (nodes) { nodes[4 * i] = n.skip; nodes[4 * i + 1] = n.first; nodes[4 * i + 2] = n.count; nodes[4 * i + 3] = n.pad; }
  }
  return (int)c->free_tree.size();
}

extern "C" int rrt_get_search_tree4(const rrt_ctx* c, float* boxes, int32_t* kids) {
  if (!c || !c->has_scene) return RRT_E_INVALID;
  for (size_t i = 0; i < c->free4.size(); ++i) {
    const DNode4& n = c->free4[i];
    for (int j = 0; j < 4; ++j) {
      if (boxes) {
        float* b = boxes + 24 * i + 6 * j;
        b[0] = n.mnx[j]; b[1] = n.mny[j]; b[2] = n.mnz[j]; b[3] = n.mxx[j]; b[4] = n.mxy[j]; b[5] = n.mxz[j];
      }
      if (kids) { kids[12 * i + 3 * j] = n.child[j]; kids[12 * i + 3 * j + 1] = n.first[j]; kids[12 * i + 3 * j + 2] = n.count[j]; }
    }
  }
  return (int)c->free4.size();
}

extern "C" int rrt_get_clean_tree(const rrt_ctx* c, double* boxes, int32_t* nodes, double* big_boxes,
                                  int32_t* big) {
  if (!c || !c->has_scene) return RRT_E_INVALID;
  if (!c->has_clean) return 0;
  for (size_t i = 0; i < c->clean.size(); ++i) {
    const DNode& n = c->clean[i];
    if (boxes) for (int k = 0; k < 3; ++k) { boxes[6 * i + k] = n.mn[k]; boxes[6 * i + 3 + k] = n.mx[k]; }
    if (nodes) { nodes[4 * i] = n.skip; nodes[4 * i + 1] = n.first; nodes[4 * i + 2] = n.count; nodes[4 * i + 3] = n.pad; }
  }
  for (size_t i = 0; i < c->big.size(); ++i) {
    const DBig& b = c->big[i];
    if (big_boxes) for (int k = 0; k < 3; ++k) { big_boxes[6 * i + k] = b.mn[k]; big_boxes[6 * i + 3 + k] = b.mx[k]; }
    if (big) { big[3 * i] = b.first; big[3 * i + 1] = b.count; big[3 * i + 2] = b.dfs; }
  }
  return (int)c->clean.size();
}

extern "C" int rrt_get_bvh(const rrt_ctx* c, double* boxes, int32_t* nodes, uint32_t* prims) {
  if (!c || !c->has_scene) return RRT_E_INVALID;
  for (size_t i = 0; i < c->nodes.size(); ++i) {
    const BNode& n = c->nodes[i];
    if (boxes) {
      double b[6] = {n.bb.mn.x, n.bb.mn.y, n.bb.mn.z, n.bb.mx.x, n.bb.mx.y, n.bb.mx.z};
      std::memcpy(boxes + 6 * i, b, sizeof(b));
    }
    if (nodes) { nodes[4 * i] = n.first; nodes[4 * i + 1] = n.count; nodes[4 * i + 2] = n.left; nodes[4 * i + 3] = n.right; }
  }
  if (prims) std::memcpy(prims, c->leaf.data(), c->leaf.size() * sizeof(uint32_t));
  return RRT_OK;
}

// ---------------------------------------------------------------------------- file helpers
static bool rd(FILE* f, void* p, size_t n) { return std::fread(p, 1, n, f) == n; }

extern "C" int rrt_scene_file_load(const char* path, rrt_scene_file** out) {
  if (!path || !out) return RRT_E_INVALID;
  *out = nullptr;
  FILE* f = std::fopen(path, "rb");
  if (!f) return RRT_E_IO;
  std::unique_ptr<rrt_scene_file> s(new rrt_scene_file());
  char magic[8];
  uint32_t hdr[4];
  bool ok = rd(f, magic, 8) && std::memcmp(magic, RRT_SCENE_MAGIC, 8) == 0 && rd(f, hdr, 16);
  if (ok) {
    s->bsdfs.resize(hdr[0]);
    for (auto& b : s->bsdfs) {
      uint32_t tp[2];
      ok = ok && rd(f, tp, 8) && rd(f, b.params, 56);
      b.type = tp[0];
    }
    s->objects.resize(hdr[1]);
    s->dbl.reserve(2 * hdr[1]);
    s->idx.reserve(hdr[1]);
    for (auto& o : s->objects) {
      if (!ok) break;
      uint32_t oh[4];
      ok = rd(f, oh, 16);
      std::memset(&o, 0, sizeof(o));
      o.kind = oh[0]; o.bsdf = oh[1];
      if (ok && oh[0] == RRT_OBJ_MESH) {
        o.n_vertices = oh[2]; o.n_triangles = oh[3];
        s->dbl.emplace_back((size_t)oh[2] * 3);
        s->dbl.emplace_back((size_t)oh[2] * 3);
        s->idx.emplace_back((size_t)oh[3] * 3);
        auto& P = s->dbl[s->dbl.size() - 2];
        auto& N = s->dbl.back();
        auto& I = s->idx.back();
        ok = rd(f, P.data(), P.size() * 8) && rd(f, N.data(), N.size() * 8) && rd(f, I.data(), I.size() * 4);
        o.positions = P.data(); o.normals = N.data(); o.indices = I.data();
      } else if (ok && oh[0] == RRT_OBJ_SPHERE) {
        double sp[4];
        ok = rd(f, sp, 32);
        o.center[0] = sp[0]; o.center[1] = sp[1]; o.center[2] = sp[2]; o.radius = sp[3];
      } else {
        ok = false;
      }
    }
    s->lights.resize(hdr[2]);
    for (auto& l : s->lights) {
      if (!ok) break;
      uint32_t th[2]; float fv[4];
      ok = rd(f, th, 8) && rd(f, fv, 16) && rd(f, l.v, 96);
      l.type = th[0]; l.is_delta = th[1];
      l.radiance[0] = fv[0]; l.radiance[1] = fv[1]; l.radiance[2] = fv[2]; l.area = fv[3];
    }
  }
  std::fclose(f);
  if (!ok) return RRT_E_IO;
  s->finalize();
  *out = s.release();
  return RRT_OK;
}
extern "C" const rrt_scene_desc* rrt_scene_file_desc(const rrt_scene_file* f) { return f ? &f->desc : nullptr; }
extern "C" void rrt_scene_file_free(rrt_scene_file* f) { delete f; }

extern "C" int rrt_camera_file_load(const char* path, rrt_camera_desc* out) {
  if (!path || !out) return RRT_E_INVALID;
  FILE* f = std::fopen(path, "rb");
  if (!f) return RRT_E_IO;
  char magic[8];
  double d[RRT_CAMERA_NDOUBLES];
  bool ok = rd(f, magic, 8) && std::memcmp(magic, RRT_CAMERA_MAGIC, 8) == 0 && rd(f, d, sizeof(d));
  std::fclose(f);
  if (!ok) return RRT_E_IO;
  std::memset(out, 0, sizeof(*out));
  out->hFov = d[0]; out->vFov = d[1]; out->nClip = d[3]; out->fClip = d[4];
  for (int i = 0; i < 3; ++i) out->pos[i] = d[5 + i];
  std::memcpy(out->c2w, d + 16, 9 * sizeof(double));
  out->focalDistance = d[28]; out->lensRadius = d[29];
  return RRT_OK;
}

// ------------------------------------------------------------------------------ device groups
// One frame region over several contexts (one per GPU): the reference's worker pool over tiles
// (pathtracer.cpp:251-255, 279-281, 611-644) as one launch per GPU.  The region's 32x32 tiles
// are dealt over the members as a lattice (rrt_partition_tiles' rule), every member renders
// its tiles into one packed buffer on its own stream, and the buffers are gathered to member 0
// -- over RCCL (grouped ncclSend / ncclRecv, xGMI between MI355X) when the members sit on
// distinct devices, by device copies when several members share one device (a one-GPU run of
// the same plan) -- and unpacked there into the region.  Pixels are independent under the keyed
// RNG, so the result equals a one-context render bit for bit.  RCCL is loaded on first use
// (dlopen, local symbols), so librrt needs no RCCL unless a group spans several devices.
#include <dlfcn.h>
#include <rccl/rccl.h>

struct rrt_group {
  std::vector<rrt_ctx*> ctx;  // not owned
  bool distinct = false;      // every member on its own device: RCCL
  void* rccl = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) err_str = nullptr;
  std::vector<ncclComm_t> comm;  // empty after a failed collective (the group then refuses to render)
  decltype(&ncclCommAbort) comm_abort = nullptr;
  std::vector<int32_t*> packed;  // per member, on its device: [n_max * T^2 * 3] f32 rgb, [n_max * T^2] i32 count
  std::vector<int32_t*> inbox;   // on member 0's device, one per other member
  size_t words = 0;              // capacity of each packed / inbox buffer, int32 words
  float* frame_rgb = nullptr;    // the whole frame on member 0 (unpack target)
  int32_t* frame_cnt = nullptr;
  size_t frame_px = 0;
  std::vector<hipEvent_t> ready;  // per member: its packed buffer is written (device-copy gather)
};

static int group_fail(rrt_group* g, int code, const std::string& msg) { return fail(g->ctx[0], code, msg); }
#define GCHK(g, x)                                                                                    \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) return group_fail(g, RRT_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCHK(g, x)                                                                                   \
  do {                                                                                               \
    ncclResult_t r_ = (x);                                                                           \
    if (r_ != ncclSuccess) return group_fail(g, RRT_E_HIP, std::string(#x) + ": " + g->err_str(r_)); \
  } while (0)

static int group_load_rccl(rrt_group* g) {
  g->rccl = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!g->rccl) g->rccl = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
  if (!g->rccl) return group_fail(g, RRT_E_HIP, std::string("cannot load RCCL: ") + dlerror());
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(g->rccl, name));
    return fn != nullptr;
  };
  if (!(sym(g->comm_init_all, "ncclCommInitAll") && sym(g->comm_destroy, "ncclCommDestroy") &&
        sym(g->group_start, "ncclGroupStart") && sym(g->group_end, "ncclGroupEnd") && sym(g->send, "ncclSend") &&
        sym(g->recv, "ncclRecv") && sym(g->err_str, "ncclGetErrorString") && sym(g->comm_abort, "ncclCommAbort")))
    return group_fail(g, RRT_E_HIP, "RCCL lacks ncclSend / ncclRecv / ncclCommInitAll");
  std::vector<int> devs;
  for (rrt_ctx* c : g->ctx) devs.push_back(c->device);
  g->comm.assign(g->ctx.size(), nullptr);
  NCHK(g, g->comm_init_all(g->comm.data(), (int)devs.size(), devs.data()));
  return RRT_OK;
}

extern "C" void rrt_group_destroy(rrt_group* g) {
  if (!g) return;
  for (size_t i = 0; i < g->ctx.size(); ++i) {
    hipSetDevice(g->ctx[i]->device);
    if (i < g->packed.size()) hipFree(g->packed[i]);
    if (i < g->ready.size() && g->ready[i]) hipEventDestroy(g->ready[i]);
  }
  if (!g->ctx.empty()) {
    hipSetDevice(g->ctx[0]->device);
    for (int32_t* b : g->inbox) hipFree(b);
    hipFree(g->frame_rgb);
    hipFree(g->frame_cnt);
  }
  for (ncclComm_t cm : g->comm)
    if (cm && g->comm_destroy) g->comm_destroy(cm);
  if (g->rccl) dlclose(g->rccl);
  delete g;
}

extern "C" int rrt_group_create(rrt_ctx* const* ctxs, uint32_t n, rrt_group** out) {
  if (!out || !ctxs || n == 0) return RRT_E_INVALID;
  *out = nullptr;
  std::unique_ptr<rrt_group, void (*)(rrt_group*)> g(new rrt_group(), rrt_group_destroy);
  for (uint32_t i = 0; i < n; ++i) {
    if (!ctxs[i]) return RRT_E_INVALID;
    if (ctxs[i]->device < 0) return fail(ctxs[i], RRT_E_NO_DEVICE, "host-only context cannot join a device group");
    g->ctx.push_back(ctxs[i]);
  }
  std::vector<int> devs;
  for (rrt_ctx* c : g->ctx) devs.push_back(c->device);
  std::sort(devs.begin(), devs.end());
  g->distinct = n > 1 && std::adjacent_find(devs.begin(), devs.end()) == devs.end();
  g->ready.assign(n, nullptr);
  for (uint32_t i = 0; i < n; ++i) {
    GCHK(g.get(), hipSetDevice(g->ctx[i]->device));
    GCHK(g.get(), hipEventCreateWithFlags(&g->ready[i], hipEventDisableTiming));
  }
  if (g->distinct)
    if (int rc = group_load_rccl(g.get())) return rc;
  *out = g.release();
  return RRT_OK;
}

extern "C" int rrt_group_render(rrt_group* g, const rrt_render_params* p, uint32_t x0, uint32_t y0, uint32_t w,
                                uint32_t h, float* rgb_out, int32_t* count_out, const volatile int* cancel) {
  if (!g || !p || !rgb_out || !count_out) return RRT_E_INVALID;
  if (w == 0 || h == 0) return RRT_OK;
  if ((uint64_t)x0 + w > p->frame_w || (uint64_t)y0 + h > p->frame_h)
    return group_fail(g, RRT_E_INVALID, "region outside frame");
  const uint32_t n = (uint32_t)g->ctx.size(), ts = 32, T2 = ts * ts;
  if (g->distinct && g->comm.empty())
    return group_fail(g, RRT_E_HIP, "the group's RCCL communicators were aborted after a failed gather");
  // the region's tiles, dealt over the members as a lattice (rrt_region_tiles)
  std::vector<std::vector<uint32_t>> tiles(n);
  for (uint32_t i = 0; i < n; ++i) {
    const int nt = rrt_region_tiles(x0, y0, w, h, ts, i, n, nullptr, 0);
    tiles[i].resize(2 * (size_t)nt);
    if (nt > 0) rrt_region_tiles(x0, y0, w, h, ts, i, n, tiles[i].data(), (uint32_t)nt);
  }
  size_t n_max = 0;
  for (const auto& t : tiles) n_max = std::max(n_max, t.size() / 2);
  const size_t words = n_max * T2 * 4;
  if (words > g->words) {  // (re)allocate the packed buffers and member 0's inbox
    for (uint32_t i = 0; i < n; ++i) {
      GCHK(g, hipSetDevice(g->ctx[i]->device));
      if (i < g->packed.size()) hipFree(g->packed[i]);
    }
    g->packed.assign(n, nullptr);
    for (uint32_t i = 0; i < n; ++i) {
      GCHK(g, hipSetDevice(g->ctx[i]->device));
      GCHK(g, hipMalloc(&g->packed[i], words * 4));
    }
    GCHK(g, hipSetDevice(g->ctx[0]->device));
    for (int32_t* b : g->inbox) hipFree(b);
    g->inbox.assign(n, nullptr);
    for (uint32_t i = 1; i < n; ++i) GCHK(g, hipMalloc(&g->inbox[i], words * 4));
    g->words = words;
  }
  const size_t fpx = (size_t)p->frame_w * p->frame_h;
  if (fpx > g->frame_px) {
    GCHK(g, hipSetDevice(g->ctx[0]->device));
    hipFree(g->frame_rgb); hipFree(g->frame_cnt);
    g->frame_rgb = nullptr; g->frame_cnt = nullptr;
    GCHK(g, hipMalloc(&g->frame_rgb, fpx * 3 * sizeof(float)));
    GCHK(g, hipMalloc(&g->frame_cnt, fpx * sizeof(int32_t)));
    g->frame_px = fpx;
  }
  const size_t cnt_off = g->words / 4 * 3;  // first count word of a packed buffer
  // every member renders its tiles (launches are asynchronous: the GPUs run together)
  for (uint32_t i = 0; i < n; ++i) {
    if (cancel && *cancel) return group_fail(g, RRT_E_CANCELLED, "cancelled");
    rrt_ctx* c = g->ctx[i];
    const uint32_t nt = (uint32_t)(tiles[i].size() / 2);
    if (nt == 0) continue;
    int32_t* buf = g->packed[i];
    if (int rc = launch(c, p, tiles[i].data(), nt, ts, x0, y0, x0 + w, y0 + h, (float*)buf, buf + cnt_off, nullptr,
                        nullptr, c->stream)) {
      // the group reports through member 0's context (rrt_last_error(ctx[0]))
      if (i > 0) g->ctx[0]->err = "group member " + std::to_string(i) + ": " + c->err;
      return rc;
    }
    GCHK(g, hipEventRecord(g->ready[i], c->stream));
  }
  // gather to member 0: the frame's only exchange
  rrt_ctx* c0 = g->ctx[0];
  if (g->distinct) {
    // Every member's send is paired with member 0's receive of it, both skipped together for a
    // member without tiles (so no rank waits on a message that is never sent); each call runs
    // with its communicator's device current.  A failed call aborts every communicator (their
    // state after a failed group is undefined) and the group refuses later renders.
    auto abort_all = [&](const std::string& what, ncclResult_t r) {
      for (uint32_t i = 0; i < n && i < g->comm.size(); ++i) {
        hipSetDevice(g->ctx[i]->device);
        if (g->comm[i]) g->comm_abort(g->comm[i]);
      }
      g->comm.clear();
      return group_fail(g, RRT_E_HIP, what + ": " + g->err_str(r));
    };
    ncclResult_t r = g->group_start();
    if (r != ncclSuccess) return abort_all("ncclGroupStart", r);
    for (uint32_t i = 1; i < n && r == ncclSuccess; ++i) {
      if (tiles[i].empty()) continue;
      (void)hipSetDevice(g->ctx[i]->device);  // (no early return inside the group)
      r = g->send(g->packed[i], g->words, ncclInt32, 0, g->comm[i], g->ctx[i]->stream);
      if (r != ncclSuccess) break;
      (void)hipSetDevice(c0->device);
      r = g->recv(g->inbox[i], g->words, ncclInt32, (int)i, g->comm[0], c0->stream);
    }
    const ncclResult_t re = g->group_end();  // closes the group even after a failed call inside it
    if (r != ncclSuccess) return abort_all("ncclSend / ncclRecv", r);
    if (re != ncclSuccess) return abort_all("ncclGroupEnd", re);
  } else {
    GCHK(g, hipSetDevice(c0->device));
    for (uint32_t i = 1; i < n; ++i) {
      if (tiles[i].empty()) continue;
      GCHK(g, hipStreamWaitEvent(c0->stream, g->ready[i], 0));
      GCHK(g, hipMemcpyPeerAsync(g->inbox[i], c0->device, g->packed[i], g->ctx[i]->device, g->words * 4, c0->stream));
    }
  }
  // unpack every member's tiles into the frame on member 0, then copy the region out
  GCHK(g, hipSetDevice(c0->device));
  for (uint32_t i = 0; i < n; ++i) {
    if (tiles[i].empty()) continue;
    const int32_t* buf = i == 0 ? g->packed[0] : g->inbox[i];
    if (int rc = rrt_unpack_tiles_device(c0, tiles[i].data(), (uint32_t)(tiles[i].size() / 2), ts, p->frame_w,
                                         p->frame_h, (const float*)buf, buf + cnt_off, g->frame_rgb, g->frame_cnt,
                                         c0->stream))
      return rc;
  }
  GCHK(g, hipMemcpy2DAsync(rgb_out, (size_t)w * 3 * sizeof(float), g->frame_rgb + ((size_t)y0 * p->frame_w + x0) * 3,
                           (size_t)p->frame_w * 3 * sizeof(float), (size_t)w * 3 * sizeof(float), h,
                           hipMemcpyDeviceToHost, c0->stream));
  GCHK(g, hipMemcpy2DAsync(count_out, (size_t)w * sizeof(int32_t), g->frame_cnt + (size_t)y0 * p->frame_w + x0,
                           (size_t)p->frame_w * sizeof(int32_t), (size_t)w * sizeof(int32_t), h,
                           hipMemcpyDeviceToHost, c0->stream));
  GCHK(g, hipStreamSynchronize(c0->stream));
  for (uint32_t i = 1; i < n; ++i) {  // the members' streams are done too (their buffers are reused next)
    GCHK(g, hipSetDevice(g->ctx[i]->device));
    GCHK(g, hipStreamSynchronize(g->ctx[i]->stream));
  }
  return RRT_OK;
}
