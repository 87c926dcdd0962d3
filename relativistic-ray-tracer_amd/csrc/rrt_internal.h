// rrt_internal.h -- device data layout shared by the host side (rrt_host.cpp) and the
// kernels (rrt_kernel.hip).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <stdint.h>

#define RRT_MAX_LIGHTS 16
#define RRT_MAX_BSDFS 64
#define RRT_MAX_DEPTH 16
#define RRT_PATH_FIELDS 13  // the path pool kernel's stack: words per recursion level (rrt_path.hip)
#define RRT_PATH_WAVES 4    // ... and its default register budget (waves per SIMD)
#define RRT_BIG_REACH 10   // oversized-leaf cell masks: dilation radius in grid cells (rrt_host.cpp)

// BVH node, 64 B, left-first pre-order (the reference's recursion order, bvh.cpp:115-138).
// Left child of an inner node is always index + 1; `skip` is the pre-order successor of the
// whole subtree, so "bbox missed or leaf done -> skip, else -> index + 1" visits exactly the
// nodes the reference's left-then-right recursion visits, in the same order, with no stack.
struct alignas(16) DNode {
  double mn[3];
  double mx[3];
  int32_t skip;    // next node after this subtree (-1: done)
  int32_t first;   // leaf: first slot in the leaf arrays
  int32_t count;   // leaf: number of slots (0: inner node)
  int32_t pad;
};
static_assert(sizeof(DNode) == 64, "DNode must be 64 bytes");

// 4-wide node of the search tree (rrt_host.cpp build_free4; rrt_device.h traverse_free4): the boxes of
// up to four children -- the search tree's nodes two levels down -- as structure of arrays, in f32
// rounded outward and widened by KParams::free4_pad: a conservative pre-test only (a leaf child that
// passes it takes the exact test on its own f64 box, kp.free_nodes[child]).  A child is an inner node
// (count 0: child = DNode4 index), a leaf of the search tree (count > 0: slots [first, first + count),
// child = its search-tree node index, the replay's ref) or empty (count < 0).
struct alignas(16) DNode4 {
  float mnx[4], mny[4], mnz[4], mxx[4], mxy[4], mxz[4];
  int32_t child[4], first[4], count[4], pad[4];
};
static_assert(sizeof(DNode4) == 160, "DNode4 must be 160 bytes");

// Oversized leaf of the reference tree, tested directly by the clean-tree walk
// (rrt_device.h traverse_clean): its box, leaf slots and left-first leaf ordinal.
struct alignas(16) DBig {
  double mn[3];
  double mx[3];
  int32_t first, count, dfs, pad;
};

// Leaf-slot geometry, 72 B (9 doubles) per slot, slots in leaf order.
//   triangle: p0, e1 = p1 - p0, e2 = p2 - p0 (exactly the values triangle.cpp:31-32 computes)
//   sphere:   c.x, c.y, c.z, r2, r, 0...
struct DPrimGeo { double v[9]; };
// Leaf-slot supporting plane (unit normal n, offset c = n . p0) for the cull in
// rrt_device.h leaf_prims; n = 0, c = 0 (never culls) for spheres and sliver triangles.
struct DPlane { double n[3]; double c; };
// Leaf-slot shading data: vertex normals n0, n1, n2 (triangle) -- read only on an accepted hit.
struct DPrimNrm { double n[9]; };
// Leaf-slot metadata: bit 0 = sphere, bits 8..15 = bsdf index.
typedef uint32_t DPrimMeta;

struct DBsdf {
  uint32_t type;
  float p[14];
};
struct DLight {
  uint32_t type, is_delta;
  float rad[3];
  float area;
  double v[4][3];
};

// Environment light (EnvironmentLight, environment_light.cpp:21-148): texels and the sampling
// tables the reference builds in init() (pdf, per-row conditional CDFs, marginal CDF), all on
// the host with the reference's arithmetic.  w == 0: no environment map.
struct DEnv {
  const float* tex;      // [h][w][3] Spectrum
  const double* pdf;     // [h][w] normalised pdf_envmap
  const double* conds;   // [h][w] conds_y
  const double* marg;    // [h]    marginal_y
  uint32_t w, h;
};

struct DCamera {
  double pos[3];
  double c2w0[3], c2w1[3], c2w2[3];   // columns
  double blx, bly;                     // -tan(radians(fov)/2), host libm (part1_code.cpp:183)
};
enum { HOLE_SCHWARZSCHILD = 0, HOLE_KERR = 1 };  // rrt_spacetime_desc.kind
struct DHole {
  double c[3];
  double r, r2, dt, cos_dt, sin_dt;    // cos/sin(dt) from host libm (blackhole.cpp:36-37)
  int32_t steps;                        // #{j : j * dt < 2 pi}  (bvh.cpp:105)
  int32_t kind;                         // HOLE_SCHWARZSCHILD / HOLE_KERR (= RRT_METRIC_*, include/rrt.h)
  // Kerr (rrt_device.h kerr_*): M = r_s / 2, a = spin * M, local frame (ez = spin axis)
  double m, a, a2, r_hor;               // r_hor = M + sqrt(M^2 - a^2) (outer horizon)
  double ex[3], ey[3], ez[3];
  double r_esc2;                        // per launch: max(|root box corner - c|^2, (4M)^2)
  int32_t kerr_max_steps, pad2;         // 4 * steps
};

// Empty-space grid over the root box (rrt_host.cpp build_free_grid): cell value k = Chebyshev
// distance, in cells, to the nearest cell touched by a BVH leaf box (cells of leaf boxes
// widened by one, capped at 255).  Every point of cell c lies at least (k - 2) * h from every
// leaf box, so a micro segment starting in c that is shorter than that reaches no leaf box:
// every leaf slab test fails, no primitive is tested, and the reference's traversal returns
// "no hit" -- the traversal can be skipped without changing any result.
struct DGrid {
  const uint8_t* k;   // [n[2]][n[1]][n[0]]; null = no grid
  double g0[3];       // root box minimum
  double inv_h;       // 1 / cell size
  double h_free;      // cell size * (1 - 2^-20): the free radius of value k is (k - 2) * h_free
  int32_t n[3];
  int32_t pad;
};

// Camera-ray miss proof (rrt_device.h camera_miss_proof): the constants of the
// planar recurrence that the reference's Schwarzschild march follows, and the margins.
struct DMissProof {
  double co1, si1;        // cos_dt / rho, sin_dt / rho  (rho = |(cos_dt, sin_dt)|)
  double rho, inv_rho, inv_si;
  double k15;             // 1.5 * r_s: f(u) = -u + k15 u^2 (blackhole.cpp:13-15)
  double dt2_4, dt2_6;    // dt^2 / 4, dt^2 / 6
  double kappa;           // a step whose |v| < kappa (|s| + |up dt|) is not certain: no proof
  double eta;             // relative position margin (>= 1e3 x the measured deviation bound)
  double scale;           // scene distance scale about the hole (margin floor)
  double lo[3], hi[3];    // root box
  double r_ball;          // distance from the hole to the farthest root-box corner (x (1 + 1e-9))
  uint32_t on, pad;
};

// Shadow-ray occlusion proof (rrt_device.h shadow_occluded_proof): triangles that
// lie along the root box's faces (a Cornell box's walls), as the reference intersects them
// (p0, p0 + e1, p0 + e2).  Face f: axis f % 3, the box's low face for f < 3, else its high face.
// n . x - d: signed distance from the triangle's plane, positive on the box's inner side;
// en[i] . x - eo[i]: distance inside edge i within the plane (unit, inward).  A segment end past
// the trigger box [in_lo, in_hi] (the root box shrunk past every kept triangle by a margin) is
// tested against the triangles of the faces it is past.
#define RRT_OCC_PER_FACE 4
struct DOccluder { double n[3], d, en[3][3], eo[3]; };
struct DShadowProof {
  DOccluder tri[6][RRT_OCC_PER_FACE];
  double in_lo[3], in_hi[3];
  double w[6];            // host: the kept triangles' largest vertex distance from their face
  uint32_t n[6];
  uint32_t on, pad;
};

// Kerr shadow-ray occlusion proof (rrt_device.h kerr_occluded_proof): a coarse march
// (steps stretch x delta_theta x r) whose chords the exact march's stay within delta of
// A wall piece of the Kerr proof: an occluder triangle, or two coplanar ones of the same face that
// share an edge and form a convex quad (a Cornell-box wall), as one convex polygon: plane (normal
// toward the box's inside) and four inward in-plane edge normals (a triangle repeats one edge).
struct DOccQuad { double n[3], d, en[4][3], eo[4]; };
struct DKerrProof {
  DOccQuad quad[6][RRT_OCC_PER_FACE];  // per root-box face (rrt_host.cpp build_occluders)
  uint32_t nq[6];
  double stretch;     // coarse step length over the exact march's
  double r_near2;     // no proof once the coarse march comes within sqrt(r_near2) of the hole
  double delta;       // crossing margin (tools/kerr_proof_sweep.py: >= 3x the largest deviation seen)
  double swept_max;   // the coarse march's swept polar angle stays below it (the exact budget: 2 pi)
  int32_t max_steps;  // coarse steps (so the exact march's step budget reaches the crossing)
  uint32_t on;
};

// Claim order within a tile (every kernel that turns a claim index ix into a pixel: tile
// tile_order[ix / ts^2], then claim_r(ix % ts^2) = the pixel's row-major index in the tile): 8x8
// blocks in row-major order, row-major inside each (ts is a multiple of 8), so 64 consecutive
// claims -- a wave of the pixel pass, a strip of its first level -- are a square of pixels.
// (Row-major claims measured slower: profiles/r04_ab_claim_block8.txt.)
__host__ __device__ __forceinline__ uint32_t claim_r(uint32_t c, uint32_t ts) {
  const uint32_t b = c >> 6, w = c & 63u, nb = ts >> 3;
  return ((b / nb) * 8u + (w >> 3)) * ts + (b % nb) * 8u + (w & 7u);
}

#define RRT_MAX_QUEUES 8
#define RRT_QUEUE_STRIDE 16  // counters 64 B apart

// A pixel handed from rrt_batch_kernel to rrt_heavy_kernel between two adaptive steps (a
// continuation): its position, the samples folded so far and their sums in the
// reference's accumulation types (raytrace_pixel, part1_code.cpp:136-158), and the next sample's
// draw offset.  seq = the launch's KParams::cont_seq once the record is written.
struct ContRec {
  double s1, s2;
  float r, g, b;
  uint32_t x, y, slot, i, O;
  uint32_t seq, pad[3];
};
// KParams::cont_ctl words (RRT_QUEUE_STRIDE apart): records reserved, records taken, blocks waiting
// for one, batch waves past their last pixel (no record can come once all are)
enum { RRT_CONT_TAIL = 0, RRT_CONT_HEAD = 1, RRT_CONT_IDLE = 2, RRT_CONT_DONE = 3, RRT_CONT_WORDS = 4 };
// rrt_heavy_kernel launches: the heavy list then continuations (side stream), untaken records
// behind the batch and heavy kernels (main stream)
enum { RRT_HEAVY_LIST = 0, RRT_HEAVY_DRAIN = 1 };

struct KParams {
  // scene
  const DNode* nodes;
  const DPrimGeo* geo;
  const DPrimNrm* nrm;
  const DPrimMeta* meta;
  const DBsdf* bsdfs;
  const DLight* lights;
  uint32_t n_lights;
  uint32_t fast_div;  // scene bounds allow the Markstein-corrected slab quotients
  DGrid grid;
  const DNode* clean_nodes;   // clean tree (pad = first leaf ordinal); null: reference walk only
  const DPlane* planes;       // per leaf slot; null: no plane cull
  double root_lo[3], root_hi[3];  // root box widened by plane_eps (segment_outside_root)
  double plane_eps;           // plane-cull margin (scene-scaled, ~1e6 x rounding error)
  const DBig* big;            // oversized leaves by left-first ordinal
  const uint32_t* big_mask;   // per grid cell: oversized leaves with a primitive in reach, or null
  double big_reach;           // segments shorter than this may use big_mask ((RRT_BIG_REACH - 1) h_free)
  int32_t clean_root;         // 0, or -1 if every leaf is oversized
  uint32_t n_big;
  const DNode* free_nodes;    // search tree over the clean tree's leaves (traverse_free), or null
  const DNode4* free4;        // the same tree 4 wide (traverse_free4), or null (binary walk)
  double free4_omax;          // segments starting farther out (max |coordinate|) take the binary walk
  DCamera cam;
  DHole hole;
  DMissProof miss;
  DEnv env;
  // render
  uint32_t ns_aa, max_ray_depth, ns_area_light, samples_per_batch;
  float max_tolerance;
  uint32_t direct_hemisphere;
  uint32_t diag;  // RRT_RENDER_DIAG_* bits >> 30 (bit 0: no traversal, bit 1: clear-segment stats)
  uint32_t count_exec;  // with counters: count the executed work (RRT_RENDER_COUNT_EXECUTED)
  uint64_t seed;
  double frame_w, frame_h;
  uint32_t frame_wi, frame_hi;
  // work: list of tiles (x, y), each split into 8x8 pixel blocks pulled by waves
  const uint32_t* tiles;
  uint32_t n_tiles, tile_size;
  uint32_t blocks_per_tile_side, n_blocks;
  uint32_t* block_counter;
  // sample-parallel kernel (rrt_sample.hip rrt_batch_kernel)
  uint32_t n_pixels;     // n_tiles * tile_size^2 (pixel work items)
  const uint32_t* tile_order;  // claim order over the caller's tile list
  // claim queues (one per XCD): queue q holds claim indices [q_end[q-1], q_end[q]) of tile_order,
  // its counter is block_counter[RRT_QUEUE_STRIDE * q]; a block starts on queue blockIdx % n_queues
  uint32_t n_queues;
  uint32_t q_end[RRT_MAX_QUEUES];
  uint32_t q_stripe;     // 1: queue q holds claims q, q + n_queues, ... of the whole order (q_end unused)
  // pixel miss proof (rrt_pixel_proof_kernel): the claim indices whose pixels were not proven
  // all-miss, in claim order per wave, and their count; null: every pixel is claimed
  uint32_t* claim_list;
  uint32_t* claim_count;
  struct FirstSample { float r, g, b; uint32_t hit; };
  FirstSample* first;          // sample 0 of every pixel slot (rrt_first_kernel), or null
  uint32_t group;        // lanes per pixel (power of two, 2..32)
  uint32_t draws_miss;   // RNG draws of a camera sample whose query misses (jitter: 2)
  uint32_t draws_hit;    // ... and of one that hits (jitter + the direct-lighting sampler draws)
  uint32_t clip_x0, clip_y0, clip_x1, clip_y1;  // region actually requested (exclusive end)
  // outputs, packed per tile: pixel (i, j) of tile t at t*tile_size^2 + j*tile_size + i
  float* rgb;
  int32_t* count;
  uint32_t* draws;      // optional
  uint32_t* counters;   // optional [4] per pixel
  DShadowProof occ;     // the hot fields above keep their offsets
  // heavy pixels (rrt_pixel_proof_kernel pixel_heavy -> rrt_heavy_kernel): listed pixels rendered
  // slot-parallel, one wave per pixel and a step's 64 draw-offset slots per round
  uint32_t* heavy_list;   // claim indices (null: no heavy path)
  uint32_t* heavy_count;  // [0]: entries appended by the pass (capped at heavy_cap); [1]: entries taken
  uint32_t heavy_cap;     // list capacity
  uint32_t claim_back;    // batch kernel: hinted list entries at the front (claim_count[0] of them),
                          // the others from the list's end backwards (claim_count[1])
  double heavy_r2;        // (RRT_HEAVY_NEAR x r_s)^2: rays passing this close make a pixel heavy
  uint64_t free_big_mask; // oversized leaves traverse_free tests from its list (the others are in
                          // the search tree); ~0 for the clean-tree and reference-tree walks
  // the reference's compile-time switches as run-time flags (include/rrt.h RRT_RENDER_THIN_LENS ..
  // RRT_RENDER_ILLUM_MASK; kernel variant V_SW only): flag bits 22..27 >> 22, the camera's lens
  double lens_r, focal;   // Camera::lensRadius / focalDistance (camera.cpp:176-184)
  uint32_t sw;            // bit 0 thin lens, 1 no adaptive, 2 env hemi, 3 microfacet hemi, 4..5 ILLUM ^ 2
  // the heavy pixels' kernel beside the batch kernel: its grid (blocks of heavy_nw waves); the
  // batch kernel's top blocks make room for as many of them as there are heavy pixels (0: none)
  uint32_t heavy_grid, heavy_nw;
  uint32_t sw_pad;
  // the path pool kernel (rrt_path.hip, depth >= 2): each path's per-level terms of
  // at_least_one_bounce_radiance, [level][field][path] (RRT_PATH_FIELDS floats a level)
  float* path_stack;
  // batch kernel: a wave whose oldest pixel has run this long (wall-clock ticks, 100 MHz) takes
  // issue priority 2, four times as long priority 3 (rrt_sample.hip tail_prio)
  uint32_t prio_ticks;
  uint32_t prio_pad;
  DKerrProof kproof;      // Kerr builds: the shadow rays' occlusion proof (kp.occ's face triangles)
  // the pixel pass's first level (rrt_strip_proof_kernel): strips of 64 consecutive claim indices
  // proven as wholes -- flag 1 per strip -- before the per-pixel level (null: per-pixel pass only)
  uint32_t* strip_list;
  // run-time proof audit (rrt_device.h audit_pick): counting launches re-check every
  // 2^audit_shift-th proven ray (and pixel) against the exact march; tallies [2 k] checked,
  // [2 k + 1] violations per proof k (RRT_AUDIT_*); null: no audit
  unsigned long long* audit;  // 64-bit: a 1080p frame audited at every_log2 = 0 exceeds 2^32 checks
  uint32_t audit_shift, audit_pad;
  // continuations: a batch-kernel group whose pixel still has >= cont_min_left
  // samples to go after an adaptive check hands it to a heavy block that is waiting for work
  // (cont_ctl[RRT_CONT_IDLE] > 0), which renders the remaining steps' draw-offset slots in parallel.
  // cont null: off.  Waiting blocks stop once all batch_waves batch waves are past their last pixel.
  ContRec* cont;
  uint32_t* cont_ctl;
  uint32_t cont_cap, cont_min_left;
  uint32_t cont_seq, batch_waves;
  uint32_t cont_room;     // batch blocks that leave at once, room for the waiting heavy blocks
  uint32_t cont_ticks;    // a heavy block stops waiting after this long without work (wall clock)
  uint32_t cont_waiters;  // heavy blocks blockIdx < cont_waiters wait for continuations; the others
                          // leave once the heavy list is done (their slots go back to the batch kernel)
#if RRT_PROFILE
  // diagnostic build: per-wave progress records in host-coherent memory (RRT_WATCHDOG_MS), read by
  // the host while the kernels run: [wave][4] = {iteration, state, pixel, marker}; batch waves
  // first, the heavy kernel's blocks from RRT_WD_HEAVY on
  uint32_t* wd;
#endif
};
#define RRT_WD_WORDS (1u << 18)
#define RRT_WD_HEAVY (1u << 17)
