/* rrt.h -- C ABI of the MI355X-native relativistic path-tracer hot path (librrt.so).
 *
 * Drop-in boundary for the reference's per-pixel radiance loop.  The reference has no
 * plugin/FFI API for this path; the seam it replaces is the private C++ call chain
 *   PathTracer::raytrace_tile  (pathtracer.cpp:549-581, pathtracer.h:212)
 *     -> PathTracer::raytrace_pixel (part1_code.cpp:125-163)
 *        -> BVHAccel::intersect (bvh.cpp:103-138) -> BlackHole::next_micro_ray (blackhole.cpp:17-40)
 *        -> BSDF::sample_f / SceneLight::sample_L (bsdf.cpp, light.cpp)
 * plus the state its callers install: PathTracer::set_scene (pathtracer.cpp:95-117, which also
 * builds the BVH, :304-328), set_camera (:119-134), set_frame_size (:136-149) and the `-B`
 * black-hole override of main.cpp:139-145.  Each entry point below names the reference
 * interface it replaces.  Plain C types only; no exceptions cross the ABI; every function
 * returns RRT_OK (0) or a negative RRT_E* code, with a message in rrt_last_error().
 *
 * RNG: the reference draws from one shared glibc rand() stream; this library uses the keyed
 * per-pixel stream of csrc/rrt_rng.h (seed, x, y), which the oracle harness also links into
 * the reference, so outputs are comparable pixel by pixel.
 */
#ifndef RRT_H
#define RRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RRT_ABI_VERSION 5  /* 2: rrt_spacetime_desc gained spin + axis (Kerr)
                              3: rrt_stats gained last_main_kernel_ms / last_heavy_pixels (callers
                                 built against 2 pass a smaller struct: rebuild), the
                                 RRT_RENDER_WAVEFRONT selects the path pool kernel (depth >= 2;
                                 RRT_E_INVALID elsewhere),
                                 rrt_libm_eval added
                              4: rrt_set_proof_audit / rrt_get_proof_audit added
                              5: rrt_stats gained last_cont_pixels (continuations); the proof-audit
                                 tallies are 64-bit on the device too */

enum {
  RRT_OK = 0,
  RRT_E_INVALID = -1,     /* bad argument / unsupported scene feature */
  RRT_E_HIP = -2,         /* HIP runtime error (message has the HIP error string) */
  RRT_E_CANCELLED = -3,   /* render stopped through the cancel flag (PathTracer::stop) */
  RRT_E_NO_DEVICE = -4,   /* context created host-only (device < 0) or no GPU */
  RRT_E_IO = -5           /* file helpers */
};

typedef struct rrt_ctx rrt_ctx;

/* ---------------------------------------------------------------- context */
typedef struct {
  int device;              /* HIP device ordinal; -1 = host-only context (BVH build, tests) */
  uint32_t free_grid_res;  /* empty-space grid: cells along the root box's longest axis
                              (0 = default 128, 1 = no grid).  Result-neutral. */
  uint32_t reserved[6];
} rrt_device_cfg;

/* Replaces: PathTracer::PathTracer (pathtracer.cpp:32-85) device-side state. */
int rrt_create(rrt_ctx** out, const rrt_device_cfg* cfg);
void rrt_destroy(rrt_ctx* ctx);
const char* rrt_last_error(const rrt_ctx* ctx);
int rrt_abi_version(void);

/* ---------------------------------------------------------------- scene */
enum { RRT_OBJ_MESH = 0, RRT_OBJ_SPHERE = 1 };
/* BSDF kinds and parameter slots: include/rrt_scene_format.h (bsdf.h:74-199) */
enum { RRT_BSDF_DIFFUSE = 0, RRT_BSDF_EMISSION = 1, RRT_BSDF_MIRROR = 2, RRT_BSDF_GLASS = 3,
       RRT_BSDF_MICROFACET = 4, RRT_BSDF_REFRACTION = 5 };
/* Light kinds (light.h): area, point, directional, infinite hemisphere */
enum { RRT_LIGHT_AREA = 0, RRT_LIGHT_POINT = 1, RRT_LIGHT_DIRECTIONAL = 2, RRT_LIGHT_HEMISPHERE = 3 };

typedef struct {
  uint32_t kind;              /* RRT_OBJ_* */
  uint32_t bsdf;              /* index into rrt_scene_desc.bsdfs */
  uint32_t n_vertices, n_triangles;
  const double* positions;    /* mesh: [n_vertices][3]   (StaticScene::Mesh::positions) */
  const double* normals;      /* mesh: [n_vertices][3]   (StaticScene::Mesh::normals) */
  const uint32_t* indices;    /* mesh: [n_triangles][3], mesh-local (object.cpp:28-33) */
  double center[3];           /* sphere (SphereObject::o) */
  double radius;              /* sphere (SphereObject::r) */
} rrt_object_desc;

typedef struct { uint32_t type; float params[14]; } rrt_bsdf_desc;

typedef struct {
  uint32_t type, is_delta;
  float radiance[3];
  float area;                 /* area light: (float)(|dim_x| * |dim_y|), light.cpp:78 */
  double v[4][3];             /* area: position, direction, dim_x, dim_y; point: position;
                                 directional: dirToLight; hemisphere: sampleToWorld columns */
} rrt_light_desc;

typedef struct {
  uint32_t n_objects, n_bsdfs, n_lights, reserved;
  const rrt_object_desc* objects;   /* StaticScene::Scene::objects order = BVH build order */
  const rrt_bsdf_desc* bsdfs;
  const rrt_light_desc* lights;     /* StaticScene::Scene::lights order */
} rrt_scene_desc;

/* Replaces: PathTracer::set_scene + build_accel (pathtracer.cpp:95-117, 304-328;
 * BVHAccel::construct_bvh bvh.cpp:49-96).  The library copies everything (the caller keeps
 * ownership), builds the reference BVH on the host and uploads a flattened copy to HBM. */
int rrt_set_scene(rrt_ctx* ctx, const rrt_scene_desc* scene);

/* ---------------------------------------------------------------- camera / spacetime */
typedef struct {
  double hFov, vFov;          /* degrees (Camera::hFov / vFov after configure/set_screen_size) */
  double nClip, fClip;
  double pos[3];
  double c2w[9];              /* row-major c2w(i, j), as Camera::dump_settings writes it */
  double lensRadius, focalDistance;
} rrt_camera_desc;
/* Replaces: PathTracer::set_camera (pathtracer.cpp:119-134). */
int rrt_set_camera(rrt_ctx* ctx, const rrt_camera_desc* cam);

enum { RRT_METRIC_SCHWARZSCHILD = 0, RRT_METRIC_KERR = 1 };
typedef struct {
  uint32_t kind;              /* RRT_METRIC_SCHWARZSCHILD (r_s = 0: the reference's flat limit)
                                 or RRT_METRIC_KERR (build-defined, no reference) */
  uint32_t reserved;
  double center[3];           /* global_black_hole.o   (blackhole.cpp:5 default (0,1,0)) */
  double r_s;                 /* global_black_hole.r   (default 0.1); Kerr: 2M */
  double delta_theta;         /* global_black_hole.delta_theta (default 0.1); Kerr: the step's
                                 angular size seen from the hole (h = delta_theta * r / |dx/dl|) */
  /* Kerr only (ignored for Schwarzschild): */
  double spin;                /* dimensionless a/M in [0, 1) */
  double axis[3];             /* spin axis (world; normalised by the library; 0 = scene up (0,1,0)) */
} rrt_spacetime_desc;
/* Replaces: the `-B x y z r dtheta` override of the global black hole (main.cpp:139-145).
 * RRT_METRIC_KERR swaps BlackHole::next_micro_ray for an RK4 null-geodesic step in Kerr-Schild
 * coordinates; the rest of BVHAccel::intersect (segment tests, capture = no hit) is unchanged. */
int rrt_set_spacetime(rrt_ctx* ctx, const rrt_spacetime_desc* st);
/* The validated envelope of the camera / pixel / shadow proofs (profiles/
 * r03_proof_sweep.json): delta_theta in [RRT_PROOF_DT_MIN, RRT_PROOF_DT_MAX] and r_s <=
 * RRT_PROOF_RS_OVER_EXTENT x the scene's largest root-box extent.  Outside it the kernels march
 * every ray exactly.  Returns 1 if the context's scene and Schwarzschild hole are inside it. */
#define RRT_PROOF_DT_MIN 0.04
#define RRT_PROOF_DT_MAX 0.6
#define RRT_PROOF_RS_OVER_EXTENT 0.5
int rrt_proof_envelope(const rrt_ctx* ctx);
/* The Kerr local frame for a spin axis (ez = unit(axis), ex, ey completing a right-handed
 * basis), so a checker can restate the integrator in the same coordinates. */
void rrt_kerr_frame(const double* axis3, double* ex3, double* ey3, double* ez3);

/* ---------------------------------------------------------------- environment map */
typedef struct {
  uint32_t width, height;     /* equirectangular map, HDRImageBuffer layout: row y covers
                                 theta = (y + 0.5) / height * pi from +y (environment_light.cpp) */
  const float* texels;        /* [height][width][3] linear RGB (Spectrum), main.cpp:64-75 order */
} rrt_envmap_desc;
/* Replaces: the envmap argument of PathTracer::PathTracer -> EnvironmentLight
 * (pathtracer.cpp:61-63, environment_light.cpp:21-148): importance-sampled light and the miss
 * radiance.  The library copies the texels and builds the sampling CDFs.  NULL removes it. */
int rrt_set_envmap(rrt_ctx* ctx, const rrt_envmap_desc* envmap);

/* ---------------------------------------------------------------- render */
typedef struct {
  uint32_t ns_aa;             /* -s   (AppConfig default 1) */
  uint32_t max_ray_depth;     /* -m   (default 1) */
  uint32_t ns_area_light;     /* -l   (default 1) */
  uint32_t samples_per_batch; /* -a n (default 32) */
  float max_tolerance;        /* -a t (default 0.05f) */
  uint32_t direct_hemisphere; /* -H */
  uint64_t seed;              /* keyed RNG seed */
  uint32_t frame_w, frame_h;  /* sampleBuffer.w / h (set_frame_size) */
  uint32_t flags;             /* RRT_RENDER_* */
  uint32_t variant;           /* A/B measurements, 0 = defaults.  Bits 0..7: waves/SIMD the
                                 depth<=1 kernel is built for (1..6, register budget); bits
                                 8..11: the sample-0 pre-pass's waves/SIMD; bits 16..19: the heavy-pixel
                                 threshold (1: capture boundary only; 2 / 3 / 4: rays within
                                 1.1 / 1.5 / 2.0 r_s; 0: 1.2); bits 12..15: blocks per CU the
                                 batch grid leaves free besides the heavy kernel's; bits 20..21:
                                 waves per heavy pixel (0: 2, 1: 1, 2: 4); bit 23: no room left
                                 for the heavy kernel; bits 24..27: the heavy-pixel kernel's
                                 waves/SIMD (4 or 5; 0: 4); bits 28..31: its waves in multiples
                                 of the CU count (0: 2) */
} rrt_render_params;
enum {
  RRT_RENDER_COUNTERS = 1u << 0, /* also produce per-pixel work counters (slower variant) */
  RRT_RENDER_DRAWS = 1u << 1,    /* also produce per-pixel RNG draw counts */
  RRT_RENDER_WAVEFRONT = 1u << 2, /* depth >= 2 (Schwarzschild): the path pool kernel -- one ray per
                                     lane per round, the paths' state between rays in LDS -- instead
                                     of the per-pixel loop (A/B, slower on m3); RRT_E_INVALID with
                                     Kerr, counters, switches or depth <= 1 */
  RRT_RENDER_EXACT_DIV = 1u << 3, /* slab tests by true division instead of the
                                     Markstein-corrected reciprocal (A/B testing) */
  RRT_RENDER_PIXEL_LOOP = 1u << 4, /* depth <= 1: per-pixel-loop kernel instead of the default
                                     per-sample kernel (A/B testing) */
  RRT_RENDER_NO_SKIP = 1u << 5,   /* traverse every micro segment, ignoring the empty-space
                                     grid (A/B testing; results are identical) */
  RRT_RENDER_NO_CLEAN = 1u << 6,  /* walk the reference tree as is, not the clean tree with
                                     its oversized leaves listed apart (A/B testing; results
                                     are identical) */
  RRT_RENDER_PER_PIXEL = 1u << 7, /* depth <= 1: one lane per pixel (per-sample kernel) instead
                                     of the sample-parallel kernel (A/B testing) */
  RRT_RENDER_ORDERED = 1u << 9,   /* sample-parallel kernel: claim tiles in list order instead
                                     of centre-first (A/B testing) */
  RRT_RENDER_NO_FIRST = 1u << 10, /* sample-parallel kernel: no sample-0 pre-pass (the
                                     default; overrides RRT_RENDER_PREPASS) */
  RRT_RENDER_ONE_QUEUE = 1u << 11, /* sample-parallel kernel: one chip-wide claim queue (A/B
                                     testing; results are identical) */
  RRT_RENDER_XCD_QUEUES = 1u << 12, /* sample-parallel kernel: one claim queue per XCD (A/B
                                     testing; results are identical).  Default: per-XCD queues
                                     for the general and Kerr builds, one queue for LEAN builds */
  RRT_RENDER_STRIPED_QUEUES = 1u << 15, /* sample-parallel kernel: the centre-first claim order
                                     dealt round-robin over one claim counter per XCD (A/B;
                                     the default of the area/point-light builds) */
  RRT_RENDER_PREPASS = 1u << 14, /* sample-parallel kernel: render sample 0 of every pixel in a
                                     pre-pass whose hit status seeds the pixel's first hypothesis
                                     (A/B testing; results are identical) */
  RRT_RENDER_NO_MISS_PROOF = 1u << 13, /* march every camera ray exactly instead of first trying
                                     the planar-recurrence miss proof (A/B testing; results
                                     are identical) */
  RRT_RENDER_NO_PIXEL_PROOF = 1u << 17, /* sample-parallel kernel: no pixel miss proof pass (every
                                     pixel's camera rays are marched or proven one by one) */
  RRT_RENDER_NO_SHADOW_PROOF = 1u << 16, /* march every shadow ray exactly instead of first trying
                                     the occlusion proof (a certain crossing of a root-box face
                                     triangle before any possible capture; A/B and parity) */
  RRT_RENDER_NO_SEARCH_TREE = 1u << 18, /* walk the clean tree (left-first, the reference's order)
                                     instead of the SAH search tree over the same leaves with the
                                     ordered replay of accepted primitives (A/B; results are
                                     identical) */
  RRT_RENDER_NO_HEAVY = 1u << 20, /* sample-parallel kernel: no slot-parallel path for heavy
                                     pixels (those whose rays straddle the hole's capture boundary
                                     or pass close to it; A/B and parity, results are identical) */
  RRT_RENDER_HEAVY = 1u << 21,    /* sample-parallel kernel: the heavy pixels' path for every
                                     launch (by default it runs for launches of at most 60% of the
                                     frame's pixels, e.g. one rank's tiles of a multi-GPU frame,
                                     and when ns_aa >= 4 samples_per_batch; results are identical) */
  RRT_RENDER_DEEP_SAMPLE = 1u << 19, /* depth >= 2 (Schwarzschild): the per-sample refill kernel
                                     instead of the per-pixel loop (A/B; results are identical) */
  /* The reference's compile-time switches (pathtracer.h:4-6, environment_light.h:4, bsdf.h:4) as
   * run-time flags; 0 is the reference build's setting.  Any of them selects the general
   * per-pixel-loop kernel build that carries them (every ray marched exactly; Schwarzschild only;
   * parity against the restatement: the reference's switches are #defines this harness cannot flip): */
  RRT_RENDER_THIN_LENS = 1u << 22, /* THIN_LENS 1: Camera::generate_ray_for_thin_lens (camera.cpp:176-184)
                                     with the camera's lensRadius / focalDistance; its lens sample comes
                                     from the grid sampler after the pixel jitter (part1_code.cpp:137-139) */
  RRT_RENDER_NO_ADAPTIVE = 1u << 23, /* ADAPTIVE 0: every pixel takes ns_aa samples (part1_code.cpp:147-159) */
  RRT_RENDER_ENV_HEMI = 1u << 24, /* ENV_HEMI 1: EnvironmentLight::sample_L samples the uniform sphere
                                     (environment_light.cpp:139-142, sampler.cpp:33-40) */
  RRT_RENDER_MICROFACET_HEMI = 1u << 25, /* MICROFACET_HEMI 1: MicrofacetBSDF::sample_f takes the
                                     cosine hemisphere sampler (bsdf.cpp:93-94) */
  /* bits 26..27: ILLUM (pathtracer.h:4) xor 2, see RRT_RENDER_ILLUM: 0 normal shading,
     1 direct lighting only, 2 the default, 3 at_least_one_bounce_radiance alone (part1_code.cpp:78-122) */
  RRT_RENDER_ILLUM_MASK = 3u << 26,
  RRT_RENDER_COUNT_EXECUTED = 1u << 8, /* with COUNTERS: count the work the renderer executes
                                     (AABB tests incl. oversized leaves, primitive tests after
                                     the plane cull, micro steps, and plane tests in place of
                                     queries) instead of the reference's */
  /* diagnostics only -- results are NOT the reference's: */
  RRT_RENDER_DIAG_NO_INTERIOR = 1u << 28, /* skip walks of segments starting in the root box */
  RRT_RENDER_DIAG_NO_EXTERIOR = 1u << 29, /* skip walks of segments starting outside it */
  RRT_RENDER_DIAG_NO_TRAVERSE = 1u << 30, /* skip every BVH traversal (cost of the rest) */
  RRT_RENDER_DIAG_CLEAR_STATS = 1u << 31  /* with COUNTERS: counter 3 = grid-clear segments,
                                             counter 2 = AABB tests outside them */
};
#define RRT_RENDER_ILLUM(n) ((((uint32_t)(n)) ^ 2u) << 26)  /* ILLUM n as flag bits (ILLUM 2: 0) */
void rrt_render_params_default(rrt_render_params* p);

/* Replaces: PathTracer::raytrace_tile / raytrace_cell over the region [x0,x0+w) x [y0,y0+h)
 * of the frame (y = 0 at the bottom, sampleBuffer rows).  Host buffers, row-major over the
 * region: rgb_out [h][w][3] (sampleBuffer Spectrum), count_out [h][w]
 * (sampleCountBuffer, part1_code.cpp:161).  draws_out [h][w] and counters_out [h][w][4]
 * (AABB tests, micro steps, primitive tests, BVH queries) are optional (NULL).
 * cancel: polled between launches (continueRaytracing, pathtracer.cpp:566); may be NULL. */
int rrt_render(rrt_ctx* ctx, const rrt_render_params* p, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
               float* rgb_out, int32_t* count_out, uint32_t* draws_out, uint32_t* counters_out,
               const volatile int* cancel);

/* Device-resident variant for multi-GPU / benchmarking.  Renders the listed square tiles
 * (tile t covers x in [tiles[2t], +tile_size), y in [tiles[2t+1], +tile_size), clipped to
 * the frame) into PACKED device buffers: pixel (i, j) of list entry t goes to
 * rgb[(t * tile_size * tile_size + j * tile_size + i) * 3], count[...] likewise.  Asynchronous
 * on `stream` (a hipStream_t, NULL = default stream); no host synchronisation.
 * tiles is a host array of 2*n_tiles uint32.  A context owns one launch workspace (parameters,
 * claim counters, tile list): a launch or unpack on a different stream than the context's
 * previous one makes its stream wait for that previous use first (hipStreamWaitEvent), so
 * launches of one context never overlap; use one context per stream to overlap renders.
 * The heavy pixels' kernel (RRT_RENDER_HEAVY) runs on the context's own high-priority side
 * stream, forked from `stream` after the pixel proof pass and joined back into it (events)
 * before the launch ends: work the caller enqueues on `stream` afterwards sees the whole frame. */
int rrt_render_tiles_device(rrt_ctx* ctx, const rrt_render_params* p, const uint32_t* tiles, uint32_t n_tiles,
                            uint32_t tile_size, float* d_rgb, int32_t* d_count, uint32_t* d_counters,
                            void* stream);
/* Unpack packed tiles (as written above) into frame-layout device buffers [frame_h][frame_w]. */
int rrt_unpack_tiles_device(rrt_ctx* ctx, const uint32_t* tiles, uint32_t n_tiles, uint32_t tile_size,
                            uint32_t frame_w, uint32_t frame_h, const float* d_rgb_packed,
                            const int32_t* d_count_packed, float* d_rgb, int32_t* d_count, void* stream);
/* Gamma tonemap to RGBA8, HDRImageBuffer::toColor + ImageBuffer::update_pixel
 * (image.h:53-62, 183-198), frame layout on the device. */
int rrt_tonemap_device(rrt_ctx* ctx, uint32_t n_pixels, const float* d_rgb, uint32_t* d_rgba, void* stream);

/* Multi-GPU group: one frame region over several contexts, one per GPU (the
 * reference's tile worker pool, pathtracer.cpp:251-255, 279-281, 611-644, as one launch per GPU).
 * The region's 32x32 tiles are dealt over the members as a lattice (rrt_region_tiles), every member renders its
 * tiles into a packed buffer on its own stream, member 0 gathers them -- RCCL grouped
 * send / recv over xGMI when the members are on distinct devices, device copies when several
 * share one -- and unpacks them.  Output as rrt_render (host buffers [h][w]).  The contexts must
 * hold the same scene, camera and spacetime; the group does not own them. */
typedef struct rrt_group rrt_group;
int rrt_group_create(rrt_ctx* const* ctxs, uint32_t n, rrt_group** out);
int rrt_group_render(rrt_group* g, const rrt_render_params* p, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                     float* rgb_out, int32_t* count_out, const volatile int* cancel);
void rrt_group_destroy(rrt_group* g);

/* Tile partition of a frame over `world` ranks (the multi-GPU split of SURVEY 8(e)): tile (tx, ty)
 * goes to rank (tx + S ty) % world, S the integer nearest 0.382 world that is prime to it (1 for
 * world <= 4, 2 for 5, 3 for 7 and 8), tiles listed row by row.  Writes up to max_tiles (x, y)
 * pairs for `rank` into tiles_out and returns the number of tiles (or a negative error). */
int rrt_partition_tiles(uint32_t frame_w, uint32_t frame_h, uint32_t tile_size, uint32_t rank, uint32_t world,
                        uint32_t* tiles_out, uint32_t max_tiles);
/* The same deal over the tiles of a region (x0, y0, w x h pixels; tiles from its origin): the split
 * rrt_group_render uses for its members.  rrt_partition_tiles is the region (0, 0, frame). */
int rrt_region_tiles(uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t tile_size, uint32_t rank,
                     uint32_t world, uint32_t* tiles_out, uint32_t max_tiles);

/* ---------------------------------------------------------------- introspection */
typedef struct {
  uint32_t n_prims, n_nodes, n_leaf_refs, max_depth;
  uint64_t device_bytes;      /* HBM held by the scene */
  uint32_t grid_n[3];         /* empty-space grid cells per axis (0 = none) */
  uint32_t n_clean, n_big;    /* clean-tree nodes and oversized leaves (0 = reference walk) */
  float grid_free_frac;       /* fraction of grid cells with free radius > 0 */
  float last_kernel_ms;       /* HIP-event time of the last render launch */
  uint32_t grid_blocks, block_threads;
  char kernel[64];            /* name of the last render kernel(s) launched */
  float last_main_kernel_ms;  /* HIP-event time of the last launch's main kernel alone (after
                                 any pre-pass such as rrt_pixel_proof_kernel) */
  uint32_t last_heavy_pixels;  /* pixels the last launch rendered slot-parallel (heavy pixels) */
  uint32_t last_cont_pixels;   /* pixels the last launch's batch kernel handed to the heavy kernel
                                  between adaptive steps (continuations) */
} rrt_stats;
int rrt_get_stats(const rrt_ctx* ctx, rrt_stats* out);
/* Diagnostics: evaluate the device's restatement of the host C library's transcendentals
 * (csrc/rrt_glibm.h -- the reference's sin/cos (sampler.cpp:53-55, environment_light.cpp:97-137),
 * acos (sampler.cpp:20, bsdf.h:166, environment_light.cpp:88), atan2 (environment_light.cpp:89),
 * sinf/cosf (sampler.cpp:23-25), and the microfacet BSDF's exp, log, erf, atan and tan
 * (bsdf.cpp:45-96, bsdf.h:159-191)) on n host arguments: fn 0 sin(a), 1 cos(a), 2 acos(a),
 * 3 atan2(a, b), 4 sinf((float)a), 5 cosf((float)a) (float results widened to double), 6 exp(a),
 * 7 log(a), 8 erf(a), 9 atan(a), 10 tan(a). */
int rrt_libm_eval(rrt_ctx* ctx, int fn, const double* a, const double* b, double* out, uint64_t n);
/* Run-time proof audit.  The renderer skips marches whose results its proofs
 * determine (camera-ray miss, shadow-ray occlusion, pixel and strip miss, Kerr occlusion); their
 * margins are validated by sweeps.  With the audit set, every counting launch that runs the proofs
 * (RRT_RENDER_COUNTERS | RRT_RENDER_COUNT_EXECUTED) also marches every 2^every_log2-th proven ray
 * (every 2^every_log2-th pixel for the pixel pass) exactly and tallies disagreements.  Render
 * outputs are unchanged.  rrt_get_proof_audit (synchronises the device) returns and resets the
 * tallies: out[2 k] rays checked, out[2 k + 1] violations, k = RRT_AUDIT_CAMERA .. RRT_AUDIT_ZERO. */
enum { RRT_AUDIT_CAMERA = 0, RRT_AUDIT_SHADOW = 1, RRT_AUDIT_PIXEL = 2, RRT_AUDIT_STRIP = 3, RRT_AUDIT_KERR = 4,
       RRT_AUDIT_ZERO = 5 /* reserved: the zero-sample variant (round 5) was removed; always 0 */,
       RRT_AUDIT_KINDS = 6 };
int rrt_set_proof_audit(rrt_ctx* ctx, int every_log2 /* < 0: off (the default) */);
int rrt_get_proof_audit(rrt_ctx* ctx, uint64_t* out /* [2 * RRT_AUDIT_KINDS] */);
/* HIP-event times of the last n (<= 32) render launches, oldest first: the whole launch and its
 * main kernel alone (bench.py's roofline divides by the latter).  Returns the count filled. */
int rrt_get_launch_times(const rrt_ctx* ctx, uint32_t n, float* total_ms, float* main_ms);
/* Host copy of the flattened BVH: boxes [n][6] (min, max), nodes [n][4] (first, count, left,
 * right; count 0 = inner node), prims [n_leaf_refs] (build-order primitive ids) -- the layout
 * of the oracle's reference-BVH dump.  Any pointer may be NULL to query sizes via stats. */
int rrt_get_bvh(const rrt_ctx* ctx, double* boxes, int32_t* nodes, uint32_t* prims);

/* The clean tree the renderer walks: boxes [n][6], nodes [n][4] = (skip, first
 * slot, slot count (0 = inner), left-first ordinal of the first leaf); oversized leaves:
 * big_boxes [nb][6], big [nb][3] = (first slot, slot count, ordinal).  Returns n (0 = none);
 * query nb through rrt_get_stats.  Any pointer may be NULL. */
int rrt_get_clean_tree(const rrt_ctx* ctx, double* boxes, int32_t* nodes, double* big_boxes, int32_t* big);
/* The search tree: an SAH hierarchy over the clean tree's leaves in pre-order,
 * boxes [n][6], nodes [n][4] = (skip, first slot, slot count (0 = inner), the leaf's left-first
 * ordinal).  Returns n (0 = none); call with NULL pointers to get n. */
int rrt_get_search_tree(const rrt_ctx* ctx, double* boxes, int32_t* nodes);

/* The search tree 4 wide (the walk's 4-wide nodes): boxes [n][4][6] f32 (min, max;
 * rounded outward and widened: a conservative pre-test), kids [n][4][3] = (child, first slot, count):
 * count 0 an inner node (child = its 4-wide index), > 0 a search-tree leaf (child = its search-tree
 * node index), < 0 empty.  Returns n (0 = none: the binary walk); any pointer may be NULL. */
int rrt_get_search_tree4(const rrt_ctx* ctx, float* boxes, int32_t* kids);

/* The empty-space grid: k [n[2]][n[1]][n[0]] uint8 Chebyshev cell distances,
 * geom = {g0.x, g0.y, g0.z, 1/h, h_free}.  Returns the number of cells (0 = no grid); any
 * pointer may be NULL.  For host-side tests of its conservativeness. */
int rrt_get_free_grid(const rrt_ctx* ctx, uint8_t* k, double* geom, int32_t* n);
/* Per grid cell, the oversized leaves (rrt_get_clean_tree's big list, bit = index) with a
 * primitive within reach; *reach = the segment length below which a clear bit lets the walk skip
 * that leaf.  Returns the number of cells (0 = no masks).  Host-side tests. */
int rrt_get_big_masks(const rrt_ctx* ctx, uint32_t* mask, double* reach);
/* The shadow-ray occlusion proof's triangles: per root-box face f (axis f % 3;
 * the low face for f < 3, else the high face) up to 4 triangles lying along it, each as 16
 * doubles: unit plane normal n (toward the box's inside) and offset d, then the three in-plane
 * inward unit edge normals en[3][3] and their offsets eo[3]: tris [6][4][16], counts [6].
 * Returns the total (0 = the proof never applies).  Any pointer may be NULL.  Host-side tests. */
int rrt_get_occluders(const rrt_ctx* ctx, double* tris, uint32_t* counts);

/* ---------------------------------------------------------------- file helpers (.rrts/.rrtc) */
typedef struct rrt_scene_file rrt_scene_file;
int rrt_scene_file_load(const char* path, rrt_scene_file** out);
const rrt_scene_desc* rrt_scene_file_desc(const rrt_scene_file* f);
void rrt_scene_file_free(rrt_scene_file* f);
int rrt_camera_file_load(const char* path, rrt_camera_desc* out);
/* .rrts writer (the layout rrt_scene_file_load reads). */
int rrt_scene_file_save(const char* path, const rrt_scene_desc* scene);

/* ---------------------------------------------------------------- image output (host only) */
/* HDRImageBuffer::toColor + ImageBuffer::update_pixel for one pixel (image.h:53-62, 183-198):
 * RGBA8 packed R in the low byte. */
uint32_t rrt_tonemap_pixel(const float rgb[3]);
/* PNG file of w x h RGBA8 pixels, rows top to bottom (what lodepng::encode writes for
 * PathTracer::save_image, pathtracer.cpp:646-684). */
int rrt_write_png(const char* path, const uint32_t* rgba, uint32_t w, uint32_t h);

/* OpenEXR environment maps (main.cpp:42-79 load_exr): single-part scanline files without
 * compression, HALF or FLOAT channels; R, G, B = the file's channels 2, 1, 0 (main.cpp:69-75).
 * *texels_out = [h][w][3] floats, released with rrt_exr_free.  rrt_exr_save writes FLOAT B,G,R. */
int rrt_exr_load(const char* path, float** texels_out, uint32_t* w_out, uint32_t* h_out);
void rrt_exr_free(float* texels);
int rrt_exr_save(const char* path, const float* rgb, uint32_t w, uint32_t h);

/* ---------------------------------------------------------------- native scene ingest (host only)
 * The full CGL::Camera record: the fields Camera::dump_settings / load_settings exchange
 * (camera.cpp:138-169), in that order; also the .rrtc payload (include/rrt_scene_format.h). */
typedef struct {
  double hFov, vFov, ar, nClip, fClip;
  double pos[3], targetPos[3];
  double phi, theta, r, minR, maxR;
  double c2w[9];              /* row-major c2w(i, j) */
  double screenW, screenH, screenDist;
  double focalDistance, lensRadius;
} rrt_camera_state;

typedef struct {
  uint32_t screen_w, screen_h;   /* -r W H (Application::resize -> Camera::set_screen_size) */
  double lens_radius;            /* -b (AppConfig default 0.25; PathTracer::set_camera copies it) */
  double focal_distance;         /* -d (default 4.7) */
  uint32_t reserved[4];
} rrt_collada_options;
void rrt_collada_options_default(rrt_collada_options* opt);   /* 800x600, 0.25, 4.7 */

/* Replaces: Collada::ColladaParser::load (collada/collada.cpp:131-936) + Application::load
 * (application.cpp:219-295: scene objects/lights, bbox camera placement) +
 * DynamicScene::Scene::get_static_scene (dynamic_scene/scene.cpp:133-145; halfedge vertex
 * normals, halfEdgeMesh.cpp:29-397).  Produces the StaticScene PathTracer::set_scene receives and
 * the Camera PathTracer::set_camera receives (cam_out may be NULL).  Host only; no GPU needed.
 * On failure returns RRT_E_INVALID / RRT_E_IO and writes a message into err (may be NULL). */
int rrt_collada_load(const char* path, const rrt_collada_options* opt, rrt_scene_file** scene_out,
                     rrt_camera_state* cam_out, char* err, size_t err_len);
/* Camera::load_settings / dump_settings text files (the `-c` flag, main.cpp). */
int rrt_camera_settings_load(const char* path, rrt_camera_state* out);
int rrt_camera_settings_save(const char* path, const rrt_camera_state* cam);
/* .rrtc binary record <-> rrt_camera_state */
int rrt_camera_state_file_load(const char* path, rrt_camera_state* out);
int rrt_camera_state_file_save(const char* path, const rrt_camera_state* cam);
/* The subset rrt_set_camera takes. */
int rrt_camera_state_desc(const rrt_camera_state* cam, rrt_camera_desc* out);

#ifdef __cplusplus
}
#endif
#endif /* RRT_H */
