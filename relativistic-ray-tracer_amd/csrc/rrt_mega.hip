// rrt_mega.hip -- the hot path (max_ray_depth <= 1) as a persistent wavefront state machine.
//
// Reference: PathTracer::raytrace_pixel (part1_code.cpp:125-163) -> est_radiance_global_illumination
// (:103-123, ILLUM 2) -> estimate_direct_lighting_importance / _hemisphere (:15-57) ->
// BVHAccel::intersect (bvh.cpp:103-138) -> BlackHole::next_micro_ray (blackhole.cpp:17-40).
//
// Why a state machine: written as nested calls, every query site (camera ray, shadow ray,
// hemisphere ray) inlines its own copy of the geodesic march + traversal and the kernel needs
// > 256 VGPRs (one wave per SIMD).  Here each lane carries a small explicit state (pixel
// accumulators, shading record, one in-flight query) and one loop iteration advances every
// lane by one step of whatever it is doing: take a pixel, start a camera sample, march one
// micro segment of its current query (capture test + full segment traversal), or resolve a
// finished query (shade, issue the next shadow ray, close the sample / pixel).  A lane that
// finishes early immediately takes new work (per-wave 8x8 pixel pools refilled by one atomic),
// so the wave is not held back by its slowest pixel or its longest geodesic.
//
// Slab test: the reference divides by the segment direction (bbox.cpp:11-16).  Per segment we
// form y = RN(1/d) once and get each quotient with two Markstein correction steps
// (q0 = a*y; q1 = q0 + (a - d*q0)*y; q = q1 + (a - d*q1)*y, residuals exact by FMA), which
// equals the correctly rounded a/d when nothing under/overflows (Markstein's theorem).  The
// host enables it only when every BVH coordinate is 0 or in [2^-800, 2^20] in magnitude, and
// a segment whose origin/direction leaves that range uses true division -- so every decision
// is the reference's.
#include "rrt_device.h"

namespace rrt {

// BVHAccel::intersect_micro (bvh.cpp:115-138) over one micro segment, stackless (skip pointers)
template <bool EXACT, bool COUNT>
__device__ __forceinline__ bool seg_traverse(const KParams& kp, v3 o, v3 d, v3 y, double max_t, bool any,
                                             int& slot_out, double& t_out, double& b1_out, double& b2_out,
                                             Counters& cn) {
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
        max_t = t; hit = true; slot_out = slot; t_out = t; b1_out = b1; b2_out = b2;
        if (any) break;
      }
    }
    if (hit && any) break;
    node = n.skip;
  }
  return hit;
}

enum : uint32_t { PH_IDLE = 0, PH_NEED = 1, PH_SAMPLE = 2, PH_QUERY = 3, PH_RESOLVE = 4 };
enum : uint32_t { Q_CAMERA = 0, Q_SHADOW = 1, Q_HEMI = 2 };

}  // namespace rrt

template <bool COUNT, int WAVES>
__global__ __launch_bounds__(256, WAVES) void rrt_mega_kernel(const KParams* __restrict__ kpp) {
  const KParams& kp = *kpp;
  using namespace rrt;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
  const uint32_t bpt = kp.blocks_per_tile_side;
  const uint32_t tpix = kp.tile_size * kp.tile_size;
  const v3 hc = V(kp.hole.c[0], kp.hole.c[1], kp.hole.c[2]);

  // wave-uniform pixel pool: one 8x8 block of the tile list at a time
  uint32_t pool_blk = 0, pool_next = 64;
  bool pool_empty = false;

  uint32_t phase = PH_NEED;
  // pixel state
  uint32_t slot_out = 0;
  uint32_t px = 0, py = 0;
  Rng g; g.key = 0; g.ctr = 0;
  uint32_t ns = 0;
  double s1 = 0.0, s2 = 0.0;
  spec ret = S(0, 0, 0), e = S(0, 0, 0), L = S(0, 0, 0), pend = S(0, 0, 0);
  float pend_wz = 0.f;
  Counters cn = {0, 0, 0, 0};
  // shading record (camera hit)
  v3 hp = V(0, 0, 0), nn = V(0, 0, 0), wol = V(0, 0, 0);
  uint32_t bsdf = 0, li = 0, lk = 0;
  int total = 0;
  // in-flight query
  v3 qo = V(0, 0, 0), qd = V(0, 0, 0);
  double qmax = 0.0, qt = 0.0, qb1 = 0.0, qb2 = 0.0;
  int qstep = 0, qslot = -1;
  uint32_t qkind = Q_CAMERA;
  bool qhit = false;

  for (;;) {
    // ---------------------------------------------------------------- refill
    for (;;) {
      const uint64_t need = __ballot(phase == PH_NEED);
      if (need == 0) break;
      if (pool_next >= 64) {
        if (pool_empty) {
          if (phase == PH_NEED) phase = PH_IDLE;
          break;
        }
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(kp.block_counter, 1u);
        b = __shfl(b, 0);
        if (b >= kp.n_blocks) { pool_empty = true; continue; }
        pool_blk = b;
        pool_next = 0;
      }
      const uint32_t avail = 64u - pool_next;
      const uint32_t rank = (uint32_t)__popcll(need & lt_mask);
      if (phase == PH_NEED && rank < avail) {
        const uint32_t k = pool_next + rank;
        const uint32_t t = pool_blk / (bpt * bpt), b = pool_blk % (bpt * bpt);
        const uint32_t lx = (b % bpt) * 8 + (k & 7u), ly = (b / bpt) * 8 + (k >> 3);
        const uint32_t x = kp.tiles[2 * t] + lx, y = kp.tiles[2 * t + 1] + ly;
        if (lx < kp.tile_size && ly < kp.tile_size && x >= kp.clip_x0 && y >= kp.clip_y0 && x < kp.clip_x1 &&
            y < kp.clip_y1) {
          px = x; py = y;
          slot_out = t * tpix + ly * kp.tile_size + lx;
          g.key = rrt_pixel_key(kp.seed, x, y); g.ctr = 0;
          ns = 0; s1 = 0.0; s2 = 0.0; ret = S(0, 0, 0);
          cn.bbox = 0; cn.micro = 0; cn.prim = 0; cn.query = 0;
          phase = PH_SAMPLE;
          if (kp.ns_aa == 0) {  // the reference's loop does not run: ret / 0
            spec r = ret / (float)0;
            kp.rgb[3 * slot_out] = r.r; kp.rgb[3 * slot_out + 1] = r.g; kp.rgb[3 * slot_out + 2] = r.b;
            kp.count[slot_out] = 0;
            if (kp.draws) kp.draws[slot_out] = 0;
            phase = PH_NEED;
          }
        }
      }
      const uint32_t n_need = (uint32_t)__popcll(need);
      pool_next += (n_need < avail) ? n_need : avail;
    }
    if (__ballot(phase != PH_IDLE) == 0) break;

    // ---------------------------------------------------------------- camera sample
    if (phase == PH_SAMPLE) {
      double sx = (double)px, sy = (double)py;
      if (kp.ns_aa == 1) { sx += 0.5; sy += 0.5; }
      else { double jx, jy; g.grid(jx, jy); sx += jx; sy += jy; }
      const DCamera& cam = kp.cam;  // Camera::generate_ray (part1_code.cpp:182-187)
      double cx = sx / kp.frame_w, cy = sy / kp.frame_h;
      double vx = (1 - cx) * cam.blx + cx * -cam.blx, vy = (1 - cy) * cam.bly + cy * -cam.bly;
      v3 w = (smul(vx, ld3(cam.c2w0)) + smul(vy, ld3(cam.c2w1))) + smul(-1.0, ld3(cam.c2w2));
      qo = ld3(cam.pos); qd = unit(w); qmax = 0.0; qstep = 0; qkind = Q_CAMERA;
      if (COUNT) cn.query++;
      phase = PH_QUERY;
    }

    // ---------------------------------------------------------------- one micro segment
    if (phase == PH_QUERY) {
      next_micro(kp.hole, qo, qd, qmax);
      ++qstep;
      if (COUNT) cn.micro++;
      double tc;
      qhit = false;
      bool done;
      if (sphere_t(hc, kp.hole.r2, qo, qd, qmax, tc)) {
        done = true;  // captured by the hole: "no hit" (bvh.cpp:107-108)
      } else if (!COUNT && segment_clear(kp.grid, qo, qmax)) {
        done = qstep >= kp.hole.steps;  // no leaf box within reach: traversal would miss
      } else {
        const v3 y = V(xdiv(1.0, qd.x), xdiv(1.0, qd.y), xdiv(1.0, qd.z));
        const bool fast = segment_fast(kp, qo, qd);
        const bool any = (qkind == Q_SHADOW);
        if (fast) qhit = seg_traverse<false, COUNT>(kp, qo, qd, y, qmax, any, qslot, qt, qb1, qb2, cn);
        else qhit = seg_traverse<true, COUNT>(kp, qo, qd, y, qmax, any, qslot, qt, qb1, qb2, cn);
        done = qhit || qstep >= kp.hole.steps;
      }
      if (done) phase = PH_RESOLVE;
    }

    // ---------------------------------------------------------------- resolve / shade
    if (phase == PH_RESOLVE) {
      bool sample_done = false;
      spec s = S(0, 0, 0);
      bool issue = false;  // scan lights for the next shadow / hemisphere query
      if (qkind == Q_CAMERA) {
        if (!qhit) {
          sample_done = true;  // no environment light in this path
        } else {
          const DPrimMeta meta = kp.meta[qslot];
          bsdf = (meta >> 8) & 0xffu;
          hp = qo + vmul(qd, qt);
          const v3 wout = -qd;
          if (meta & 1u) {
            const DPrimGeo gp = kp.geo[qslot];
            nn = unit((qo + vmul(qd, qt)) - V(gp.v[0], gp.v[1], gp.v[2]));
          } else {
            const DPrimNrm q = kp.nrm[qslot];
            const double b0 = 1 - qb1 - qb2;
            nn = (smul(b0, V(q.n[0], q.n[1], q.n[2])) + smul(qb1, V(q.n[3], q.n[4], q.n[5]))) +
                 smul(qb2, V(q.n[6], q.n[7], q.n[8]));
          }
          const DBsdf bs = kp.bsdfs[bsdf];
          e = emission(bs);
          if (kp.max_ray_depth == 0) {
            s = e;
            sample_done = true;
          } else {
            const Frame f = coord_space(nn);
            wol = to_local(f, wout);
            L = S(0, 0, 0);
            li = 0; lk = 0;
            total = kp.direct_hemisphere ? (int)(kp.n_lights * kp.ns_area_light) : 0;
            issue = true;
          }
        }
      } else if (qkind == Q_SHADOW) {
        if (!qhit) L = L + pend;
        issue = true;
      } else {  // Q_HEMI
        if (qhit) L = L + (emission(kp.bsdfs[(kp.meta[qslot] >> 8) & 0xffu]) * pend) * pend_wz;
        issue = true;
      }
      if (issue) {
        const DBsdf bs = kp.bsdfs[bsdf];
        if (kp.direct_hemisphere) {  // estimate_direct_lighting_hemisphere (:15-31)
          if ((int)lk < total) {
            ++lk;
            const v3 w_in = hemisphere_sample(g);
            const Frame f = coord_space(nn);
            const v3 wi = to_world(f, w_in);
            pend = bsdf_f(bs, wol, w_in);
            pend_wz = (float)w_in.z;
            qo = hp + smul(EPS_D, wi); qd = wi; qmax = 0.0; qstep = 0; qkind = Q_HEMI;
            if (COUNT) cn.query++;
            phase = PH_QUERY;
          } else {
            s = e + ((L * 2.0f) * (float)PI_D) / (float)total;
            sample_done = true;
          }
        } else {  // estimate_direct_lighting_importance (:33-57)
          for (;;) {
            if (li >= kp.n_lights) {
              s = e + L / (float)total;
              sample_done = true;
              break;
            }
            const DLight& l = kp.lights[li];
            const uint32_t num = l.is_delta ? 1u : kp.ns_area_light;
            if (lk == 0) total += (int)num;
            if (lk >= num) { ++li; lk = 0; continue; }
            ++lk;
            v3 wi; float dist, pdf;
            const spec smp = light_sample_L(kp.env, l, g, hp, wi, dist, pdf);
            const Frame f = coord_space(nn);
            const v3 w_in = to_local(f, wi);
            if (w_in.z < 0) continue;
            pend = ((smp * bsdf_f(bs, wol, w_in)) * (float)w_in.z) / pdf;
            qo = hp + smul(EPS_D, wi); qd = wi; qmax = 0.0; qstep = 0; qkind = Q_SHADOW;
            if (COUNT) cn.query++;
            phase = PH_QUERY;
            break;
          }
        }
      }
      if (sample_done) {  // raytrace_pixel loop body tail, ADAPTIVE == 1 (:145-159)
        ret = ret + s;
        const double il = illum(s);
        s1 += il;
        s2 += il * il;
        ++ns;
        bool stop = false;
        if (ns % kp.samples_per_batch == 0) {
          const double avg = s1 / ns, sd = sqrt((s2 - avg * s1) / (ns - 1));
          if (1.96 * sd / sqrt((double)ns) <= (double)kp.max_tolerance * avg) stop = true;
        }
        if (stop || ns >= kp.ns_aa) {
          const spec r = ret / (float)ns;
          kp.rgb[3 * slot_out] = r.r; kp.rgb[3 * slot_out + 1] = r.g; kp.rgb[3 * slot_out + 2] = r.b;
          kp.count[slot_out] = (int32_t)ns;
          if (kp.draws) kp.draws[slot_out] = g.ctr;
          if (COUNT && kp.counters) {
            kp.counters[4 * slot_out] = cn.bbox; kp.counters[4 * slot_out + 1] = cn.micro;
            kp.counters[4 * slot_out + 2] = cn.prim; kp.counters[4 * slot_out + 3] = cn.query;
          }
          phase = PH_NEED;
        } else {
          phase = PH_SAMPLE;
        }
      }
    }
  }
}

// waves: minimum waves per SIMD the register allocation must allow (1..4); A/B knob
hipError_t rrt_launch_mega(const KParams& kp, const KParams* d_kp, int count, int waves, uint32_t grid, hipStream_t stream) {
#define RRT_MEGA_CASE(W)                                                                         \
  case W:                                                                                        \
    if (count) hipLaunchKernelGGL((rrt_mega_kernel<true, W>), dim3(grid), dim3(256), 0, stream, d_kp); \
    else hipLaunchKernelGGL((rrt_mega_kernel<false, W>), dim3(grid), dim3(256), 0, stream, d_kp);      \
    break;
  switch (waves) {
    RRT_MEGA_CASE(1)
    RRT_MEGA_CASE(3)
    RRT_MEGA_CASE(4)
    default:
    RRT_MEGA_CASE(2)
  }
#undef RRT_MEGA_CASE
  return hipGetLastError();
}
