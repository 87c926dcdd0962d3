// Minimal reproducer of the round-3 heavy-pixel hang: a wave claims work items with
// lane 0's atomic and broadcasts the claim with __shfl; the body is wave-uniform (ballots,
// shuffles) and lane 0 stores the result.  With the body inlined, hipcc (ROCm 7.2, gfx950, -O3)
// splits the claim loop: the broadcast lands in an inner loop that the atomic is outside of, whose
// exit mask is `lane == 0` and whose back edge zeroes the claim register -- after the first item
// lanes 1..63 re-run the claim check without lane 0 and redo item 0 forever.  COMPILE ONLY: never
// launch this kernel on a GPU (it does not terminate).  check_isa.py reads the listing; run.sh
// builds the variants.
#include <hip/hip_runtime.h>
#include <cstdint>
#ifndef BODY_ATTR
#define BODY_ATTR __forceinline__
#endif
#ifndef BROADCAST
#define BROADCAST(k) __shfl((k), 0)
#endif
// claim loop: lane 0 claims, __shfl broadcasts; a wave-uniform body with a step loop; lane 0 stores
__device__ BODY_ATTR void body(const float* in, float* out, uint32_t k, uint32_t lane, uint32_t nsteps) {
  float acc = 0.0f;
  uint32_t i = 0, m0 = 0;
  for (;;) {
    const float s = in[(k * 64u + m0 + lane) & 4095u];
    const uint64_t b = __ballot(s > 0.5f);
    uint32_t m = 0;
    for (uint32_t j = 0; j < 8u; ++j) {
      acc += __shfl(s, (int)m);
      m += ((b >> m) & 1ull) ? 2u : 1u;
    }
    m0 += m;
    i += 8u;
    if (i >= nsteps || acc > 1e30f) break;
  }
  if (lane == 0) out[k] = acc;
}
__global__ __launch_bounds__(256) void claim_loop(uint32_t* counter, uint32_t n, const float* in, float* out, uint32_t nsteps) {
  const uint32_t lane = threadIdx.x & 63u;
  for (;;) {
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(counter, 1u);
    k = BROADCAST(k);
    if (k >= n) break;
    body(in, out, k, lane, nsteps);
  }
}
