// tools/ubench_f64.hip -- FP64 VALU micro-benchmark on gfx950: cycles per wave64 instruction for
// dependent / independent v_fma_f64 chains, v_rcp_f64 / v_rsq_f64, and the correctly rounded
// division / sqrt sequences, at 1..8 waves per SIMD.  Diagnostic only (not part of librrt).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_f64.hip -o /tmp/ubench_f64
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define N_ITER 4096

template <int ILP>
__global__ void fma_chain(double* out, double a, double b) {
  double x[ILP];
  for (int k = 0; k < ILP; ++k) x[k] = threadIdx.x * 1e-9 + k;
  for (int i = 0; i < N_ITER; ++i) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) x[k] = fma(x[k], a, b);
  }
  double s = 0;
  for (int k = 0; k < ILP; ++k) s += x[k];
  if (s == 12345.678) out[0] = s;
}

template <int ILP>
__global__ void div_chain(double* out, double a) {
  double x[ILP];
  for (int k = 0; k < ILP; ++k) x[k] = 1.5 + threadIdx.x * 1e-9 + k;
  for (int i = 0; i < N_ITER / 8; ++i) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) x[k] = a / x[k] + 1.0;
  }
  double s = 0;
  for (int k = 0; k < ILP; ++k) s += x[k];
  if (s == 12345.678) out[0] = s;
}

template <int ILP>
__global__ void sqrt_chain(double* out, double a) {
  double x[ILP];
  for (int k = 0; k < ILP; ++k) x[k] = 1.5 + threadIdx.x * 1e-9 + k;
  for (int i = 0; i < N_ITER / 8; ++i) {
#pragma unroll
    for (int k = 0; k < ILP; ++k) x[k] = sqrt(x[k]) + a;
  }
  double s = 0;
  for (int k = 0; k < ILP; ++k) s += x[k];
  if (s == 12345.678) out[0] = s;
}

template <class F>
float time_it(F launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double* out; hipMalloc(&out, 8);
  int ncu = 256;
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0); ncu = p.multiProcessorCount;
  const double clk = 2.4e9;
  for (int wps : {1, 2, 4, 8}) {  // waves per SIMD
    const int blocks = ncu * wps;  // 256-thread blocks = 1 wave per SIMD each
    // per SIMD: wps waves; each wave executes N_ITER*ILP fma
    auto report = [&](const char* name, float ms, double instr_per_wave) {
      double cyc = ms * 1e-3 * clk;
      double per_simd_instr = instr_per_wave * wps;
      printf("%-22s waves/SIMD=%d  %.2f cycles per wave-instruction per SIMD\n", name, wps, cyc / per_simd_instr);
    };
    report("fma dep (ILP1)", time_it([&] { hipLaunchKernelGGL(fma_chain<1>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 1e-9); }), N_ITER * 1.0);
    report("fma ILP4", time_it([&] { hipLaunchKernelGGL(fma_chain<4>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 1e-9); }), N_ITER * 4.0);
    report("fma ILP8", time_it([&] { hipLaunchKernelGGL(fma_chain<8>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 1e-9); }), N_ITER * 8.0);
    report("div dep (per div)", time_it([&] { hipLaunchKernelGGL(div_chain<1>, dim3(blocks), dim3(256), 0, 0, out, 1.25); }), N_ITER / 8 * 1.0);
    report("div ILP4 (per div)", time_it([&] { hipLaunchKernelGGL(div_chain<4>, dim3(blocks), dim3(256), 0, 0, out, 1.25); }), N_ITER / 8 * 4.0);
    report("sqrt dep (per sqrt)", time_it([&] { hipLaunchKernelGGL(sqrt_chain<1>, dim3(blocks), dim3(256), 0, 0, out, 0.25); }), N_ITER / 8 * 1.0);
    report("sqrt ILP4 (per sqrt)", time_it([&] { hipLaunchKernelGGL(sqrt_chain<4>, dim3(blocks), dim3(256), 0, 0, out, 0.25); }), N_ITER / 8 * 4.0);
  }
  return 0;
}
