// f64 VALU issue rate per SIMD vs waves per SIMD (diagnostics only).
// Each wave runs ILP independent chains of v_add_f64 / v_mul_f64 / v_fma_f64 (unrolled);
// grid = 256 CUs x 4 SIMDs x W waves (one wave per block; launch_bounds keep 1..8 waves/SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
template <int ILP, int OP>
__global__ __launch_bounds__(64) void k_f64(double* out, int iters, double a, double b) {
  double x[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) x[i] = threadIdx.x * 1e-3 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) {
        if constexpr (OP == 0) x[i] = x[i] + a;
        else if constexpr (OP == 1) x[i] = x[i] * b;
        else x[i] = __builtin_fma(x[i], b, a);
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s += x[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}
template <int ILP>
__global__ __launch_bounds__(64) void k_f32(float* out, int iters, float a) {
  float x[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) x[i] = x[i] + a;
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s += x[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}
template <typename F>
double timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms;
}
int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double* out; hipMalloc(&out, (size_t)cus * 4 * 8 * 64 * 8);
  const int iters = 4096;
  for (int w : {1, 2, 4, 8}) {
    const int blocks = cus * 4 * w;
    const double instrs = (double)blocks * iters * 16 * 8;   // wave-instructions (ILP 8)
    double ms;
    ms = timeit([&] { hipLaunchKernelGGL((k_f64<8, 0>), dim3(blocks), dim3(64), 0, 0, out, iters, 1e-9, 0.999); });
    printf("waves/SIMD %d  add_f64 ILP8: %.3f ms  %.2f cyc@2.4GHz per wave-instr per SIMD\n", w, ms, ms * 1e-3 * 2.4e9 * cus * 4 / instrs);
    ms = timeit([&] { hipLaunchKernelGGL((k_f64<8, 1>), dim3(blocks), dim3(64), 0, 0, out, iters, 1e-9, 0.999); });
    printf("waves/SIMD %d  mul_f64 ILP8: %.3f ms  %.2f cyc\n", w, ms, ms * 1e-3 * 2.4e9 * cus * 4 / instrs);
    ms = timeit([&] { hipLaunchKernelGGL((k_f64<8, 2>), dim3(blocks), dim3(64), 0, 0, out, iters, 1e-9, 0.999); });
    printf("waves/SIMD %d  fma_f64 ILP8: %.3f ms  %.2f cyc\n", w, ms, ms * 1e-3 * 2.4e9 * cus * 4 / instrs);
    ms = timeit([&] { hipLaunchKernelGGL((k_f64<2, 0>), dim3(blocks), dim3(64), 0, 0, out, iters, 1e-9, 0.999); });
    printf("waves/SIMD %d  add_f64 ILP2: %.3f ms  %.2f cyc\n", w, ms, ms * 1e-3 * 2.4e9 * cus * 4 / (instrs / 4));
    ms = timeit([&] { hipLaunchKernelGGL((k_f32<8>), dim3(blocks), dim3(64), 0, 0, (float*)out, iters, 1e-9f); });
    printf("waves/SIMD %d  add_f32 ILP8: %.3f ms  %.2f cyc\n", w, ms, ms * 1e-3 * 2.4e9 * cus * 4 / instrs);
  }
  return 0;
}
