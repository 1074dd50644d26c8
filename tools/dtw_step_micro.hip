// Micro-benchmark of the DTW sweep wave's step (diagnostics only; not part of the product).
// One wave per block runs S steps of the min-chain of dtw_band_kernel with parts switched off,
// timed with s_memtime (shader clocks) and s_memrealtime (100 MHz).  Build and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/dtw_step_micro.hip -o /tmp/dtw_step && /tmp/dtw_step
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#pragma clang fp contract(off)

__device__ __forceinline__ double vmin_f64(double x, double y) {
  double r;
  asm volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ double shr1(double v, double lane0) {
  const int2 a = __builtin_bit_cast(int2, v), o = __builtin_bit_cast(int2, lane0);
  const int lo = __builtin_amdgcn_update_dpp(o.x, a.x, 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(o.y, a.y, 0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double rshr1(double v, double lane0) {   // row_shr:1 (timing only)
  const int2 a = __builtin_bit_cast(int2, v), o = __builtin_bit_cast(int2, lane0);
  const int lo = __builtin_amdgcn_update_dpp(o.x, a.x, 0x111, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(o.y, a.y, 0x111, 0xf, 0xf, false);
  return __builtin_bit_cast(double, make_int2(lo, hi));
}

// V: 0 full step, 1 no global store, 2 no ds_write, 3 no DPP (v_mov), 4 row_shr DPP, 5 no code,
//    6 nothing but DPP + min + add, 7 float32 chain
// 8 full step, setprio 3;  9 full step + chunk end (release fence, LDS counter store, C-ring read of
//    lane 63 + 8-value sc1 store);  10 full step + next chunk's 19 LDS reads issued at the chunk start
//    (used at its end);  11 = 8 + 9 + 10 without the code (the production sweep's shape)
template <int V>
__global__ __launch_bounds__(64) void step_kernel(const double* d, double* out, uint32_t* dn, int S,
                                                  uint64_t* stamps) {
  __shared__ double erow[32][64];
  __shared__ double dq[32][64];
  __shared__ double eqs[256];
  __shared__ int cnt[4];
  const int lane = threadIdx.x;
  for (int k = 0; k < 32; ++k) dq[k][lane] = d[k * 64 + lane];
  for (int k = lane; k < 256; k += 64) eqs[k] = __builtin_inf();
  if (lane < 4) cnt[lane] = 1 << 30;
  __syncthreads();
  if constexpr (V == 8 || V == 11) __builtin_amdgcn_s_setprio(3);
  double dcn[8], echn[8], ech[8];
  for (int u = 0; u < 8; ++u) { echn[u] = __builtin_inf(); ech[u] = echn[u]; dcn[u] = 0; }
  uint64_t* E = reinterpret_cast<uint64_t*>(out) + 4;
  int guard = 0;
  double o = __builtin_inf(), upp = lane == 0 ? 0.0 : __builtin_inf();
  float of = __builtin_inff(), uppf = lane == 0 ? 0.f : __builtin_inff();
  uint32_t dacc = 0;
  double* cs = out + blockIdx.x * (size_t)S * 64 + lane;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int s0 = 0; s0 < S; s0 += 8) {
    double dc[8];
    int c0 = 0, c1 = 0, c2 = 0;
    if constexpr (V == 10 || V == 11) {
#pragma unroll
      for (int u = 0; u < 8; ++u) dc[u] = dcn[u];
      c0 = __hip_atomic_load(&cnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      c1 = __hip_atomic_load(&cnt[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      c2 = __hip_atomic_load(&cnt[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int u = 0; u < 8; ++u) dcn[u] = dq[(s0 + 8 + u) & 31][lane];
#pragma unroll
      for (int u = 0; u < 8; ++u) echn[u] = eqs[(s0 + 9 + u) & 255];
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) dc[u] = dq[(s0 + u) & 31][lane];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (V == 7) {
        const float up = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, __builtin_inff()),
                                                                              __builtin_bit_cast(int, of), 0x138, 0xf, 0xf, false));
        const float b = fminf(up, fminf(of, uppf));
        of = (float)dc[u] + b;
        uppf = up;
        if (lane == 63 && of == 1.f) out[0] = of;
      } else {
        double up;
        if constexpr (V == 3) up = o;
        else if constexpr (V == 4) up = rshr1(o, __builtin_inf());
        else if constexpr (V == 10 || V == 11) up = shr1(o, ech[u]);
        else up = shr1(o, __builtin_inf());
        const double best = vmin_f64(up, vmin_f64(o, upp));
        uint32_t code = 0;
        if constexpr (V != 5 && V != 6 && V != 11) code = best == up ? 0u : (best == o ? 1u : 2u);
        o = dc[u] + best;
        upp = up;
        if constexpr (V != 1 && V != 6) cs[((int64_t)(s0 + u)) << 6] = o;
        if constexpr (V != 2 && V != 6) erow[(s0 + u) & 31][lane] = o;
        dacc |= code << (2 * ((s0 & 8) + u));
      }
    }
    if constexpr (V != 11) {
      if (s0 & 8) { dn[(blockIdx.x * (size_t)S / 16 + (s0 >> 4)) * 64 + lane] = dacc; dacc = 0; }
    }
    if constexpr (V == 9 || V == 11) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&cnt[3], s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const double ev = erow[(s0 + (lane & 7)) & 31][63];
      if (lane < 8 && blockIdx.x == 0)
        __hip_atomic_store(E + s0 + lane, __builtin_bit_cast(uint64_t, ev), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (V == 10 || V == 11) {
      if (c0 < s0 || c1 < s0 || c2 < s0) ++guard;     // never (counters are 2^30)
#pragma unroll
      for (int u = 0; u < 8; ++u) ech[u] = echn[u] > 1e300 ? __builtin_inf() : echn[u];
    }
  }
  if (guard) out[2] = guard;
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) { stamps[2 * blockIdx.x] = t1 - t0; stamps[2 * blockIdx.x + 1] = r1 - r0; }
  if (lane == 0 && o == 12345.0 && of == 1.f) out[1] = erow[0][0];
}

template <int V>
void run(const char* name, const double* d, double* out, uint32_t* dn, int S, int blocks, uint64_t* st) {
  hipLaunchKernelGGL(step_kernel<V>, dim3(blocks), dim3(64), 0, 0, d, out, dn, S, st);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(step_kernel<V>, dim3(blocks), dim3(64), 0, 0, d, out, dn, S, st);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b);
  uint64_t h[2];
  hipMemcpy(h, st, 16, hipMemcpyDeviceToHost);
  printf("%-28s blocks %4d: %7.1f clk/step  %6.1f ns/step (realtime)  kernel %.3f ms\n", name, blocks,
         (double)h[0] / S, (double)h[1] * 10.0 / S, ms);
}

int main() {
  const int S = 51712;
  double* d; double* out; uint32_t* dn; uint64_t* st;
  hipMalloc(&d, 32 * 64 * 8);
  hipMemset(d, 0, 32 * 64 * 8);
  const int maxb = 1024;
  hipMalloc(&out, (size_t)maxb * S * 64 * 8 / 8);   // blocks beyond 128 share (timing only)
  hipMalloc(&dn, (size_t)maxb * (S / 16 + 1) * 64 * 4);
  hipMalloc(&st, maxb * 16);
  for (int blocks : {1, 128}) {
    double* o = out;
    (void)o;
    run<0>("full step", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<1>("no global store", d, out, dn, S, blocks, st);
    run<2>("no ds_write", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<3>("no DPP", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<4>("row_shr DPP", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<5>("no code", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<6>("DPP+min+add only", d, out, dn, S, blocks, st);
    run<7>("f32 chain", d, out, dn, S, blocks, st);
    run<8>("full step + setprio", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<9>("full step + chunk end", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<10>("full step + prefetch", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
    run<11>("production sweep shape", d, out, dn, S, blocks > 128 ? 128 : blocks, st);
  }
  return 0;
}
