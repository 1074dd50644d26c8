// music_kernels.hip -- the per-frame parts of MusicFeatureExtractor.ExtractFeatures that the
// fused STFT kernel does not produce (fingerprint/extractors/music.go:178-583):
//
//  music_frame_kernel  per magnitude row: SpectralContrast.Compute with 6 bands
//                      (algorithms/spectral/spectral_contrast.go:26-137: |X|^2 of each band, an
//                      ascending sort, mean of the bottom and top 20 % in sorted order,
//                      10 log10(peak / valley)), and extractEnergyFeatures' low / high band energy
//                      ratios (music.go:487-519: bins < K/4 and > 3K/4, sums in bin order)
//  abs_stats_kernel    max |y| and sum |y| in sample order (extractTemporalFeatures' peak and
//                      average amplitude, music.go:388-397), one wave, Go's sequential chain
//  frame_peak_kernel   max |y| of consecutive frames (the per-frame crest factor, :421-440)
//
// float64 throughout, no FMA contraction: the sums follow Go's order operation for operation.
#include "kernels.h"

#pragma clang fp contract(off)

namespace sonar {

// One 64-lane block per frame.  LDS: the frame's power row (K doubles) and a sort buffer of the
// next power of two >= the widest band.  The band is sorted by a bitonic network over P slots
// (+Inf padding sorts to the end), then lane 0 adds the bottom vc and top pc values in ascending
// order exactly as calculateBandContrast does after its insertion sort (:88-126).
__global__ __launch_bounds__(64) void music_frame_kernel(const double* mag, int64_t F, int K, const int* edges,
                                                         int nbands, int P, double* contrast, double* lo_ratio,
                                                         double* hi_ratio) {
  extern __shared__ double sm[];
  double* pw = sm;              // [K]
  double* sb = sm + K;          // [P]
  const int64_t t = blockIdx.x;
  if (t >= F) return;
  const int lane = threadIdx.x;
  const double* row = mag + t * (int64_t)K;
  for (int i = lane; i < K; i += 64) {
    const double m = row[i];
    pw[i] = __dmul_rn(m, m);
  }
  __syncthreads();
  for (int b = 0; b < nbands; ++b) {
    const int s0 = edges[b];
    const int e0 = min(edges[b + 1], K);
    double c = 0.0;
    if (s0 < e0) {
      const int L = e0 - s0;
      int Pb = 1;
      while (Pb < L) Pb <<= 1;
      for (int i = lane; i < Pb; i += 64) sb[i] = i < L ? pw[s0 + i] : __builtin_inf();
      __syncthreads();
      for (int k = 2; k <= Pb; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = lane; i < Pb; i += 64) {
            const int ixj = i ^ j;
            if (ixj > i) {
              const double a = sb[i], d = sb[ixj];
              const bool up = (i & k) == 0;
              if (up ? a > d : a < d) { sb[i] = d; sb[ixj] = a; }
            }
          }
          __syncthreads();
        }
      }
      if (lane == 0) {
        int vc = (int)(0.2 * (double)L), pc = (int)(0.2 * (double)L);
        if (vc == 0) vc = 1;
        if (pc == 0) pc = 1;
        double valley = 0.0;
        for (int i = 0; i < vc; ++i) valley = __dadd_rn(valley, sb[i]);
        valley = __ddiv_rn(valley, (double)vc);
        double peak = 0.0;
        for (int i = L - pc; i < L; ++i) peak = __dadd_rn(peak, sb[i]);
        peak = __ddiv_rn(peak, (double)pc);
        if (valley <= 0) valley = 1e-10;
        c = peak <= 0 ? 0.0 : __dmul_rn(10.0, log10(__ddiv_rn(peak, valley)));
      }
      __syncthreads();
    }
    if (lane == 0) contrast[t * nbands + b] = c;
  }
  if (lo_ratio && lane == 0) {
    const int lc = K / 4, hc = 3 * K / 4;
    double tot = 0.0, lo = 0.0, hi = 0.0;
    for (int i = 0; i < K; ++i) {
      const double e = pw[i];
      tot = __dadd_rn(tot, e);
      if (i < lc) lo = __dadd_rn(lo, e);
      else if (i > hc) hi = __dadd_rn(hi, e);
    }
    lo_ratio[t] = tot > 0 ? __ddiv_rn(lo, tot) : 0.0;
    hi_ratio[t] = tot > 0 ? __ddiv_rn(hi, tot) : 0.0;
  }
}

// One wave: 64 consecutive samples per step, every lane runs the same sequential chain through
// v_readlane broadcasts (Go's order); out[0] = max |y|, out[1] = sum |y|.
__global__ __launch_bounds__(64) void abs_stats_kernel(const double* y, int64_t n, double* out) {
  const int lane = threadIdx.x;
  double mx = 0.0, sum = 0.0;
  double cur = lane < n ? y[lane] : 0.0;
  for (int64_t i = 0; i < n; i += 64) {
    const double nxt = i + 64 + lane < n ? y[i + 64 + lane] : 0.0;
    const int m = (int)min((int64_t)64, n - i);
    const double a = fabs(cur);
    for (int k = 0; k < m; ++k) {
      const int2 v = __builtin_bit_cast(int2, a);
      const double ak = __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(v.x, k),
                                                             __builtin_amdgcn_readlane(v.y, k)));
      if (ak > mx) mx = ak;
      sum = __dadd_rn(sum, ak);
    }
    cur = nxt;
  }
  if (lane == 0) { out[0] = mx; out[1] = sum; }
}

// out[i] = max |y[i fs .. min(i fs + fs, n))|, one thread per frame (exact: order-free maximum)
__global__ __launch_bounds__(256) void frame_peak_kernel(const double* y, int64_t n, int64_t frames, int64_t fs,
                                                         double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= frames) return;
  const int64_t s = i * fs, e = min(s + fs, n);
  double pk = 0.0;
  for (int64_t j = s; j < e; ++j) {
    const double a = fabs(y[j]);
    if (a > pk) pk = a;
  }
  out[i] = pk;
}

int launch_music_frames(const double* mag, int64_t F, int K, const int* edges, int nbands, int maxband,
                        double* contrast, double* lo_ratio, double* hi_ratio, hipStream_t s) {
  if (F <= 0) return 0;
  int P = 1;
  while (P < maxband) P <<= 1;
  const size_t lds = (size_t)(K + P) * sizeof(double);
  if (lds > 160 * 1024) return -1;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)music_frame_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(music_frame_kernel, dim3((unsigned)F), dim3(64), lds, s, mag, F, K, edges, nbands, P, contrast,
                     lo_ratio, hi_ratio);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_abs_stats(const double* y, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(abs_stats_kernel, dim3(1), dim3(64), 0, s, y, n, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_frame_peak(const double* y, int64_t n, int64_t frames, int64_t fs, double* out, hipStream_t s) {
  if (frames <= 0) return 0;
  hipLaunchKernelGGL(frame_peak_kernel, dim3((unsigned)((frames + 255) / 256)), dim3(256), 0, s, y, n, frames, fs,
                     out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace sonar
