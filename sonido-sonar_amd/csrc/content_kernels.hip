// content_kernels.hip -- ContentDetector.DetectFromAudio (fingerprint/content_detector.go:72-153)
// on the device: the whole-PCM passes and the 2048-point direct DFT.  float64, no FMA
// contraction (Makefile), Go's summation order inside every frame.
//   detect_scan_kernel    zero crossings (:220-233) and max / min |x| (> 1e-10) (:306-330):
//                         integer counts and order-free extrema -> exact
//   frame_sums_kernel     per-frame sum of squares, one thread per frame, sequential in j as
//                         the Go loops (:236-247 / :267-272 with 1024 / 512; :402-412 with the
//                         100 ms frames) -> each frame's sum is bit-identical to Go's
//   dft_mag_kernel        |X_k| of the direct DFT of the first min(2048, n) samples
//                         (computeBasicSpectrum :452-467), one block per bin
#include <hip/hip_runtime.h>

#include <cmath>

#include "kernels.h"

namespace sonar {
namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void detect_scan_kernel(const double* x, int64_t n,
                                                             unsigned long long* crossings,
                                                             unsigned long long* max_bits,
                                                             unsigned long long* min_bits) {
  __shared__ unsigned long long s_c[kBlock], s_max[kBlock], s_min[kBlock];
  unsigned long long c = 0, mx = 0, mn = 0x7ff0000000000000ull;   // mn starts at +Inf
  auto visit = [&](int64_t i, double v, double p) {
    if (i > 0) c += (p >= 0 && v < 0) || (p < 0 && v >= 0);
    const double a = fabs(v);
    const unsigned long long b = (unsigned long long)__double_as_longlong(a);   // order-preserving for a >= 0
    if (a > 0.0 && b > mx) mx = b;                 // maxVal starts at 0: only a > 0 can raise it
    if (a > 1e-10 && b < mn) mn = b;
  };
  // pairs (2i, 2i + 1) by 16-B loads when x is 16-B aligned; the previous sample of 2i is
  // the neighbour pair's second element (a cache hit)
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int64_t np = n / 2;
    for (int64_t q = t0; q < np; q += stride) {
      const double2 v = reinterpret_cast<const double2*>(x)[q];
      const int64_t i = 2 * q;
      visit(i, v.x, i > 0 ? x[i - 1] : 0.0);
      visit(i + 1, v.y, v.x);
    }
    if (t0 == 0 && (n & 1)) visit(n - 1, x[n - 1], n > 1 ? x[n - 2] : 0.0);
  } else {
    for (int64_t i = t0; i < n; i += stride) visit(i, x[i], i > 0 ? x[i - 1] : 0.0);
  }
  s_c[threadIdx.x] = c;
  s_max[threadIdx.x] = mx;
  s_min[threadIdx.x] = mn;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      s_c[threadIdx.x] += s_c[threadIdx.x + w];
      s_max[threadIdx.x] = max(s_max[threadIdx.x], s_max[threadIdx.x + w]);
      s_min[threadIdx.x] = min(s_min[threadIdx.x], s_min[threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    atomicAdd(crossings, s_c[0]);
    atomicMax(max_bits, s_max[0]);
    atomicMin(min_bits, s_min[0]);
  }
}

// sum_{j < fs, start + j < n} x[start + j]^2 for frame f, start = f * hop, added in Go's j order.
// The adds are a serial chain per frame; the loads are issued kFsBatch at a time (and the next
// batch while the current one is summed) so the chain does not wait on memory per element.
constexpr int kFsBatch = 32;
__global__ __launch_bounds__(64) void frame_sums_kernel(const double* x, int64_t n, int64_t frames, int64_t hop,
                                                            int64_t fs, double* out) {
  const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (f >= frames) return;
  const int64_t s = f * hop;
  const int64_t e = min(n, s + fs);
  double acc = 0.0;
  int64_t i = s;
  double cur[kFsBatch], nxt[kFsBatch];
  // 16-B loads when the frame start is 16-B aligned (hop and the base pointer even)
  const bool v2 = ((reinterpret_cast<uintptr_t>(x + s) & 15) == 0);
  auto load = [&](double* d, int64_t at) {
    if (v2) {
#pragma unroll
      for (int q = 0; q < kFsBatch; q += 2) {
        const double2 t = *reinterpret_cast<const double2*>(x + at + q);
        d[q] = t.x;
        d[q + 1] = t.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < kFsBatch; q++) d[q] = x[at + q];
    }
  };
  if (i + kFsBatch <= e) {
    load(cur, i);
    while (i + 2 * kFsBatch <= e) {
      load(nxt, i + kFsBatch);
#pragma unroll
      for (int q = 0; q < kFsBatch; q++) acc += cur[q] * cur[q];
#pragma unroll
      for (int q = 0; q < kFsBatch; q++) cur[q] = nxt[q];
      i += kFsBatch;
    }
#pragma unroll
    for (int q = 0; q < kFsBatch; q++) acc += cur[q] * cur[q];
    i += kFsBatch;
  }
  for (; i < e; i++) acc += x[i] * x[i];
  out[f] = acc;
}

// |X_k|, X_k = sum_n x[n] (cos + i sin)(-2 pi k n / N), angle evaluated as Go writes it.  One
// block per bin, the n-sum split over the block and tree-reduced in a fixed order (the sin/cos
// already differ from Go's by an ulp, so the sequential order would not make it bit-exact).
__global__ __launch_bounds__(kBlock) void dft_mag_kernel(const double* x, int N, double* mag) {
  __shared__ double s_re[kBlock], s_im[kBlock];
  const int k = blockIdx.x;
  double re = 0.0, im = 0.0;
  for (int t = threadIdx.x; t < N; t += kBlock) {
    const double ang = -2.0 * M_PI * (double)k * (double)t / (double)N;
    double sn, cs;
    sincos(ang, &sn, &cs);
    re += x[t] * cs;
    im += x[t] * sn;
  }
  s_re[threadIdx.x] = re;
  s_im[threadIdx.x] = im;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      s_re[threadIdx.x] += s_re[threadIdx.x + w];
      s_im[threadIdx.x] += s_im[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) mag[k] = sqrt(s_re[0] * s_re[0] + s_im[0] * s_im[0]);
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

int launch_detect_scan(const double* x, int64_t n, unsigned long long* words /* [3] */, hipStream_t s) {
  const unsigned long long init[3] = {0ull, 0ull, 0x7ff0000000000000ull};
  if (hipMemcpyAsync(words, init, sizeof(init), hipMemcpyHostToDevice, s) != hipSuccess) return -1;
  if (n <= 0) return 0;
  const unsigned g = (unsigned)std::min<int64_t>(blocks(n), 2048);    // 3 atomics per block
  hipLaunchKernelGGL(detect_scan_kernel, dim3(g), dim3(kBlock), 0, s, x, n, words, words + 1, words + 2);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_frame_sums(const double* x, int64_t n, int64_t frames, int64_t hop, int64_t fs, double* out,
                      hipStream_t s) {
  if (frames <= 0) return 0;
  // 64-thread blocks: the frame count is n / hop, often too few 256-thread blocks for 256 CUs
  hipLaunchKernelGGL(frame_sums_kernel, dim3((unsigned)((frames + 63) / 64)), dim3(64), 0, s, x, n, frames, hop, fs,
                     out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dft_mag(const double* x, int N, double* mag, hipStream_t s) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(dft_mag_kernel, dim3(N / 2 + 1), dim3(kBlock), 0, s, x, N, mag);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sonar
