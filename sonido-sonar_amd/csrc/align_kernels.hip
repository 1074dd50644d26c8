// align_kernels.hip -- path B of the hot path on gfx950: normalized
// cross-correlation and DTW, float64 like the Go reference.
//
//  NCC  CrossCorrelation.Compute with NormalizedCrossCorrelation / TimeDomain
//       (algorithms/stats/correlation.go:131-228, 373-409, 452-501) as configured by
//       NewAlignmentAnalyzer (algorithms/stats/alignment.go:60-81).
//       One thread per lag; every sum runs in Go's index order with unfused
//       mul/add (__d*_rn), so correlations -- and therefore the peak lag -- are
//       bit-identical to a sequential float64 evaluation.
//  DTW  DTWAlignment.Align / fillCostMatrix / findPreviousStep / backtrack
//       (algorithms/stats/dtw.go:55-217) with EuclideanDistanceFunc (distance.go:29-36).
//       dtw_dist_kernel   : C[i][j] = ||q_{i-1} - r_{j-1}||, C[0][*] = C[*][0] = +Inf, C[0][0] = 0
//                           (fully parallel, the matrix lives in HBM: 288 GB fits 51,676^2 doubles)
//       dtw_wave_kernel   : one launch per anti-diagonal of 64 x 64 tiles; one wave per tile
//                           sweeps its tile anti-diagonally (lane = row), neighbours through
//                           DPP shuffles, and records Go's backtrack choice (vertical <=
//                           horizontal <= diagonal, strict <) as a direction byte per cell.
//       dtw_backtrack_kernel: one wave walks the direction bytes from (N, M) through
//                           64 x 64 LDS-cached blocks.
#include "kernels.h"

#pragma clang fp contract(off)

namespace sonar {

namespace {
// math.Min (Go): NaN propagates, -Inf wins, -0 < +0
__device__ __forceinline__ double go_min(double x, double y) {
  if (__builtin_isinf(x) && x < 0) return x;
  if (__builtin_isinf(y) && y < 0) return y;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0 && x == y) return __builtin_signbit(x) ? x : y;
  return x < y ? x : y;
}
}  // namespace

// ---------------------------------------------------------------- NCC ----
// stats[0..3] = mean_a, sd_a, mean_b, sd_b  (correlation.go:464-501, sequential sums)
__global__ void ncc_stats_kernel(const double* a, int64_t na, const double* b, int64_t nb, double* stats) {
  const int w = threadIdx.x;
  if (w > 1) return;
  const double* s = w ? b : a;
  const int64_t n = w ? nb : na;
  double mean = 0.0;
  for (int64_t i = 0; i < n; ++i) mean = __dadd_rn(mean, s[i]);
  mean = __ddiv_rn(mean, (double)n);
  double var = 0.0;
  for (int64_t i = 0; i < n; ++i) { const double d = __dsub_rn(s[i], mean); var = __dadd_rn(var, __dmul_rn(d, d)); }
  var = __ddiv_rn(var, (double)n);
  stats[2 * w] = mean;
  stats[2 * w + 1] = sqrt(var);
}

__global__ void ncc_norm_kernel(const double* a, int64_t na, const double* b, int64_t nb, const double* stats,
                                double* xa, double* xb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < na) {
    const double d = __dsub_rn(a[i], stats[0]);
    xa[i] = stats[1] < 1e-10 ? d : __ddiv_rn(d, stats[1]);
  }
  if (i < nb) {
    const double d = __dsub_rn(b[i], stats[2]);
    xb[i] = stats[3] < 1e-10 ? d : __ddiv_rn(d, stats[3]);
  }
}

// one lag per thread (normalizedCrossCorrelation, correlation.go:373-409)
__global__ __launch_bounds__(256) void ncc_lag_kernel(const double* x, int64_t na, const double* y, int64_t nb,
                                                      int64_t L, double* corr) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 2 * L + 1) return;
  const int64_t lag = idx - L;
  int64_t s1, e1, s2, e2;                       // calculateOverlapRegion :421-449
  if (lag >= 0) { s1 = 0; e1 = na; s2 = lag; e2 = nb; if (e1 > nb - lag) e1 = nb - lag; if (e2 > nb) e2 = nb; }
  else { s1 = -lag; e1 = na; s2 = 0; e2 = nb; if (e1 > na) e1 = na; if (e2 > na + lag) e2 = na + lag; }
  const int64_t ov = (e1 - s1) < (e2 - s2) ? (e1 - s1) : (e2 - s2);
  double c = 0.0;
  if (ov > 0) {
    double sm = 0.0, q1 = 0.0, q2 = 0.0;
    const double* px = x + s1;
    const double* py = y + s2;
    for (int64_t k = 0; k < ov; ++k) {
      const double v1 = px[k], v2 = py[k];
      sm = __dadd_rn(sm, __dmul_rn(v1, v2));
      q1 = __dadd_rn(q1, __dmul_rn(v1, v1));
      q2 = __dadd_rn(q2, __dmul_rn(v2, v2));
    }
    const double dn = sqrt(__dmul_rn(q1, q2));
    c = dn < 1e-10 ? 0.0 : __ddiv_rn(sm, dn);
  }
  corr[idx] = c;
}

int launch_ncc(const double* a, int64_t na, const double* b, int64_t nb, int64_t L, double* xa, double* xb,
               double* stats, double* corr, hipStream_t s) {
  hipLaunchKernelGGL(ncc_stats_kernel, dim3(1), dim3(64), 0, s, a, na, b, nb, stats);
  const int64_t nmax = na > nb ? na : nb;
  hipLaunchKernelGGL(ncc_norm_kernel, dim3((unsigned)((nmax + 255) / 256)), dim3(256), 0, s, a, na, b, nb, stats, xa,
                     xb);
  const int64_t nl = 2 * L + 1;
  hipLaunchKernelGGL(ncc_lag_kernel, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, xa, na, xb, nb, L, corr);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------- DTW ----
constexpr int DTW_T = 64;   // tile rows (= lanes) and columns

__global__ __launch_bounds__(256) void dtw_dist_kernel(const double* q, int64_t nq, const double* r, int64_t nr,
                                                       int dim, int band, double* C) {
  const int64_t pitch = nr + 1;
  const int64_t total = (nq + 1) * pitch;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx / pitch, j = idx - i * pitch;
    double v;
    if (i == 0 || j == 0) {
      v = (i == 0 && j == 0) ? 0.0 : __builtin_inf();
    } else if (band > 0 && (i - j > band || j - i > band)) {
      v = __builtin_inf();                       // outside Sakoe-Chiba band: never filled (dtw.go:115-119)
    } else {
      const double* a = q + (i - 1) * dim;
      const double* b = r + (j - 1) * dim;
      double s = 0.0;
      for (int d = 0; d < dim; ++d) { const double df = __dsub_rn(a[d], b[d]); s = __dadd_rn(s, __dmul_rn(df, df)); }
      v = sqrt(s);
    }
    C[idx] = v;
  }
}

// One wave per 64x64 tile on anti-diagonal `diag` of the tile grid.
__global__ __launch_bounds__(64) void dtw_wave_kernel(double* C, uint8_t* dir, int64_t nq, int64_t nr, int band,
                                                      int64_t diag, int64_t ntr, int64_t ntc) {
  __shared__ double above[DTW_T + 1];            // C[i0-1][j0-1 .. j0+63]
  const int lane = threadIdx.x;
  const int64_t tr_lo = diag - (ntc - 1) > 0 ? diag - (ntc - 1) : 0;
  const int64_t tr = tr_lo + blockIdx.x;
  const int64_t tc = diag - tr;
  if (tr >= ntr || tc < 0) return;
  const int64_t pitch = nr + 1;
  const int64_t i0 = 1 + tr * DTW_T, j0 = 1 + tc * DTW_T;
  const int64_t i = i0 + lane;
  const bool row_ok = i <= nq;
  for (int k = lane; k <= DTW_T; k += 64) {
    const int64_t j = j0 - 1 + k;
    above[k] = (j <= nr) ? C[(i0 - 1) * pitch + j] : __builtin_inf();
  }
  if (lane == 0 && j0 + DTW_T - 1 <= nr) above[DTW_T] = C[(i0 - 1) * pitch + j0 + DTW_T - 1];
  const double left0 = row_ok ? C[i * pitch + (j0 - 1)] : __builtin_inf();
  __syncthreads();
  double diag0 = __shfl_up(left0, 1, 64);
  if (lane == 0) diag0 = above[0];

  double out = left0;      // my value at the previous column
  double up_prev = 0.0;    // value received from the lane above at the previous step
  for (int s = 0; s < DTW_T + 63; ++s) {
    double up = __shfl_up(out, 1, 64);
    const int cj = s - lane;
    if (lane == 0) up = above[(s + 1) <= DTW_T ? (s + 1) : DTW_T];
    const int64_t j = j0 + cj;
    const bool act = row_ok && cj >= 0 && cj < DTW_T && j <= nr;
    if (act) {
      const double left = (cj == 0) ? left0 : out;
      const double dg = (cj == 0) ? diag0 : up_prev;
      const int64_t o = i * pitch + j;
      const double d = C[o];
      const bool inband = !(band > 0 && (i - j > band || j - i > band));
      double v = d;
      if (inband) v = __dadd_rn(d, go_min(go_min(up, left), dg));
      // findPreviousStep (dtw.go:191-217): vertical, horizontal, diagonal; strict <
      uint8_t code = 0; double best = up;
      if (left < best) { code = 1; best = left; }
      if (dg < best) code = 2;
      C[o] = v;
      dir[(i - 1) * nr + (j - 1)] = code;
      out = v;
    }
    up_prev = up;
  }
}

// Single wave: backtrack (dtw.go:165-188) through 64x64 LDS-cached blocks.
// Records points in reverse order: rev_q[k] = i-1, rev_r[k] = j-1.
__global__ __launch_bounds__(64) void dtw_backtrack_kernel(const uint8_t* dir, int64_t nq, int64_t nr, int32_t* rev_q,
                                                           int32_t* rev_r, int64_t* plen) {
  __shared__ uint8_t blk[64][64];
  const int lane = threadIdx.x;
  int64_t i = nq, j = nr, P = 0;
  int64_t r0 = 1 << 30, c0 = 1 << 30;   // block rows [r0, r0+63], cols [c0, c0+63]
  while (i > 0 || j > 0) {
    if (lane == 0) { rev_q[P] = (int32_t)(i - 1); rev_r[P] = (int32_t)(j - 1); }
    ++P;
    if (i == 0) { --j; continue; }
    if (j == 0) { --i; continue; }
    if (i < r0 || i > r0 + 63 || j < c0 || j > c0 + 63) {
      __syncthreads();
      r0 = i - 63 > 1 ? i - 63 : 1;
      c0 = j - 63 > 1 ? j - 63 : 1;
      const int64_t row = r0 + lane;
      if (row <= nq) {
        const uint8_t* src = dir + (row - 1) * nr + (c0 - 1);
        const int64_t ncols = (nr - (c0 - 1)) < 64 ? (nr - (c0 - 1)) : 64;
        for (int k = 0; k < ncols; ++k) blk[lane][k] = src[k];
      }
      __syncthreads();
    }
    const uint8_t code = blk[i - r0][j - c0];
    if (code == 0) --i;
    else if (code == 1) --j;
    else { --i; --j; }
  }
  if (lane == 0) *plen = P;
}

// path cost C[i][j] - C[i-1][j-1] (0 on the borders), forward order
__global__ void dtw_path_cost_kernel(const double* C, int64_t nr, const int32_t* rev_q, const int32_t* rev_r,
                                     int64_t P, int32_t* pq, int32_t* pr, double* pc) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P) return;
  const int64_t src = P - 1 - k;
  const int64_t qi = rev_q[src], ri = rev_r[src];   // i-1, j-1
  const int64_t pitch = nr + 1;
  double c = 0.0;
  if (qi >= 0 && ri >= 0) c = __dsub_rn(C[(qi + 1) * pitch + (ri + 1)], C[qi * pitch + ri]);
  pq[k] = (int32_t)qi; pr[k] = (int32_t)ri; pc[k] = c;
}

int launch_dtw(const double* q, int64_t nq, const double* r, int64_t nr, int dim, int band, double* C, uint8_t* dir,
               int32_t* rev_q, int32_t* rev_r, int64_t* plen, hipStream_t s) {
  const int64_t total = (nq + 1) * (nr + 1);
  int64_t blocks = (total + 255) / 256;
  if (blocks > 256 * 64) blocks = 256 * 64;
  hipLaunchKernelGGL(dtw_dist_kernel, dim3((unsigned)blocks), dim3(256), 0, s, q, nq, r, nr, dim, band, C);
  const int64_t ntr = (nq + DTW_T - 1) / DTW_T, ntc = (nr + DTW_T - 1) / DTW_T;
  for (int64_t d = 0; d < ntr + ntc - 1; ++d) {
    const int64_t lo = d - (ntc - 1) > 0 ? d - (ntc - 1) : 0;
    const int64_t hi = d < ntr - 1 ? d : ntr - 1;
    const int64_t cnt = hi - lo + 1;
    hipLaunchKernelGGL(dtw_wave_kernel, dim3((unsigned)cnt), dim3(64), 0, s, C, dir, nq, nr, band, d, ntr, ntc);
  }
  hipLaunchKernelGGL(dtw_backtrack_kernel, dim3(1), dim3(64), 0, s, dir, nq, nr, rev_q, rev_r, plen);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_dtw_path_cost(const double* C, int64_t nr, const int32_t* rev_q, const int32_t* rev_r,
                         const int64_t* /*plen_dev*/, int64_t P, int32_t* pq, int32_t* pr, double* pc,
                         hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(dtw_path_cost_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, C, nr, rev_q, rev_r,
                     P, pq, pr, pc);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace sonar
