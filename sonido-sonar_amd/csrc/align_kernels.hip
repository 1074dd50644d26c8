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
//       dtw_band_kernel   : ONE persistent launch; 64-row bands pipelined through an sc1
//                           edge hand-off, lane = row, DPP neighbours, distance inline
//                           (see the DTW section below for the layout)
//       dtw_walk_kernel   : one wave walks the 2-bit direction codes from (N, M)
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include <cstdio>
#include <mutex>

#include "kernels.h"

#pragma clang fp contract(off)

namespace sonar {

namespace {
// math.Min (Go): NaN propagates, -Inf wins, -0 < +0
// sqrt(x) for x in [2^-767, +Inf): LLVM's correctly rounded f64 sqrt sequence (v_rsq_f64 + two
// Goldschmidt/Newton refinements) without its range scaling (an ldexp by 0 there) and its
// 0 / Inf class fix-up (not taken there), so the same bits as sqrt() in 10 instructions instead
// of 18.  The caller checks the range for the whole wave.
__device__ __forceinline__ double sqrt_normal(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
constexpr double DTW_SQRT_MIN = 0x1p-767;   // below: the full sqrt() (its scaled range)

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
// Global z-score statistics (normalize :464-501): mean and population std of each input, every
// sum sequential in Go's index order (bit-exact).  One wave per input: the wave loads 64
// consecutive values per step (coalesced, the next step in flight), and every lane runs the
// same sequential add chain over them through v_readlane broadcasts.
__device__ __forceinline__ double lane_bcast(double v, int j) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), j);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// a batched launch's job (blockIdx.y) into SGPRs
template <class J>
__device__ __forceinline__ J load_job(const J* p) {
  static_assert(sizeof(J) % 4 == 0, "read as dwords");
  J r;
  const int* src = reinterpret_cast<const int*>(p);
  int* dst = reinterpret_cast<int*>(&r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(J) / 4); ++k) dst[k] = __builtin_amdgcn_readfirstlane(src[k]);
  return r;
}

// BJ (this and the two NCC kernels below): one pair per blockIdx.y, its arguments from jobs[]
template <bool BJ = false>
__global__ __launch_bounds__(64) void ncc_stats_kernel(const double* a, int64_t na, const double* b, int64_t nb,
                                                       double* stats, const NccJob* jobs) {
  SONAR_FEAT_PRIO();
  if constexpr (BJ) {
    const NccJob j = load_job(jobs + blockIdx.y);
    a = j.a; na = j.na; b = j.b; nb = j.nb; stats = j.stats;
  }
  const int w = blockIdx.x;
  const int lane = threadIdx.x;
  const double* s = w ? b : a;
  const int64_t n = w ? nb : na;
  // full 64-value steps are unrolled (constant readlane indices, broadcasts issued ahead of the
  // add chain); the tail runs the same chain with a runtime index
  double mean = 0.0;
  {
    double cur = lane < n ? s[lane] : 0.0;
    int64_t i = 0;
    for (; i + 64 <= n; i += 64) {
      const double nxt = i + 64 + lane < n ? s[i + 64 + lane] : 0.0;
#pragma unroll
      for (int j = 0; j < 64; j++) mean = __dadd_rn(mean, lane_bcast(cur, j));
      cur = nxt;
    }
    for (int j = 0; j < (int)(n - i); j++) mean = __dadd_rn(mean, lane_bcast(cur, j));
  }
  mean = __ddiv_rn(mean, (double)n);
  double var = 0.0;
  {
    double cur = lane < n ? __dsub_rn(s[lane], mean) : 0.0;
    int64_t i = 0;
    for (; i + 64 <= n; i += 64) {
      const double nxt = i + 64 + lane < n ? __dsub_rn(s[i + 64 + lane], mean) : 0.0;
#pragma unroll
      for (int j = 0; j < 64; j++) {
        const double d = lane_bcast(cur, j);
        var = __dadd_rn(var, __dmul_rn(d, d));
      }
      cur = nxt;
    }
    for (int j = 0; j < (int)(n - i); j++) {
      const double d = lane_bcast(cur, j);
      var = __dadd_rn(var, __dmul_rn(d, d));
    }
  }
  var = __ddiv_rn(var, (double)n);
  if (lane == 0) {
    stats[2 * w] = mean;
    stats[2 * w + 1] = sqrt(var);
  }
}

template <bool BJ = false>
__global__ void ncc_norm_kernel(const double* a, int64_t na, const double* b, int64_t nb, const double* stats,
                                double* xa, double* xb, const NccJob* jobs) {
  SONAR_FEAT_PRIO();
  if constexpr (BJ) {
    const NccJob j = load_job(jobs + blockIdx.y);
    a = j.a; na = j.na; b = j.b; nb = j.nb; stats = j.stats; xa = j.xa; xb = j.xb;
  }
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

// one lag per thread (normalizedCrossCorrelation, correlation.go:373-409), sums in Go's index
// order (bit-exact).  A block owns 256 consecutive lags; their overlap windows start within 255
// samples of each other (s1 = max(0, -lag), s2 = max(0, lag)), so each k-tile of both inputs is
// staged once in LDS (coalesced) and every thread walks its own offsets there.
constexpr int kNccTile = 1024;
template <bool BJ = false>
__global__ __launch_bounds__(256) void ncc_lag_kernel(const double* x, int64_t na, const double* y, int64_t nb,
                                                      int64_t L, double* corr, const NccJob* jobs) {
  SONAR_FEAT_PRIO();
  __shared__ double xs[kNccTile + 256], ys[kNccTile + 256];
  __shared__ int64_t ovmax_s;
  if constexpr (BJ) {
    const NccJob j = load_job(jobs + blockIdx.y);
    x = j.xa; na = j.na; y = j.xb; nb = j.nb; L = j.L; corr = j.corr;
  }
  const int64_t nl = 2 * L + 1;
  const int64_t idx0 = (int64_t)blockIdx.x * 256;
  if (idx0 >= nl) return;
  const int64_t idx = idx0 + threadIdx.x;
  const bool active = idx < nl;
  const int64_t lag = idx - L;
  int64_t s1 = 0, e1 = 0, s2 = 0, e2 = 0;         // calculateOverlapRegion :421-449
  if (lag >= 0) { s1 = 0; e1 = na; s2 = lag; e2 = nb; if (e1 > nb - lag) e1 = nb - lag; if (e2 > nb) e2 = nb; }
  else { s1 = -lag; e1 = na; s2 = 0; e2 = nb; if (e1 > na) e1 = na; if (e2 > na + lag) e2 = na + lag; }
  int64_t ov = (e1 - s1) < (e2 - s2) ? (e1 - s1) : (e2 - s2);
  if (!active || ov < 0) ov = 0;
  // window origins over the block's lags [idx0 - L, last - L]
  const int64_t lastlag = (idx0 + 255 < nl ? idx0 + 255 : nl - 1) - L;
  const int64_t x0 = lastlag < 0 ? -lastlag : 0;   // min s1
  const int64_t y0 = idx0 - L > 0 ? idx0 - L : 0;   // min s2
  if (threadIdx.x == 0) ovmax_s = 0;
  __syncthreads();
  atomicMax(reinterpret_cast<unsigned long long*>(&ovmax_s), (unsigned long long)ov);
  __syncthreads();
  const int64_t ovmax = ovmax_s;
  const int ox = (int)(s1 - x0), oy = (int)(s2 - y0);   // 0..255 for active lags
  double sm = 0.0, q1 = 0.0, q2 = 0.0;
  for (int64_t k0 = 0; k0 < ovmax; k0 += kNccTile) {
    for (int j = threadIdx.x; j < kNccTile + 256; j += 256) {
      const int64_t gx = x0 + k0 + j, gy = y0 + k0 + j;
      xs[j] = gx < na ? x[gx] : 0.0;
      ys[j] = gy < nb ? y[gy] : 0.0;
    }
    __syncthreads();
    int kend = ov - k0 < kNccTile ? (int)(ov - k0) : kNccTile;
    if (kend < 0) kend = 0;
    const double* px = xs + ox;
    const double* py = ys + oy;
    int k = 0;
    for (; k + 4 <= kend; k += 4) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const double c1 = px[k + j], c2 = py[k + j];
        sm = __dadd_rn(sm, __dmul_rn(c1, c2));
        q1 = __dadd_rn(q1, __dmul_rn(c1, c1));
        q2 = __dadd_rn(q2, __dmul_rn(c2, c2));
      }
    }
    for (; k < kend; k++) {
      const double c1 = px[k], c2 = py[k];
      sm = __dadd_rn(sm, __dmul_rn(c1, c2));
      q1 = __dadd_rn(q1, __dmul_rn(c1, c1));
      q2 = __dadd_rn(q2, __dmul_rn(c2, c2));
    }
    __syncthreads();
  }
  if (!active) return;
  double c = 0.0;
  if (ov > 0) {
    const double dn = sqrt(__dmul_rn(q1, q2));
    c = dn < 1e-10 ? 0.0 : __ddiv_rn(sm, dn);
  }
  corr[idx] = c;
}

int launch_ncc(const double* a, int64_t na, const double* b, int64_t nb, int64_t L, double* xa, double* xb,
               double* stats, double* corr, hipStream_t s) {
  const NccJob* none = nullptr;
  hipLaunchKernelGGL((ncc_stats_kernel<false>), dim3(2), dim3(64), 0, s, a, na, b, nb, stats, none);
  const int64_t nmax = na > nb ? na : nb;
  hipLaunchKernelGGL((ncc_norm_kernel<false>), dim3((unsigned)((nmax + 255) / 256)), dim3(256), 0, s, a, na, b, nb, stats, xa,
                     xb, none);
  const int64_t nl = 2 * L + 1;
  hipLaunchKernelGGL((ncc_lag_kernel<false>), dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, xa, na, xb, nb, L, corr,
                     none);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// launch_ncc over many pairs in three launches (blockIdx.y = pair); the same kernels, arithmetic
// and order per pair, so the same bits
int launch_ncc_batch(const NccJob* hjobs, const NccJob* djobs, int nj, hipStream_t s) {
  if (nj <= 0) return 0;
  if (nj > 65535) return -1;
  int64_t nmax = 1, nlmax = 1;
  for (int k = 0; k < nj; ++k) {
    nmax = std::max(nmax, std::max(hjobs[k].na, hjobs[k].nb));
    nlmax = std::max(nlmax, 2 * hjobs[k].L + 1);
  }
  hipLaunchKernelGGL((ncc_stats_kernel<true>), dim3(2, (unsigned)nj), dim3(64), 0, s, nullptr, 0, nullptr, 0, nullptr,
                     djobs);
  hipLaunchKernelGGL((ncc_norm_kernel<true>), dim3((unsigned)((nmax + 255) / 256), (unsigned)nj), dim3(256), 0, s,
                     nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, djobs);
  hipLaunchKernelGGL((ncc_lag_kernel<true>), dim3((unsigned)((nlmax + 255) / 256), (unsigned)nj), dim3(256), 0, s,
                     nullptr, 0, nullptr, 0, 0, nullptr, djobs);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// AlignmentAnalyzer.addNoise (alignment.go:737-749): out[i][j] = q + (sin(i*j+i+j) * level) * q
__global__ void perturb_kernel(const double* q, int64_t nq, int dim, double level, double* out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nq * dim) return;
  const int64_t i = idx / dim, j = idx - i * dim;
  const double v = q[idx];
  out[idx] = __dadd_rn(v, __dmul_rn(__dmul_rn(sin((double)(i * j + i + j)), level), v));
}
// flatten2DFeatures (:363-378): the first component of every frame
__global__ void first_column_kernel(const double* x, int64_t n, int dim, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = x[i * dim];
}
int launch_perturb(const double* q, int64_t nq, int dim, double level, double* out, hipStream_t s) {
  const int64_t n = nq * dim;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(perturb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, nq, dim, level, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
int launch_first_column(const double* x, int64_t n, int dim, double* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(first_column_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n, dim, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------- DTW ----
// Forward sweep (fillCostMatrix + applyStepPattern "symmetric2", dtw.go:106-135,138-143)
// as ONE persistent launch.  Rows are cut into bands of 64; one wave owns a band
// (lane l = row 64b+1+l) and sweeps it in S = nr + 63 skewed steps: at step s lane
// l relaxes column j = s - l + 1, so C[i-1][j] (lane l-1, previous step) and
// C[i-1][j-1] (what this lane received one step earlier) arrive through one
// DPP wave_shr:1 per step and C[i][j-1] is the lane's own register.  Bands are
// handed out by an atomic ticket in order, so a wave only ever waits for an
// earlier, already running band: band b's last row goes to band b+1 through the
// edge buffer E as 8-byte sc1 stores that ARE the flag (the buffer is pre-filled
// with a signalling-NaN sentinel no arithmetic can produce; MI355X_MICROARCH.md
// "Valid forms", R2).  The local distance (EuclideanDistanceFunc, distance.go:29-36,
// unfused, Go's summation order) is computed inline from the lane's query row in
// registers and a 128-row LDS ring of reference rows (row s-l for lane l).
//   Cn[b][s][l]  C[64b+1+l][s-l+1]    one coalesced 512-B store per step (8 B/cell)
//   Dn[b][w][l]  2-bit findPreviousStep codes (dtw.go:191-217) of steps 16w..16w+15
// The walk (backtrack, dtw.go:165-188) is one wave reading Dn through 16-word
// register windows (readlane), s = j-1+l strictly decreases along the path.
constexpr int DTW_ECH = 8;                          // edge values polled per chunk
#ifndef DTW_G
#define DTW_G 4                                     // steps per scheduling group in the sweep
#endif
constexpr uint64_t DTW_SENT = 0x7FF000017FF00001ull;  // signalling NaN: never an arithmetic result
// Every inter-workgroup access of the band pipeline is a GLOBAL instruction.  The batched band
// kernels read their DtwArgs through readfirstlane, so the compiler cannot prove that E and the
// sync words are global and emitted FLAT accesses for them: a flat_load_dwordx2 sc1 edge poll was
// measured to keep returning the sentinel for milliseconds after the producer's store (every
// agent-scope acquire issued after 1 ms without progress was followed by new values: 20,027 of
// 20,053 in four C5 repetitions), which is what timed out the round-2 C5 runs.  The single-DTW
// kernels got global_load sc1 and never stalled.  MI355X_MICROARCH.md: "global_/buffer_ sc1 loads
// to registers (never flat_)".
typedef __attribute__((address_space(1))) uint64_t dtw_gu64;
typedef __attribute__((address_space(1))) int32_t dtw_gi32;
__device__ __forceinline__ uint64_t g_load_agent(const uint64_t* p) {
  return __hip_atomic_load((const dtw_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t g_load_system(const uint64_t* p) {
  return __hip_atomic_load((const dtw_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int32_t g_load_agent(const int32_t* p) {
  return __hip_atomic_load((const dtw_gi32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_store_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store((dtw_gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a plain access through a pointer known to address global memory (global_* instead of flat_*;
// a flat access also counts against lgkmcnt, so the LDS waits of the role would wait for it)
#define DTW_GLOBAL(p) ((__attribute__((address_space(1))) std::remove_pointer_t<decltype(p)>*)(p))
typedef double dtw_d2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void g_add_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_fetch_add((dtw_gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Liveness bound of every wait in the band kernel: a wait gives up when it has seen no progress
// for DTW_STALL_TICKS of s_memrealtime (100 MHz) AND has polled at least DTW_STALL_POLLS times (a
// wave that was switched out does not time out on wall time alone).  The first wave to give up
// writes the DTW's diagnostic record (DtwArgs::diag) and raises the block's LDS abort word, which
// every other wait of the block checks; the edge poller also watches the DTW's global error word,
// so the bands below a failed one stop within milliseconds instead of each running out its bound.
#ifndef DTW_STALL_MS
#define DTW_STALL_MS 1000
#endif
constexpr uint64_t DTW_STALL_TICKS = (uint64_t)DTW_STALL_MS * 100000ull;
constexpr uint32_t DTW_STALL_POLLS = 1u << 18;
// the edge poller's refresh: after 1 ms without a new edge value it issues one agent-scope acquire
// (buffer_inv sc1) and counts it in diag[13] (diag[14] when the next poll found new values)
constexpr uint64_t DTW_REFRESH_TICKS = 100000ull;
#ifndef DTW_SPIN_SLEEP
#define DTW_SPIN_SLEEP 4                            // s_sleep between LDS counter polls (A/B 0,1,4,8,16: 4-8 best)
#endif

static_assert(sizeof(DtwArgs) % 4 == 0, "read as dwords");

// Many independent DTWs in one band-kernel launch: a block's ticket t runs over every DTW's bands
// in order (DTW k owns tickets [start[k], start[k+1])), so each DTW's bands still start in band
// order, and a DTW's first band starts as soon as the previous DTW's last band holds a slot.
struct DtwBatch {
  const DtwArgs* args;
  const int64_t* start;
  int n;
  int32_t* ticket;
  const int2* map;   // nullable: ticket -> (DTW, band) in any order where a band's predecessor
                     // has the smaller ticket; null: DTW-major through `start`
};

namespace {

// a DtwArgs at a wave-uniform address into SGPRs (every field read through readfirstlane).  The
// compiler cannot tell that its pointers address global memory: accesses through them that matter
// go through DTW_GLOBAL / g_load_agent / g_store_agent (global_* instead of flat_*)
__device__ __forceinline__ DtwArgs load_args_uniform(const DtwArgs* p) {
  DtwArgs r;
  const int* src = reinterpret_cast<const int*>(p);
  int* dst = reinterpret_cast<int*>(&r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(DtwArgs) / 4); ++k) dst[k] = __builtin_amdgcn_readfirstlane(src[k]);
  return r;
}
}  // namespace

namespace {
__device__ __forceinline__ double shr1(double v, double lane0) {
  const int2 a = __builtin_bit_cast(int2, v), o = __builtin_bit_cast(int2, lane0);
  const int lo = __builtin_amdgcn_update_dpp(o.x, a.x, 0x138, 0xf, 0xf, false);   // wave_shr:1
  const int hi = __builtin_amdgcn_update_dpp(o.y, a.y, 0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double shl1(double v) {      // lane l <- lane l+1 (lane 63 <- +Inf)
  const int2 a = __builtin_bit_cast(int2, v);
  const int lo = __builtin_amdgcn_update_dpp(0, a.x, 0x130, 0xf, 0xf, false);   // wave_shl:1
  const int hi = __builtin_amdgcn_update_dpp(0x7FF00000, a.y, 0x130, 0xf, 0xf, false);
  return __builtin_bit_cast(double, make_int2(lo, hi));
}
// v_min_f64 without the canonicalising v_max_f64 x, x the compiler adds around fmin in IEEE mode
// (the operands here are never signalling NaNs: FAST inputs are finite)
__device__ __forceinline__ double vmin_f64(double x, double y) {
  double r;
  asm volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int2 a = __builtin_bit_cast(int2, v);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(a.x, l), __builtin_amdgcn_readlane(a.y, l)));
}
}  // namespace

// Block = 4 + DTW_NDW waves, all coupled through LDS counters (a wave reads data only after it
// has read the count that covers it; LDS requests of one wave complete in order, so data loads
// issued AFTER a counter load see everything the counter covers).  Wave order: sweep, NDW
// distance waves, feeder, code, edge -- a block's waves go to SIMDs in the cyclic order 0, 2, 1,
// 3 (MI355X_MICROARCH.md, LDS).  NDW = 4 (A/B against 3, 5, 6 and DG 4 in
// tools/scratch/ab_ndw.sh: C3 band 21.1 -> 20.3 ms, C5 +1 %; 5 or 6 waves need DG 4 to keep two
// blocks per CU and lose more to the shorter interleave).
//  sweep     the min-chain of every cell and the band's bottom edge.  Per step only DPP -> min
//            -> add is on the chain.  A single wave issues LDS and memory instructions slowly
//            (each moves its 64 lanes' data), so the sweep does few: per 8-step chunk 4 paired
//            C-ring writes, 10 reads for the NEXT chunk (its counters, distances and top-edge
//            values, issued while the current chunk runs) and one 8-value edge store.  It never
//            loads from global memory (on gfx9 a vmcnt wait would also drain its own stores).
//  feeder    reference rows into the LDS ring (16-row blocks, prefetched into registers and
//            written once every distance chunk that reads the overwritten rows is done).
//  edge      C[64b][j] polled from E with sc1 loads into two edge rings (slot j-1 for the
//            sweep's aligned pair reads, slot j for the code wave's).
//  code      the C store (8 B/cell, paired dwordx4) and findPreviousStep's 2-bit directions
//            (dtw.go:191-217) recomputed from the sweep's C values (an LDS ring of the last
//            DTW_OQ steps) into Dn, off the sweep's critical path.
//  distance  8-step chunks round-robin; the unfused Euclidean distance of every lane's cell into
//            an LDS distance ring, the chunk's 8 cells interleaved.
// The distance and C rings are [lane][step] with rows of DQ + 2 / OQ + 2 doubles (68 / 132 dwords,
// 4 mod 64: a lane's pair of steps is one 16-B access, and every 16-lane b128 read group and
// 8-lane b128 write group covers distinct banks).
#ifndef DTW_RROWS_CFG
#define DTW_RROWS_CFG 128
#endif
constexpr int DTW_RROWS = DTW_RROWS_CFG;   // reference rows in the LDS ring
constexpr int DTW_RBLK = 16;               // rows per ring refill
#ifndef DTW_DQ_CFG
#define DTW_DQ_CFG 32
#endif
constexpr int DTW_DQ = DTW_DQ_CFG;         // steps of distances held in LDS (a power of two), batched
#ifndef DTW_DQ_SINGLE_CFG
#define DTW_DQ_SINGLE_CFG 64
#endif
// ... and for the single-DTW instance (C3): 64 steps let the distance waves run further ahead of the
// sweep.  Same box, three rounds (profiles/r06ah_dtw_rings_ab.log): C3 band 14.9-15.2 against
// 15.7-16.1 ms; in the batched instance the larger LDS footprint costs C5 4 % (2,134-2,146 against
// 2,216-2,229 pairs/s), so it keeps 32.  The split confirmed on another box (r06ai_dtw_dq_single_ab.log):
// C3 band 14.9-15.1 against 15.6-16.3 ms, C5 unchanged.  68.5 KB of LDS, 104-108 VGPRs: still 2 per CU
constexpr int DTW_DQ_SINGLE = DTW_DQ_SINGLE_CFG;
#ifndef DTW_SWEEP_PRIO_CFG
#define DTW_SWEEP_PRIO_CFG 3
#endif
constexpr int DTW_SWEEP_PRIO = DTW_SWEEP_PRIO_CFG;  // s_setprio of the sweep (the min-chain is the critical path)
#ifndef DTW_CODE_PRIO
#define DTW_CODE_PRIO 2           // s_setprio of the code wave (A/B: 0, 1, 2, 3)
#endif
#ifndef DTW_DIST_PRIO
#define DTW_DIST_PRIO 0           // s_setprio of the distance waves while they compute (A/B).  At 1,
                                  // C5 ran 1.3 % faster (profiles/r05q_dtw_prio_ab.log) but a
                                  // process's first C5 call lost DTWs to the 1 s bound again, in round
                                  // 4 (profiles/r04pq_ab.log) and round 5 (r05s_c5_workers_ab.log),
                                  // even with every wait at 0: busy distance waves of one band block
                                  // outrank the OTHER block's edge poller on a shared SIMD (DESIGN.md,
                                  // Kernel 6)
#endif
#ifndef DTW_AUX_PRIO
#define DTW_AUX_PRIO 0            // s_setprio of the ring feeder (A/B)
#endif
#ifndef DTW_EDGE_PRIO
#define DTW_EDGE_PRIO 3           // s_setprio of the edge poller (round 6): the top level, the same as
                                  // the sweep that produces the edge it polls.  The edge poll is the
                                  // kernel's only wait on ANOTHER block; at the top level no wave of any
                                  // block outranks it (Kernel 6, "Liveness by construction")
#endif
#ifndef DTW_OQ_CFG
#define DTW_OQ_CFG 32
#endif
constexpr int DTW_OQ = DTW_OQ_CFG;         // steps of C values held in LDS for the code wave
constexpr int DTW_DROW = DTW_DQ + 2;       // doubles per lane row of the transposed rings: a
constexpr int DTW_OROW = DTW_OQ + 2;       // multiple of 4 dwords plus 4 (mod 64 dwords)
constexpr int DTW_EQ = 128;       // edge values in the LDS rings
constexpr int DTW_EAHEAD = 64;    // the feeder fetches edge columns up to min(prog, cprog) + EAHEAD
#ifndef DTW_NDW
#define DTW_NDW 4                 // distance waves per block (A/B: tools/scratch/ab_ndw.sh)
#endif
#ifndef DTW_DG
#define DTW_DG 8                  // distance cells interleaved per pass (a divisor of DTW_ECH)
#endif
#ifndef DTW_BATCH_MINWAVES
#define DTW_BATCH_MINWAVES 6      // the batched (C5) instance: 80 VGPRs instead of 98 (launch_dtw_batch)
#endif
#ifndef DTW_BATCH_PAD
#define DTW_BATCH_PAD 2560        // dynamic LDS bytes per batched band block: unused, caps it at 2 per CU
#endif
#ifndef DTW_MINWAVES
#define DTW_MINWAVES 4            // waves per SIMD the register budget must allow
#endif
constexpr int DTW_WAVES = 4 + DTW_NDW;
// wave roles: 0 sweep, 1..NDW distance, then the ring feeder, the code wave and the edge poller
// DTW_SWAP_FEEDER: the feeder takes wave 4 (the sweep's SIMD under the 0,2,1,3 order) and the
// last distance wave moves to the feeder's slot (NDW >= 4 only; A/B knob)
#ifndef DTW_SWAP_FEEDER
#define DTW_SWAP_FEEDER 0
#endif
constexpr bool DTW_SWAP = DTW_SWAP_FEEDER && DTW_NDW >= 4;
constexpr int DTW_FEEDER_WAVE = DTW_SWAP ? 4 : DTW_NDW + 1;
constexpr int DTW_CODE_WAVE = DTW_NDW + 2;
constexpr int DTW_EDGE_WAVE = DTW_NDW + 3;
// distance-wave index of wave `wave` (1..NDW+1 minus the feeder)
__device__ __forceinline__ int dtw_dist_index(int wave) { return DTW_SWAP && wave == DTW_NDW + 1 ? 3 : wave - 1; }
static_assert(DTW_NDW >= 1 && DTW_NDW <= 7, "distance counters live in ctr[0..6]");
// counter slots: NDW <= 3 keeps {dchunk[0..2], efill} in one 16-B quad (one LDS read for the
// sweep); more distance waves use ctr[0..NDW-1] + efill in ctr[7] (two quads)
constexpr int DTW_CTR_EFILL = DTW_NDW <= 3 ? 3 : 7;
constexpr int DTW_CTR_CPROG = DTW_NDW <= 3 ? 4 : 8;
constexpr int DTW_CTR_PROG = DTW_NDW <= 3 ? 5 : 9;
constexpr int DTW_CTR_RDY = DTW_NDW <= 3 ? 6 : 10;
constexpr int DTW_CTR_ABORT = 12;   // set by the first wave of the block that gives up
constexpr int DTW_CTR_TICKET = 13;  // the block's ticket (diagnostics)
// Ring row stride in doubles.  A distance wave's lane l reads row t-l, so consecutive lanes sit
// one stride apart; 12-dim rows padded to 14 doubles (112 B, 28 dwords: 16 distinct 4-dword bank
// quads in every 16-lane group of ds_read_b128) make those reads conflict-free (96 B is 2-way).
template <int D>
constexpr int dtw_ring_stride() { return D == 12 ? 14 : (D > 0 ? D : 1); }
// The first DTW_ECH ring rows are mirrored after the ring, so one chunk's DTW_ECH consecutive rows
// never wrap and a lane addresses them as one base plus immediate offsets.
constexpr int DTW_RMIR = DTW_ECH;

// The Dn allocation (dtw_dn_bytes) holds, after the nb * SW * 64 direction words, the band exit
// map Xm[nb][nr64] and its segment boundaries Xr[nb][nseg][64] (int32, dtw_exit_map_kernel), and
// the band walk's meta words: ent[nb] (the column at which the path crosses the band's last valid
// row), cnt[nb] (its moves inside the band) and off[nb] (moves of the later bands: where its
// moves start in the walk's order).
constexpr int DTW_XSEG = 1024;    // columns per exit-map segment (a multiple of 64)
__host__ __device__ __forceinline__ int64_t dtw_nr64(int64_t nr) { return (nr + 63) & ~(int64_t)63; }
__host__ __device__ __forceinline__ int64_t dtw_nseg(int64_t nr) { return (nr + DTW_XSEG - 1) / DTW_XSEG; }
__device__ __forceinline__ int32_t* dtw_xmap(uint32_t* Dn, int64_t nb, int64_t SW) {
  return reinterpret_cast<int32_t*>(Dn + ((nb * SW) << 6));
}
__device__ __forceinline__ int32_t* dtw_xbound(uint32_t* Dn, int64_t nb, int64_t SW, int64_t nr) {
  return dtw_xmap(Dn, nb, SW) + nb * dtw_nr64(nr);
}
__device__ __forceinline__ int32_t* dtw_walk_meta(uint32_t* Dn, int64_t nb, int64_t SW, int64_t nr) {
  return dtw_xbound(Dn, nb, SW, nr) + nb * dtw_nseg(nr) * 64;
}

// C[i][j] of band-step (b, s), lane l in the paired layout Cn[b][s/2][l][s%2]
__device__ __forceinline__ int64_t dtw_cn_off(int64_t b, int64_t S2, int64_t s, int64_t l) {
  return ((b * S2 + (s >> 1)) << 7) + 2 * l + (s & 1);
}

// A wait of the band kernel gave up (called by the whole wave, uniformly): raise the block's abort
// word and the DTW's error bit for this role, and, if this is the DTW's first such wave, write its
// diagnostic record (layout at DtwArgs::diag).  The record re-reads the band above's edge word at
// the first column this band lacks in four ways -- sc1 load, sc1 load after an agent acquire,
// system-scope load, atomic fetch_or(0) at agent and system scope -- so a value that never left the
// producer can be told apart from one the consumer's caches did not show, and scans that edge row
// for the first column still holding the sentinel (how far the producer got).
__device__ __attribute__((noinline)) void dtw_stall(
    int32_t* sync, uint64_t* diag, int role, int64_t b, int* ctr,
                                                     const uint64_t* Ein, int64_t nr, uint32_t polls, uint64_t t0) {
  const int lane = threadIdx.x & 63;
  const uint64_t now = __builtin_amdgcn_s_memrealtime();
  const int prog = __hip_atomic_load(&ctr[DTW_CTR_PROG], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int cprog = __hip_atomic_load(&ctr[DTW_CTR_CPROG], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int efill = __hip_atomic_load(&ctr[DTW_CTR_EFILL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int rdy = __hip_atomic_load(&ctr[DTW_CTR_RDY], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const int ticket = __hip_atomic_load(&ctr[DTW_CTR_TICKET], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  uint64_t dch = 0;
#pragma unroll
  for (int w = 0; w < 4 && w < DTW_NDW; ++w)
    dch |= (uint64_t)(uint16_t)__hip_atomic_load(&ctr[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) << (16 * w);
  int claimed = 0;
  if (lane == 0) {
    __hip_atomic_store(&ctr[DTW_CTR_ABORT], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or((dtw_gi32*)&sync[1], 1 << (role - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (diag) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&diag[15]), 1ull);
      const uint64_t hdr = (1ull << 63) | ((uint64_t)role << 56) | ((uint64_t)(ticket & 0xFFFFFF) << 32) |
                           (uint64_t)(uint32_t)b;
      claimed = atomicCAS(reinterpret_cast<unsigned long long*>(&diag[0]), 0ull, (unsigned long long)hdr) == 0;
    }
  }
  claimed = __builtin_amdgcn_readfirstlane(claimed);
  if (!claimed) return;
  const int64_t lo = prog < cprog ? prog : cprog;
  const int64_t want = lo + DTW_EAHEAD < nr ? lo + DTW_EAHEAD : nr;
  uint64_t e[5] = {0, 0, 0, 0, 0};
  int64_t first = -1;
  if (Ein) {
    uint64_t* E = const_cast<uint64_t*>(Ein);
    const int64_t col = efill + 1 <= nr ? efill + 1 : nr;
    if (lane == 0) e[0] = g_load_agent(E + col);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (lane == 0) {
      e[1] = g_load_agent(E + col);
      e[2] = g_load_system(E + col);
      e[3] = __hip_atomic_fetch_or((dtw_gu64*)(E + col), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      e[4] = __hip_atomic_fetch_or((dtw_gu64*)(E + col), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    for (int64_t c0 = 1; c0 <= nr; c0 += 64) {
      const int64_t j = c0 + lane;
      const uint64_t v = j <= nr ? g_load_agent(E + j) : 0ull;
      const uint64_t m = __builtin_amdgcn_ballot_w64(j <= nr && v == DTW_SENT);
      if (m) { first = c0 + (int64_t)__builtin_ctzll(m); break; }
    }
  }
  if (lane == 0) {
    uint64_t* d = diag;
    d[1] = (uint32_t)prog | ((uint64_t)(uint32_t)cprog << 32);
    d[2] = (uint32_t)efill | ((uint64_t)(uint32_t)rdy << 32);
    d[3] = dch;
    d[4] = (uint32_t)want | ((uint64_t)(uint32_t)nr << 32);
    for (int k = 0; k < 5; ++k) d[5 + k] = e[k];
    d[10] = (uint64_t)first;
    // (a wait of another wave of the block, reported here by the edge poller: the bound itself)
    d[11] = ((t0 ? now - t0 : DTW_STALL_TICKS) & 0xFFFFFFFFFFull) | ((uint64_t)(polls >> 10) << 40);
    const uint64_t hw = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const uint64_t xcc = (uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20); // HW_REG_XCC_ID
    d[12] = (xcc & 0xFF) | (hw << 32);
  }
}

// A bounded LDS wait (SONAR_SPIN_UNTIL) checks the block's abort word and the clock every
// DTW_SPIN_CHECK polls (~10 ms); after DTW_STALL_TICKS without progress (and >= 16 checks, so a wave
// that was switched out does not time out on wall time alone) it gives up: it records its role in
// the block's LDS stall word, raises the abort word and its bit of the DTW's error word, and
// stops waiting: it sets the wave's dead_ flag, which ends this and every later wait at once, so the
// wave runs out its loop on stale LDS data (in-bounds: every index comes from loop counters) and
// its DTW is reported failed.  Neither a call nor a `return` inside the wait loops: a call costs the
// sweep's, code wave's and distance waves' loops their register allocation (C5 -10 %), and a
// `return` is a divergent exit from those loops (the abort word is an LDS load), which turns their
// uniform loop state into per-lane values (sweep 87 -> 128 VGPRs, C5 -15 %).  The edge poller (or
// the ring feeder), whose loop already holds the call, sees the abort word and writes the DTW's
// diagnostic record for the stalled role (dtw_stall).
constexpr uint32_t DTW_SPIN_CHECK = 1u << 16;
constexpr int DTW_CTR_STALLED = 14;   // role of the block's first wave that timed out (0: none)
__device__ __forceinline__ void dtw_local_stall(int role, int32_t* sync, int* ctr, int lane) {
  if (lane == 0) {
    int expect = 0;
    __hip_atomic_compare_exchange_strong(&ctr[DTW_CTR_STALLED], &expect, role, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&ctr[DTW_CTR_ABORT], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or((__attribute__((address_space(1))) int32_t*)&sync[1], 1 << (role - 1), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int D, bool FAST, bool BANDED, bool BATCH = false>
// (2 blocks of 8 waves per CU: at least 4 waves per SIMD, <= 128 VGPRs)
__global__ __launch_bounds__(64 * DTW_WAVES, BATCH ? DTW_BATCH_MINWAVES : DTW_MINWAVES)
void dtw_band_kernel(DtwArgs a_in, DtwBatch bt) {
  constexpr int DR = D > 0 ? D : 1;
  constexpr int DS = dtw_ring_stride<D>();
  constexpr int FEEDER_WAVE = DTW_FEEDER_WAVE;
  constexpr int CODE_WAVE = DTW_CODE_WAVE;
  constexpr int EDGE_WAVE = DTW_EDGE_WAVE;
  __shared__ __attribute__((aligned(16))) double ring[(DTW_RROWS + DTW_RMIR) * DS];
  constexpr int DQ = BATCH ? DTW_DQ : DTW_DQ_SINGLE;
  __shared__ __attribute__((aligned(16))) double dring[64][DQ + 2];     // distance of step t at [l][t % DQ]
  __shared__ __attribute__((aligned(16))) double oring[64][DTW_OROW];   // C of step t at [l][t % OQ]
  __shared__ __attribute__((aligned(16))) double eqa[DTW_EQ];           // C[64b][c] at slot c - 1
  __shared__ __attribute__((aligned(16))) double eqb[DTW_EQ];           // C[64b][c] at slot c
  // dchunk[w] (per distance wave: 1 + its last finished chunk) in ctr[0..NDW-1], then efill (edge
  // columns in the rings), cprog (code steps done), prog (sweep steps done), rdy (highest ring
  // block ready) at the DTW_CTR_* slots
  __shared__ __attribute__((aligned(16))) int ctr[16];
  __shared__ int64_t shb;
  __shared__ int shk;
#define SONAR_LDS_LD(x) __hip_atomic_load(&(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define SONAR_LDS_ST(x, v) __hip_atomic_store(&(x), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
  int& efill = ctr[DTW_CTR_EFILL];
  int& cprog = ctr[DTW_CTR_CPROG];
  int& prog = ctr[DTW_CTR_PROG];
  int& rdy = ctr[DTW_CTR_RDY];
  // (wave is uniform: readfirstlane keeps it, and every address derived from it, in SGPRs)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double inf = __builtin_inf();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 16; ++k) ctr[k] = 0;
    if constexpr (BATCH) {
      const int64_t t = atomicAdd(bt.ticket, 1);
      ctr[DTW_CTR_TICKET] = (int)t;
      if (bt.map) {
        if (t < bt.start[bt.n]) {
          const int2 pb = bt.map[t];
          shk = pb.x;
          shb = pb.y;
        } else {
          shk = 0;
          shb = INT64_MAX;                            // past the last ticket: the block exits
        }
      } else {
        int lo = 0, hi = bt.n;                        // start[lo] <= t < start[lo + 1]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (bt.start[mid] <= t) lo = mid; else hi = mid;
        }
        shk = lo;
        shb = t - bt.start[lo];                       // >= nb past the last DTW: the block exits
      }
    } else {
      shb = atomicAdd(&a_in.sync[0], 1);
      ctr[DTW_CTR_TICKET] = (int)shb;
    }
    rdy = -1;
  }
  if (threadIdx.x < 64) {        // steps -1 and -2: C[i][j] for j <= 0 is +Inf (column 0) / unset
    oring[lane][DTW_OQ - 1] = inf;
    oring[lane][DTW_OQ - 2] = inf;
  }
  __syncthreads();
  const int64_t b = shb;
  const DtwArgs a = BATCH ? load_args_uniform(bt.args + __builtin_amdgcn_readfirstlane(shk)) : a_in;
  if (b >= a.nb) return;
  const int64_t nq = a.nq, nr = a.nr, S = a.S, S2 = (a.S + 1) >> 1;
  const int dim = D > 0 ? D : a.dim;
  constexpr uint64_t INF_BITS = 0x7FF0000000000000ull;
  const uint64_t* Ein = b > 0 ? a.E + (b - 1) * (nr + 1) : nullptr;       // C[64b][j] at index j
  const int64_t nblk = (nr + DTW_RBLK - 1) / DTW_RBLK;
  const int64_t i = 64 * b + 1 + lane;
  const bool row_ok = i <= nq;
  const int64_t qrow = row_ok ? i - 1 : 0;
  uint64_t spins_total = 0;
  uint32_t dead_ = 0;
  // spin (LDS only) until `cond` holds; bounded, see DTW_SPIN_CHECK.  A wave that gives up, or sees
  // the block's abort word, sets dead_ and runs out its loop without waiting again.  `prio` is the
  // wave's working s_setprio level (a constant): while it spins the wave drops to 0 and takes it back
  // once `cond` holds, so a waiting wave never outranks the producer it waits for (DESIGN.md,
  // Kernel 6, "Issue priorities and liveness").
#define SONAR_SPIN_UNTIL(role, prio, cond)                                            \
  do {                                                                                \
    if (!dead_ && !(cond)) {                                                          \
      if ((prio) > 0) __builtin_amdgcn_s_setprio(0);                                  \
      const uint64_t tr0_ = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;           \
      uint64_t w0_ = 0;                                                               \
      uint32_t sp_ = 0, rounds_ = 0;                                                  \
      while (!(cond)) {                                                               \
        __builtin_amdgcn_s_sleep(DTW_SPIN_SLEEP);                                     \
        if (++sp_ > DTW_SPIN_CHECK) {                                                 \
          sp_ = 0;                                                                    \
          if (SONAR_LDS_LD(ctr[DTW_CTR_ABORT])) { dead_ = 1; break; }                 \
          const uint64_t now_ = __builtin_amdgcn_s_memrealtime();                     \
          if (!w0_) w0_ = now_;                                                       \
          else if (++rounds_ >= 16 && now_ - w0_ > DTW_STALL_TICKS) {                 \
            dtw_local_stall((role), a.sync, ctr, lane);                               \
            dead_ = 1; break;                                                         \
          }                                                                           \
        }                                                                             \
      }                                                                               \
      if (a.trace) spins_total += __builtin_amdgcn_s_memrealtime() - tr0_;            \
      if ((prio) > 0) __builtin_amdgcn_s_setprio(prio);                               \
    }                                                                                 \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");                            \
  } while (0)

  if (wave == FEEDER_WAVE || wave == EDGE_WAVE) {
    // ------------------------------------------------ ring feeder / edge poller
    if (wave == FEEDER_WAVE) {
      if (DTW_AUX_PRIO) __builtin_amdgcn_s_setprio(DTW_AUX_PRIO);
    } else {
      if (DTW_EDGE_PRIO) __builtin_amdgcn_s_setprio(DTW_EDGE_PRIO);
    }
    // two waves, so the edge poll's global-load latency never delays a ring refill
    const bool do_ring = wave == FEEDER_WAVE;
    int64_t nextblk = 0, have = 0;
    // polls without work since the last one that found work, the realtime of the 64th of them,
    // and the edge poller's refresh state
    uint32_t idle = 0;
    uint64_t t_idle = 0, t_fence = 0;
    bool fenced = false;
    const int64_t ecols = Ein ? nr : 0;
    // block nextblk's rows are loaded into registers as soon as the previous block is written
    // (lanes < RBLK, one row each), so the global-load latency is off the distance waves' path
    double pv[DR];
    auto prefetch = [&](int64_t blk) {
      const int64_t row = DTW_RBLK * blk + lane;
#pragma unroll
      for (int k = 0; k < DR; ++k) pv[k] = (lane < DTW_RBLK && row < nr) ? DTW_GLOBAL(a.r)[row * D + k] : 0.0;
    };
    if constexpr (D > 0) prefetch(0);
    while (true) {
      const int64_t p = SONAR_LDS_LD(prog), cp = SONAR_LDS_LD(cprog);
      bool work = false, wait_edge = false;
      if (D > 0 && do_ring) {
        // block m overwrites rows up to r = RBLK*m - RROWS + RBLK - 1, which distance chunks up to
        // index (r + 63) / ECH read (chunk t0 reads rows t0-63 .. t0+7): all of them are done once
        // every distance wave's counter is above that index (wave w has finished every chunk
        // c = w mod NDW below ctr[w])
        int mind = SONAR_LDS_LD(ctr[0]);
#pragma unroll
        for (int w = 1; w < DTW_NDW; ++w) {
          const int x = SONAR_LDS_LD(ctr[w]);
          mind = x < mind ? x : mind;
        }
        if (nextblk < nblk &&
            (nextblk < DTW_RROWS / DTW_RBLK ||
             (int64_t)mind > (DTW_RBLK * nextblk - DTW_RROWS + DTW_RBLK - 1 + 63) / DTW_ECH)) {
          if (lane < DTW_RBLK) {
            const int64_t row = DTW_RBLK * nextblk + lane;
            const int slot = (int)(row & (DTW_RROWS - 1));
            double* dst = ring + slot * DS;
            double* mir = ring + (DTW_RROWS + slot) * DS;
#pragma unroll
            for (int k = 0; k < DR; ++k) dst[k] = pv[k];
            if (slot < DTW_RMIR) {
#pragma unroll
              for (int k = 0; k < DR; ++k) mir[k] = pv[k];
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) SONAR_LDS_ST(rdy, (int)nextblk);
          ++nextblk;
          if (nextblk < nblk) prefetch(nextblk);
          work = true;
        }
      }
      if (!do_ring && have < ecols) {
        // the slots of column c are rewritten for column c + EQ: the sweep reads columns
        // <= prog + 16, the code wave columns <= cprog + 8
        const int64_t lo = p < cp ? p : cp;
        const int64_t want = lo + DTW_EAHEAD < ecols ? lo + DTW_EAHEAD : ecols;
        if (have < want) {
          wait_edge = true;
          const int64_t jj = have + 1 + lane;
          uint64_t v = INF_BITS;
          if (jj <= want) v = g_load_agent(Ein + jj);
          const uint64_t bad = __builtin_amdgcn_ballot_w64(jj <= want && v == DTW_SENT);
          const int64_t lim = want - have < 64 ? want - have : 64;
          const int64_t got = bad ? (int64_t)__builtin_ctzll(bad) : lim;   // contiguous ready prefix
          if (lane < got) {
            eqa[(jj - 1) & (DTW_EQ - 1)] = __builtin_bit_cast(double, v);
            eqb[jj & (DTW_EQ - 1)] = __builtin_bit_cast(double, v);
          }
          if (got > 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            have += got;
            if (lane == 0) SONAR_LDS_ST(efill, (int)have);
            work = true;
          }
        }
      }
      if (do_ring ? (D == 0 || nextblk >= nblk) : have >= ecols) break;
      if (work) {
        // diag[14]: the first poll after a refresh found new values
        if (fenced && lane == 0 && a.diag) g_add_agent(&a.diag[14], 1ull);
        fenced = false;
        idle = 0;
      } else {
        fenced = false;
        __builtin_amdgcn_s_sleep(1);   // (the poller at 2 or 4: no different, profiles/r06z_*)
        if ((++idle & 63) == 0) {
          if (SONAR_LDS_LD(ctr[DTW_CTR_ABORT])) {
            // a wave of this block timed out (SONAR_SPIN_UNTIL): write its diagnostic record here
            const int st = SONAR_LDS_LD(ctr[DTW_CTR_STALLED]);
            if (st) dtw_stall(a.sync, a.diag, st, b, ctr, Ein, nr, 0, 0);
            return;
          }
          const uint64_t now = __builtin_amdgcn_s_memrealtime();
          if (idle == 64) t_idle = now;
          if (wait_edge) {
            // another band of this DTW gave up: its edge (and so this band's) will never come
            if (g_load_agent(&a.sync[1])) {
              if (lane == 0) SONAR_LDS_ST(ctr[DTW_CTR_ABORT], 1);
              return;
            }
            if (now - t_idle > DTW_REFRESH_TICKS && now - t_fence > DTW_REFRESH_TICKS) {
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
              t_fence = now;
              fenced = true;
              if (lane == 0 && a.diag) g_add_agent(&a.diag[13], 1ull);
            }
          }
          if (idle >= DTW_STALL_POLLS && now - t_idle > DTW_STALL_TICKS) {
            dtw_stall(a.sync, a.diag, do_ring ? DTW_ROLE_FEEDER : DTW_ROLE_EDGE, b, ctr, Ein, nr, idle, t_idle);
            return;
          }
        }
      }
    }
    return;
  }

  if (wave == CODE_WAVE) {
    // --------------------------------------------------------------- code wave
    // above the distance waves in issue arbitration (below the sweep's 3): the sweep spins on
    // the code wave's progress once the C ring is full, and the four distance waves, which run
    // ahead of the sweep, otherwise take the code wave's issue slots.  Trace of a C5 call
    // (profiles/r04j_c5_band_trace.txt): half of the sweep's spins were on the code wave.
    // Measured (profiles/r04k_ab.log): C5 1,862-1,880 -> 2,087-2,116 pairs/s.
    __builtin_amdgcn_s_setprio(DTW_CODE_PRIO);
    // step s, lane l: up = C of lane l-1 at step s-1, left = own at s-1, diag = lane l-1 at s-2;
    // lane 0's left neighbour is the band's top edge: C[64b][s+1] / C[64b][s]
    __attribute__((address_space(1))) uint32_t* Db = DTW_GLOBAL(a.Dn) + ((b * a.SW) << 6) + lane;
    __attribute__((address_space(1))) double* Cb = DTW_GLOBAL(a.Cn) + dtw_cn_off(b, S2, 0, lane);
    uint32_t dacc = 0;
    double ckv = 0.0;                                  // the lane's C at the latest multiple-of-64 column
    for (int64_t s0 = 0; s0 < S; s0 += DTW_ECH) {
      const int need = (int)(s0 + DTW_ECH < S ? s0 + DTW_ECH : S);
      SONAR_SPIN_UNTIL(DTW_ROLE_CODE, DTW_CODE_PRIO, SONAR_LDS_LD(prog) >= need);
      // steps s0-2 .. s0+7 as 5 pairs (the last value unused); lane 0's neighbour pairs are the
      // edge columns (t+2, t+3) at eqb slots (t+2, t+3) (per-lane addresses, no divergence)
      double cv[DTW_ECH + 2], nv[DTW_ECH + 2];
#pragma unroll
      for (int k = 0; k < DTW_ECH / 2 + 1; ++k) {
        const int64_t t = s0 - 2 + 2 * k;
        const double2 o = *reinterpret_cast<const double2*>(&oring[lane][t & (DTW_OQ - 1)]);
        const double2 n = lane > 0 ? *reinterpret_cast<const double2*>(&oring[lane - 1][t & (DTW_OQ - 1)])
                                   : *reinterpret_cast<const double2*>(&eqb[(t + 2) & (DTW_EQ - 1)]);
        cv[2 * k] = o.x; cv[2 * k + 1] = o.y;
        nv[2 * k] = n.x; nv[2 * k + 1] = n.y;
      }
      if (lane == 0) {
#pragma unroll
        for (int u = 0; u < DTW_ECH + 1; ++u) {
          const int64_t c = s0 + u;                      // nv[u] = C[64b][c]
          nv[u] = (c == 0 || !Ein || c > nr) ? ((c == 0 && b == 0) ? 0.0 : inf) : nv[u];
        }
      }
#pragma unroll
      for (int u = 0; u < DTW_ECH; ++u) {
        const double up = nv[u + 1], left = cv[u + 1], dg = nv[u];
        uint32_t code;
        if constexpr (FAST) {
          const double best = vmin_f64(up, vmin_f64(left, dg));
          code = best == up ? 0u : (best == left ? 1u : 2u);
        } else {
          double best = up;
          code = 0;
          if (left < best) { code = 1; best = left; }
          if (dg < best) code = 2;
        }
        dacc |= code << (2 * ((s0 & 8) + u));
      }
      // the chunk's C values: cv[2 + u] = step s0 + u, stored as pairs (Cn[b][s/2][l][s%2])
      if (a.Cn) {
#pragma unroll
        for (int k = 0; k < DTW_ECH / 2; ++k)
          if (s0 + 2 * k < S)
            *(__attribute__((address_space(1))) dtw_d2*)(Cb + ((s0 + 2 * k) << 6)) = dtw_d2{cv[2 + 2 * k], cv[3 + 2 * k]};
      } else {
        // checkpoint columns only.  Lane l meets column J = 64m at step J + l - 1, so every lane
        // has C[i][J] once the chunk holding step J + 62 is done (s0 % 64 == 56, J = s0 - 56):
        // one coalesced 512-B store per 64 steps.  In that chunk lanes 57-63 take their value of
        // column J and lane 0 already its value of column J + 64.
        const int u = (int)((lane - 1 - s0) & 63);      // the chunk step at which the lane's column is 64m
        // (one LDS read of the C ring, still holding the chunk, instead of a select over cv[])
        const double cap = u < DTW_ECH ? oring[lane][(s0 + u) & (DTW_OQ - 1)] : ckv;
        const int64_t J = s0 - 56;
        if ((s0 & 63) == 56 && J >= 64 && J <= nr)
          DTW_GLOBAL(a.CK)[((b * (nr >> 6) + (J >> 6) - 1) << 6) + lane] = (u < DTW_ECH && lane != 0) ? cap : ckv;
        ckv = cap;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) SONAR_LDS_ST(cprog, need);
      if ((s0 & 8) || s0 + DTW_ECH >= S) {             // steps 16w .. 16w+15 complete (or the last one)
        Db[(int64_t)(s0 >> 4) << 6] = dacc;
        dacc = 0;
      }
    }
    if (a.trace && lane == 0) DTW_GLOBAL(a.trace)[8 * b + 7] = spins_total;   // code wave's waits
    return;
  }

  double qv[DR];
  if constexpr (D > 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) qv[k] = DTW_GLOBAL(a.q)[qrow * D + k];
  }
  // local distance of the lane's cell at step t for a runtime dimension (D == 0), from global
  // memory (EuclideanDistanceFunc order, unfused)
  auto dist_rt = [&](int64_t t) -> double {
    double sum = 0.0;
    const int64_t jj = t - lane + 1;
    if (row_ok && jj >= 1 && jj <= nr) {
      const double* qa = a.q + qrow * dim;
      const double* rb = a.r + (jj - 1) * dim;
      for (int k = 0; k < dim; ++k) {
        const double df = qa[k] - rb[k];
        sum = sum + df * df;
      }
    }
    return sqrt(sum);
  };

  if (wave >= 1) {   // (every other role returned above)
    // ---------------------------------------------------------- distance waves
    if (DTW_DIST_PRIO) __builtin_amdgcn_s_setprio(DTW_DIST_PRIO);
    const int w = dtw_dist_index(wave);
    for (int64_t c = w; DTW_ECH * c < S; c += DTW_NDW) {
      const int64_t t0 = DTW_ECH * c;
      // ring slots of steps t0..t0+7 were last read by the sweep for steps t0-DQ..t0-DQ+7
      SONAR_SPIN_UNTIL(DTW_ROLE_DIST, DTW_DIST_PRIO, SONAR_LDS_LD(prog) >= t0 + DTW_ECH - DQ);
      double dv[DTW_ECH];
      if constexpr (D > 0) {
        const int64_t need = (t0 + DTW_ECH - 1) / DTW_RBLK;             // rows up to t0+7
        const int64_t needc = need < nblk - 1 ? need : nblk - 1;
        SONAR_SPIN_UNTIL(DTW_ROLE_DIST, DTW_DIST_PRIO, SONAR_LDS_LD(rdy) >= needc);
        // rows t0-l .. t0-l+7 sit at consecutive slots (mirror), so one base + immediate offsets;
        // steps past S and rows outside [0, nr) give values the sweep never stores.  The chunk's
        // cells advance together, one dimension at a time: each sum is Go's sequential chain,
        // the chains interleave.
        const double* rw0 = ring + (int)((t0 - lane) & (DTW_RROWS - 1)) * DS;
#pragma unroll
        for (int g0 = 0; g0 < DTW_ECH; g0 += DTW_DG) {   // DTW_DG interleaved chains at a time
          double sum[DTW_DG];
          if constexpr (D % 2 == 0) {
#pragma unroll
            for (int k = 0; k < D; k += 2) {
              double2 rv[DTW_DG];
#pragma unroll
              for (int u = 0; u < DTW_DG; ++u) rv[u] = *reinterpret_cast<const double2*>(rw0 + (g0 + u) * DS + k);
#pragma unroll
              for (int u = 0; u < DTW_DG; ++u) {
                const double d0 = qv[k] - rv[u].x;
                sum[u] = k == 0 ? d0 * d0 : sum[u] + d0 * d0;   // 0.0 + x == x for x >= +0 or NaN
                const double d1 = qv[k + 1] - rv[u].y;
                sum[u] = sum[u] + d1 * d1;
              }
            }
          } else {
#pragma unroll
            for (int k = 0; k < D; ++k) {
#pragma unroll
              for (int u = 0; u < DTW_DG; ++u) {
                const double d0 = qv[k] - rw0[(g0 + u) * DS + k];
                sum[u] = k == 0 ? d0 * d0 : sum[u] + d0 * d0;
              }
            }
          }
          if constexpr (FAST) {
            // finite inputs: sums are finite and >= 0; the short sqrt when every lane's DG sums
            // are in its range (all but exact or near-exact zero distances), else sqrt()
            double mn = sum[0];
#pragma unroll
            for (int u = 1; u < DTW_DG; ++u) mn = vmin_f64(mn, sum[u]);
            if (__builtin_amdgcn_ballot_w64(!(mn >= DTW_SQRT_MIN)) == 0) {
#pragma unroll
              for (int u = 0; u < DTW_DG; ++u) dv[g0 + u] = sqrt_normal(sum[u]);
            } else {
#pragma unroll
              for (int u = 0; u < DTW_DG; ++u) dv[g0 + u] = sqrt(sum[u]);
            }
          } else {
#pragma unroll
            for (int u = 0; u < DTW_DG; ++u) dv[g0 + u] = sqrt(sum[u]);
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < DTW_ECH; ++u) dv[u] = dist_rt(t0 + u);
      }
      double* drow = &dring[lane][t0 & (DQ - 1)];
#pragma unroll
      for (int u = 0; u < DTW_ECH; u += 2)
        *reinterpret_cast<double2*>(drow + u) = make_double2(dv[u], dv[u + 1]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) SONAR_LDS_ST(ctr[w], (int)(c + 1));
    }
    if (a.trace && lane == 0 && w == 0) DTW_GLOBAL(a.trace)[8 * b + 6] = spins_total;   // distance wave 0's waits
    return;
  }

  // ---------------------------------------------------------------- sweep wave
  // the min-chain is the pipeline's critical path: it wins VALU arbitration over the distance
  // waves sharing its SIMD (MI355X_MICROARCH.md, "VALU issue is arbitrated ... by priority")
  __builtin_amdgcn_s_setprio(DTW_SWEEP_PRIO);
  const uint64_t t_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t t_first = 0;
  uint64_t* Eout = (b + 1 < a.nb) ? a.E + b * (nr + 1) : nullptr;         // C[64b+64][j]
  double out = inf;                                   // C[i][j-1]; C[i][0] = +Inf
  double up_prev = (lane == 0 && b == 0) ? 0.0 : inf; // C[i-1][j-1]; C[0][0] = 0
  const int64_t band = a.band;

  // chunk of steps [s0, s0+8) may start once its distances, its top-edge columns (through s0+8)
  // and the code wave's progress (C-ring slots reused after DTW_OQ steps) are there.  32-bit
  // compares: nq + nr < 2^31 is checked on the host.
  const int nr32 = (int)nr;
  // the counters the sweep reads: dchunk[0..NDW-1], efill, cprog (scalars, not an array, so
  // nothing lands in scratch)
  struct Ctrs { int d0, d1, d2, d3, d4, d5, d6, ef, cp; };
  auto ready = [&](int s0, Ctrs k) -> bool {
    const int c = s0 / DTW_ECH, w = c % DTW_NDW;
    int dchk = k.d0;
    if (DTW_NDW > 1 && w == 1) dchk = k.d1;
    if (DTW_NDW > 2 && w == 2) dchk = k.d2;
    if (DTW_NDW > 3 && w == 3) dchk = k.d3;
    if (DTW_NDW > 4 && w == 4) dchk = k.d4;
    if (DTW_NDW > 5 && w == 5) dchk = k.d5;
    if (DTW_NDW > 6 && w == 6) dchk = k.d6;
    const int neede = s0 + DTW_ECH < nr32 ? s0 + DTW_ECH : nr32;
    return dchk > c && (!Ein || k.ef >= neede) && k.cp >= s0 + DTW_ECH - DTW_OQ + 2;
  };
  // trace only: which producer a spin started on (1 distances, 2 the band above's edge, 3 the code
  // wave), and the spin ticks per cause (trace words 4 and 5; the rest of word 3's total is code)
  uint64_t spin_dist = 0, spin_edge = 0;
  auto spin_cause = [&](int s0, Ctrs k) -> int {
    const int c = s0 / DTW_ECH, w = c % DTW_NDW;
    int dchk = k.d0;
    if (DTW_NDW > 1 && w == 1) dchk = k.d1;
    if (DTW_NDW > 2 && w == 2) dchk = k.d2;
    if (DTW_NDW > 3 && w == 3) dchk = k.d3;
    if (DTW_NDW > 4 && w == 4) dchk = k.d4;
    if (DTW_NDW > 5 && w == 5) dchk = k.d5;
    if (DTW_NDW > 6 && w == 6) dchk = k.d6;
    if (dchk <= c) return 1;
    const int neede = s0 + DTW_ECH < nr32 ? s0 + DTW_ECH : nr32;
    if (Ein && k.ef < neede) return 2;
    return 3;
  };
  auto account = [&](int cause, uint64_t before) {
    if (cause == 1) spin_dist += spins_total - before;
    else if (cause == 2) spin_edge += spins_total - before;
  };
  // {dchunk, efill} as one (NDW <= 3) or two 16-B volatile LDS reads, cprog as one 4-B read
  typedef int ctr4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) volatile ctr4 lds_ctr4;   // LDS, not flat
  typedef __attribute__((address_space(3))) volatile int lds_int;
  auto load_ctr = [&]() -> Ctrs {
    Ctrs k;
    const ctr4 x = *(lds_ctr4*)(&ctr[0]);
    k.d0 = x.x; k.d1 = x.y; k.d2 = x.z; k.d3 = x.w;
    if constexpr (DTW_NDW > 3) {
      const ctr4 y = *(lds_ctr4*)(&ctr[4]);
      k.d4 = y.x; k.d5 = y.y; k.d6 = y.z; k.ef = y.w;
    } else {
      k.d4 = k.d5 = k.d6 = 0;
      k.ef = x.w;
    }
    k.cp = *(lds_int*)(&ctr[DTW_CTR_CPROG]);
    return k;
  };
  // raw loads only: the border selects come after the steps, so the loads' latency overlaps the
  // chunk instead of stalling its start.  Volatile like the counter loads: the compiler keeps them
  // behind the counter read that covers them (LDS returns one wave's requests in order), with no
  // wait between the two
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) volatile d2v lds_d2;
  auto load_chunk = [&](int64_t s0, double (&dc)[DTW_ECH], double (&ech)[DTW_ECH]) {
    const double* dr = &dring[lane][s0 & (DQ - 1)];
    const double* er = &eqa[s0 & (DTW_EQ - 1)];        // columns s0+1 .. s0+8
#pragma unroll
    for (int u = 0; u < DTW_ECH; u += 2) {
      const d2v d2 = *(lds_d2*)(dr + u);
      const d2v e2 = *(lds_d2*)(er + u);
      dc[u] = d2.x; dc[u + 1] = d2.y;
      ech[u] = e2.x; ech[u + 1] = e2.y;
    }
  };
  // columns s0+1.. >= 1; the values are uniform (broadcast reads), so they move to SGPRs
  auto fix_edges = [&](int64_t s0, double (&ech)[DTW_ECH]) {
#pragma unroll
    for (int u = 0; u < DTW_ECH; ++u) {
      const double e = (!Ein || s0 + 1 + u > nr) ? inf : ech[u];
      const int2 e2 = __builtin_bit_cast(int2, e);
      ech[u] = __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readfirstlane(e2.x),
                                                    __builtin_amdgcn_readfirstlane(e2.y)));
    }
  };
  // one sweep step: lane l relaxes C[i][s-l+1] with local distance d; l0up = C[64b][s+1] for lane
  // 0.  FULL: every lane's column is in [1, nr] (s in [63, nr-1]), so no per-lane predicate is
  // needed (rows past nq compute values nobody reads).
  auto step = [&](auto full_tag, int64_t s, double l0up, double d) {
    constexpr bool FULL = decltype(full_tag)::value;
    const double up = shr1(out, l0up);               // C[i-1][j]; lane 0 takes l0up
    const double left = out, dg = up_prev;
    double best;
    if constexpr (FAST) best = vmin_f64(up, vmin_f64(left, dg));   // all >= +0 or +Inf: order-free
    else best = go_min(go_min(up, left), dg);                      // math.Min: NaN / -Inf / -0 rules
    double v = d + best;
    const int64_t j = s - lane + 1;
    if constexpr (BANDED) {
      if (i - j > band || j - i > band) v = inf;      // outside the Sakoe-Chiba band: never filled
    }
    if constexpr (FULL) {
      out = v;
    } else {
      if (row_ok && j >= 1 && j <= nr) out = v;
    }
    up_prev = up;
  };
  // a pair of steps, then one 16-B C-ring write for both
  auto pair = [&](auto full_tag, int64_t s, double e0, double e1, double d0, double d1) {
    step(full_tag, s, e0, d0);
    const double o0 = out;
    step(full_tag, s + 1, e1, d1);
    *reinterpret_cast<double2*>(&oring[lane][s & (DTW_OQ - 1)]) = make_double2(o0, out);
  };

  double dc[DTW_ECH], ech[DTW_ECH];
  Ctrs kc = load_ctr();
  if (!ready(0, kc)) {
    const int cause = a.trace ? spin_cause(0, kc) : 0;
    const uint64_t before = spins_total;
    SONAR_SPIN_UNTIL(DTW_ROLE_SWEEP, DTW_SWEEP_PRIO, (kc = load_ctr(), ready(0, kc)));
    if (a.trace) account(cause, before);
  }
  if (a.trace) t_first = __builtin_amdgcn_s_memrealtime();
  load_chunk(0, dc, ech);
  fix_edges(0, ech);
  for (int64_t s0 = 0; s0 < S; s0 += DTW_ECH) {
    const int64_t s1 = s0 + DTW_ECH;
    if (b == a.dbg_stall && s0 >= 1024) return;        // fault injection (tests only)
    // next chunk: counters first, then its data (LDS completes a wave's requests in order)
    double dcn[DTW_ECH], echn[DTW_ECH];
    if (s1 < S) {
      kc = load_ctr();
      load_chunk(s1, dcn, echn);
    }
    if (s0 >= 63 && s1 <= nr) {
#pragma unroll
      for (int u = 0; u < DTW_ECH; u += 2) pair(std::true_type{}, s0 + u, ech[u], ech[u + 1], dc[u], dc[u + 1]);
    } else {
      // the last pair may run one step past S: its value lands in the pair's spare slot
#pragma unroll
      for (int u = 0; u < DTW_ECH; u += 2)
        if (s0 + u < S) pair(std::false_type{}, s0 + u, ech[u], ech[u + 1], dc[u], dc[u + 1]);
    }
    // the chunk's 8 edge values (lane 63's C) are read back before the release, so the one
    // LDS drain covers both the ring writes and this read
    const double ev = oring[63][(s0 + (lane & (DTW_ECH - 1))) & (DTW_OQ - 1)];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) SONAR_LDS_ST(prog, (int)(s1 < S ? s1 : S));   // steps < s1 are done
    if (Eout) {                                        // one sc1 store of the chunk's 8 edge values
      const int64_t je = s0 + lane - 62;               // lane 63's column at step s0 + lane
      if (lane < DTW_ECH && je >= 1 && je <= nr)
        g_store_agent(Eout + je, __builtin_bit_cast(uint64_t, ev));
    }
    if (s1 >= S) break;
    if (!ready((int)s1, kc)) {
      // the counters read at the chunk's start were stale.  When the band is gated by its
      // predecessor's edge (every chunk, once it has caught up) the data usually arrived during
      // the chunk, so the fresh counters and the chunk's data are read back to back (LDS
      // completes a wave's requests in order: data read after a count that covers it is valid),
      // one LDS round trip instead of two; only a still-missing producer spins.
      kc = load_ctr();
      load_chunk(s1, dcn, echn);
      if (!ready((int)s1, kc))
      {
        const int cause = a.trace ? spin_cause((int)s1, kc) : 0;
        const uint64_t before = spins_total;
        SONAR_SPIN_UNTIL(DTW_ROLE_SWEEP, DTW_SWEEP_PRIO, (kc = load_ctr(), ready((int)s1, kc)));
        if (a.trace) account(cause, before);
        load_chunk(s1, dcn, echn);
      }
    }
    fix_edges(s1, echn);
#pragma unroll
    for (int u = 0; u < DTW_ECH; ++u) { dc[u] = dcn[u]; ech[u] = echn[u]; }
  }
#undef SONAR_SPIN_UNTIL
#undef SONAR_LDS_LD
#undef SONAR_LDS_ST
  if (a.trace && lane == 0) {
    auto* tr = DTW_GLOBAL(a.trace);
    tr[8 * b + 0] = t_start;
    tr[8 * b + 1] = t_first;
    tr[8 * b + 2] = __builtin_amdgcn_s_memrealtime();
    // spins (10 ns ticks, low 24 bits), XCC id (bits 24-31) and HW_ID (high word: SIMD bits 4-5,
    // CU/SH/SE bits 8-15) of the sweep wave, so the probe can see which sweeps shared a SIMD
    const uint64_t hw = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const uint64_t xcc = (uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20); // HW_REG_XCC_ID
    tr[8 * b + 3] = (spins_total & 0xFFFFFFull) | ((xcc & 0xFF) << 24) | (hw << 32);
    tr[8 * b + 4] = spin_dist;                        // the sweep's spins on its distance waves
    tr[8 * b + 5] = spin_edge;                        // ... on the band above's edge (rest: the code wave)
  }
}

// Single wave: backtrack (dtw.go:165-188) over the 2-bit direction codes.  The walk is
// inherently sequential, so it only emits its own moves (2 bits per step, 16 per word, stored
// 64 words at a time); dtw_path_decode_kernel turns them into points and costs in parallel.
// Moves: 0 = vertical (i-1), 1 = horizontal (j-1), 2 = diagonal.
//
// Position inside band b: lane l = (i-1) % 64 and sweep step s = j-1+l; every move lowers s by
// 1 or 2 and l by 0 or 1, so inside a band the walk only goes down through the code words
// Dn[b][s/16][l].  The band's words sit in a 16-word register window (win[k] = word wlo+k, one
// lane per row), and each window slot has its own copy of the step loop (STEP_SLOT below), so
// the code of a step is one v_readlane of a FIXED register with the lane in an SGPR -- no
// dynamic register indexing -- followed by scalar bit-field work.  The next band's window is
// prefetched on band entry around the current column.
#define DTW_WIN 16
// The steps while the walk stays in its band, window slot K and the matrix interior (l >= 0,
// s >= 16 * w, j >= 1), for window slot kw (uniform).  A move: 0 up (l-1, s-1), 1 left (j-1, s-1),
// 2 diagonal (both, s-2), as arithmetic on the code: dl = 1 - (c & 1), dj = (c + 1) >> 1,
// dbp = 2 + (c & 2).  The words of the current lane (wc) and of the lane above (wu) are held in
// SGPRs; an up/diagonal move takes wu and fetches the next lane's word with a v_readlane whose
// result is needed only a move later, so the readlane latency is off the move-to-move chain.
// Uses win[], ll, bp, jj and emit() of the enclosing walk.
#define DTW_STEP_SLOT(K)                                                              \
    case K: {                                                                         \
      uint32_t wc = __builtin_amdgcn_readlane(win[K], ll);                            \
      uint32_t wu = __builtin_amdgcn_readlane(win[K], ll > 0 ? ll - 1 : 0);           \
      do {                                                                            \
        const uint32_t code = (wc >> bp) & 3u;                                        \
        emit(code);                                                                   \
        const int dl = 1 - (int)(code & 1u);                                          \
        ll -= dl;                                                                     \
        jj -= (int)((code + 1u) >> 1);                                                \
        bp -= 2 + (int)(code & 2u);                                                   \
        wc = dl ? wu : wc;                                                            \
        wu = __builtin_amdgcn_readlane(win[K], ll > 0 ? ll - 1 : 0);                  \
      } while ((ll | bp | (jj - 1)) >= 0);                                            \
      break;                                                                          \
    }
#define DTW_WALK_SLOTS(kw)                                                                                     \
  switch (kw) {                                                                                                \
    DTW_STEP_SLOT(0) DTW_STEP_SLOT(1) DTW_STEP_SLOT(2) DTW_STEP_SLOT(3) DTW_STEP_SLOT(4) DTW_STEP_SLOT(5)       \
    DTW_STEP_SLOT(6) DTW_STEP_SLOT(7) DTW_STEP_SLOT(8) DTW_STEP_SLOT(9) DTW_STEP_SLOT(10) DTW_STEP_SLOT(11)     \
    DTW_STEP_SLOT(12) DTW_STEP_SLOT(13) DTW_STEP_SLOT(14) DTW_STEP_SLOT(15)                                     \
    default: break;                                                                                            \
  }
__device__ __forceinline__ void dtw_walk_body(const uint32_t* Dn, int64_t nq, int64_t nr, int64_t SW,
                                              uint32_t* codes, int64_t* plen) {
  const int lane = threadIdx.x;
  uint32_t win[DTW_WIN], nxt[DTW_WIN];
#pragma unroll
  for (int k = 0; k < DTW_WIN; ++k) { win[k] = 0u; nxt[k] = 0u; }
  const int sw = (int)SW;
  int i = (int)nq, j = (int)nr, P = 0;
  int wb = -1, wlo = 0, pb = -1, plo = 0;
  uint32_t cacc = 0, vacc = 0;
  // the open word is built in an SGPR; a completed word moves into lane (word % 64) of vacc, and
  // the 64 words of vacc are stored once every 1,024 moves
  auto emit = [&](uint32_t code) {
    cacc |= code << (2 * (P & 15));
    ++P;
    if ((P & 15) == 0) {
      const int wi = (P >> 4) - 1;
      vacc = lane == (wi & 63) ? cacc : vacc;
      cacc = 0;
      if ((P & 1023) == 0) codes[wi - 63 + lane] = vacc;
    }
  };
  auto load_win = [&](uint32_t (&dst)[DTW_WIN], int bnd, int lo) {
    const uint32_t* src = Dn + (((int64_t)bnd * sw + lo) << 6) + lane;
#pragma unroll
    for (int k = 0; k < DTW_WIN; ++k) dst[k] = (lo + k < sw) ? src[k << 6] : 0u;
  };
  while (i > 0 && j > 0) {
    const int l = (i - 1) & 63, bnd = (i - 1) >> 6;
    const int s = j - 1 + l, w = s >> 4;
    if (bnd != wb || w < wlo) {
      if (bnd == pb && w >= plo && w < plo + DTW_WIN) {   // prefetched on entry to the band below
#pragma unroll
        for (int k = 0; k < DTW_WIN; ++k) win[k] = nxt[k];
        wlo = plo;
      } else {
        wlo = w - (DTW_WIN - 1) > 0 ? w - (DTW_WIN - 1) : 0;
        load_win(win, bnd, wlo);
      }
      if (bnd != wb && bnd > 0) {                       // the walk enters band bnd-1 at a column <= j
        pb = bnd - 1;
        const int wt = (j - 1 + 63) >> 4;
        plo = wt - (DTW_WIN - 1) > 0 ? wt - (DTW_WIN - 1) : 0;
        load_win(nxt, pb, plo);
      }
      wb = bnd;
    }
    // steps while the walk stays in this band, this window slot, and the matrix interior:
    // l >= 0, s >= 16 * w (bit position >= 0), j >= 1
    const int kw = __builtin_amdgcn_readfirstlane(w - wlo);
    int ll = __builtin_amdgcn_readfirstlane(l);
    int bp = __builtin_amdgcn_readfirstlane(2 * (s & 15));          // bit position of step s
    int jj = __builtin_amdgcn_readfirstlane(j);
    DTW_WALK_SLOTS(kw);
    i = 64 * bnd + ll + 1;
    j = jj;
  }
  while (i > 0 || j > 0) {    // findPreviousStep on the borders: i == 0 -> left, j == 0 -> up
    emit(i == 0 ? 1u : 0u);
    if (i == 0) --j; else --i;
  }
  if (P & 15) vacc = lane == ((P >> 4) & 63) ? cacc : vacc;   // the partial last word
  if (P & 1023) {             // the last, partly filled block of 64 words
    const int base = (P >> 10) << 6, nw = (P + 15) >> 4;
    if (lane < nw - base) codes[base + lane] = vacc;
  }
  if (lane == 0) *plen = P;
}

__global__ __launch_bounds__(64) void dtw_walk_kernel(const uint32_t* Dn, int64_t nq, int64_t nr, int64_t SW,
                                                      uint32_t* codes, int64_t* plen) {
  dtw_walk_body(Dn, nq, nr, SW, codes, plen);
}

// one block per DTW of a batch (the walks are independent)
__global__ __launch_bounds__(64) void dtw_walk_batch_kernel(const DtwArgs* args) {
  const DtwArgs a = load_args_uniform(args + blockIdx.x);
  dtw_walk_body(a.Dn, a.nq, a.nr, a.SW, a.codes, a.plen);
}

// ------------------------------------------------------- backtrack by bands ----
// The serial walk above is a chain of nq + nr dependent moves (5.3 ms at 51,676^2).  With the
// exit map Xm the chain shrinks to one dependent load per band, and the bands' own stretches of
// the path are walked in parallel; the moves land in the same 2-bit stream, in the same order,
// as the serial walk's (dtw.go:165-188):
//  dtw_exit_map_kernel     Xm and the segment boundaries (above), every band and segment at once.
//  dtw_walk_chain_kernel   one lane: ent[nb-1] = nr (the walk starts at (nq, nr)), then
//                          ent[b-1] = Xm[b][ent[b] - 1] (0 stays 0; a segment symbol resolved).
//  dtw_walk_band_kernel<false>  one wave per band: from (64b + lv + 1, ent[b]) until the path
//                          reaches row 64b (band 0: to (0, 0), border moves included); cnt[b].
//  dtw_walk_scan_kernel    off[b] = moves of the bands below b in the walk order (b' > b), the
//                          total P, and the move words zeroed.
//  dtw_walk_band_kernel<true>   the same walks again, ORing their moves into the stream at off[b].
// (BATCH: blockIdx.y, or the block, is the DTW of a batch)
// Exit map of band b (dtw_exit_map_kernel, grid (segment, band[, DTW])): X(l, j) = the column
// at which the backtrack from cell (64b+1+l, j) reaches row 64b.  It follows the codes as C
// follows the costs: X(l, j) = X(l-1, j) (up), X(l, j-1) (left), X(l-1, j-1) (diagonal), with
// X(-1, j) = j (the edge row) and X(l, 0) = 0 (the path then runs up column 0), so one wave
// sweeps a segment of DTW_XSEG columns in the band kernel's skew (lane = row, DPP from lane l-1),
// reading the 2-bit codes 16 steps per word.  A segment does not wait for its left neighbour: its
// left boundary X(l, J0-1) enters as the symbol -(l+1), and the chain resolves a symbol through
// the neighbour's right boundary Xr[b][k-1][l] (a path crosses a segment's left edge before
// reaching row 64b only within ~64 columns of it, so this is rare and one hop).
// 64 steps of the exit-map recurrence (4 code words); row lv's X after step t0 + u -> hrow[u]
template <bool GUARD>
__device__ __forceinline__ void dtw_xm_block(const uint32_t (&cw)[4], int t0, int J0, int ncol, int lane, int lv,
                                             int& x, int& xdg, int* hrow) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int hist[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int t = t0 + 16 * q + u;
      // code 0 up, 1 left, 2 diagonal as two sign-extended bit masks and two bit-selects
      const int mleft = (int)(cw[q] << (31 - 2 * u)) >> 31, mdiag = (int)(cw[q] << (30 - 2 * u)) >> 31;
      const int xup = __builtin_amdgcn_update_dpp(J0 + t, x, 0x138, 0xf, 0xf, false);   // wave_shr:1
      const int xud = (mdiag & xdg) | (~mdiag & xup);
      const int xn = (mleft & x) | (~mleft & xud);
      xdg = xup;
      if constexpr (GUARD) x = (unsigned)(t - lane) < (unsigned)ncol ? xn : x;
      else x = xn;
      hist[u] = x;
    }
    if (lane == lv) {
#pragma unroll
      for (int u = 0; u < 16; ++u) hrow[16 * q + u] = hist[u];
    }
  }
}

template <bool BATCH>
__global__ __launch_bounds__(64) void dtw_exit_map_kernel(DtwArgs a_in, const DtwArgs* args) {
  const DtwArgs a = BATCH ? load_args_uniform(args + blockIdx.z) : a_in;
  const int64_t b = blockIdx.y, k = blockIdx.x;
  const int64_t nq = a.nq, nr = a.nr, nb = a.nb, SW = a.SW, nseg = dtw_nseg(nr);
  if (b >= nb || k >= nseg) return;
  const int lane = threadIdx.x;
  const int64_t J0 = 1 + k * DTW_XSEG, J1 = J0 + DTW_XSEG < nr + 1 ? J0 + DTW_XSEG : nr + 1;   // columns [J0, J1)
  const int lv = (int)(b == nb - 1 ? nq - 1 - 64 * b : 63);
  const uint32_t* Db = a.Dn + ((b * SW) << 6) + lane;
  int32_t* Xb = dtw_xmap(a.Dn, nb, SW) + b * dtw_nr64(nr);
  const int ncol = (int)(J1 - J0);
  const int T = ncol + lv;                         // steps until row lv has reached column J1-1
  const int64_t w0 = (J0 - 1) >> 4;                // the segment's first code word (J0-1 = 1024k)
  const int nblk = (T + 63) >> 6;                  // 64-step blocks (4 code words each)
  __shared__ int hrow[64];                         // row lv's X over a block's 64 steps
  int x = k == 0 ? 0 : -(lane + 1);                // own X of the previous step (the left boundary)
  int xdg = (int)(J0 - 1);                         // lane 0: X(-1, J0-1)
  auto ldw = [&](int q) -> uint32_t {
    const int64_t w = w0 + q;
    return (q < 4 * nblk && w < SW) ? Db[w << 6] : 0u;
  };
  // code words two blocks ahead of the recurrence (HBM latency is a few blocks of steps)
  uint32_t cur[4], nx1[4], nx2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) { cur[q] = ldw(q); nx1[q] = ldw(4 + q); }
  for (int blk = 0; blk < nblk; ++blk) {
#pragma unroll
    for (int q = 0; q < 4; ++q) nx2[q] = ldw(4 * (blk + 2) + q);
    const int t0 = 64 * blk;
    // the guards (a lane before its first or past its last column keeps its X) only where the
    // block crosses the skewed start or end
    if (t0 < 64 || t0 + 64 > ncol) dtw_xm_block<true>(cur, t0, (int)J0, ncol, lane, lv, x, xdg, hrow);
    else dtw_xm_block<false>(cur, t0, (int)J0, ncol, lane, lv, x, xdg, hrow);
    // row lv's 64 values (steps t0 .. t0+63 = Xm columns J0-1+t0-lv+u) -> one coalesced store
    __syncthreads();
    const int tu = t0 + lane - lv;
    if (tu >= 0 && tu < ncol) Xb[J0 - 1 + tu] = hrow[lane];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) { cur[q] = nx1[q]; nx1[q] = nx2[q]; }
  }
  dtw_xbound(a.Dn, nb, SW, nr)[(b * nseg + k) * 64 + lane] = x;   // X(l, J1-1) (rows <= lv)
}

template <bool BATCH>
__global__ __launch_bounds__(64) void dtw_walk_chain_kernel(DtwArgs a_in, const DtwArgs* args) {
  const DtwArgs a = BATCH ? load_args_uniform(args + blockIdx.x) : a_in;
  if (threadIdx.x != 0) return;
  const int64_t nb = a.nb, nr64 = dtw_nr64(a.nr), nseg = dtw_nseg(a.nr);
  const int32_t* X = dtw_xmap(a.Dn, nb, a.SW);
  const int32_t* Xr = dtw_xbound(a.Dn, nb, a.SW, a.nr);
  int32_t* ent = dtw_walk_meta(a.Dn, nb, a.SW, a.nr);
  int e = (int)a.nr;
  ent[nb - 1] = e;
  for (int64_t b = nb - 1; b > 0; --b) {
    if (e > 0) {
      int v = X[b * nr64 + e - 1];
      int64_t k = (e - 1) / DTW_XSEG;
      while (v < 0 && k > 0) v = Xr[(b * nseg + --k) * 64 + (-v - 1)];   // a segment's left boundary
      e = v < 0 ? 0 : v;
    }
    ent[b - 1] = e;
  }
}

template <bool EMIT, bool BATCH>
__global__ __launch_bounds__(64) void dtw_walk_band_kernel(DtwArgs a_in, const DtwArgs* args) {
  const DtwArgs a = BATCH ? load_args_uniform(args + blockIdx.y) : a_in;
  const int64_t nb = a.nb;
  const int bnd = (int)blockIdx.x;
  if (bnd >= nb) return;
  const int lane = threadIdx.x;
  const int64_t nq = a.nq, SW = a.SW;
  const int sw = (int)SW;
  int32_t* meta = dtw_walk_meta(a.Dn, nb, SW, a.nr);
  const int lv = (int)(bnd == nb - 1 ? nq - 1 - 64 * (int64_t)bnd : 63);
  const int ilo = 64 * bnd;
  int i = ilo + lv + 1, j = __builtin_amdgcn_readfirstlane(meta[bnd]);
  int64_t g = EMIT ? __builtin_amdgcn_readfirstlane(meta[2 * nb + bnd]) : 0;   // the next move's index
  int P = 0;
  uint32_t cacc = 0;
  uint32_t* codes = a.codes;
  auto emit = [&](uint32_t code) {
    if constexpr (EMIT) {
      cacc |= code << (2 * (g & 15));
      ++g;
      if ((g & 15) == 0) {                         // a word complete (shared with a neighbour band
        if (lane == 0) atomicOr(&codes[(g >> 4) - 1], cacc);   // at the segment's ends: OR)
        cacc = 0;
      }
    }
    ++P;
  };
  const uint32_t* Db = a.Dn + (((int64_t)bnd * sw) << 6) + lane;
  uint32_t win[DTW_WIN];
  int wlo = -1;
  while (i > ilo && j > 0) {
    const int l = (i - 1) & 63;
    const int s = j - 1 + l, w = s >> 4;
    if (w < wlo || wlo < 0) {
      wlo = w - (DTW_WIN - 1) > 0 ? w - (DTW_WIN - 1) : 0;
#pragma unroll
      for (int k = 0; k < DTW_WIN; ++k) win[k] = (wlo + k < sw) ? Db[(int64_t)(wlo + k) << 6] : 0u;
    }
    const int kw = __builtin_amdgcn_readfirstlane(w - wlo);
    int ll = __builtin_amdgcn_readfirstlane(l);
    int bp = __builtin_amdgcn_readfirstlane(2 * (s & 15));
    int jj = __builtin_amdgcn_readfirstlane(j);
    DTW_WALK_SLOTS(kw);
    i = ilo + ll + 1;
    j = jj;
  }
  if (bnd == 0) {
    while (i > 0 || j > 0) {                       // findPreviousStep on the borders
      emit(i == 0 ? 1u : 0u);
      if (i == 0) --j; else --i;
    }
  } else {
    while (i > ilo) { emit(0u); --i; }             // j == 0: up column 0 to the band's top
  }
  if constexpr (EMIT) {
    if ((g & 15) && lane == 0) atomicOr(&codes[g >> 4], cacc);
  } else {
    if (lane == 0) meta[nb + bnd] = P;
  }
}

// any block of 64..1024 threads (a multiple of 64).  Batches launch 256: a 1024-thread block needs
// 4 waves on every SIMD of one CU at once, which a CU that also holds a DTW wave (320 registers of
// 512) cannot give, so under C5 the block waited for a CU to drain (4.1 ms average in the r03c trace)
template <bool BATCH>
__global__ __launch_bounds__(1024) void dtw_walk_scan_kernel(DtwArgs a_in, const DtwArgs* args) {
  __shared__ int64_t wsum[16];
  const DtwArgs a = BATCH ? load_args_uniform(args + blockIdx.x) : a_in;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, NT = (int)blockDim.x, NWV = NT >> 6;
  const int64_t nb = a.nb;
  int32_t* meta = dtw_walk_meta(a.Dn, nb, a.SW, a.nr);
  const int32_t* cnt = meta + nb;
  int32_t* off = meta + 2 * nb;
  // thread t owns bands in walk order k = nb-1-b over [k0, k1)
  const int64_t per = (nb + NT - 1) / NT;
  const int64_t k0 = t * per < nb ? t * per : nb, k1 = (t + 1) * per < nb ? (t + 1) * per : nb;
  int64_t sum = 0;
  for (int64_t k = k0; k < k1; ++k) sum += cnt[nb - 1 - k];
  int64_t inc = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int64_t base = 0, tot = 0;
  for (int w = 0; w < NWV; ++w) { base += w < wv ? wsum[w] : 0; tot += wsum[w]; }
  int64_t o = base + inc - sum;
  for (int64_t k = k0; k < k1; ++k) {
    off[nb - 1 - k] = (int32_t)o;
    o += cnt[nb - 1 - k];
  }
  const int64_t nw = (tot + 15) >> 4;
  for (int64_t w = t; w < nw; w += NT) a.codes[w] = 0u;
  if (t == 0) *a.plen = tot;
}

namespace {
__device__ __forceinline__ double cn_at(const double* Cn, int64_t S, int64_t i, int64_t j) {
  if (i == 0) return j == 0 ? 0.0 : __builtin_inf();
  if (j == 0) return __builtin_inf();
  const int64_t b = (i - 1) >> 6, l = (i - 1) & 63;
  return Cn[dtw_cn_off(b, (S + 1) >> 1, j - 1 + l, l)];
}
}  // namespace

// Path points and costs from the walk's moves (dtw.go:165-188), in two launches.
//  dtw_path_scan_kernel (one block): per 16-move code word, its (di, dj) from two popcounts (a
//    move is 0 = up, 1 = left, 2 = diag: di counts moves != 1, dj moves != 0; padding fields
//    of the last word are 0 and excluded), then the block's exclusive scan gives every word's
//    starting cell (i, j).
//  dtw_path_points_kernel (one thread per word): replays its 16 moves from that cell.  Point k
//    of the walk is (i_k - 1, j_k - 1) with cost C[i][j] - C[i-1][j-1] (0 on the borders);
//    output is in forward order (index P-1-k).  The 32 cost loads of a thread are independent.
// (BATCH: one block per DTW of a batch, its P read from the walk's output, and C[nq][nr] saved)
template <bool BATCH>
__global__ __launch_bounds__(1024) void dtw_path_scan_kernel(const uint32_t* codes, int64_t P, int64_t nq,
                                                             int64_t nr, int2* wstart, const DtwArgs* args) {
  __shared__ int64_t wsum[2][16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, NT = (int)blockDim.x;   // 64..1024 (see walk scan)
  if constexpr (BATCH) {
    const DtwArgs a = load_args_uniform(args + blockIdx.x);
    codes = a.codes; P = *a.plen; nq = a.nq; nr = a.nr; wstart = a.wstart;
    if (t == 0 && a.Cn) *a.cnm = cn_at(a.Cn, a.S, nq, nr);   // (CK mode: the tile pass writes it)
  }
  const int64_t nw = (P + 15) >> 4;
  const int64_t per = (nw + NT - 1) / NT;
  const int64_t w0 = t * per < nw ? t * per : nw, w1 = (t + 1) * per < nw ? (t + 1) * per : nw;
  auto counts = [&](int64_t w, int64_t& di, int64_t& dj) {
    const uint32_t x = codes[w];
    const int n = (int)(P - 16 * w < 16 ? P - 16 * w : 16);
    const int c1 = __builtin_popcount(x & 0x55555555u), c2 = __builtin_popcount(x & 0xAAAAAAAAu);
    di = n - c1;
    dj = c1 + c2;
  };
  int64_t di = 0, dj = 0;
  for (int64_t w = w0; w < w1; ++w) {
    int64_t a, b;
    counts(w, a, b);
    di += a;
    dj += b;
  }
  int64_t si = di, sj = dj;                         // block exclusive scan of (di, dj)
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t ui = __shfl_up(si, o, 64), uj = __shfl_up(sj, o, 64);
    if (lane >= o) { si += ui; sj += uj; }
  }
  if (lane == 63) { wsum[0][wv] = si; wsum[1][wv] = sj; }
  __syncthreads();
  int64_t oi = 0, oj = 0;
  for (int w = 0; w < wv; ++w) { oi += wsum[0][w]; oj += wsum[1][w]; }
  int64_t i = nq - (oi + si - di), j = nr - (oj + sj - dj);
  for (int64_t w = w0; w < w1; ++w) {
    wstart[w] = make_int2((int)i, (int)j);
    int64_t a, b;
    counts(w, a, b);
    i -= a;
    j -= b;
  }
}

// (BATCH: blockIdx.y = the DTW of a batch)
template <bool BATCH>
__global__ __launch_bounds__(256) void dtw_path_points_kernel(const uint32_t* codes, const int2* wstart, int64_t P,
                                                              const double* Cn, int64_t S, int32_t* pq, int32_t* pr,
                                                              double* pc, const DtwArgs* args) {
  if constexpr (BATCH) {
    const DtwArgs a = load_args_uniform(args + blockIdx.y);
    codes = a.codes; wstart = a.wstart; P = *a.plen; Cn = a.Cn; S = a.S; pq = a.pq; pr = a.pr; pc = a.pc;
  }
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= ((P + 15) >> 4)) return;
  const uint32_t x = codes[w];
  const int n = (int)(P - 16 * w < 16 ? P - 16 * w : 16);
  int i = wstart[w].x, j = wstart[w].y;
  // one move at a time, stored at once (no per-word arrays: 108 -> ~30 VGPRs, so these blocks fit
  // on a CU beside the band kernel's two under C5)
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k < n) {
      const int64_t f = P - 1 - (16 * w + k);
      pq[f] = i - 1; pr[f] = j - 1;
      double c = 0.0;
      if (Cn && i > 0 && j > 0) c = __dsub_rn(cn_at(Cn, S, i, j), cn_at(Cn, S, i - 1, j - 1));
      if (Cn || i == 0 || j == 0) pc[f] = c;            // (CK mode: the tile pass writes the rest)
    }
    const uint32_t m = (x >> (2 * k)) & 3u;
    i -= m != 1u;
    j -= m != 0u;
  }
}

// ---------------------------------------------------------------- path tiles (CK mode)
// Without the cost matrix, a path point's cost C[i][j] - C[i-1][j-1] (dtw.go:165-188) is
// recomputed: the path visits at most nb + ceil(nr/64) tiles of 64 x 64 cells (tile (bi, bj) =
// rows 64bi+1 .., columns 64bj+1 ..), and a tile's cells follow from its top row C[64bi][*] (the
// band edge E of band bi-1, or row 0) and its left column C[*][64bj] (checkpoint CK, or column
// 0), both written by the band kernel.  The recurrence, the distance (Go's sequential sum,
// unfused, then a correctly rounded sqrt) and math.Min are the band kernel's, so every value is
// bit-identical to the full store's.
//  dtw_path_runs_kernel: thread per path point; a point whose tile differs from its
//    predecessor's starts a run (the path is monotone, so a tile's points are contiguous); runs
//    are appended through an atomic counter in any order.
//  dtw_path_tile_kernel: one wave per run: the tile's anti-diagonal recurrence in registers
//    (127 steps, lane = row, distances inline), each path point's cost taken at its own step.
template <bool BATCH>
__global__ __launch_bounds__(256) void dtw_path_runs_kernel(DtwArgs a_in, const DtwArgs* args) {
  const DtwArgs a = BATCH ? load_args_uniform(args + blockIdx.y) : a_in;
  const int64_t P = *a.plen;
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= P) return;
  const int pi = a.pq[f], pj = a.pr[f];
  if (pi < 0 || pj < 0) return;                      // border point: cost 0, written by the points pass
  bool start = f == 0;
  if (!start) {
    const int qi = a.pq[f - 1], qj = a.pr[f - 1];
    start = qi < 0 || qj < 0 || (qi >> 6) != (pi >> 6) || (qj >> 6) != (pj >> 6);
  }
  if (start) {
    const int k = atomicAdd(&a.runs[0], 1);
    a.runs[1 + k] = (int)f;
  }
}

template <bool BATCH, int D>
__global__ __launch_bounds__(64) void dtw_path_tile_kernel(DtwArgs a_in, const DtwArgs* args) {
  // Registers only for the recurrence (the band kernel's sweep shape: lane = row, at step st lane l
  // relaxes column c = st - l, C[i-1][j] by DPP from lane l-1, C[i-1][j-1] one step later, C[i][j-1]
  // its own), so the block needs ~7 KB of LDS and co-resides with the band kernel's blocks (the
  // earlier T/Dl tile arrays took 73 KB and waited for whole CUs to drain under C5's streams).
  __shared__ __attribute__((aligned(16))) double Rt[D > 0 ? 64 * D : 2];   // D > 0: the tile's reference rows
  __shared__ double top[66];                         // C[64bi][jb + c], c = 0 .. 64
  __shared__ int rlo[64], rhi[64], rf[64];           // the run's points in row li: columns, first index
  const DtwArgs a = BATCH ? load_args_uniform(args + blockIdx.y) : a_in;
  const int lane = threadIdx.x;
  if ((int)blockIdx.x >= a.runs[0]) return;
  const int64_t P = *a.plen, nq = a.nq, nr = a.nr;
  const int f0 = a.runs[1 + blockIdx.x];
  const int bi = a.pq[f0] >> 6, bj = a.pr[f0] >> 6;
  const double inf = __builtin_inf();
  const int64_t i = 64 * (int64_t)bi + 1 + lane;     // the lane's row
  const int64_t jb = 64 * (int64_t)bj;               // column of the tile's left boundary
  for (int c = lane; c <= 64; c += 64) {
    const int64_t j = jb + c;
    double v = inf;
    if (bi == 0) v = j == 0 ? 0.0 : inf;
    else if (j >= 1 && j <= nr) v = __builtin_bit_cast(double, a.E[(int64_t)(bi - 1) * (nr + 1) + j]);
    top[c] = v;
  }
  const double leftc = bj == 0 ? inf : a.CK[(((int64_t)bi * (nr >> 6) + bj - 1) << 6) + lane];   // C[i][jb]
  rlo[lane] = 64; rhi[lane] = -1; rf[lane] = INT32_MAX;
  const int dim = a.dim;
  const double* qrow = a.q + (i <= nq ? i - 1 : 0) * dim;
  double qv[D > 0 ? D : 1];
  if constexpr (D > 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) qv[k] = qrow[k];
    const int64_t jl = jb + 1 + lane;
    const double* rrow = a.r + (jl <= nr ? jl - 1 : 0) * D;
#pragma unroll
    for (int k = 0; k < D; ++k) Rt[lane * D + k] = rrow[k];
  }
  __syncthreads();
  // the run's points: at most 127 (a monotone path inside one tile), contiguous from f0; a row's
  // points are consecutive columns at consecutive indices
  for (int64_t f = f0 + lane; f < P && f < f0 + 128; f += 64) {
    const int pi = a.pq[f], pj = a.pr[f];
    if (pi < 0 || pj < 0 || (pi >> 6) != bi || (pj >> 6) != bj) continue;
    const int li = pi - 64 * bi, lj = pj - 64 * bj;
    atomicMin(&rlo[li], lj);
    atomicMax(&rhi[li], lj);
    atomicMin(&rf[li], (int)f);
  }
  __syncthreads();
  const int mlo = rlo[lane], mhi = rhi[lane], mf = rf[lane];
  // own C of the previous step (before the lane's first column: C[i][jb], which its lower
  // neighbour takes as the diagonal of ITS first cell), and the previous step's up
  double v = leftc, upp = top[0];
  for (int st = 0; st < 127; ++st) {
    const int c = st - lane;                         // column jb + 1 + c
    const double up = shr1(v, top[st + 1 < 65 ? st + 1 : 64]);   // lane 0: the top row
    const double dg = upp;
    upp = up;
    if (c >= 0 && c < 64) {
      const int64_t j = jb + 1 + c;
      const double left = v;
      double sum = 0.0;
      if constexpr (D > 0) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double df = qv[k] - Rt[c * D + k];
          sum = sum + df * df;
        }
      } else {
        const double* rrow = a.r + (j <= nr ? j - 1 : 0) * dim;
        for (int k = 0; k < dim; ++k) {
          const double df = qrow[k] - rrow[k];
          sum = sum + df * df;
        }
      }
      double nv = sqrt(sum) + go_min(go_min(up, left), dg);
      if (a.band > 0 && (i - j > a.band || j - i > a.band)) nv = inf;   // outside the Sakoe-Chiba band
      v = nv;
      if (c >= mlo && c <= mhi) {
        const int64_t f = mf + (c - mlo);
        a.pc[f] = __dsub_rn(nv, dg);
        if (i == nq && j == nr) *a.cnm = nv;
      }
    }
  }
}

// costMatrix[1:] row-major: block = one band x 64 columns, staged through LDS so
// both the skewed reads and the row-major writes are coalesced.
__global__ __launch_bounds__(256) void dtw_cost_rowmajor_kernel(const double* Cn, int64_t nq, int64_t nr, int64_t S,
                                                                double* out) {
  __shared__ double tile[64][65];
  const int64_t b = blockIdx.y, j0 = 1 + (int64_t)blockIdx.x * 64;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int u = wv; u < 127; u += 4) {             // steps s = j0-1+u cover columns j0..j0+63 of every row
    const int64_t s = j0 - 1 + u;
    const int64_t col = u - lane;                  // j - j0
    if (s < S && col >= 0 && col < 64) tile[lane][col] = Cn[dtw_cn_off(b, (S + 1) >> 1, s, lane)];
  }
  __syncthreads();
  const int64_t pitch = nr + 1;
  for (int rr = wv; rr < 64; rr += 4) {
    const int64_t i = 64 * b + 1 + rr;
    const int64_t j = j0 + lane;
    if (i <= nq && j <= nr) out[(i - 1) * pitch + j] = tile[rr][lane];
    if (i <= nq && blockIdx.x == 0 && lane == 0) out[(i - 1) * pitch] = __builtin_inf();
  }
}

__global__ void nonfinite_kernel(const double* x, int64_t n, int32_t* flag) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    if (!__builtin_isfinite(x[k])) *flag = 1;
}

// the probe over both sequences of every DTW of a batch (blockIdx.y = the DTW): one launch per
// batch instead of two per pair on the batch's stream
// Also fills the DTW's band-edge rows E with the sentinel the band kernel polls for and zeroes its
// path-tile run counters (what a hipMemsetD32Async and a hipMemsetAsync per batch did before).
// Same stream, earlier kernel: the stores are visible to the band kernel's sc1 polls.
__global__ void nonfinite_batch_kernel(const DtwArgs* args) {
  const DtwArgs a = load_args_uniform(args + blockIdx.y);
  const int64_t nqe = a.nq * a.dim, n = nqe + a.nr * a.dim;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride)
    if (!__builtin_isfinite(k < nqe ? a.q[k] : a.r[k - nqe])) a.sync[2] = 1;
  if (a.nb > 1) {   // E[b][j], b < nb - 1, j <= nr (dtw_edge_bytes)
    const int64_t ne = (a.nb - 1) * (a.nr + 1);
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < ne; k += stride)
      a.E[k] = 0x7FF000017FF00001ull;
  }
  if (a.runs) {     // the path-tile run counters (dtw_run_words), read after the band kernel
    const int64_t nw = a.nb + (a.nr + 63) / 64 + 2;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nw; k += stride) a.runs[k] = 0;
  }
}

// SONAR_DTW_DBG_STALL=<band> (tests only): fault injection, see DtwArgs::dbg_stall; "b<band>"
// injects it into batched launches only (launch_dtw_batch), so the single-pair redo runs clean
int32_t dtw_dbg_stall_band(bool batch) {
  const char* e = std::getenv("SONAR_DTW_DBG_STALL");
  if (!e) return -1;
  if (e[0] == 'b') return batch ? (int32_t)std::atoi(e + 1) : -1;
  return (int32_t)std::atoi(e);
}

// threads of the batched walk / path scans (one block per DTW): 256, so the block fits beside the
// DTW waves of other batches (1,024 threads waited for a whole CU to drain under C5)
constexpr unsigned kBatchScanThreads = 256;

// SONAR_DTW_SERIAL_WALK=1: the one-wave serial backtrack instead of the backtrack by bands (A/B)
static bool dtw_serial_walk() {
  const char* e = std::getenv("SONAR_DTW_SERIAL_WALK");
  return e && e[0] == '1';
}

DtwGeom dtw_geom(int64_t nq, int64_t nr) {
  DtwGeom g;
  g.nq = nq; g.nr = nr;
  g.nb = (nq + 63) / 64;
  g.S = nr + 63;
  g.SW = (g.S + 15) / 16;
  return g;
}
size_t dtw_cn_bytes(const DtwGeom& g) { return (size_t)g.nb * ((g.S + 1) / 2) * 128 * 8; }
size_t dtw_dn_bytes(const DtwGeom& g) {   // direction words + exit map + walk meta (dtw_walk_meta)
  return ((size_t)g.nb * g.SW * 64 + (size_t)g.nb * dtw_nr64(g.nr) + (size_t)g.nb * dtw_nseg(g.nr) * 64 +
          3 * (size_t)g.nb + 3) / 4 * 16;
}
size_t dtw_ck_bytes(const DtwGeom& g) { return (size_t)g.nb * (g.nr >= 64 ? g.nr / 64 : 1) * 64 * 8; }
int64_t dtw_run_words(const DtwGeom& g) { return g.nb + (g.nr + 63) / 64 + 2; }
size_t dtw_edge_bytes(const DtwGeom& g) { return (size_t)(g.nb > 1 ? g.nb - 1 : 1) * (g.nr + 1) * 8; }
int64_t dtw_cn_index(const DtwGeom& g, int64_t i, int64_t j) {
  const int64_t b = (i - 1) >> 6, l = (i - 1) & 63, s = j - 1 + l;
  return ((b * ((g.S + 1) / 2) + (s >> 1)) << 7) + 2 * l + (s & 1);
}

int launch_dtw(const double* q, const double* r, int dim, int band, bool fast, const DtwGeom& g, double* Cn,
               uint32_t* Dn, uint64_t* E, int32_t* sync_words, uint32_t* codes, int64_t* plen, uint64_t* trace,
               hipStream_t s, hipEvent_t mid, double* CK) {
  // sync_words: [0] ticket, [1] error bits, [2] non-finite flag (set by the caller's probe), [3]
  // unused, then the DTW_DIAG_WORDS-word diagnostic record at byte 16 (DTW_SYNC_BYTES in all)
  if (hipMemsetAsync(sync_words, 0, 2 * sizeof(int32_t), s) != hipSuccess) return -5;
  if (hipMemsetAsync(sync_words + 4, 0, DTW_DIAG_WORDS * 8, s) != hipSuccess) return -5;
  if (g.nb > 1 && hipMemsetD32Async((hipDeviceptr_t)E, 0x7FF00001u, dtw_edge_bytes(g) / 4, s) != hipSuccess) return -5;
  DtwArgs a{q, r, dim, band, g.nq, g.nr, g.nb, g.S, g.SW, Cn, Dn, reinterpret_cast<uint64_t*>(E), sync_words,
            trace};
  a.CK = CK;
  a.diag = reinterpret_cast<uint64_t*>(sync_words + 4);
  a.dbg_stall = dtw_dbg_stall_band(false);
  if (!Cn && !CK) return -1;
  const DtwBatch nob{};
  const dim3 grid((unsigned)g.nb), block(64 * DTW_WAVES);
#define SONAR_DTW_LAUNCH(DD)                                                                          \
  do {                                                                                                \
    if (band > 0) {                                                                                   \
      if (fast) hipLaunchKernelGGL((dtw_band_kernel<DD, true, true>), grid, block, 0, s, a, nob);     \
      else hipLaunchKernelGGL((dtw_band_kernel<DD, false, true>), grid, block, 0, s, a, nob);         \
    } else {                                                                                          \
      if (fast) hipLaunchKernelGGL((dtw_band_kernel<DD, true, false>), grid, block, 0, s, a, nob);    \
      else hipLaunchKernelGGL((dtw_band_kernel<DD, false, false>), grid, block, 0, s, a, nob);        \
    }                                                                                                 \
  } while (0)
  if (dim == 12) SONAR_DTW_LAUNCH(12);
  else if (dim == 1) SONAR_DTW_LAUNCH(1);
  else SONAR_DTW_LAUNCH(0);
#undef SONAR_DTW_LAUNCH
  if (mid) hipEventRecord(mid, s);
  if (dtw_serial_walk()) {
    hipLaunchKernelGGL(dtw_walk_kernel, dim3(1), dim3(64), 0, s, Dn, g.nq, g.nr, g.SW, codes, plen);
  } else {
    a.codes = codes;
    a.plen = plen;
    const DtwArgs* none = nullptr;
    hipLaunchKernelGGL(dtw_exit_map_kernel<false>, dim3((unsigned)dtw_nseg(g.nr), (unsigned)g.nb), dim3(64), 0, s, a,
                       none);
    hipLaunchKernelGGL(dtw_walk_chain_kernel<false>, dim3(1), dim3(64), 0, s, a, none);
    hipLaunchKernelGGL((dtw_walk_band_kernel<false, false>), dim3((unsigned)g.nb), dim3(64), 0, s, a, none);
    hipLaunchKernelGGL(dtw_walk_scan_kernel<false>, dim3(1), dim3(1024), 0, s, a, none);
    hipLaunchKernelGGL((dtw_walk_band_kernel<true, false>), dim3((unsigned)g.nb), dim3(64), 0, s, a, none);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_dtw_path_cost(const double* Cn, const DtwGeom& g, const uint32_t* codes, int64_t P, int2* wstart,
                         int32_t* pq, int32_t* pr, double* pc, hipStream_t s) {
  if (P <= 0) return 0;
  const int64_t nw = (P + 15) >> 4;
  hipLaunchKernelGGL(dtw_path_scan_kernel<false>, dim3(1), dim3(1024), 0, s, codes, P, g.nq, g.nr, wstart,
                     (const DtwArgs*)nullptr);
  hipLaunchKernelGGL(dtw_path_points_kernel<false>, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, codes,
                     (const int2*)wstart, P, Cn, g.S, pq, pr, pc, (const DtwArgs*)nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_dtw_path_tiles(const DtwArgs& a, int64_t P, hipStream_t s) {
  if (P <= 0) return 0;
  const DtwGeom g = dtw_geom(a.nq, a.nr);
  if (hipMemsetAsync(a.runs, 0, 4, s) != hipSuccess) return -5;
  hipLaunchKernelGGL(dtw_path_runs_kernel<false>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, a,
                     (const DtwArgs*)nullptr);
  if (a.dim == 12)
    hipLaunchKernelGGL((dtw_path_tile_kernel<false, 12>), dim3((unsigned)(dtw_run_words(g) - 2)), dim3(64), 0, s, a,
                       (const DtwArgs*)nullptr);
  else
    hipLaunchKernelGGL((dtw_path_tile_kernel<false, 0>), dim3((unsigned)(dtw_run_words(g) - 2)), dim3(64), 0, s, a,
                       (const DtwArgs*)nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_dtw_batch(const DtwArgs* hargs, const DtwArgs* dargs, const int64_t* dstart, int n, int64_t total_bands,
                     int64_t max_cap, int32_t* ticket, hipStream_t s, const int2* dmap) {
  if (n <= 0 || total_bands <= 0) return 0;
  if (total_bands > INT32_MAX) return -1;
  const DtwArgs none{};
  const DtwBatch bt{dargs, dstart, n, ticket, dmap};
  // the batched instance is built for 6 waves per SIMD (80 VGPRs) but launched with DTW_BATCH_PAD
  // bytes of dynamic LDS it never touches, so LDS still holds it to 2 blocks per CU (3 x 52 KB would
  // fit; 3 x 54.7 KB do not): the 18 registers per wave it gives up leave room on each SIMD for
  // the other worker streams' short kernels beside two band blocks.  C5 2,143-2,162 ->
  // 2,216-2,235 pairs/s (Kernel 6, "Register budget of the batched instance")
  // the 2-blocks-per-CU cap above rests on LDS arithmetic only (static LDS + DTW_BATCH_PAD > 160 KB / 3):
  // checked once per process against the runtime's occupancy calculator, so a change of DTW_DQ or of
  // the static LDS that lets a third block fit (measured slower) does not go unnoticed
  static std::once_flag occ_once;
  std::call_once(occ_once, [] {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, dtw_band_kernel<12, true, false, true>,
                                                     64 * DTW_WAVES, DTW_BATCH_PAD) == hipSuccess && blocks != 2)
      std::fprintf(stderr, "sonar: batched dtw_band_kernel fits %d blocks per CU (sized for 2: DTW_BATCH_PAD)\n",
                   blocks);
  });
  hipLaunchKernelGGL((dtw_band_kernel<12, true, false, true>), dim3((unsigned)total_bands), dim3(64 * DTW_WAVES),
                     DTW_BATCH_PAD, s, none, bt);
  if (dtw_serial_walk()) {
    hipLaunchKernelGGL(dtw_walk_batch_kernel, dim3((unsigned)n), dim3(64), 0, s, dargs);
  } else {
    int64_t max_nb = 1;
    for (int k = 0; k < n; ++k) max_nb = hargs[k].nb > max_nb ? hargs[k].nb : max_nb;
    int64_t max_seg = 1;
    for (int k = 0; k < n; ++k) max_seg = dtw_nseg(hargs[k].nr) > max_seg ? dtw_nseg(hargs[k].nr) : max_seg;
    hipLaunchKernelGGL(dtw_exit_map_kernel<true>, dim3((unsigned)max_seg, (unsigned)max_nb, (unsigned)n), dim3(64), 0,
                       s, none, dargs);
    hipLaunchKernelGGL(dtw_walk_chain_kernel<true>, dim3((unsigned)n), dim3(64), 0, s, none, dargs);
    hipLaunchKernelGGL((dtw_walk_band_kernel<false, true>), dim3((unsigned)max_nb, (unsigned)n), dim3(64), 0, s, none,
                       dargs);
    hipLaunchKernelGGL(dtw_walk_scan_kernel<true>, dim3((unsigned)n), dim3(kBatchScanThreads), 0, s, none, dargs);
    hipLaunchKernelGGL((dtw_walk_band_kernel<true, true>), dim3((unsigned)max_nb, (unsigned)n), dim3(64), 0, s, none,
                       dargs);
  }
  hipLaunchKernelGGL(dtw_path_scan_kernel<true>, dim3((unsigned)n), dim3(kBatchScanThreads), 0, s, (const uint32_t*)nullptr,
                     (int64_t)0, (int64_t)0, (int64_t)0, (int2*)nullptr, dargs);
  const int64_t nw = (max_cap + 15) >> 4;
  hipLaunchKernelGGL(dtw_path_points_kernel<true>, dim3((unsigned)((nw + 255) / 256), (unsigned)n), dim3(256), 0, s,
                     (const uint32_t*)nullptr, (const int2*)nullptr, (int64_t)0, (const double*)nullptr, (int64_t)0,
                     (int32_t*)nullptr, (int32_t*)nullptr, (double*)nullptr, dargs);
  if (!hargs[0].Cn) {   // CK mode (every DTW of a batch alike): the path-tile pass; runs zeroed by the caller
    int64_t max_tiles = 1;
    for (int k = 0; k < n; ++k) {
      const int64_t t = dtw_run_words(dtw_geom(hargs[k].nq, hargs[k].nr)) - 2;
      max_tiles = t > max_tiles ? t : max_tiles;
    }
    hipLaunchKernelGGL(dtw_path_runs_kernel<true>, dim3((unsigned)((max_cap + 255) / 256), (unsigned)n), dim3(256), 0,
                       s, none, dargs);
    hipLaunchKernelGGL((dtw_path_tile_kernel<true, 12>), dim3((unsigned)max_tiles, (unsigned)n), dim3(64), 0, s, none,
                       dargs);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_dtw_cost_rowmajor(const double* Cn, const DtwGeom& g, double* out, hipStream_t s) {
  const dim3 grid((unsigned)((g.nr + 63) / 64), (unsigned)g.nb);
  hipLaunchKernelGGL(dtw_cost_rowmajor_kernel, grid, dim3(256), 0, s, Cn, g.nq, g.nr, g.S, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_nonfinite_batch(const DtwArgs* dargs, int n, int64_t max_elems, hipStream_t s) {
  if (n <= 0) return 0;
  if (max_elems < 1) max_elems = 1;
  int64_t blocks = (max_elems + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(nonfinite_batch_kernel, dim3((unsigned)blocks, (unsigned)n), dim3(256), 0, s, dargs);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// sonar_align_pairs' scorer reductions on the device (alignment.go:380-643, correlation.go:526-667):
// one wave per pair over its warping path and energy correlation -- host::path_sums and
// host::corr_sums, bit for bit -- so a batch copies back ~150 bytes per pair instead of its path
// (16 B per point) and correlation, and its host thread only combines scalars.  Counts, extrema
// and the peak index (the first index of the largest |corr|, as Go's strict > scan) are order-free;
// the float sums keep Go's sequential order: 64 terms are formed at once (a smoothed cost is Go's
// window sum, a deviation is squared before it is added, as Go does) and then added one by one in
// index order (seq_add below).
namespace {
__device__ __forceinline__ int64_t wave_isum(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// the largest a over the wave (ties: the smallest index); a = -1 for "none"
__device__ __forceinline__ void wave_argmax(double& a, int64_t& i) {
  for (int o = 32; o > 0; o >>= 1) {
    const double ao = __shfl_xor(a, o, 64);
    const int64_t io = __shfl_xor(i, o, 64);
    if (ao > a || (ao == a && io < i)) { a = ao; i = io; }
  }
}
}  // namespace

// Sequential sums of 64 terms at a time (acc += v[lane 0], += v[lane 1], ... in lane order, for
// NC independent sums at once).  Round 6: the terms go through LDS and every lane runs the add chain
// on broadcast reads, so a term costs one dependent v_add_f64 (the reads are independent and issue
// ahead) instead of two v_readlane + the SGPR hazard + the add (3.2 -> 2.0 ms per launch).
template <int NC>
__device__ __forceinline__ void seq_add(double (&acc)[NC], const double (&v)[NC], int cnt, double* buf) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NC; ++c) buf[64 * c + lane] = v[c];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // 32 terms per sum into registers with every read issued up front, then the adds in order
  for (int k0 = 0; k0 < cnt; k0 += 32) {
    double r[NC][32];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int q = 0; q < 32; q += 2) {
        const double2 v2 = *reinterpret_cast<const double2*>(&buf[64 * c + k0 + q]);
        r[c][q] = v2.x; r[c][q + 1] = v2.y;
      }
    if (k0 + 32 <= cnt) {
#pragma unroll
      for (int q = 0; q < 32; ++q)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] += r[c][q];
    } else {
#pragma unroll
      for (int q = 0; q < 32; ++q)
        if (k0 + q < cnt) {
#pragma unroll
          for (int c = 0; c < NC; ++c) acc[c] += r[c][q];
        }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");     // the next block's stores after every read
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

constexpr int SU = 4;   // 64-term steps whose terms are formed before their adds (loads in flight)
__global__ __launch_bounds__(64) void pair_score_kernel(const ScoreJob* jobs) {
  const ScoreJob j = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  __shared__ __attribute__((aligned(16))) double sbuf[2 * 64];
  // ---- warping path
  const int64_t P = *j.plen;
  host::PathSums ps;
  ps.P = P;
  if (P > 0) {
    int64_t off = 0, dg = 0, ch = 0;
    const int64_t w = max((int64_t)2, min((int64_t)5, P / 4)), h = w / 2;
    auto smooth = [&](int64_t i) {                  // calculateCostConsistency's window mean
      double t = 0.0;
      const int64_t lo = max((int64_t)0, i - h), hi = min(P - 1, i + h);
      for (int64_t q = lo; q <= hi; ++q) t += j.pc[q];
      return t / (double)(hi - lo + 1);
    };
    double sc = 0.0, ss = 0.0;                       // Go's sequential sums (wave-uniform)
    // SU steps of 64 terms are formed first (their path loads all in flight at once), then added
    for (int64_t b0 = 0; b0 < P; b0 += 64 * SU) {
      double cu[SU], mu[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int64_t i = b0 + 64 * u + lane;
        double c = 0.0, m = 0.0;
        if (i < P) {
          off += j.pr[i] - j.pq[i];
          c = j.pc[i];
          if (P > 1) m = smooth(i);
          if (i >= 1) {
            const int d0 = j.pq[i] - j.pq[i - 1], d1 = j.pr[i] - j.pr[i - 1];
            if (d0 > 0 && d1 > 0) dg++;
            if (i >= 2 && (d0 != j.pq[i - 1] - j.pq[i - 2] || d1 != j.pr[i - 1] - j.pr[i - 2])) ch++;
          }
        }
        cu[u] = c; mu[u] = m;
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int64_t b = b0 + 64 * u;
        if (b < P) {
          const int cnt = (int)min((int64_t)64, P - b);
          double acc[2] = {sc, ss};
          const double v[2] = {cu[u], mu[u]};
          seq_add<2>(acc, v, cnt, sbuf);
          sc = acc[0]; ss = acc[1];
        }
      }
    }
    ps.offset_sum = wave_isum(off);
    ps.diag_steps = wave_isum(dg);
    ps.changes = wave_isum(ch);
    ps.sum_cost = sc;
    ps.p0q = j.pq[0]; ps.p0r = j.pr[0]; ps.p1q = j.pq[P - 1]; ps.p1r = j.pr[P - 1];
    if (P > 1) {
      ps.sum_smooth = ss;
      const double mean = ss / (double)P;
      double vv = 0.0;
      for (int64_t b0 = 0; b0 < P; b0 += 64 * SU) {
        double du[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int64_t i = b0 + 64 * u + lane;
          double d2 = 0.0;
          if (i < P) { const double d = smooth(i) - mean; d2 = d * d; }
          du[u] = d2;
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int64_t b = b0 + 64 * u;
          if (b < P) {
            const int cnt = (int)min((int64_t)64, P - b);
            double acc[1] = {vv};
            const double v[1] = {du[u]};
            seq_add<1>(acc, v, cnt, sbuf);
            vv = acc[0];
          }
        }
      }
      ps.var_smooth = vv;
    }
  }
  if (lane == 0) *j.path = ps;
  // ---- energy correlation
  if (!j.corr) return;
  const int64_t nl = j.nl;
  host::CorrSums cs;
  cs.num_lags = nl;
  if (nl > 0) {
    // findPeak: Go keeps corr[0] unless a strictly larger |corr| follows (a NaN corr[0] is kept)
    double a = -1.0;
    int64_t pi = nl;
    for (int64_t i = lane; i < nl; i += 64) {
      const double v = fabs(j.corr[i]);
      if (v > a) { a = v; pi = i; }                  // NaN never wins
    }
    wave_argmax(a, pi);
    const double c0 = j.corr[0];
    if (isnan(c0) || !(a > fabs(c0))) pi = 0;        // nothing strictly larger than |corr[0]|
    cs.peak_index = pi;
    cs.peak = j.corr[pi];
    double ns = 0.0, sa = -1.0, ms = 0.0;
    int64_t nc = 0, si = nl;
    for (int64_t b0 = 0; b0 < nl; b0 += 64 * SU) {
      double qu[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int64_t i = b0 + 64 * u + lane;
        double sq = 0.0;                             // terms outside the mask add an exact +0
        if (i < nl) {
          const double c = j.corr[i], v = fabs(c);
          const int64_t d = i > pi ? i - pi : pi - i;
          if (d > 5) { sq = c * c; nc++; }
          if (i != pi && v > sa) { sa = v; si = i; }
          if (d > 10 && v > ms) ms = v;
        }
        qu[u] = sq;
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int64_t b = b0 + 64 * u;
        if (b < nl) {
          const int cnt = (int)min((int64_t)64, nl - b);
          double acc[1] = {ns};
          const double v[1] = {qu[u]};
          seq_add<1>(acc, v, cnt, sbuf);
          ns = acc[0];
        }
      }
    }
    cs.noise_sum = ns;
    cs.noise_count = wave_isum(nc);
    wave_argmax(sa, si);
    cs.second_peak = (si < nl && sa > 0.0) ? j.corr[si] : 0.0;   // Go starts from 0 with a strict >
    int64_t mi = 0;
    wave_argmax(ms, mi);                             // a max of non-negative values
    cs.max_sidelobe = ms;
    if (nl >= 3 && pi > 0 && pi < nl - 1) cs.sharpness = -(j.corr[pi + 1] - 2 * j.corr[pi] + j.corr[pi - 1]);
  }
  if (lane == 0) *j.corr_out = cs;
}

int launch_pair_scores(const ScoreJob* djobs, int n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(pair_score_kernel, dim3((unsigned)n), dim3(64), 0, s, djobs);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_nonfinite(const double* x, int64_t n, int32_t* flag, hipStream_t s) {
  if (n <= 0) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(nonfinite_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, n, flag);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace sonar
