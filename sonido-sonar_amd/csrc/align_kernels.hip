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
#include <type_traits>

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

__global__ __launch_bounds__(64) void ncc_stats_kernel(const double* a, int64_t na, const double* b, int64_t nb,
                                                       double* stats) {
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

// one lag per thread (normalizedCrossCorrelation, correlation.go:373-409), sums in Go's index
// order (bit-exact).  A block owns 256 consecutive lags; their overlap windows start within 255
// samples of each other (s1 = max(0, -lag), s2 = max(0, lag)), so each k-tile of both inputs is
// staged once in LDS (coalesced) and every thread walks its own offsets there.
constexpr int kNccTile = 1024;
__global__ __launch_bounds__(256) void ncc_lag_kernel(const double* x, int64_t na, const double* y, int64_t nb,
                                                      int64_t L, double* corr) {
  __shared__ double xs[kNccTile + 256], ys[kNccTile + 256];
  __shared__ int64_t ovmax_s;
  const int64_t nl = 2 * L + 1;
  const int64_t idx0 = (int64_t)blockIdx.x * 256;
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
  hipLaunchKernelGGL(ncc_stats_kernel, dim3(2), dim3(64), 0, s, a, na, b, nb, stats);
  const int64_t nmax = na > nb ? na : nb;
  hipLaunchKernelGGL(ncc_norm_kernel, dim3((unsigned)((nmax + 255) / 256)), dim3(256), 0, s, a, na, b, nb, stats, xa,
                     xb);
  const int64_t nl = 2 * L + 1;
  hipLaunchKernelGGL(ncc_lag_kernel, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, xa, na, xb, nb, L, corr);
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
constexpr int DTW_SPIN_LIMIT = 1 << 22;

struct DtwArgs {
  const double* q;
  const double* r;
  int dim, band;
  int64_t nq, nr, nb, S, SW;
  double* Cn;
  uint32_t* Dn;
  uint64_t* E;
  int32_t* sync;   // [0] band ticket, [1] error flag
  uint64_t* trace; // optional [nb][4]: t_start, t_first_edge, t_end, sweep wait ticks (s_memrealtime, 100 MHz)
};

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
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int2 a = __builtin_bit_cast(int2, v);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(a.x, l), __builtin_amdgcn_readlane(a.y, l)));
}
}  // namespace

// Block = 2 + DTW_NDW waves, all coupled through LDS counters (a wave reads data
// only after it has read the count that covers it):
//  wave 0  sweep: the min-chain of every cell, the C / direction / edge stores.  It
//          never loads from global memory (on gfx9 a vmcnt wait would also drain
//          its own Cn stores, ~0.5 us per step), reading distances and the band's
//          top edge from LDS.
//  wave 1  feeder: reference rows into a 256-row LDS ring (32-row blocks, written
//          once the sweep's progress shows the overwritten rows dead) and C[64b][j]
//          polled from E with sc1 loads into an edge ring.
//  wave 2+ distance: 8-step chunks round-robin; the unfused Euclidean distance
//          of every lane's cell into a DTW_DQ-step LDS distance ring.
// The sweep's critical path is then ~20 VALU ops per step instead of ~70, and the
// distance work runs on other SIMDs in parallel.
#ifndef DTW_RROWS_CFG
#define DTW_RROWS_CFG 128
#endif
#ifndef DTW_DQ_CFG
#define DTW_DQ_CFG 32
#endif
constexpr int DTW_RROWS = DTW_RROWS_CFG;   // reference rows in the LDS ring
constexpr int DTW_RBLK = 32;               // rows per ring refill
constexpr int DTW_DQ = DTW_DQ_CFG;         // steps of distances held in LDS
constexpr int DTW_EQ = 256;       // edge values in the LDS ring
constexpr int DTW_EAHEAD = 128;   // the feeder fetches edge columns up to prog + EAHEAD
#ifndef DTW_NDW
#define DTW_NDW 3                 // distance waves per block
#endif

template <int D, bool FAST, bool BANDED>
__global__ __launch_bounds__(64 * (2 + DTW_NDW)) void dtw_band_kernel(DtwArgs a) {
  constexpr int DR = D > 0 ? D : 1;
  __shared__ __attribute__((aligned(16))) double ring[DTW_RROWS * DR];
  __shared__ double dring[DTW_DQ][64];
  __shared__ double eq[DTW_EQ];
  __shared__ double erow[DTW_ECH][64];      // the sweep's last 8 rows of C (lane 63 = the band's edge)
  __shared__ int64_t shb;
  __shared__ int prog, rdy, efill;          // sweep steps done; highest ring block ready; edge columns in eq
  __shared__ int dchunk[DTW_NDW];           // per distance wave: 1 + index of its last finished chunk
#define SONAR_LDS_LD(x) __hip_atomic_load(&(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define SONAR_LDS_ST(x, v) __hip_atomic_store(&(x), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    shb = atomicAdd(&a.sync[0], 1);
    prog = 0; rdy = -1; efill = 0;
    for (int w = 0; w < DTW_NDW; ++w) dchunk[w] = 0;
  }
  __syncthreads();
  const int64_t b = shb;
  if (b >= a.nb) return;
  const int64_t nq = a.nq, nr = a.nr, S = a.S;
  const int dim = D > 0 ? D : a.dim;
  const double inf = __builtin_inf();
  constexpr uint64_t INF_BITS = 0x7FF0000000000000ull;
  const uint64_t* Ein = b > 0 ? a.E + (b - 1) * (nr + 1) : nullptr;       // C[64b][j] at index j
  const int64_t nblk = (nr + DTW_RBLK - 1) / DTW_RBLK;
  const int64_t i = 64 * b + 1 + lane;
  const bool row_ok = i <= nq;
  const int64_t qrow = row_ok ? i - 1 : 0;
  uint64_t spins_total = 0;
  // spin (LDS only) until `cond` holds; bounded, flags the error word instead of hanging
#define SONAR_SPIN_UNTIL(cond)                                                        \
  do {                                                                                \
    uint64_t sp_ = 0;                                                                 \
    if (!(cond)) {                                                                    \
      const uint64_t w0_ = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;            \
      while (!(cond)) {                                                               \
        __builtin_amdgcn_s_sleep(1);                                                  \
        if (++sp_ > (uint64_t)DTW_SPIN_LIMIT * 4) { if (lane == 0) atomicOr(&a.sync[1], 2); break; } \
      }                                                                               \
      if (a.trace) spins_total += __builtin_amdgcn_s_memrealtime() - w0_;             \
    }                                                                                 \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");                            \
  } while (0)

  if (wave == 1) {
    // ------------------------------------------------------------ feeder wave
    int64_t nextblk = 0, have = 0;
    uint64_t idle = 0;
    const int64_t ecols = Ein ? nr : 0;
    while (true) {
      const int64_t p = SONAR_LDS_LD(prog);
      bool work = false;
      if constexpr (D > 0) {
        // block m overwrites block m - RROWS/RBLK, whose last row RBLK*m - RROWS + RBLK - 1 is
        // read (by lane 63) for step row + 63: the sweep has consumed it once prog >= row + 64
        if (nextblk < nblk &&
            (nextblk < DTW_RROWS / DTW_RBLK || p >= DTW_RBLK * nextblk - DTW_RROWS + DTW_RBLK + 63)) {
          if (lane < DTW_RBLK) {
            const int64_t row = DTW_RBLK * nextblk + lane;
            double* dst = ring + (row & (DTW_RROWS - 1)) * D;
#pragma unroll
            for (int k = 0; k < DR; ++k) dst[k] = row < nr ? a.r[row * D + k] : 0.0;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) SONAR_LDS_ST(rdy, (int)nextblk);
          ++nextblk;
          work = true;
        }
      }
      if (have < ecols) {
        const int64_t want = p + DTW_EAHEAD < ecols ? p + DTW_EAHEAD : ecols;
        if (have < want) {
          const int64_t jj = have + 1 + lane;
          uint64_t v = INF_BITS;
          if (jj <= want) v = __hip_atomic_load(Ein + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint64_t bad = __builtin_amdgcn_ballot_w64(jj <= want && v == DTW_SENT);
          const int64_t lim = want - have < 64 ? want - have : 64;
          const int64_t got = bad ? (int64_t)__builtin_ctzll(bad) : lim;   // contiguous ready prefix
          if (lane < got) eq[jj & (DTW_EQ - 1)] = __builtin_bit_cast(double, v);
          if (got > 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            have += got;
            if (lane == 0) SONAR_LDS_ST(efill, (int)have);
            work = true;
          }
        }
      }
      if ((D == 0 || nextblk >= nblk) && have >= ecols) break;
      if (!work) {
        __builtin_amdgcn_s_sleep(1);
        if (++idle > (uint64_t)DTW_SPIN_LIMIT * 4) {   // producer band never arrived: flag, release the rest
          if (lane == 0) { atomicOr(&a.sync[1], 1); SONAR_LDS_ST(efill, (int)ecols); SONAR_LDS_ST(rdy, (int)nblk); }
          break;
        }
      }
    }
    return;
  }

  double qv[DR];
  if constexpr (D > 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) qv[k] = a.q[qrow * D + k];
  }
  // local distance of the lane's cell at step t (EuclideanDistanceFunc order, unfused)
  auto dist = [&](int64_t t) -> double {
    if constexpr (D > 0) {
      const double* rw = ring + ((t - lane) & (DTW_RROWS - 1)) * D;
      double df = qv[0] - rw[0];
      double sum = df * df;                            // 0.0 + x == x for x >= +0 or NaN
#pragma unroll
      for (int k = 1; k < D; ++k) {
        df = qv[k] - rw[k];
        sum = sum + df * df;
      }
      return sqrt(sum);
    } else {
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
    }
  };

  if (wave >= 2) {
    // ---------------------------------------------------------- distance waves
    const int w = wave - 2;
    for (int64_t c = w; DTW_ECH * c < S; c += DTW_NDW) {
      const int64_t t0 = DTW_ECH * c;
      // ring slots of steps t0..t0+7 were last read by the sweep for steps t0-DQ..t0-DQ+7
      SONAR_SPIN_UNTIL(SONAR_LDS_LD(prog) >= t0 + DTW_ECH - DTW_DQ);
      if constexpr (D > 0) {
        const int64_t need = (t0 + DTW_ECH - 1) / DTW_RBLK;             // rows up to t0+7
        const int64_t needc = need < nblk - 1 ? need : nblk - 1;
        SONAR_SPIN_UNTIL(SONAR_LDS_LD(rdy) >= needc);
      }
#pragma unroll
      for (int g0 = 0; g0 < DTW_ECH; g0 += DTW_G) {
        double dv[DTW_G];
#pragma unroll
        for (int u = 0; u < DTW_G; ++u) dv[u] = t0 + g0 + u < S ? dist(t0 + g0 + u) : 0.0;
#pragma unroll
        for (int u = 0; u < DTW_G; ++u) dring[(t0 + g0 + u) & (DTW_DQ - 1)][lane] = dv[u];
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) SONAR_LDS_ST(dchunk[w], (int)(c + 1));
    }
    return;
  }

  // ---------------------------------------------------------------- sweep wave
  const uint64_t t_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t t_first = 0;
  uint64_t* Eout = (b + 1 < a.nb) ? a.E + b * (nr + 1) : nullptr;         // C[64b+64][j]
  double out = inf;                                   // C[i][j-1]; C[i][0] = +Inf
  double up_prev = (lane == 0 && b == 0) ? 0.0 : inf; // C[i-1][j-1]; C[0][0] = 0
  uint32_t dacc = 0;
  const int64_t band = a.band;
  double* Cb = a.Cn + ((b * S) << 6) + lane;
  uint32_t* Db = a.Dn + ((b * a.SW) << 6) + lane;

  // one sweep step: lane l relaxes C[i][s-l+1] with local distance d; l0up = C[64b][s+1]
  // for lane 0.  FULL: every lane's column is in [1, nr] (s in [63, nr-1]), so no
  // per-lane predicate is needed (rows past nq compute values nobody reads).
  auto step = [&](auto full_tag, int s, double l0up, double d, double* cs) -> uint32_t {
    constexpr bool FULL = decltype(full_tag)::value;
    const double up = shr1(out, l0up);               // C[i-1][j]; lane 0 takes l0up's lane 0
    const int j = s - lane + 1;
    const double left = out, dg = up_prev;
    // findPreviousStep: vertical, horizontal, diagonal; strict < (NaN compares false)
    uint32_t code = 0;
    double best = up;
    if (left < best) { code = 1; best = left; }
    if (dg < best) { code = 2; best = dg; }
    if constexpr (!FAST) best = go_min(go_min(up, left), dg);   // math.Min: NaN / -Inf / -0 rules
    double v = d + best;
    if constexpr (BANDED) {
      if (i - j > band || j - i > band) v = inf;      // outside the Sakoe-Chiba band: never filled
    }
    if constexpr (FULL) {
      out = v;
    } else {
      if (row_ok && j >= 1 && j <= nr) out = v;
    }
    *cs = out;
    up_prev = up;
    return code;
  };

  // the band's sweep, specialised on whether it has a band above (edge in) and below (edge out)
  auto sweep = [&](auto ein_tag, auto eout_tag) {
    constexpr bool EIN = decltype(ein_tag)::value, EOUT = decltype(eout_tag)::value;
    for (int s0 = 0; s0 < S; s0 += DTW_ECH) {
      if (lane == 0) SONAR_LDS_ST(prog, s0);           // steps < s0 are done
      const int64_t c = s0 / DTW_ECH;
      SONAR_SPIN_UNTIL(SONAR_LDS_LD(dchunk[c % DTW_NDW]) > c);
      double ech = inf;                                // lane k: C[64b][s0+1+k]; shifted down one lane per step
      if constexpr (EIN) {
        const int need = (int)(s0 + DTW_ECH < nr ? s0 + DTW_ECH : nr);
        SONAR_SPIN_UNTIL(SONAR_LDS_LD(efill) >= need);
        if (a.trace && s0 == 0) t_first = __builtin_amdgcn_s_memrealtime();
        const int64_t jj = s0 + 1 + lane;
        if (lane < DTW_ECH && jj <= nr) ech = eq[jj & (DTW_EQ - 1)];
      }
      double dc[DTW_ECH];
#pragma unroll
      for (int u = 0; u < DTW_ECH; ++u) dc[u] = dring[(s0 + u) & (DTW_DQ - 1)][lane];
      double* cs = Cb + ((int64_t)s0 << 6);
      auto body = [&](auto full_tag) {
#pragma unroll
        for (int u = 0; u < DTW_ECH; ++u) {
          if (decltype(full_tag)::value || s0 + u < S) {
            const uint32_t code = step(full_tag, s0 + u, ech, dc[u], cs + (u << 6));
            dacc |= code << (2 * ((s0 & 8) + u));
            if constexpr (EOUT) erow[u][lane] = out;   // lane 63's value is this band's edge
            if constexpr (EIN) ech = shl1(ech);
          }
        }
      };
      if (s0 >= 63 && s0 + DTW_ECH <= nr) body(std::true_type{});
      else body(std::false_type{});
      if constexpr (EOUT) {                            // one sc1 store of the chunk's 8 edge values
        const int64_t je = (int64_t)s0 + lane - 62;
        if (lane < DTW_ECH && je >= 1 && je <= nr)
          __hip_atomic_store(Eout + je, __builtin_bit_cast(uint64_t, erow[lane & (DTW_ECH - 1)][63]),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if ((s0 & 8) || s0 + DTW_ECH >= S) {             // steps 16w .. 16w+15 complete (or the last one)
        Db[(int64_t)(s0 >> 4) << 6] = dacc;
        dacc = 0;
      }
    }
  };
  if (Ein) {
    if (Eout) sweep(std::true_type{}, std::true_type{});
    else sweep(std::true_type{}, std::false_type{});
  } else {
    if (Eout) sweep(std::false_type{}, std::true_type{});
    else sweep(std::false_type{}, std::false_type{});
  }
  if (lane == 0) SONAR_LDS_ST(prog, (int)S);
#undef SONAR_SPIN_UNTIL
#undef SONAR_LDS_LD
#undef SONAR_LDS_ST
  if (a.trace && lane == 0) {
    a.trace[4 * b + 0] = t_start;
    a.trace[4 * b + 1] = t_first;
    a.trace[4 * b + 2] = __builtin_amdgcn_s_memrealtime();
    a.trace[4 * b + 3] = spins_total;
  }
}

// Single wave: backtrack (dtw.go:165-188) over the 2-bit direction codes.  The walk
// is inherently sequential, so it only emits its own moves (2 bits per step, 16 per
// word, stored 64 words at a time); dtw_path_decode_kernel turns them into points and
// costs in parallel.  Interior steps read lane l's code word of band (i-1)/64 from a
// 16-word register window (s = j-1+l only decreases inside a band, so only the
// lower bound is checked); the next band's window is prefetched on band entry.
// Moves: 0 = vertical (i-1), 1 = horizontal (j-1), 2 = diagonal.
__global__ __launch_bounds__(64) void dtw_walk_kernel(const uint32_t* Dn, int64_t nq, int64_t nr, int64_t SW,
                                                      uint32_t* codes, int64_t* plen) {
  const int lane = threadIdx.x;
  uint32_t win[16], nxt[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { win[k] = 0u; nxt[k] = 0u; }
  int i = (int)nq, j = (int)nr, P = 0;
  int wb = -1, wlo = 0, pb = -1, plo = 0;
  const int sw = (int)SW;
  uint32_t cacc = 0, vacc = 0;
  auto emit = [&](uint32_t code) {
    cacc |= code << (2 * (P & 15));
    ++P;
    if ((P & 15) == 0) {
      const int wi = (P >> 4) - 1;
      vacc = lane == (wi & 63) ? cacc : vacc;
      cacc = 0;
      if ((wi & 63) == 63) codes[wi - 63 + lane] = vacc;
    }
  };
  auto load_win = [&](uint32_t (&dst)[16], int bnd, int lo) {
    const uint32_t* src = Dn + (((int64_t)bnd * sw + lo) << 6) + lane;
#pragma unroll
    for (int k = 0; k < 16; ++k) dst[k] = (lo + k < sw) ? src[k << 6] : 0u;
  };
  while (i > 0 && j > 0) {
    const int l = (i - 1) & 63, bnd = (i - 1) >> 6;
    const int s = j - 1 + l, w = s >> 4;
    if (bnd != wb || w < wlo) {
      if (bnd == pb && w >= plo && w < plo + 16) {     // prefetched on entry to the band below
#pragma unroll
        for (int k = 0; k < 16; ++k) win[k] = nxt[k];
        wlo = plo;
      } else {
        wlo = w - 15 > 0 ? w - 15 : 0;
        load_win(win, bnd, wlo);
        __builtin_amdgcn_s_waitcnt(0x0F70);             // vmcnt(0) here, before the prefetch is issued
      }
      if (bnd != wb && bnd > 0) {                       // the walk enters band bnd-1 at a column <= j
        pb = bnd - 1;
        const int wt = (j - 1 + 63) >> 4;
        plo = wt - 15 > 0 ? wt - 15 : 0;
        load_win(nxt, pb, plo);
      }
      wb = bnd;
    }
    const int kw = __builtin_amdgcn_readfirstlane(w - wlo);      // uniform: keeps the index scalar
    const uint32_t word = __builtin_amdgcn_readlane(win[kw], __builtin_amdgcn_readfirstlane(l));
    const uint32_t code = (word >> ((s & 15) << 1)) & 3u;
    emit(code);
    i -= code != 1u;
    j -= code != 0u;
  }
  while (i > 0 || j > 0) {    // findPreviousStep on the borders: i == 0 -> left, j == 0 -> up
    emit(i == 0 ? 1u : 0u);
    if (i == 0) --j; else --i;
  }
  const int nw = (P + 15) >> 4;
  if (P & 15) vacc = lane == ((nw - 1) & 63) ? cacc : vacc;
  if (nw > 0 && (nw & 63) != 0) {
    const int base = (nw - 1) & ~63;
    if (lane < nw - base) codes[base + lane] = vacc;
  }
  if (lane == 0) *plen = P;
}

namespace {
__device__ __forceinline__ double cn_at(const double* Cn, int64_t S, int64_t i, int64_t j) {
  if (i == 0) return j == 0 ? 0.0 : __builtin_inf();
  if (j == 0) return __builtin_inf();
  const int64_t b = (i - 1) >> 6, l = (i - 1) & 63;
  return Cn[((b * S + (j - 1 + l)) << 6) + l];
}
}  // namespace

// Path points and costs from the walk's moves (dtw.go:165-188): one block; each
// thread replays a contiguous run of moves from the exclusive prefix sum of the
// earlier runs' (di, dj).  Point k of the walk is (i_k - 1, j_k - 1) with cost
// C[i][j] - C[i-1][j-1] (0 on the borders); output is in forward order (index P-1-k).
__global__ __launch_bounds__(1024) void dtw_path_decode_kernel(const uint32_t* codes, int64_t P, int64_t nq,
                                                               int64_t nr, const double* Cn, int64_t S, int32_t* pq,
                                                               int32_t* pr, double* pc) {
  __shared__ int64_t wsum[2][16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t seg = (P + 1023) / 1024;
  const int64_t k0 = t * seg < P ? t * seg : P, k1 = (t + 1) * seg < P ? (t + 1) * seg : P;
  auto code_at = [&](int64_t k) -> uint32_t { return (codes[k >> 4] >> ((k & 15) << 1)) & 3u; };
  int64_t di = 0, dj = 0;
  for (int64_t k = k0; k < k1; ++k) {
    const uint32_t c = code_at(k);
    di += c != 1u;
    dj += c != 0u;
  }
  // block exclusive scan of (di, dj)
  int64_t si = di, sj = dj;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t ui = __shfl_up(si, o, 64), uj = __shfl_up(sj, o, 64);
    if (lane >= o) { si += ui; sj += uj; }
  }
  if (lane == 63) { wsum[0][wv] = si; wsum[1][wv] = sj; }
  __syncthreads();
  int64_t oi = 0, oj = 0;
  for (int w = 0; w < wv; ++w) { oi += wsum[0][w]; oj += wsum[1][w]; }
  int64_t i = nq - (oi + si - di), j = nr - (oj + sj - dj);
  for (int64_t k = k0; k < k1; ++k) {
    const int64_t f = P - 1 - k;
    double c = 0.0;
    if (i > 0 && j > 0) c = __dsub_rn(cn_at(Cn, S, i, j), cn_at(Cn, S, i - 1, j - 1));
    pq[f] = (int32_t)(i - 1); pr[f] = (int32_t)(j - 1); pc[f] = c;
    const uint32_t m = code_at(k);
    i -= m != 1u;
    j -= m != 0u;
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
    if (s < S && col >= 0 && col < 64) tile[lane][col] = Cn[((b * S + s) << 6) + lane];
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

DtwGeom dtw_geom(int64_t nq, int64_t nr) {
  DtwGeom g;
  g.nq = nq; g.nr = nr;
  g.nb = (nq + 63) / 64;
  g.S = nr + 63;
  g.SW = (g.S + 15) / 16;
  return g;
}
size_t dtw_cn_bytes(const DtwGeom& g) { return (size_t)g.nb * g.S * 64 * 8; }
size_t dtw_dn_bytes(const DtwGeom& g) { return (size_t)g.nb * g.SW * 64 * 4; }
size_t dtw_edge_bytes(const DtwGeom& g) { return (size_t)(g.nb > 1 ? g.nb - 1 : 1) * (g.nr + 1) * 8; }
int64_t dtw_cn_index(const DtwGeom& g, int64_t i, int64_t j) {
  const int64_t b = (i - 1) >> 6, l = (i - 1) & 63;
  return ((b * g.S + (j - 1 + l)) << 6) + l;
}

int launch_dtw(const double* q, const double* r, int dim, int band, bool fast, const DtwGeom& g, double* Cn,
               uint32_t* Dn, uint64_t* E, int32_t* sync_words, uint32_t* codes, int64_t* plen, uint64_t* trace,
               hipStream_t s) {
  if (hipMemsetAsync(sync_words, 0, 2 * sizeof(int32_t), s) != hipSuccess) return -5;
  if (g.nb > 1 && hipMemsetD32Async((hipDeviceptr_t)E, 0x7FF00001u, dtw_edge_bytes(g) / 4, s) != hipSuccess) return -5;
  DtwArgs a{q, r, dim, band, g.nq, g.nr, g.nb, g.S, g.SW, Cn, Dn, reinterpret_cast<uint64_t*>(E), sync_words,
            trace};
  const dim3 grid((unsigned)g.nb), block(64 * (2 + DTW_NDW));
#define SONAR_DTW_LAUNCH(DD)                                                                          \
  do {                                                                                                \
    if (band > 0) {                                                                                   \
      if (fast) hipLaunchKernelGGL((dtw_band_kernel<DD, true, true>), grid, block, 0, s, a);          \
      else hipLaunchKernelGGL((dtw_band_kernel<DD, false, true>), grid, block, 0, s, a);              \
    } else {                                                                                          \
      if (fast) hipLaunchKernelGGL((dtw_band_kernel<DD, true, false>), grid, block, 0, s, a);         \
      else hipLaunchKernelGGL((dtw_band_kernel<DD, false, false>), grid, block, 0, s, a);             \
    }                                                                                                 \
  } while (0)
  if (dim == 12) SONAR_DTW_LAUNCH(12);
  else if (dim == 1) SONAR_DTW_LAUNCH(1);
  else SONAR_DTW_LAUNCH(0);
#undef SONAR_DTW_LAUNCH
  hipLaunchKernelGGL(dtw_walk_kernel, dim3(1), dim3(64), 0, s, Dn, g.nq, g.nr, g.SW, codes, plen);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_dtw_path_cost(const double* Cn, const DtwGeom& g, const uint32_t* codes, int64_t P, int32_t* pq,
                         int32_t* pr, double* pc, hipStream_t s) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(dtw_path_decode_kernel, dim3(1), dim3(1024), 0, s, codes, P, g.nq, g.nr, Cn, g.S, pq, pr, pc);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_dtw_cost_rowmajor(const double* Cn, const DtwGeom& g, double* out, hipStream_t s) {
  const dim3 grid((unsigned)((g.nr + 63) / 64), (unsigned)g.nb);
  hipLaunchKernelGGL(dtw_cost_rowmajor_kernel, grid, dim3(256), 0, s, Cn, g.nq, g.nr, g.S, out);
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
