// compare_kernels.hip -- FingerprintComparator (fingerprint/comparison.go) on a device gallery.
//
// Three stages, all float64 like the reference:
//   colstats_*      per-fingerprint statistics (gonum stat.Mean / corrected two-pass
//                   stat.Variance) of the MFCC columns, chroma columns and the compared
//                   sequences, reduced over row chunks in a fixed order (deterministic);
//                   HBM-bound streaming of the feature arrays, once per fingerprint.
//   coherence       gonum stat.Correlation of SpectralCentroid / SpectralRolloff for each
//                   pair (EnableDetailedMetrics only, comparison.go:977-1008): one block per
//                   (pair, sequence) streams both sequences.
//   compare         one thread per (query, candidate): calculateFeatureSimilarity and the
//                   scorers over two gallery records (comparison.go:133-194, 266-402,
//                   646-1037); a few hundred float64 operations per pair.
// FindBestMatches adds two stable device-wide radix sorts (hipCUB) of the per-pair keys.
// Built with -ffp-contract=off: Go on amd64 rounds every product and sum separately.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>

#include "kernels.h"

namespace sonar {
namespace {

constexpr int kBlock = 256;

// ---- Go math helpers (NaN behaviour of math.Max / math.Min) ---------------------------
__device__ __forceinline__ double go_max(double x, double y) {
  if (isinf(x) && x > 0) return x;
  if (isinf(y) && y > 0) return y;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? y : x;
  return x > y ? x : y;
}
__device__ __forceinline__ double go_min(double x, double y) {
  if (isinf(x) && x < 0) return x;
  if (isinf(y) && y < 0) return y;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? x : y;
  return x < y ? x : y;
}

// gonum floats.Norm(x, 2) = f64.L2NormUnitary: scaled sum of squares
__device__ double l2norm(const double* x, int n) {
  double scale = 0.0, ss = 1.0;
  for (int i = 0; i < n; i++) {
    const double v = x[i];
    if (v == 0.0) continue;
    const double a = fabs(v);
    if (isnan(a)) return NAN;
    if (scale < a) {
      const double s = scale / a;
      ss = 1.0 + ss * s * s;
      scale = a;
    } else {
      const double s = a / scale;
      ss += s * s;
    }
  }
  if (isinf(scale)) return INFINITY;
  return scale * sqrt(ss);
}

// cosineSimilarity (comparison.go:858-873)
__device__ double cosine(const double* a, int na, const double* b, int nb) {
  if (na != nb || na == 0) return 0.0;
  double dot = 0.0;
  for (int i = 0; i < na; i++) dot += a[i] * b[i];
  const double n1 = l2norm(a, na), n2 = l2norm(b, nb);
  if (n1 == 0 || n2 == 0) return 0.0;
  return dot / (n1 * n2);
}

// compareSequenceStats (:827-842): cosine of (mean, std)
__device__ double seq_sim(const FpRec& A, const FpRec& B, int s) {
  const double a[2] = {A.seq_mean[s], A.seq_std[s]}, b[2] = {B.seq_mean[s], B.seq_std[s]};
  return cosine(a, 2, b, 2);
}

// compareScalarFeatures (:844-856)
__device__ double scalar_sim(double v1, double v2) {
  if (v1 == 0 && v2 == 0) return 1.0;
  const double mx = go_max(fabs(v1), fabs(v2));
  if (mx == 0) return 1.0;
  return go_max(0.0, 1.0 - fabs(v1 - v2) / mx);
}

__device__ double mean_of(const double* v, int n) {   // stat.Mean(v, nil) = floats.Sum / n
  double s = 0.0;
  for (int i = 0; i < n; i++) s += v[i];
  return s / (double)n;
}

// ---- column statistics ----------------------------------------------------------------
// One pass over HBM: a block owns a chunk of rows, holds its kRegs values per thread in
// registers, and writes the chunk's column sums and its corrected two-pass M2 around the
// chunk mean (ss - comp^2 / n_k, gonum's form).  The final kernel merges the chunks
// (Chan et al.: M2 = sum_k M2_k + n_k (mean_k - mean)^2): the same quantity as gonum's
// corrected two-pass variance over the whole column, rounded differently (~1e-16 rel.).
// Thread layout for cols <= 256: 256 / cols rows per step, thread t owns column t % cols
// (each step's reads are one contiguous run); wider matrices: thread t owns columns t,
// t + 256, ... and reads the chunk's rows twice (L2-resident).
constexpr int kRegs = 16;

__host__ __device__ inline int64_t colstats_chunk_rows(int cols) {
  return cols <= kBlock ? (int64_t)(kBlock / cols) * kRegs : kRegs;
}

__device__ double block_sum(double v, double* s_v) {
  s_v[threadIdx.x] = v;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_v[threadIdx.x] += s_v[threadIdx.x + w];
    __syncthreads();
  }
  const double r = s_v[0];
  __syncthreads();
  return r;
}

// Chunk merge (own launch, one block per job): mean = Sum / n; variance = M2 / (n - 1)
// (n = 1 -> 0 / 0 = NaN, as gonum).  All columns at once with the chunk kernel's thread
// layout; fixed thread assignment + fixed-order sums (deterministic).  A fused "last block
// merges" variant needs agent-scope release fences, which write back the XCD's L2 per block
// and measured 20x slower.
__device__ void colstats_merge(const StatJob& J, const double* part_sum, const double* part_m2, double* s_a) {
  const int C = J.cols, t = threadIdx.x;
  const double n = (double)J.rows;
  auto nk_of = [&](int q) {
    return (double)(min(J.rows, (int64_t)(q + 1) * J.chunk_rows) - (int64_t)q * J.chunk_rows);
  };
  if (C <= kBlock) {
    const int rpi = kBlock / C, active = rpi * C, c = t % C, g = t / C;
    double s = 0.0;
    if (t < active)
      for (int q = g; q < J.nchunks; q += rpi) s += part_sum[J.part_off + (int64_t)q * C + c];
    s_a[t] = s;
    __syncthreads();
    double tot = 0.0;
    for (int q = 0; q < rpi; q++) tot += s_a[c + q * C];
    const double mean = tot / n;
    __syncthreads();
    double m2 = 0.0;
    if (t < active)
      for (int q = g; q < J.nchunks; q += rpi) {
        const int64_t o = J.part_off + (int64_t)q * C + c;
        const double nk = nk_of(q), dm = part_sum[o] / nk - mean;
        m2 += part_m2[o] + nk * dm * dm;
      }
    s_a[t] = m2;
    __syncthreads();
    if (t < C) {
      double mm = 0.0;
      for (int q = 0; q < rpi; q++) mm += s_a[t + q * C];
      J.out_mean[t] = mean;
      if (J.out_std) J.out_std[t] = sqrt(mm / (n - 1.0));
    }
  } else {
    for (int c = 0; c < C; c++) {
      double s = 0.0;
      for (int q = t; q < J.nchunks; q += kBlock) s += part_sum[J.part_off + (int64_t)q * C + c];
      const double mean = block_sum(s, s_a) / n;
      double m2 = 0.0;
      for (int q = t; q < J.nchunks; q += kBlock) {
        const int64_t o = J.part_off + (int64_t)q * C + c;
        const double nk = nk_of(q), dm = part_sum[o] / nk - mean;
        m2 += part_m2[o] + nk * dm * dm;
      }
      m2 = block_sum(m2, s_a);
      if (t == 0) {
        J.out_mean[c] = mean;
        if (J.out_std) J.out_std[c] = sqrt(m2 / (n - 1.0));
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void colstats_kernel(const StatJob* jobs, const int* chunk_job,
                                                          const int* chunk_k, double* part_sum, double* part_m2) {
  __shared__ double s_a[kBlock], s_b[kBlock];
  const StatJob J = jobs[chunk_job[blockIdx.x]];
  const int k = chunk_k[blockIdx.x];
  const int C = J.cols, t = threadIdx.x;
  const int64_t r0 = (int64_t)k * J.chunk_rows, r1 = min(J.rows, r0 + J.chunk_rows);
  const double nk = (double)(r1 - r0);
  if (C <= kBlock) {
    const int rpi = kBlock / C, active = rpi * C, c = t % C;
    double v[kRegs];
    double a = 0.0;
#pragma unroll
    for (int i = 0; i < kRegs; i++) {
      const int64_t r = r0 + t / C + (int64_t)i * rpi;
      v[i] = (t < active && r < r1) ? J.src[r * C + c] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < kRegs; i++) a += v[i];
    s_a[t] = a;
    __syncthreads();
    double sum = 0.0;                                   // chunk column sum, fixed order
    for (int q = 0; q < rpi; q++) sum += s_a[c + q * C];
    const double mu = sum / nk;
    double ss = 0.0, comp = 0.0;
#pragma unroll
    for (int i = 0; i < kRegs; i++) {
      const int64_t r = r0 + t / C + (int64_t)i * rpi;
      if (t < active && r < r1) {
        const double d = v[i] - mu;
        ss += d * d;
        comp += d;
      }
    }
    __syncthreads();
    s_a[t] = ss;
    s_b[t] = comp;
    __syncthreads();
    if (t < C) {
      double sss = 0.0, sc = 0.0;
      for (int q = 0; q < rpi; q++) { sss += s_a[t + q * C]; sc += s_b[t + q * C]; }
      const int64_t o = J.part_off + (int64_t)k * C + t;
      part_sum[o] = sum;
      part_m2[o] = sss - sc * sc / nk;
    }
  } else {
    for (int c = t; c < C; c += kBlock) {
      double sum = 0.0;
      for (int64_t r = r0; r < r1; r++) sum += J.src[r * C + c];
      const double mu = sum / nk;
      double ss = 0.0, comp = 0.0;
      for (int64_t r = r0; r < r1; r++) {
        const double d = J.src[r * C + c] - mu;
        ss += d * d;
        comp += d;
      }
      const int64_t o = J.part_off + (int64_t)k * C + c;
      part_sum[o] = sum;
      part_m2[o] = ss - comp * comp / nk;
    }
  }
}

__global__ __launch_bounds__(kBlock) void colstats_final_kernel(const StatJob* jobs, const double* part_sum,
                                                                const double* part_m2) {
  __shared__ double s_a[kBlock];
  colstats_merge(jobs[blockIdx.x], part_sum, part_m2, s_a);
}

// ---- spectral coherence ----------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void coherence_kernel(const FpRec* recs, const int64_t* q_idx,
                                                           const int64_t* c_idx, int64_t nc, double* coh) {
  __shared__ double s_v[5][kBlock];
  const int64_t pair = blockIdx.x >> 1;
  const int seq = blockIdx.x & 1;             // 0 centroid, 1 rolloff
  const FpRec& A = recs[q_idx[pair / nc]];
  const FpRec& B = recs[c_idx ? c_idx[pair % nc] : pair % nc];
  const int s = seq ? SEQ_ROLLOFF : SEQ_CENTROID;
  const bool both = (A.present & B.present & SONAR_FEAT_SPECTRAL) && A.seq_len[s] > 0 && B.seq_len[s] > 0;
  if (!both) {                                // not compared: no coherence entry
    if (threadIdx.x == 0) coh[2 * pair + seq] = NAN;
    return;
  }
  const double* x = seq ? A.rolloff : A.centroid;
  const double* y = seq ? B.rolloff : B.centroid;
  const int64_t n = A.seq_len[s];             // == B.seq_len[s], checked on the host
  const double xu = A.seq_mean[s], yu = B.seq_mean[s];
  double sxx = 0.0, syy = 0.0, sxy = 0.0, xc = 0.0, yc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) {
    const double xd = x[i] - xu, yd = y[i] - yu;
    sxx += xd * xd;
    syy += yd * yd;
    sxy += xd * yd;
    xc += xd;
    yc += yd;
  }
  s_v[0][threadIdx.x] = sxx; s_v[1][threadIdx.x] = syy; s_v[2][threadIdx.x] = sxy;
  s_v[3][threadIdx.x] = xc; s_v[4][threadIdx.x] = yc;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w)
      for (int v = 0; v < 5; v++) s_v[v][threadIdx.x] += s_v[v][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double nn = (double)n;
    double a = s_v[0][0], b = s_v[1][0], c = s_v[2][0];
    const double xcs = s_v[3][0], ycs = s_v[4][0];
    a -= xcs * xcs / nn;
    b -= ycs * ycs / nn;
    c -= xcs * ycs / nn;
    coh[2 * pair + seq] = c / sqrt(a * b);
  }
}

// ---- compare ---------------------------------------------------------------------------
__device__ __forceinline__ sonar_similarity compare_pair(const CompareArgs& a, const FpRec& A, const FpRec& B,
                                                         int64_t pair) {
  sonar_similarity r;
  r.overall_similarity = 0.0;
  r.feature_similarity = 0.0;
  r.confidence = 0.0;
  for (int i = 0; i < 6; i++) r.feature_distances[i] = 0.0;
  r.data_availability = r.feature_coverage = r.temporal_alignment = 0.0;
  r.noise_level = r.dynamic_range_match = r.spectral_coherence = 0.0;
  r.distance_mask = 0;
  r.has_quality = 0;
  r.status = (A.id == B.id) ? 1 : 0;
  r.content_type_match = A.ct == B.ct;
  if (a.content_filter && !r.content_type_match) {          // :160-166
    r.confidence = 0.25;
    return r;
  }
  // calculateFeatureSimilarity (:266-341)
  double fs = 0.0;
  if ((A.present & B.present & SONAR_FEAT_FEATURES) == 0) {
    r.status = r.status ? r.status : 2;                       // "features cannot be nil"
  } else {
    double sims[6], ws[6];
    int n = 0;
    auto add = [&](int key, double sim) {
      sims[n] = sim;
      ws[n] = A.w[key];                                       // weights of fp1 (:282)
      n++;
      r.feature_distances[key] = 1.0 - sim;
      r.distance_mask |= 1u << key;
    };
    if (A.mfcc_frames > 0 && B.mfcc_frames > 0) {             // compareMFCC (:344-402)
      double sim = 0.0;
      if (A.mfcc_C > 0 && B.mfcc_C > 0)
        sim = cosine(a.pool + A.mfcc_off, 2 * A.mfcc_C, a.pool + B.mfcc_off, 2 * B.mfcc_C);
      add(SONAR_FD_MFCC, sim);
    }
    if (A.present & B.present & SONAR_FEAT_SPECTRAL) {        // compareSpectralFeatures (:646-671)
      double v[3];
      int m = 0;
      for (int s = SEQ_CENTROID; s <= SEQ_FLUX; s++)
        if (A.seq_len[s] > 0 && B.seq_len[s] > 0) v[m++] = seq_sim(A, B, s);
      add(SONAR_FD_SPECTRAL, m ? mean_of(v, m) : 0.0);
    }
    if (A.chroma_frames > 0 && B.chroma_frames > 0) {         // compareChromaFeatures (:673-688)
      double sim = 0.0;
      if (A.chroma_B > 0 && B.chroma_B > 0)
        sim = cosine(a.pool + A.chroma_off, A.chroma_B, a.pool + B.chroma_off, B.chroma_B);
      add(SONAR_FD_CHROMA, sim);
    }
    if (A.present & B.present & SONAR_FEAT_TEMPORAL) {        // compareTemporalFeatures (:690-719)
      double v[4];
      int m = 0;
      if (A.dynamic_range > 0 && B.dynamic_range > 0) v[m++] = scalar_sim(A.dynamic_range, B.dynamic_range);
      v[m++] = scalar_sim(A.silence_ratio, B.silence_ratio);
      if (A.onset_density > 0 && B.onset_density > 0) v[m++] = scalar_sim(A.onset_density, B.onset_density);
      if (A.seq_len[SEQ_RMS] > 0 && B.seq_len[SEQ_RMS] > 0) v[m++] = seq_sim(A, B, SEQ_RMS);
      add(SONAR_FD_TEMPORAL, mean_of(v, m));
    }
    if (A.present & B.present & SONAR_FEAT_SPEECH) {          // compareSpeechFeatures (:721-747)
      double v[3];
      int m = 0;
      if (A.speech_rate > 0 && B.speech_rate > 0) v[m++] = scalar_sim(A.speech_rate, B.speech_rate);
      if (A.vtl > 0 && B.vtl > 0) v[m++] = scalar_sim(A.vtl, B.vtl);
      if (A.seq_len[SEQ_VOICING] > 0 && B.seq_len[SEQ_VOICING] > 0) v[m++] = seq_sim(A, B, SEQ_VOICING);
      add(SONAR_FD_SPEECH, m ? mean_of(v, m) : 0.0);
    }
    if (A.present & B.present & SONAR_FEAT_HARMONIC) {        // compareHarmonicFeatures (:749-770)
      double v[2];
      int m = 0;
      if (A.seq_len[SEQ_HARMONIC] > 0 && B.seq_len[SEQ_HARMONIC] > 0) v[m++] = seq_sim(A, B, SEQ_HARMONIC);
      if (A.seq_len[SEQ_PITCH] > 0 && B.seq_len[SEQ_PITCH] > 0) v[m++] = seq_sim(A, B, SEQ_PITCH);
      add(SONAR_FD_HARMONIC, m ? mean_of(v, m) : 0.0);
    }
    if (n == 0) {
      r.status = r.status ? r.status : 2;                     // "no comparable features found"
    } else {                                                  // stat.Mean(values, weights)
      double sv = 0.0, sw = 0.0;
      for (int i = 0; i < n; i++) { sv += ws[i] * sims[i]; sw += ws[i]; }
      fs = sv / sw;
    }
  }
  r.feature_similarity = fs;
  r.overall_similarity = fs;                                  // calculateOverallSimilarity (:886-889)
  const int nd = __popc(r.distance_mask);
  if (a.detailed) {                                           // calculateQualityMetrics (:892-936)
    r.has_quality = 1;
    const uint32_t both = A.present & B.present;
    const int avail = ((both & SONAR_FEAT_MFCC) != 0) + ((both & SONAR_FEAT_SPECTRAL) != 0) +
                      ((both & SONAR_FEAT_CHROMA) != 0) + ((both & SONAR_FEAT_TEMPORAL) != 0) +
                      ((both & SONAR_FEAT_SPEECH) != 0) + ((both & SONAR_FEAT_HARMONIC) != 0);
    r.data_availability = (double)avail / 6.0;
    r.feature_coverage = (double)nd / 6.0;
    const double dd = fabs(A.duration - B.duration), md = go_max(A.duration, B.duration);
    r.temporal_alignment = md > 0 ? 1.0 - go_min(1.0, dd / md) : 1.0;
    // estimateNoiseLevel (:939-958); FeatureDistances in key order (a Go map has none)
    if (nd == 0) {
      r.noise_level = 0.5;
    } else if (nd <= 1) {
      r.noise_level = 0.0;
    } else {
      double v[6];
      int m = 0;
      for (int key = 0; key < 6; key++)
        if (r.distance_mask & (1u << key)) v[m++] = 1.0 - r.feature_distances[key];
      const double mu = mean_of(v, m);
      double ss = 0.0, comp = 0.0;
      for (int i = 0; i < m; i++) {
        const double d = v[i] - mu;
        ss += d * d;
        comp += d;
      }
      const double var = (ss - comp * comp / (double)m) / (double)(m - 1);
      r.noise_level = go_min(1.0, sqrt(var));
    }
    // calculateDynamicRangeMatch (:961-974)
    if (!(both & SONAR_FEAT_TEMPORAL) || A.dynamic_range <= 0 || B.dynamic_range <= 0)
      r.dynamic_range_match = 0.5;
    else
      r.dynamic_range_match = scalar_sim(A.dynamic_range, B.dynamic_range);
    // calculateSpectralCoherence (:977-1008)
    if (!(both & SONAR_FEAT_SPECTRAL)) {
      r.spectral_coherence = 0.5;
    } else {
      double v[2];
      int m = 0;
      for (int s = 0; s < 2; s++) {
        const double c = a.coh[2 * pair + s];
        if (!isnan(c)) v[m++] = fabs(c);
      }
      r.spectral_coherence = m ? mean_of(v, m) : 0.5;
    }
  }
  // calculateConfidence (:1011-1037)
  double conf = 0.5;
  if (r.overall_similarity > 0.8) conf += 0.3;
  else if (r.overall_similarity > 0.6) conf += 0.2;
  if (r.content_type_match) conf += 0.1;
  conf += (double)nd * 0.05;
  if (r.has_quality) {
    conf += r.data_availability * 0.1;
    conf -= r.noise_level * 0.1;
  }
  r.confidence = go_max(0.0, go_min(1.0, conf));
  return r;
}

// Thread = pair (q * nc + c).  The records are written through LDS so that a block stores
// its 256 x 136 B of results as one contiguous run of 16-B stores (a per-thread struct store
// is 17 scattered 8-B stores, one cache line per lane each).
__global__ __launch_bounds__(kBlock) void compare_kernel(CompareArgs a) {
  __shared__ __attribute__((aligned(16))) sonar_similarity s_out[kBlock];
  const int64_t n = a.nq * a.nc, p0 = (int64_t)blockIdx.x * kBlock, pair = p0 + threadIdx.x;
  if (pair < n) {
    const int64_t qi = a.q_idx[pair / a.nc];
    const int64_t ci = a.c_idx ? a.c_idx[pair % a.nc] : pair % a.nc;
    s_out[threadIdx.x] = compare_pair(a, a.recs[qi], a.recs[ci], pair);
  }
  __syncthreads();
  const int64_t cnt = min((int64_t)kBlock, n - p0);
  const int words = (int)(cnt * sizeof(sonar_similarity) / 16);     // 136 B = 8.5 x 16 B
  const float4* src = reinterpret_cast<const float4*>(s_out);
  float4* dst = reinterpret_cast<float4*>(a.out + p0);
  for (int i = threadIdx.x; i < words; i += kBlock) dst[i] = src[i];
  if ((cnt & 1) && threadIdx.x == 0) {                                // odd count: trailing 8 B
    const double* s8 = reinterpret_cast<const double*>(s_out);
    double* d8 = reinterpret_cast<double*>(a.out + p0);
    const int last = (int)(cnt * sizeof(sonar_similarity) / 8) - 1;
    d8[last] = s8[last];
  }
}

// ---- FindBestMatches ---------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void match_keys_kernel(const sonar_similarity* sims, int64_t nq, int64_t nc,
                                                            double thr, double* keys, int64_t* vals,
                                                            uint8_t* pass_flag) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nq * nc) return;
  const sonar_similarity& s = sims[i];
  const bool pass = s.status != 1 && s.overall_similarity >= thr;   // :218 self skip, :232 threshold
  keys[i] = pass ? s.overall_similarity : -INFINITY;
  vals[i] = i;                                                      // pair index q * nc + c
  pass_flag[i] = pass;
}

// matches per query: one block per query, fixed-order tree sum (no atomics)
__global__ __launch_bounds__(kBlock) void match_count_kernel(const uint8_t* pass_flag, int64_t nc, int64_t* counts) {
  __shared__ int64_t s_c[kBlock];
  const uint8_t* f = pass_flag + (int64_t)blockIdx.x * nc;
  int64_t c = 0;
  for (int64_t i = threadIdx.x; i < nc; i += kBlock) c += f[i];
  s_c[threadIdx.x] = c;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) s_c[threadIdx.x] += s_c[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) counts[blockIdx.x] = s_c[0];
}

__device__ int classify(double s) {                                  // classifyMatch (:1040-1052)
  if (s >= 0.95) return SONAR_MATCH_EXACT;
  if (s >= 0.85) return SONAR_MATCH_VERY_SIMILAR;
  if (s >= 0.75) return SONAR_MATCH_SIMILAR;
  if (s >= 0.6) return SONAR_MATCH_SOMEWHAT_SIMILAR;
  return SONAR_MATCH_WEAK;
}

__global__ __launch_bounds__(kBlock) void match_gather_kernel(const sonar_similarity* sims, const int64_t* vals,
                                                              const int64_t* counts, int64_t nq, int64_t nc, int K,
                                                              sonar_match* out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nq * (int64_t)K) return;
  const int64_t q = i / K, k = i % K;
  if (k >= counts[q]) return;
  const int64_t c = vals[q * nc + k] % nc;
  sonar_match m;
  m.candidate = c;
  m.rank = (int32_t)k + 1;
  m.similarity = sims[q * nc + c];
  m.match_type = classify(m.similarity.overall_similarity);
  out[i] = m;
}

__global__ __launch_bounds__(kBlock) void pair_query_kernel(const int64_t* pairs, int64_t n, int64_t nc,
                                                            int32_t* q) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) q[i] = (int32_t)(pairs[i] / nc);
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

int64_t colstats_chunk_rows_for(int cols) { return colstats_chunk_rows(cols); }

int launch_colstats(const StatJob* jobs, int njobs, const int* chunk_job, const int* chunk_k, int nchunks,
                    double* part_sum, double* part_m2, hipStream_t s) {
  if (njobs == 0) return 0;
  hipLaunchKernelGGL(colstats_kernel, dim3(nchunks), dim3(kBlock), 0, s, jobs, chunk_job, chunk_k, part_sum, part_m2);
  hipLaunchKernelGGL(colstats_final_kernel, dim3(njobs), dim3(kBlock), 0, s, jobs, part_sum, part_m2);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_coherence(const FpRec* recs, const int64_t* q_idx, int64_t nq, const int64_t* c_idx, int64_t nc,
                     double* coh, hipStream_t s) {
  const int64_t nb = 2 * nq * nc;
  if (nb == 0) return 0;
  if (nb > 0x7fffffff) return -1;
  hipLaunchKernelGGL(coherence_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, recs, q_idx, c_idx, nc, coh);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_compare(const CompareArgs& a, hipStream_t s) {
  const int64_t n = a.nq * a.nc;
  if (n == 0) return 0;
  if (blocks(n) > 0x7fffffffu) return -1;
  hipLaunchKernelGGL(compare_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_match_keys(const sonar_similarity* sims, int64_t nq, int64_t nc, double threshold, double* keys,
                      int64_t* vals, uint8_t* pass_flag, int64_t* counts, hipStream_t s) {
  const int64_t n = nq * nc;
  if (nq == 0) return 0;
  if (n > 0)
    hipLaunchKernelGGL(match_keys_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, sims, nq, nc, threshold, keys, vals,
                       pass_flag);
  hipLaunchKernelGGL(match_count_kernel, dim3((unsigned)nq), dim3(kBlock), 0, s, pass_flag, nc, counts);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Per-query descending order in two stable device-wide radix sorts (LSD): by similarity
// (descending), then by query index -- every query keeps its candidates' similarity order and,
// for equal similarities, candidate order.  (A segmented sort would give each query one block.)
int sort_match_keys(const double* keys, double* keys2, const int64_t* vals, int64_t* vals2, int64_t* vals3,
                    int32_t* qk, int32_t* qk2, int64_t nq, int64_t nc, void* temp, size_t* temp_bytes,
                    hipStream_t s) {
  const int n = (int)(nq * nc);
  int qbits = 1;
  while ((int64_t(1) << qbits) < nq) qbits++;
  if (!temp) {
    size_t a = 0, b = 0;
    if (hipcub::DeviceRadixSort::SortPairsDescending(nullptr, a, keys, keys2, vals, vals2, n, 0, 64, s) !=
            hipSuccess ||
        hipcub::DeviceRadixSort::SortPairs(nullptr, b, qk, qk2, vals2, vals3, n, 0, qbits, s) != hipSuccess)
      return -1;
    *temp_bytes = a > b ? a : b;
    return 0;
  }
  size_t tb = *temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairsDescending(temp, tb, keys, keys2, vals, vals2, n, 0, 64, s) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(pair_query_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, vals2, (int64_t)n, nc, qk);
  tb = *temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(temp, tb, qk, qk2, vals2, vals3, n, 0, qbits, s) != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_match_gather(const sonar_similarity* sims, const int64_t* vals_sorted, const int64_t* counts,
                        int64_t nq, int64_t nc, int K, sonar_match* out, hipStream_t s) {
  const int64_t n = nq * (int64_t)K;
  if (n == 0) return 0;
  hipLaunchKernelGGL(match_gather_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, sims, vals_sorted, counts, nq, nc, K,
                     out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace sonar
