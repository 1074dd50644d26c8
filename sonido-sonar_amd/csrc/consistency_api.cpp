// consistency_api.cpp -- the two steps after the alignment path:
//
//   sonar_alignment_consistency   AlignmentAnalyzer.AnalyzeAlignmentConsistency
//                                 (algorithms/stats/alignment.go:709-800)
//   sonar_truncate_to_alignment   AlignmentExtractor.TruncateToAlignmentPCM
//                                 (fingerprint/extractors/alignment.go:223-297)
//
// The perturbation of the query (addNoise, :737-749) and the alignment itself (NCC / DTW kernels
// through sonar_ncc / sonar_dtw on device buffers) run on the GPU; the offset statistics and the
// truncation arithmetic are O(1) host epilogues, as in Go.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"
#include "host_dsp.h"
#include "kernels.h"

using sonar::detail::dbuf;
using sonar::detail::fail;

extern "C" {

int sonar_alignment_consistency(sonar_ctx* c, const double* query, int64_t nq, const double* reference, int64_t nr,
                                int32_t dim, int32_t method, int32_t max_lag, int32_t hop, int32_t sample_rate,
                                int32_t num_trials, sonar_alignment_stats* out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  std::memset(out, 0, sizeof(*out));
  if (num_trials < 2) num_trials = 5;                                 // :711-713
  // every trial fails in Go for an empty input or a method AlignFeatures does not support
  // (:85-87, :104-105); the analysis then reports no successful alignments (:730-732)
  const bool ok_method = method == SONAR_ALIGN_DTW || method == SONAR_ALIGN_XCORR || method == SONAR_ALIGN_HYBRID;
  if (nq <= 0 || nr <= 0 || !query || !reference || dim <= 0 || !ok_method)
    return fail(c, SONAR_ERR_INVALID, "no successful alignments");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  double* dq = (double*)dbuf(c, "cons.q", nq * dim * 8);
  double* dqp = (double*)dbuf(c, "cons.qp", nq * dim * 8);
  double* dr = (double*)dbuf(c, "cons.r", nr * dim * 8);
  if (!dq || !dqp || !dr) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  HIP_TRY(c, hipMemcpyAsync(dq, query, nq * dim * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(dr, reference, nr * dim * 8, hipMemcpyHostToDevice, s));
  if (sonar::launch_perturb(dq, nq, dim, 0.01, dqp, s) != 0) return fail(c, SONAR_ERR_DEVICE, "perturb launch failed");

  // AlignFeatures(perturbedQuery, reference, sampleRate) (:84-106), the offset it returns
  int64_t offset = 0;
  bool have_corr = false;
  double corr_conf = 0.0;
  if (method == SONAR_ALIGN_XCORR || method == SONAR_ALIGN_HYBRID) {   // alignWithCrossCorrelation :151-181
    double* q0 = (double*)dbuf(c, "cons.q0", nq * 8);
    double* r0 = (double*)dbuf(c, "cons.r0", nr * 8);
    if (!q0 || !r0) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    if (sonar::launch_first_column(dqp, nq, dim, q0, s) != 0 || sonar::launch_first_column(dr, nr, dim, r0, s) != 0)
      return fail(c, SONAR_ERR_DEVICE, "flatten launch failed");
    int64_t L = std::max<int64_t>(0, std::min<int64_t>({(int64_t)max_lag, nq - 1, nr - 1}));
    double* dcorr = (double*)dbuf(c, "cons.corr", (2 * L + 1) * 8);
    if (!dcorr) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    double met[10];
    const int rc = sonar_ncc(c, q0, nq, r0, nr, max_lag, dcorr, met, 1);
    if (rc != SONAR_OK) return rc;
    sonar::host::NccMetrics m;
    m.peak_corr = met[0]; m.peak_lag = (int64_t)met[1]; m.peak_index = (int64_t)met[2]; m.p_value = met[3];
    m.snr = met[4]; m.sharpness = met[5]; m.second_peak = met[6]; m.psl = met[7]; m.overlap = (int64_t)met[8];
    m.num_lags = (int64_t)met[9];
    const auto sc = sonar::host::xcorr_scores(m, hop, sample_rate, max_lag);
    offset = sc.offset;
    corr_conf = sc.confidence;
    have_corr = true;
  }
  // alignWithHybrid (:308-337): DTW only when the correlation confidence is <= 0.7; the DTW
  // result is written into the same result object, so its offset is the one returned (F8)
  if (method == SONAR_ALIGN_DTW || (method == SONAR_ALIGN_HYBRID && !(have_corr && corr_conf > 0.7))) {
    const int64_t cap = nq + nr + 1;
    int32_t* dpq = (int32_t*)dbuf(c, "cons.pq", cap * 4);
    int32_t* dpr = (int32_t*)dbuf(c, "cons.pr", cap * 4);
    double* dpc = (double*)dbuf(c, "cons.pc", cap * 8);
    if (!dpq || !dpr || !dpc) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    int64_t P = 0;
    double dist = 0.0;
    const int rc = sonar_dtw(c, dqp, nq, dr, nr, dim, -1, &dist, dpq, dpr, dpc, &P, nullptr, 1);
    if (rc != SONAR_OK) return rc;
    std::vector<int32_t> pq(P), pr(P);
    std::vector<double> pc(P);
    if (P > 0) {
      HIP_TRY(c, hipMemcpyAsync(pq.data(), dpq, P * 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipMemcpyAsync(pr.data(), dpr, P * 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipMemcpyAsync(pc.data(), dpc, P * 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipStreamSynchronize(s));
    }
    offset = sonar::host::dtw_scores(pq.data(), pr.data(), pc.data(), P, nq, nr, dist, sample_rate).offset;
  }
  // calculateOffsetStats (:751-800) over num_trials equal offsets, in Go's operation order
  std::vector<double> offs((size_t)num_trials, (double)offset);
  double sum = 0.0;
  for (double o : offs) sum += o;
  const double mean = sum / (double)offs.size();
  double ssd = 0.0;
  for (double o : offs) { const double d = o - mean; ssd += d * d; }
  const double sd = std::sqrt(ssd / (double)offs.size());
  std::vector<double> srt = offs;
  std::sort(srt.begin(), srt.end());
  const size_t n = srt.size();
  const double median = (n % 2 == 0) ? (srt[n / 2 - 1] + srt[n / 2]) / 2.0 : srt[n / 2];
  double consistency = 1.0;
  if (mean != 0) consistency = 1.0 / (1.0 + sd / std::fabs(mean));
  out->mean_offset = mean;
  out->stddev_offset = sd;
  out->median_offset = median;
  out->offset_range = srt[n - 1] - srt[0];
  out->consistency = consistency;
  out->offset = offset;
  out->trials = num_trials;
  return SONAR_OK;
}

int sonar_truncate_to_alignment(sonar_ctx* c, int64_t n1, int64_t n2, int32_t sample_rate, double temporal_offset,
                                int64_t* start1, int64_t* start2, int64_t* length) {
  if (!c) return SONAR_ERR_INVALID;
  if (!start1 || !start2 || !length) return fail(c, SONAR_ERR_INVALID, "null argument");
  const double sr = (double)sample_rate;
  // offsetSamples = int(math.Round(|offset| * sr)) (:226-228), used only when offset != 0
  auto offset_samples = [&]() { return (int64_t)std::round(std::fabs(temporal_offset) * sr); };
  int64_t s1 = 0, s2 = 0, common = 0;
  if (temporal_offset > 0) {                      // stream 2 is ahead: skip its beginning
    s2 = offset_samples();
    if (s2 >= n2)
      return fail(c, SONAR_ERR_INVALID, "offset too large: need to skip " + std::to_string(s2) +
                                            " samples but pcm2 only has " + std::to_string(n2));
    common = std::min(n1, n2 - s2);
  } else if (temporal_offset < 0) {               // stream 1 is ahead
    s1 = offset_samples();
    if (s1 >= n1)
      return fail(c, SONAR_ERR_INVALID, "offset too large: need to skip " + std::to_string(s1) +
                                            " samples but pcm1 only has " + std::to_string(n1));
    common = std::min(n1 - s1, n2);
  } else {
    common = std::min(n1, n2);
  }
  if (common <= 0) return fail(c, SONAR_ERR_INVALID, "no overlapping audio after alignment");
  const int64_t pad = (int64_t)(0.5 * sr);       // 0.5 s on both ends when there is room (:276-282)
  if (common > 2 * pad) { s1 += pad; s2 += pad; common -= 2 * pad; }
  *start1 = s1;
  *start2 = s2;
  *length = common;
  return SONAR_OK;
}

}  // extern "C"
