// hybrid_api.cpp -- the hybrid half of row a16:
//
//   sonar_analyzer_align_features   AlignmentAnalyzer.AlignFeatures (algorithms/stats/alignment.go:84-106)
//                                   for DTW, CrossCorrelation and Hybrid (alignWithHybrid :308-337)
//   sonar_align_audio               AlignmentAnalyzer.AlignAudio (:108-126) over extractEnergyFeatures
//                                   (:341-361)
//   sonar_align_audio_files         AlignmentExtractor.AlignAudioFiles
//                                   (fingerprint/extractors/alignment.go:489-553): ShortTimeEnergy
//                                   (algorithms/temporal/energy.go:25-50) + the extractor's Hybrid
//                                   analyzer (:99-126)
//
// Every O(frames) / O(cells) array runs on a HIP kernel: the RMS energy frames (energy_wave_kernel),
// the first-component flatten (first_column_kernel), the normalised cross-correlation (ncc_*_kernel)
// and the DTW band pipeline with its backtrack (dtw_band_kernel ...), through sonar_ncc / sonar_dtw on
// device buffers.  The host runs what Go runs on scalars: the scorers (host_dsp.cpp) and the hybrid
// combination.  F8: alignWithCrossCorrelation and alignWithDTW mutate and return the same result
// object, so when the correlation confidence is <= 0.7 the "correlation" confidence and similarity
// that alignWithHybrid blends are already the DTW's: Confidence = 0.6 c + 0.4 c and Similarity =
// 0.7 s + 0.3 s of the DTW values, evaluated in that order (unfused, as Go on amd64).
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

namespace {

// Go's truncating integer division (the operands here never overflow)
int64_t go_div(int64_t a, int64_t b) { return a / b; }   // C++ '/' truncates toward zero like Go

#pragma clang fp contract(off)
double blend(double w1, double a, double w2, double b) { return w1 * a + w2 * b; }

// AlignFeatures on device arrays dq [nq][dim], dr [nr][dim] (row-major float64); fills `res`
int analyzer_align(sonar_ctx* c, const double* dq, int64_t nq, const double* dr, int64_t nr, int32_t dim,
                   int32_t method, int32_t max_lag, int32_t hop, int32_t sample_rate, sonar_result* res,
                   const std::string& wrap) {
  if (nq <= 0 || nr <= 0) return fail(c, SONAR_ERR_EMPTY, wrap + "empty feature sequences provided");   // :85-87
  if (method != SONAR_ALIGN_DTW && method != SONAR_ALIGN_XCORR && method != SONAR_ALIGN_HYBRID)
    return fail(c, SONAR_ERR_INVALID, wrap + "unsupported alignment method: " + std::to_string(method));   // :103-104
  if (dim <= 0) return fail(c, SONAR_ERR_INVALID, "feature dimension must be positive");
  hipStream_t s = c->stream;
  // result := &AlignmentResult{Method, QueryLength, ReferenceLength, SampleRate} (:89-94)
  res->scalar("method", (double)method);
  res->scalar("query_length", (double)nq);
  res->scalar("reference_length", (double)nr);
  res->scalar("sample_rate", (double)sample_rate);
  double offset = 0, offset_s = 0, conf = 0, sim = 0, quality = 0, noise = 0, stability = 0;
  if (method == SONAR_ALIGN_XCORR || method == SONAR_ALIGN_HYBRID) {   // alignWithCrossCorrelation :151-181
    const double *q0 = dq, *r0 = dr;
    if (dim > 1) {                                                  // flatten2DFeatures (:363-378): frame[0]
      double* a = (double*)dbuf(c, "hy.q0", nq * 8);
      double* b = (double*)dbuf(c, "hy.r0", nr * 8);
      if (!a || !b) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
      if (sonar::launch_first_column(dq, nq, dim, a, s) != 0 || sonar::launch_first_column(dr, nr, dim, b, s) != 0)
        return fail(c, SONAR_ERR_DEVICE, "flatten launch failed");
      q0 = a; r0 = b;
    }
    const int64_t L = std::max<int64_t>(0, std::min<int64_t>({(int64_t)max_lag, nq - 1, nr - 1}));
    double* dcorr = (double*)dbuf(c, "hy.corr", (2 * L + 1) * 8);
    if (!dcorr) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    double met[10];
    int rc = sonar_ncc(c, q0, nq, r0, nr, max_lag, dcorr, met, 1);
    if (rc != SONAR_OK) return rc;
    std::vector<double> corr(2 * L + 1);
    HIP_TRY(c, hipMemcpyAsync(corr.data(), dcorr, corr.size() * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    sonar::host::NccMetrics m;
    m.peak_corr = met[0]; m.peak_lag = (int64_t)met[1]; m.peak_index = (int64_t)met[2]; m.p_value = met[3];
    m.snr = met[4]; m.sharpness = met[5]; m.second_peak = met[6]; m.psl = met[7]; m.overlap = (int64_t)met[8];
    m.num_lags = (int64_t)met[9];
    const auto sc = sonar::host::xcorr_scores(m, hop, sample_rate, max_lag);
    offset = (double)sc.offset; offset_s = sc.offset_seconds; sim = sc.similarity; conf = sc.confidence;
    quality = sc.quality; noise = sc.noise_level;
    // CrossCorrResult (correlation.go:20-40)
    res->vec("correlations", corr);
    static const char* nm[10] = {"peak_correlation", "peak_lag", "peak_index", "p_value", "snr", "sharpness",
                                 "second_peak", "peak_to_sidelobe", "overlap_length", "num_lags"};
    for (int k = 0; k < 10; k++) res->scalar(nm[k], met[k]);
  }
  const bool run_dtw = method == SONAR_ALIGN_DTW || (method == SONAR_ALIGN_HYBRID && !(conf > 0.7));   // :316-318
  if (run_dtw) {                                                    // alignWithDTW :129-148
    const int64_t cap = nq + nr + 1;
    int32_t* dpq = (int32_t*)dbuf(c, "hy.pq", cap * 4);
    int32_t* dpr = (int32_t*)dbuf(c, "hy.pr", cap * 4);
    double* dpc = (double*)dbuf(c, "hy.pc", cap * 8);
    if (!dpq || !dpr || !dpc) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    int64_t P = 0;
    double dist = 0.0;
    const int rc = sonar_dtw(c, dq, nq, dr, nr, dim, -1, &dist, dpq, dpr, dpc, &P, nullptr, 1);
    if (rc != SONAR_OK) {
      if (rc == SONAR_ERR_EMPTY) return fail(c, rc, wrap + "DTW alignment failed: " + c->err);
      return rc;                                                    // device errors have no Go counterpart
    }
    std::vector<int32_t> pq(P), pr(P);
    std::vector<double> pc(P);
    if (P > 0) {
      HIP_TRY(c, hipMemcpyAsync(pq.data(), dpq, P * 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipMemcpyAsync(pr.data(), dpr, P * 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipMemcpyAsync(pc.data(), dpc, P * 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipStreamSynchronize(s));
    }
    const auto sd = sonar::host::dtw_scores(pq.data(), pr.data(), pc.data(), P, nq, nr, dist, sample_rate);
    offset = (double)sd.offset; offset_s = sd.offset_seconds; quality = sd.quality; stability = sd.stability;
    if (method == SONAR_ALIGN_DTW) {
      conf = sd.confidence; sim = sd.similarity;
    } else {
      // alignWithHybrid (:327-334), F8: dtwResult == corrResult == result
      conf = blend(0.6, sd.confidence, 0.4, sd.confidence);
      sim = blend(0.7, sd.similarity, 0.3, sd.similarity);
    }
    // DTWResult (dtw.go:13-22; the cost matrix is not returned here)
    std::vector<double> vq(P), vr(P);
    for (int64_t i = 0; i < P; i++) { vq[i] = pq[i]; vr[i] = pr[i]; }
    res->scalar("dtw_distance", dist);
    res->vec("dtw_path_query", vq);
    res->vec("dtw_path_reference", vr);
    res->vec("dtw_path_cost", pc);
  }
  res->scalar("offset", offset);
  res->scalar("offset_seconds", offset_s);
  res->scalar("confidence", conf);
  res->scalar("similarity", sim);
  res->scalar("alignment_quality", quality);
  res->scalar("noise_level", noise);
  res->scalar("stability", stability);
  res->scalar("dtw_ran", run_dtw ? 1.0 : 0.0);
  return SONAR_OK;
}

// PCM to the device (or use it there), float64
int device_pcm(sonar_ctx* c, const double* pcm, int64_t n, int32_t dev, const char* tag, const double** out) {
  if (dev) { *out = pcm; return SONAR_OK; }
  double* d = (double*)dbuf(c, tag, std::max<int64_t>(n, 1) * 8);
  if (!d) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (pcm)");
  if (n > 0) HIP_TRY(c, hipMemcpyAsync(d, pcm, n * 8, hipMemcpyHostToDevice, c->stream));
  *out = d;
  return SONAR_OK;
}

// RMS frames sqrt(sum x^2 / W) of the raw PCM (no pre-emphasis: alpha 0 is the identity in the
// kernel), frames [i H, i H + W), Go's sequential sum per frame
int rms_frames(sonar_ctx* c, const double* dpcm, int64_t n, int64_t F, int32_t W, int32_t H, const char* tag,
               double** out) {
  double* e = (double*)dbuf(c, tag, std::max<int64_t>(F, 1) * 8);
  if (!e) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (energy)");
  if (F > 0 && sonar::launch_energy(dpcm, 1, n, F, W, H, 0.0, e, 1, c->stream) != 0)
    return fail(c, SONAR_ERR_DEVICE, "energy launch failed");
  *out = e;
  return SONAR_OK;
}

}  // namespace

extern "C" {

int sonar_analyzer_align_features(sonar_ctx* c, const double* query, int64_t nq, const double* reference, int64_t nr,
                                  int32_t dim, int32_t method, int32_t max_lag, int32_t hop, int32_t sample_rate,
                                  int32_t device_ptrs, sonar_result** out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  if (nq <= 0 || nr <= 0 || !query || !reference) return fail(c, SONAR_ERR_EMPTY, "empty feature sequences provided");
  if (dim <= 0) return fail(c, SONAR_ERR_INVALID, "feature dimension must be positive");
  HIP_TRY(c, hipSetDevice(c->device));
  const double *dq = query, *dr = reference;
  if (!device_ptrs) {
    double* a = (double*)dbuf(c, "hy.q", nq * dim * 8);
    double* b = (double*)dbuf(c, "hy.r", nr * dim * 8);
    if (!a || !b) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    HIP_TRY(c, hipMemcpyAsync(a, query, nq * dim * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(b, reference, nr * dim * 8, hipMemcpyHostToDevice, c->stream));
    dq = a; dr = b;
  }
  auto* res = new sonar_result();
  const int rc = analyzer_align(c, dq, nq, dr, nr, dim, method, max_lag, hop, sample_rate, res, "");
  if (rc != SONAR_OK) { delete res; return rc; }
  *out = res;
  return SONAR_OK;
}

int sonar_align_audio(sonar_ctx* c, const double* q_pcm, int64_t nq, const double* r_pcm, int64_t nr, int32_t method,
                      int32_t max_lag, int32_t hop, int32_t window, int32_t sample_rate, int32_t device_ptrs,
                      sonar_result** out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  if ((nq > 0 && !q_pcm) || (nr > 0 && !r_pcm)) return fail(c, SONAR_ERR_INVALID, "null PCM");
  if (hop == 0) return fail(c, SONAR_ERR_PANIC, "runtime error: integer divide by zero");   // :344
  if (window <= 0 || hop < 0)
    return fail(c, SONAR_ERR_UNSUPPORTED, "window must be positive and hop non-negative (Go divides 0 by 0 per frame)");
  if (nq <= 0 || nr <= 0)
    return fail(c, SONAR_ERR_UNSUPPORTED, "empty PCM (Go returns a 0/0 energy frame or none)");
  HIP_TRY(c, hipSetDevice(c->device));
  // extractEnergyFeatures (:341-361): numFrames = (len - W) / H + 1 (truncating); a signal shorter
  // than W but within one hop of it has one frame over its whole length (end = min(start + W, len))
  const double* src[2] = {q_pcm, r_pcm};
  const int64_t len[2] = {nq, nr};
  double* e[2] = {nullptr, nullptr};
  int64_t F[2] = {0, 0};
  for (int k = 0; k < 2; k++) {
    F[k] = go_div(len[k] - window, hop) + 1;
    if (F[k] < 0) return fail(c, SONAR_ERR_PANIC, "runtime error: makeslice: len out of range");
    const double* d = nullptr;
    int rc = device_pcm(c, src[k], len[k], device_ptrs, k ? "hy.rpcm" : "hy.qpcm", &d);
    if (rc != SONAR_OK) return rc;
    const int32_t W = len[k] >= window ? window : (int32_t)len[k];
    rc = rms_frames(c, d, len[k], F[k], W, hop, k ? "hy.re" : "hy.qe", &e[k]);
    if (rc != SONAR_OK) return rc;
  }
  auto* res = new sonar_result();
  const int rc = analyzer_align(c, e[0], F[0], e[1], F[1], 1, method, max_lag, hop, sample_rate, res, "");
  if (rc != SONAR_OK) { delete res; return rc; }
  *out = res;
  return SONAR_OK;
}

int sonar_align_audio_files(sonar_ctx* c, const double* q_pcm, int64_t nq, const double* r_pcm, int64_t nr,
                            int32_t sample_rate, int32_t feature_sample_rate, int32_t hop, int32_t window,
                            double max_lag_seconds, int32_t device_ptrs, sonar_result** out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  if ((nq > 0 && !q_pcm) || (nr > 0 && !r_pcm)) return fail(c, SONAR_ERR_INVALID, "null PCM");
  // NewAlignmentExtractorWithMaxLag (:104-107): maxLagFrames = int(maxLagSeconds * SampleRate) / HopSize
  if (hop == 0) return fail(c, SONAR_ERR_PANIC, "runtime error: integer divide by zero");
  const int64_t max_lag_samples = (int64_t)(max_lag_seconds * (double)feature_sample_rate);
  const int64_t mlf = go_div(max_lag_samples, hop);
  const int32_t max_lag = (int32_t)std::max<int64_t>(INT32_MIN, std::min<int64_t>(INT32_MAX, mlf));
  HIP_TRY(c, hipSetDevice(c->device));
  // ComputeShortTimeEnergy (energy.go:25-50): empty when len < W, W <= 0 or H <= 0
  const double* src[2] = {q_pcm, r_pcm};
  const int64_t len[2] = {nq, nr};
  double* e[2] = {nullptr, nullptr};
  int64_t F[2] = {0, 0};
  for (int k = 0; k < 2; k++) {
    F[k] = sonar_energy_frames(len[k], window, hop);
    if (F[k] <= 0) continue;
    const double* d = nullptr;
    int rc = device_pcm(c, src[k], len[k], device_ptrs, k ? "hy.rpcm" : "hy.qpcm", &d);
    if (rc != SONAR_OK) return rc;
    rc = rms_frames(c, d, len[k], F[k], window, hop, k ? "hy.re" : "hy.qe", &e[k]);
    if (rc != SONAR_OK) return rc;
  }
  auto* res = new sonar_result();
  // the extractor's analyzer: NewAlignmentAnalyzer(AlignmentHybrid, maxLagFrames, ...) (:120-126)
  const int rc = analyzer_align(c, e[0], F[0], e[1], F[1], 1, SONAR_ALIGN_HYBRID, max_lag, hop, sample_rate, res,
                                "alignment failed: ");
  if (rc != SONAR_OK) { delete res; return rc; }
  // AlignmentFeatures (:528-544): Method "energy_correlation", BestAlignment.FeatureType "energy",
  // FeatureSimilarity{"energy"}; TimeStretch is never set (zero value)
  auto get = [&](const char* k) { return res->get(k); };
  res->scalar("temporal_offset", get("offset_seconds"));
  res->scalar("offset_confidence", get("confidence"));
  res->scalar("alignment_similarity", get("similarity"));
  res->scalar("feature_similarity_energy", get("similarity"));
  res->scalar("query_length_seconds", (double)nq / (double)sample_rate);
  res->scalar("reference_length_seconds", (double)nr / (double)sample_rate);
  res->scalar("time_stretch", 0.0);
  res->scalar("max_lag_frames", (double)mlf);
  *out = res;
  return SONAR_OK;
}

}  // extern "C"
