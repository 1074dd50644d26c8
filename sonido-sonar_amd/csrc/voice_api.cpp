// voice_api.cpp -- VoiceQualityAnalyzer.AnalyzeVoiceQuality (algorithms/speech/voice_quality.go:56-111)
// above the HIP kernels.
//
//   device: the YIN scan of 1024-sample frames at hop 256 (yin_kernel, :114-127), the RMS of every
//           extracted pitch period (period_rms_kernel, :200-207) and the 2048-lag autocorrelation
//           of calculateHNR (hnr_autocorr_kernel, :255-267);
//   host:   what Go runs sequentially on O(frames) data -- the PitchDetector temporal tracking
//           (pitch_detection.go:767-921), the period walk whose start depends on the previous
//           period's end (:133-151), and the scalar formulas (:160-451).
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

double go_max(double x, double y) {            // math.Max (NaN-propagating, +0 > -0)
  if (std::isinf(x) && x > 0) return x;
  if (std::isinf(y) && y > 0) return y;
  if (std::isnan(x) || std::isnan(y)) return NAN;
  if (x == 0 && x == y) return std::signbit(x) ? y : x;
  return x > y ? x : y;
}
double go_min(double x, double y) {
  if (std::isinf(x) && x < 0) return x;
  if (std::isinf(y) && y < 0) return y;
  if (std::isnan(x) || std::isnan(y)) return NAN;
  if (x == 0 && x == y) return std::signbit(x) ? x : y;
  return x < y ? x : y;
}

}  // namespace

namespace sonar {
namespace detail {

int voice_quality(sonar_ctx* c, const double* dy, int64_t n, int32_t sr, sonar_voice_quality_result* q) {
  std::memset(q, 0, sizeof(*q));
  if (n < (int64_t)sr)                                             // :57-59
    return fail(c, SONAR_ERR_TOO_SHORT, "signal too short for voice quality analysis (need at least 1 second)");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  // extractPitchPeriodsAndF0 (:114-157): frames i = 0, 256, ... while i < n - 1024.  With exactly
  // 1024 samples calculateVoicingStrength's DetectPitch(signal) (:363-371) reads frame 0 too.
  const int64_t Fv = n > 1024 ? (n - 1025) / 256 + 1 : 0;
  const int64_t Fl = std::max<int64_t>(Fv, n == 1024 ? 1 : 0);
  std::vector<double> praw(Fl), craw(Fl), head(std::min<int64_t>(n, 1024));
  if (Fl > 0) {
    double* dp = (double*)dbuf(c, "vq.pitch", Fl * 8);
    double* dc = (double*)dbuf(c, "vq.conf", Fl * 8);
    if (!dp || !dc) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (voice quality)");
    if (sonar::launch_yin(dy, n, Fl, 256, sr, dp, dc, nullptr, s) != 0)
      return fail(c, SONAR_ERR_DEVICE, "yin launch failed");
    HIP_TRY(c, hipMemcpyAsync(praw.data(), dp, Fl * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(craw.data(), dc, Fl * 8, hipMemcpyDeviceToHost, s));
  }
  if (!head.empty()) HIP_TRY(c, hipMemcpyAsync(head.data(), dy, head.size() * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));

  // the period walk (:123-154): a fresh PitchDetector, voiced frames with Voicing and
  // Confidence > 0.5 and F0 in [50, 500]; each period starts at max(frame start, last end)
  sonar::host::YinTracker tr;
  std::vector<int64_t> st, ln;
  std::vector<double> f0;
  int64_t last_end = 0;
  for (int64_t i = 0; i < Fv; i++) {
    double p = praw[i], cf = craw[i], v = 0.0;
    tr.step(p, cf, v);
    if (v > 0.5 && cf > 0.5 && p >= 50.0 && p <= 500.0) {
      const int64_t len = (int64_t)((double)sr / p);
      const int64_t s0 = std::max<int64_t>(i * 256, last_end), e0 = s0 + len;
      if (e0 < n) { st.push_back(s0); ln.push_back(len); f0.push_back(p); last_end = e0; }
    }
  }
  double vstr = 0.0;
  if (n == 1024) { double p = praw[0], cf = craw[0]; tr.step(p, cf, vstr); }
  const int64_t np = (int64_t)st.size();
  if (np < 3)                                                      // :67-69
    return fail(c, SONAR_ERR_TOO_SHORT, "insufficient pitch periods for analysis (found " + std::to_string(np) +
                                            ", need at least 3)");

  // period amplitudes on the device
  int64_t* dst = (int64_t*)dbuf(c, "vq.start", np * 8);
  int64_t* dln = (int64_t*)dbuf(c, "vq.len", np * 8);
  double* damp = (double*)dbuf(c, "vq.amp", np * 8);
  double* dac = (double*)dbuf(c, "vq.ac", 2048 * 8);
  if (!dst || !dln || !damp || !dac) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (voice quality)");
  HIP_TRY(c, hipMemcpyAsync(dst, st.data(), np * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(dln, ln.data(), np * 8, hipMemcpyHostToDevice, s));
  if (sonar::launch_period_rms(dy, dst, dln, np, damp, s) != 0) return fail(c, SONAR_ERR_DEVICE, "period rms launch failed");
  const bool hnr_frame = n >= 2048;                                // calculateHNR :245-248
  if (hnr_frame) {
    const int64_t s0 = std::max<int64_t>(n / 2 - 1024, 0);
    if (sonar::launch_hnr_autocorr(dy + s0, dac, s) != 0) return fail(c, SONAR_ERR_DEVICE, "hnr launch failed");
  }
  std::vector<double> amp(np), ac(hnr_frame ? 2048 : 0);
  HIP_TRY(c, hipMemcpyAsync(amp.data(), damp, np * 8, hipMemcpyDeviceToHost, s));
  if (hnr_frame) HIP_TRY(c, hipMemcpyAsync(ac.data(), dac, 2048 * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));

  // calculateJitter (:160-191) and calculateShimmer (:194-229)
  double avg = 0.0, js = 0.0;
  for (int64_t k = 0; k < np; k++) avg += (double)ln[k];
  avg /= (double)np;
  for (int64_t k = 1; k < np; k++) js += std::fabs((double)ln[k] - (double)ln[k - 1]);
  const double jitter = avg == 0 ? 0.0 : (js / (double)(np - 1)) / avg * 100.0;
  double aavg = 0.0, ss = 0.0;
  for (int64_t k = 0; k < np; k++) aavg += amp[k];
  aavg /= (double)np;
  for (int64_t k = 1; k < np; k++) ss += std::fabs(amp[k] - amp[k - 1]);
  const double shimmer = aavg == 0 ? 0.0 : (ss / (double)(np - 1)) / aavg * 100.0;
  // calculateHNR (:232-294): peak of the autocorrelation within +-25 % of the mean-F0 lag
  double mf = 0.0, hnr = 0.0;
  for (double v : f0) mf += v;
  mf /= (double)np;
  if (hnr_frame) {
    const int64_t el = (int64_t)((double)sr / mf);
    if (el < 2048) {
      const int64_t r = el / 4, a = std::max<int64_t>(1, el - r), b = std::min<int64_t>(2047, el + r);
      double mc = 0.0;
      for (int64_t i = a; i <= b; i++) if (ac[i] > mc) mc = ac[i];
      if (mc > 0 && mc < ac[0]) hnr = 10.0 * std::log10(mc / (ac[0] - mc));
    }
  }
  // calculateF0Stability (:297-322), calculateAmplitudeStability (:325-360)
  double var = 0.0;
  for (double v : f0) { const double d = v - mf; var += d * d; }
  var /= (double)np;
  const double f0s = mf == 0 ? 0.0 : go_max(0.0, 1.0 - std::sqrt(var) / mf);
  double av = 0.0;
  for (double v : amp) { const double d = v - aavg; av += d * d; }
  av /= (double)np;
  const double ams = aavg == 0 ? 0.0 : go_max(0.0, 1.0 - std::sqrt(av) / aavg);
  // calculateNoiseMeasure (:374-398) on the first 1024 samples
  double nm = 0.0;
  if (n >= 1024) {
    double hf = 0.0, te = 0.0;
    for (int i = 1; i < 1024; i++) { const double d = head[i] - head[i - 1]; hf += d * d; te += head[i] * head[i]; }
    nm = te == 0 ? 0.0 : hf / te;
  }
  // calculateF0Statistics (:401-426), calculateOverallQuality (:429-437), calculateAnalysisQuality (:440-451)
  double lo = f0[0], hi = f0[0];
  for (double v : f0) { if (v < lo) lo = v; if (v > hi) hi = v; }
  q->jitter = jitter;
  q->shimmer = shimmer;
  q->hnr = hnr;
  q->noise_measure = nm;
  q->f0_stability = f0s;
  q->amplitude_stability = ams;
  q->voicing_strength = vstr;
  q->overall_quality = (go_max(0, 1.0 - jitter / 5.0) + go_max(0, 1.0 - shimmer / 10.0) +
                        go_min(1.0, go_max(0, hnr / 20.0)) + f0s) / 4.0;
  q->num_periods = np;
  q->mean_f0 = mf;
  q->f0_range = hi - lo;
  q->analysis_quality = (go_min(1.0, (double)np / 10.0) + f0s + go_min(1.0, go_max(0, hnr / 15.0))) / 3.0;
  return SONAR_OK;
}

}  // namespace detail
}  // namespace sonar

extern "C" int sonar_voice_quality(sonar_ctx* c, const double* pcm, int64_t n, int32_t sample_rate,
                                   sonar_voice_quality_result* out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  std::memset(out, 0, sizeof(*out));
  if (n < (int64_t)sample_rate)
    return fail(c, SONAR_ERR_TOO_SHORT, "signal too short for voice quality analysis (need at least 1 second)");
  if (n > 0 && !pcm) return fail(c, SONAR_ERR_INVALID, "null buffer");
  HIP_TRY(c, hipSetDevice(c->device));
  double* d = (double*)dbuf(c, "vq.pcm", (size_t)std::max<int64_t>(n, 1) * 8);
  if (!d) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (voice quality)");
  if (n > 0) HIP_TRY(c, hipMemcpyAsync(d, pcm, n * 8, hipMemcpyHostToDevice, c->stream));
  return sonar::detail::voice_quality(c, d, n, sample_rate, out);
}
