// content_api.cpp -- ContentDetector (fingerprint/content_detector.go) behind the C ABI.
// The whole-PCM passes and the direct DFT run on the device (content_kernels.hip); the
// metadata rules are string matching on the host, and the per-frame sums come back to the
// host for the scalar reductions in Go's order (frames are 1/512 of the samples).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "ctx.h"
#include "kernels.h"

using sonar::detail::dbuf;
using sonar::detail::fail;

namespace {

std::string lower(std::string s) {            // strings.ToLower (ASCII)
  for (char& ch : s) ch = (char)std::tolower((unsigned char)ch);
  return s;
}
std::string trim(const std::string& s) {      // strings.TrimSpace (ASCII whitespace)
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) a++;
  while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
  return s.substr(a, b - a);
}
bool has(const std::string& s, const char* sub) { return s.find(sub) != std::string::npos; }
bool any_of(const std::string& s, const char* const* list) {
  for (; *list; ++list)
    if (has(s, *list)) return true;
  return false;
}

// parseContentType (:615-626)
int parse_content_type(const std::string& ct) {
  const std::string v = lower(ct);
  if (v == "music" || v == "audio/music") return SONAR_CT_MUSIC;
  if (v == "news" || v == "talk" || v == "spoken") return SONAR_CT_NEWS;
  if (v == "sports") return SONAR_CT_SPORTS;
  return SONAR_CT_UNKNOWN;
}

// inferFromGenre (:501-551)
int infer_from_genre(const std::string& g0) {
  static const char* const music[] = {"rock", "pop", "jazz", "classical", "hip-hop", "hip hop", "country",
                                      "electronic", "blues", "reggae", "folk", "metal", "punk", "r&b", "soul",
                                      "funk", "dance", "techno", "house", "ambient", "indie", "alternative",
                                      "grunge", "ska", "latin", "world", "gospel", nullptr};
  static const char* const news[] = {"news", "talk", "politics", "current affairs", "public radio", "discussion",
                                     "interview", "call-in", "spoken word", "commentary", "analysis", "reporting",
                                     "journalism", "public affairs", nullptr};
  static const char* const sports[] = {"sports", "football", "basketball", "baseball", "soccer", "hockey",
                                       "tennis", "golf", "racing", "motorsports", "athletics", "cricket", "rugby",
                                       "boxing", "mma", "sports talk", "sports news", nullptr};
  const std::string g = lower(trim(g0));
  if (any_of(g, music)) return SONAR_CT_MUSIC;
  if (any_of(g, news)) return SONAR_CT_NEWS;
  if (any_of(g, sports)) return SONAR_CT_SPORTS;
  if (has(g, "talk") && !has(g, "sports")) return SONAR_CT_TALK;
  return SONAR_CT_UNKNOWN;
}

// inferFromStation (:554-599)
int infer_from_station(const std::string& station, const std::string& url) {
  static const char* const news[] = {"news", "npr", "bbc", "cnn", "cbc", "abc news", "nbc news", "fox news",
                                     "public radio", "current affairs", "talk radio", nullptr};
  static const char* const sports[] = {"sports", "espn", "fox sports", "sports radio", "the fan", "sport",
                                       "athletic", "game", "stadium", nullptr};
  static const char* const music[] = {"fm", "music", "hits", "rock", "pop", "jazz", "country", "classic", "radio",
                                      "mix", "beat", "sound", "groove", nullptr};
  const std::string combined = lower(trim(station)) + " " + lower(url);
  if (any_of(combined, news)) return SONAR_CT_NEWS;
  if (any_of(combined, sports)) return SONAR_CT_SPORTS;
  if (any_of(combined, music)) return SONAR_CT_MUSIC;
  if (has(combined, "talk") && !has(combined, "sports")) return SONAR_CT_TALK;
  return SONAR_CT_UNKNOWN;
}

// detectContentTypeFromMetadata (:602-613)
int from_metadata(const char* ct, const char* genre, const char* station, const char* url) {
  const std::string c = ct ? ct : "", g = genre ? genre : "";
  if (!c.empty()) return parse_content_type(c);
  if (!g.empty()) return infer_from_genre(g);
  return infer_from_station(station ? station : "", url ? url : "");
}

double go_max(double x, double y) {
  if (std::isinf(x) && x > 0) return x;
  if (std::isinf(y) && y > 0) return y;
  if (std::isnan(x) || std::isnan(y)) return NAN;
  if (x == 0 && x == y) return std::signbit(x) ? y : x;
  return x > y ? x : y;
}

}  // namespace

namespace sonar {
namespace detail {

// DetectFromAudio (:72-101) + extractAcousticFeatures (:118-150) + classifyFromFeatures (:153-217)
int detect_from_audio(sonar_ctx* c, const double* pcm, int64_t n, int32_t sr, double thr, int32_t* out,
                      sonar_acoustic_features* feat) {
  sonar_acoustic_features f;
  std::memset(&f, 0, sizeof(f));
  if (n <= 0 || !pcm) {                       // :73-75
    *out = SONAR_CT_UNKNOWN;
    if (feat) *feat = f;
    return SONAR_OK;
  }
  if (sr < 10) return fail(c, SONAR_ERR_INVALID, "sample rate below 10 Hz: the 100 ms frame loop of "
                                                 "calculateTemporalStability never ends (content_detector.go:392-402)");
  hipStream_t s = c->stream;
  const int N = (int)std::min<int64_t>(2048, n), K = N / 2 + 1;
  const int64_t fe = n > 1024 ? (n - 1024 + 511) / 512 : 0;               // i < n - 1024, i += 512
  const int64_t ts = sr / 10;
  const int64_t ft = n > ts ? (n - ts + ts - 1) / ts : 0;                  // i < n - ts, i += ts
  double* x = static_cast<double*>(dbuf(c, "cd.pcm", n * sizeof(double)));
  char* w = static_cast<char*>(dbuf(c, "cd.work", 64 + (K + fe + ft) * sizeof(double)));
  if (!x || !w) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  unsigned long long* words = reinterpret_cast<unsigned long long*>(w);
  double* mag = reinterpret_cast<double*>(w + 64);
  double* esum = mag + K;
  double* tsum = esum + fe;
  HIP_TRY(c, hipMemcpyAsync(x, pcm, n * sizeof(double), hipMemcpyHostToDevice, s));
  hipEvent_t tend = timed_begin(c, s);
  if (launch_detect_scan(x, n, words, s) || launch_frame_sums(x, n, fe, 512, 1024, esum, s) ||
      launch_frame_sums(x, n, ft, ts, ts, tsum, s) || launch_dft_mag(x, N, mag, s))
    return fail(c, SONAR_ERR_DEVICE, "content detection launch failed");
  timed_end(c, s, tend);
  std::vector<double> h(K + fe + ft);
  unsigned long long hw[3];
  HIP_TRY(c, hipMemcpyAsync(hw, words, sizeof(hw), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(h.data(), mag, h.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  const double* spec = h.data();
  const double* es = spec + K;
  const double* tsm = es + fe;
  // calculateZeroCrossingRate (:220-233)
  f.zero_crossing_rate = n <= 1 ? 0.0 : (double)hw[0] / (double)(n - 1);
  // calculateSpectralCentroid (:236-252)
  {
    double ws = 0.0, ms = 0.0;
    for (int i = 0; i < K; i++) {
      const double fr = (double)i * (double)sr / (double)(K * 2);
      ws += fr * spec[i];
      ms += spec[i];
    }
    f.spectral_centroid = ms == 0 ? 0.0 : ws / ms;
  }
  // calculateEnergyVariance (:255-290)
  if (n >= 2048 && fe > 1) {
    double mean = 0.0;
    for (int64_t i = 0; i < fe; i++) mean += es[i] / 1024.0;
    mean /= (double)fe;
    double var = 0.0;
    for (int64_t i = 0; i < fe; i++) {
      const double d = es[i] / 1024.0 - mean;
      var += d * d;
    }
    f.energy_variance = var / (double)fe;
  }
  // calculateSilenceRatio (:293-317)
  if (fe > 0) {
    int64_t silent = 0;
    for (int64_t i = 0; i < fe; i++) silent += std::sqrt(es[i] / 1024.0) < 0.01;
    f.silence_ratio = (double)silent / (double)fe;
  }
  // calculateDynamicRange (:320-343)
  {
    double mx, mn;
    std::memcpy(&mx, &hw[1], 8);
    std::memcpy(&mn, &hw[2], 8);
    f.dynamic_range = (mn == 0 || std::isinf(mn)) ? 0.0 : 20.0 * std::log10(mx / mn);
  }
  // calculateFreqEnergyRatio (:346-369)
  {
    const int split = K / 4;
    double lo = 0.0, hi = 0.0;
    for (int i = 0; i < split && i < K; i++) lo += spec[i] * spec[i];
    for (int i = split; i < K; i++) hi += spec[i] * spec[i];
    const double tot = lo + hi;
    if (tot != 0) { f.low_freq_energy = lo / tot; f.high_freq_energy = hi / tot; }
  }
  // calculateHarmonicRatio (:372-401)
  if (K >= 10) {
    std::vector<int> peaks;
    for (int i = 2; i < K - 2; i++)
      if (spec[i] > spec[i - 1] && spec[i] > spec[i + 1] && spec[i] > spec[i - 2] && spec[i] > spec[i + 2])
        peaks.push_back(i);
    if (peaks.size() >= 2) {
      int harm = 0;
      for (size_t q = 1; q < peaks.size(); q++) {
        const double r = (double)peaks[q] / (double)peaks[0];
        if (std::fabs(r - std::round(r)) < 0.1) harm++;
      }
      f.harmonic_ratio = (double)harm / (double)(peaks.size() - 1);
    }
  }
  // calculateTemporalStability (:404-447)
  if (n >= 3 * ts && ft > 1) {
    double mean = 0.0;
    for (int64_t i = 0; i < ft; i++) mean += tsm[i];
    mean /= (double)ft;
    if (mean != 0) {
      double var = 0.0;
      for (int64_t i = 0; i < ft; i++) {
        const double d = tsm[i] - mean;
        var += d * d;
      }
      var /= (double)ft;
      f.temporal_stability = go_max(0.0, 1.0 - std::sqrt(var) / mean);
    }
  }
  // classifyFromFeatures (:153-217); map order in Go, fixed order here
  double music = 0.0, speech = 0.0, sports = 0.0;
  if (f.zero_crossing_rate < 0.1) music += 2.0;
  if (f.harmonic_ratio > 0.3) music += 2.0;
  if (f.temporal_stability > 0.5) music += 1.0;
  if (f.dynamic_range > 20) music += 1.0;
  if (f.zero_crossing_rate > 0.05 && f.zero_crossing_rate < 0.3) speech += 2.0;
  if (f.spectral_centroid > 800 && f.spectral_centroid < 3000) speech += 2.0;
  if (f.harmonic_ratio < 0.2) speech += 1.0;
  if (f.silence_ratio > 0.1 && f.silence_ratio < 0.4) speech += 1.0;
  if (f.energy_variance > 0.3) sports += 2.0;
  if (f.dynamic_range > 30) sports += 1.5;
  if (f.temporal_stability < 0.4) sports += 1.0;
  const int types[4] = {SONAR_CT_MUSIC, SONAR_CT_NEWS, SONAR_CT_TALK, SONAR_CT_SPORTS};
  const double scores[4] = {music, speech, speech * 0.9, sports};
  int best = SONAR_CT_UNKNOWN;
  double bs = thr;
  for (int i = 0; i < 4; i++)
    if (scores[i] > bs) { bs = scores[i]; best = types[i]; }
  f.classification_confidence = bs / 6.0;
  *out = best;
  if (feat) *feat = f;
  return SONAR_OK;
}

// DetectContentType (:31-69)
int detect_content_type(sonar_ctx* c, const double* pcm, int64_t n, int32_t sr, int32_t has_md, const char* ct,
                        const char* genre, const char* station, const char* url, int32_t acoustic,
                        int32_t dflt, double thr, int32_t* out) {
  if (has_md) {
    const int m = from_metadata(ct, genre, station, url);
    if (m != SONAR_CT_UNKNOWN) { *out = m; return SONAR_OK; }
  }
  if (acoustic && n > 0) {
    int32_t a = SONAR_CT_UNKNOWN;
    const int rc = detect_from_audio(c, pcm, n, sr, thr, &a, nullptr);
    if (rc != SONAR_OK) return rc;
    if (a != SONAR_CT_UNKNOWN) { *out = a; return SONAR_OK; }
  }
  *out = dflt;
  return SONAR_OK;
}

}  // namespace detail
}  // namespace sonar

extern "C" {

int sonar_detect_from_audio(sonar_ctx* c, const double* pcm, int64_t n, int32_t sample_rate,
                            double auto_detect_threshold, int32_t* content_type, sonar_acoustic_features* features) {
  if (!c || !content_type) return fail(c, SONAR_ERR_INVALID, "null argument");
  if (n < 0) return fail(c, SONAR_ERR_INVALID, "negative length");
  return sonar::detail::detect_from_audio(c, pcm, n, sample_rate, auto_detect_threshold, content_type, features);
}

int sonar_detect_content_type(sonar_ctx* c, const double* pcm, int64_t n, int32_t sample_rate, int32_t has_metadata,
                              const char* content_type, const char* genre, const char* station, const char* url,
                              int32_t acoustic_detection, int32_t default_content_type, double auto_detect_threshold,
                              int32_t* out_content_type) {
  if (!c || !out_content_type) return fail(c, SONAR_ERR_INVALID, "null argument");
  if (n < 0) return fail(c, SONAR_ERR_INVALID, "negative length");
  return sonar::detail::detect_content_type(c, pcm, n, sample_rate, has_metadata, content_type, genre, station, url,
                                            acoustic_detection, default_content_type, auto_detect_threshold,
                                            out_content_type);
}

}  // extern "C"
