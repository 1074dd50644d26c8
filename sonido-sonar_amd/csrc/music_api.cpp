// music_api.cpp -- MusicFeatureExtractor.ExtractFeatures (fingerprint/extractors/music.go:178-583)
// as one C entry: NewMusicFeatureExtractor(cfg) (:70-137) + ExtractFeatures(STFT(pcm, W, H), pcm,
// sample_rate).  Every per-sample and per-frame pass runs on the device (the fused STFT kernel for
// the spectrogram's descriptors and |X|^4 MFCC, music_kernels.hip for the spectral contrast and
// the band energy ratios, the DC / pre-emphasis scan, chroma and energy kernels of the alignment
// path); the host runs only Go's O(frames) scalar tails.
//
// The reference panics inside extractTemporalFeatures for almost every input (DESIGN.md F15 and
// Kernel 10): music.go:403 passes the percentiles 10 and 90 where
// DynamicRange.calculatePercentileRange (temporal/dynamic_range.go:58-76) expects fractions, so
// int(10 * (L - 1)) indexes past the L RMS frames (1024 / 512) of any signal with L >= 2
// (n >= 1536 samples); and a signal with no energy frame divides by zero at music.go:383.  Such a
// call returns SONAR_ERR_PANIC with Go's runtime message, and *out holds the arrays the Go call
// had computed before the panic (spectral features, MFCC, chroma, rms_energy, envelope_shape,
// peak / average amplitude); Go itself returns nothing.  A FeatureConfig hop above the
// spectrogram's panics earlier, in extractChromaFeatures (slice bounds, :348-352), after the
// spectral features and the MFCC.  Below 1536 samples every group is
// computed as in Go, the harmonic block zero by F7 unless the frame is exactly 1024 samples.
#include "../../include/sonar_gpu.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "ctx.h"
#include "host_dsp.h"
#include "kernels.h"

using sonar::detail::dbuf;
using sonar::detail::fail;

namespace {

constexpr int kContrastBands = 6;                                 // NewSpectralContrast(sr, 6), music.go:117

// Go int(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> MinInt64
int64_t go_int(double x) {
  if (!(x >= -9.2233720368547758e18 && x < 9.2233720368547758e18)) return std::numeric_limits<int64_t>::min();
  return (int64_t)x;
}

// SpectralContrast.initializeBands (spectral_contrast.go:140-185)
std::vector<int> contrast_edges(int sample_rate, int K, int nb) {
  std::vector<int> e(nb + 1);
  const double nyquist = (double)sample_rate / 2.0;
  const double minf = 200.0;
  double maxf = nyquist;
  if (maxf <= minf) maxf = minf * 2;
  const double lmin = std::log10(minf), lmax = std::log10(maxf);
  const double step = (lmax - lmin) / (double)nb;
  for (int i = 0; i <= nb; i++) {
    const double f = std::pow(10.0, lmin + (double)i * step);
    int64_t b = go_int(f * (double)(K - 1) / nyquist);
    if (b >= K) b = K - 1;
    if (b < 0) b = 0;
    e[i] = (int)b;
  }
  for (int i = 1; i <= nb; i++)
    if (e[i] <= e[i - 1]) e[i] = e[i - 1] + 1;
  return e;
}

// gonum stat.Variance(x, nil) (v0.16.0 MeanVariance: compensated two-pass, n - 1), with the
// mean's sum sequential (gonum's amd64 kernel pairs terms: agreement to rounding, parity unpinned)
double gonum_variance(const std::vector<double>& x) {             // common/math.go:22-27
  if (x.size() < 2) return 0.0;
  double s = 0.0;
  for (double v : x) s += v;
  const double mean = s / (double)x.size();
  double ss = 0.0, comp = 0.0;
  for (double v : x) { const double d = v - mean; ss += d * d; comp += d; }
  return (ss - comp * comp / (double)x.size()) / (double)(x.size() - 1);
}

template <typename T>
int d2h(sonar_ctx* c, std::vector<T>& v, const void* d, size_t n) {
  v.resize(n);
  if (n) HIP_TRY(c, hipMemcpyAsync(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, c->stream));
  return SONAR_OK;
}

}  // namespace

extern "C" {

int sonar_extract_music_features(sonar_ctx* c, const double* pcm, int64_t n, int32_t sample_rate,
                                 const sonar_feature_config* fc, sonar_result** out) {
  if (!c || !fc || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  if (!pcm || n <= 0) return fail(c, SONAR_ERR_INVALID, "invalid input data");        // music.go:179-181
  const int W = fc->stft_window_size, H = fc->stft_hop_size;    // the spectrogram handed in
  const int64_t F = sonar_stft_frames(n, W, H);
  if (F == SONAR_ERR_INVALID) return fail(c, SONAR_ERR_INVALID, W <= 0 ? "window size must be positive" : "hop size must be positive");
  if (F < 0) return fail(c, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int csr = fc->sample_rate;                                // m.config.SampleRate
  const int K = W / 2 + 1;
  const int64_t Fz = F;

  // ---- device inputs: the PCM and preprocessAudio (:245-259: DC removal, pre-emphasis 0.95) ----
  double* dpcm = (double*)dbuf(c, "mx.pcm", n * 8);
  double* dy = (double*)dbuf(c, "mx.pre", n * 8);
  double* dcs = (double*)dbuf(c, "mx.dcscratch", sonar::dc_preemph_scratch_bytes(n));
  if (!dpcm || !dy || !dcs) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (pcm)");
  HIP_TRY(c, hipMemcpyAsync(dpcm, pcm, n * 8, hipMemcpyHostToDevice, s));
  if (sonar::launch_dc_preemph(dpcm, n, 0.995, 0.95, dy, dcs, s) != 0) return fail(c, SONAR_ERR_DEVICE, "dc launch failed");

  // ---- the spectrogram's features in one fused launch: descriptors (:270-299), |X|^4 MFCC with
  // 13 coefficients over 26 mel filters (:105-114, :304-325, F5), and the magnitude rows ------
  double* dmag = (double*)dbuf(c, "mx.mag", (size_t)Fz * K * 8);
  double* dmfcc = (double*)dbuf(c, "mx.mfcc", (size_t)Fz * 13 * 8);
  double* dspec = (double*)dbuf(c, "mx.spec", (size_t)Fz * 9 * 8);
  if (!dmag || !dmfcc || !dspec) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (spectrogram)");
  sonar_fp_cfg cfg;
  sonar_fp_cfg_default(&cfg);
  cfg.window_size = W; cfg.hop_size = H; cfg.window_type = fc->window_type;
  cfg.sample_rate = csr;
  cfg.n_mfcc = 13; cfg.n_filters = 26; cfg.use_lifter = 1; cfg.lifter = 22.0;
  cfg.low_freq = 0.0; cfg.high_freq = (double)csr / 2.0;
  cfg.mfcc_input_power = 1;                                       // MFCC.Compute fed |X|^2 (F5)
  cfg.flags = SONAR_FP_MFCC | SONAR_FP_SPECTRAL | SONAR_FP_MAGNITUDE;
  cfg.precision = fc->precision; cfg.pcm_dtype = SONAR_F64; cfg.out_dtype = SONAR_F64; cfg.device_ptrs = 1;
  sonar_fp_out fo;
  std::memset(&fo, 0, sizeof(fo));
  fo.mfcc = dmfcc; fo.magnitude = dmag;
  fo.centroid = dspec; fo.rolloff = dspec + Fz; fo.bandwidth = dspec + 2 * Fz; fo.flatness = dspec + 3 * Fz;
  fo.crest = dspec + 4 * Fz; fo.slope = dspec + 5 * Fz; fo.flux = dspec + 6 * Fz; fo.low_ratio = dspec + 7 * Fz;
  fo.high_ratio = dspec + 8 * Fz;
  int rc = sonar_fingerprint(c, dpcm, n, &cfg, &fo);
  if (rc != SONAR_OK) return rc;

  // ---- spectral contrast and extractEnergyFeatures' band ratios per magnitude row ----------
  const std::vector<int> edges = contrast_edges(csr, K, kContrastBands);
  int maxband = 1;
  for (int b = 0; b < kContrastBands; b++) maxband = std::max(maxband, std::min(edges[b + 1], K) - edges[b]);
  int* dedges = (int*)dbuf(c, "mx.edges", 64);
  double* dcon = (double*)dbuf(c, "mx.contrast", (size_t)Fz * kContrastBands * 8);
  double* dlh = (double*)dbuf(c, "mx.lohi", (size_t)Fz * 2 * 8);
  if (!dedges || !dcon || !dlh) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (contrast)");
  HIP_TRY(c, hipMemcpyAsync(dedges, edges.data(), edges.size() * sizeof(int), hipMemcpyHostToDevice, s));
  if (sonar::launch_music_frames(dmag, Fz, K, dedges, kContrastBands, maxband, dcon, dlh, dlh + Fz, s) != 0)
    return fail(c, SONAR_ERR_UNSUPPORTED, "spectral contrast launch failed (window too large for LDS?)");

  // ---- chroma (:327-376) on the preprocessed PCM -------------------------------------------
  double* dchroma = (double*)dbuf(c, "mx.chroma", (size_t)Fz * 12 * 8);
  if (!dchroma) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (chroma)");
  // FeatureConfig.HopSize <= 0: the per-frame ChromaSTFT's STFT rejects it (stft.go:54-56), and
  // ExtractFeatures returns the wrapped error (music.go:218-221, :358-361)
  if (fc->hop_size <= 0)
    return fail(c, SONAR_ERR_INVALID,
                "chroma feature extraction failed: chroma computation failed at frame 0: hop size must be positive");
  // frame f reads processedPCM[f hop : min(f hop + n/F, n)] (:348-352): a start past the end
  // (hop above the spectrogram's, so (F-1) hop > n) is Go's slice-bounds panic at the first such
  // frame; the spectral group and the MFCC were computed before it
  const int64_t chroma_bad = (F - 1) * (int64_t)fc->hop_size > n ? n / fc->hop_size + 1 : -1;
  if (chroma_bad < 0) {
    rc = sonar_chroma_stft(c, dy, n, F, fc->hop_size, csr, 0, dchroma, 1);
    if (rc != SONAR_OK) return rc;
  }

  // ---- temporal (:378-458): ShortTimeEnergy (FeatureConfig W / H), envelope, amplitudes ------
  const int64_t Fe = chroma_bad < 0 ? sonar_energy_frames(n, fc->window_size, fc->hop_size) : 0;
  double* den = (double*)dbuf(c, "mx.energy", (size_t)std::max<int64_t>(Fe, 1) * 8);
  double* dabs = (double*)dbuf(c, "mx.abs", 16);
  if (!den || !dabs) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (energy)");
  if (Fe > 0 && sonar::launch_energy(dy, 1, n, Fe, fc->window_size, fc->hop_size, 0.0, den, 1, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "energy launch failed");
  const int64_t fse = Fe > 0 ? n / Fe : 0;                        // frameSize := len(pcm) / numFrames (:383)
  const int64_t Fenv = (Fe > 0 && fse > 0 && fc->hop_size > 0 && n >= fse) ? (n - fse) / fc->hop_size + 1 : 0;
  double* denv = (double*)dbuf(c, "mx.env", (size_t)std::max<int64_t>(Fenv, 1) * 8);
  double* dpk = (double*)dbuf(c, "mx.peak", (size_t)std::max<int64_t>(Fe, 1) * 8);
  if (!denv || !dpk) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (envelope)");
  if (Fenv > 0 && sonar::launch_energy(dy, 1, n, Fenv, (int)fse, fc->hop_size, 0.0, denv, 1, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "envelope launch failed");
  if (chroma_bad < 0 && sonar::launch_abs_stats(dy, n, dabs, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "amplitude launch failed");
  if (Fe > 0 && sonar::launch_frame_peak(dy, n, Fe, fse, dpk, s) != 0) return fail(c, SONAR_ERR_DEVICE, "peak launch failed");
  // the harmonic block's one live case: a 1024-sample frame (DetectPitch's window, :539)
  const int64_t fsh = F > 0 ? n / F : 0;
  double* dyin = (double*)dbuf(c, "mx.yin", 16);
  if (!dyin) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (pitch)");
  const bool harmonic_live = fsh == 1024 && n < 1536 && chroma_bad < 0;
  if (harmonic_live && sonar::launch_yin(dy, n, 1, 1024, csr, dyin, dyin + 1, nullptr, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "yin launch failed");

  std::vector<double> mfcc, spec, con, lh, chroma, energy, env, abss, peaks, yv;
  if (d2h(c, mfcc, dmfcc, Fz * 13) || d2h(c, spec, dspec, Fz * 9) || d2h(c, con, dcon, Fz * kContrastBands) ||
      d2h(c, lh, dlh, Fz * 2) || d2h(c, chroma, dchroma, chroma_bad < 0 ? Fz * 12 : 0) ||
      d2h(c, energy, den, (size_t)Fe) ||
      d2h(c, env, denv, (size_t)Fenv) || d2h(c, abss, dabs, 2) || d2h(c, peaks, dpk, (size_t)Fe) ||
      d2h(c, yv, dyin, harmonic_live ? 2 : 0))
    return SONAR_ERR_DEVICE;
  HIP_TRY(c, hipStreamSynchronize(s));

  auto* res = new sonar_result();
  // extractSpectralFeatures (:261-302): flux[0] = 0, flux[t] = flux(t-1, t); ZCR allocated and
  // never filled (zeros)
  static const char* names[6] = {"spectral_centroid", "spectral_rolloff", "spectral_bandwidth",
                                 "spectral_flatness", "spectral_crest", "spectral_slope"};
  for (int d = 0; d < 6; d++) res->put(names[d], std::vector<double>(spec.begin() + d * Fz, spec.begin() + (d + 1) * Fz), F, 1);
  {
    std::vector<double> flux(Fz, 0.0);
    for (int64_t t = 1; t < F; t++) flux[t] = spec[6 * Fz + t - 1];
    res->put("spectral_flux", std::move(flux), F, 1);
  }
  res->put("zero_crossing_rate", std::vector<double>(Fz, 0.0), F, 1);
  res->put("spectral_contrast", std::move(con), F, kContrastBands);
  res->put("mfcc", std::move(mfcc), F, 13);
  if (chroma_bad >= 0) {
    char msg[96];
    std::snprintf(msg, sizeof(msg), "runtime error: slice bounds out of range [%lld:%lld]",
                  (long long)(chroma_bad * fc->hop_size), (long long)n);
    *out = res;
    return fail(c, SONAR_ERR_PANIC, msg);
  }
  res->put("chroma", std::move(chroma), F, 12);
  res->vec("rms_energy", energy);
  // numFrames := len(RMSEnergy); frameSize := len(pcm) / numFrames (:382-383)
  if (Fe == 0) {
    *out = res;
    return fail(c, SONAR_ERR_PANIC, "runtime error: integer divide by zero");
  }
  res->vec("envelope_shape", env);
  const double peak_amp = abss[0], avg_amp = abss[1] / (double)n;   // :386-397
  res->scalar("peak_amplitude", peak_amp);
  res->scalar("average_amplitude", avg_amp);
  // DynamicRange.ComputeRange(pcm, 10.0, 90.0) (:401-403): RMS 1024 / 512 frames, then
  // sorted[int(10 * (L - 1))]: an index past the end for every L >= 2
  const int64_t L = n >= 1024 ? (n - 1024) / 512 + 1 : 0;
  if (L >= 2) {
    char msg[96];
    std::snprintf(msg, sizeof(msg), "runtime error: index out of range [%lld] with length %lld",
                  (long long)go_int(10.0 * (double)(L - 1)), (long long)L);
    *out = res;
    return fail(c, SONAR_ERR_PANIC, msg);
  }
  // L <= 1: the single value (or none) against itself -> 0 dB (dynamic_range.go:67-76)
  res->scalar("dynamic_range", 0.0);
  // onsets (:405-425): STFT 1024 / 512 of at most one frame -> no flux values -> no onsets;
  // a signal of at most 512 samples makes that STFT fail, and the extractor with it (:412-415)
  if (n <= 512) {
    delete res;
    return fail(c, SONAR_ERR_TOO_SHORT, "temporal feature extraction failed: signal too short for given window size and hop size");
  }
  res->scalar("onset_density", 0.0);
  res->vec("attack_time", {});
  {
    std::vector<double> crest(Fe, 0.0);                           // :428-444
    for (int64_t i = 0; i < Fe; i++) if (energy[i] > 0) crest[i] = peaks[i] / energy[i];
    res->vec("crest_factor", crest);
  }
  // ComputeSilenceRatio(pcm, spectrogram.SampleRate, -40) (silence_detection.go:171-193): RMS of
  // 25 ms frames; an RMS is never below -40, so every frame is not silent
  {
    const int fs = (int)(0.025 * (double)sample_rate), hs = fs / 2;
    const int64_t ns = (fs > 0 && hs > 0 && n >= fs) ? (n - fs) / hs + 1 : 0;
    const double sil = 0.0;
    (void)ns;
    res->scalar("silence_ratio", sil);
    res->vec("activity_level", std::vector<double>(Fe, 1.0 - sil));
  }
  // extractEnergyFeatures (:460-525)
  res->vec("short_time_energy", energy);
  res->scalar("energy_variance", gonum_variance(energy));
  {
    std::vector<double> ent(Fe, 0.0);
    double mx = 0.0, mn = std::numeric_limits<double>::infinity();
    for (int64_t i = 0; i < Fe; i++) {
      const double e = energy[i];
      if (e > 0) ent[i] = -e * std::log2(e);
      if (e > mx) mx = e;
      if (e < mn && e > 0) mn = e;
    }
    res->vec("energy_entropy", ent);
    res->scalar("loudness_range", (mn != std::numeric_limits<double>::infinity() && mn > 0) ? 20 * std::log10(mx / mn) : 0.0);
    res->vec("low_energy_ratio", std::vector<double>(lh.begin(), lh.begin() + Fz));
    res->vec("high_energy_ratio", std::vector<double>(lh.begin() + Fz, lh.end()));
  }
  // extractHarmonicFeatures (:528-583): DetectPitch takes only 1024-sample frames, the harmonic
  // ratio 2048 and the inharmonicity 4096 (F7); with a fresh detector the one live frame is
  // the raw YIN result through the temporal tracking of its first frame
  {
    std::vector<double> pe(Fz, 0.0), pc(Fz, 0.0), vs(Fz, 0.0), hr(Fz, 0.0), ih(Fz, 0.0), tc(Fz, 0.0);
    if (harmonic_live) {
      sonar::host::YinTracker tr;
      double p = yv[0], q = yv[1], v = 0.0;
      tr.step(p, q, v);
      pe[0] = p; pc[0] = q; vs[0] = v;
    }
    for (int64_t t = 0; t < F; t++) tc[t] = spec[t] * vs[t];      // centroid x voicing (:580-581)
    res->vec("pitch_estimate", pe);
    res->vec("pitch_confidence", pc);
    res->vec("voicing_strength", vs);
    res->vec("harmonic_ratio", hr);
    res->vec("inharmonicity_ratio", ih);
    res->vec("tonal_centroid", tc);
  }
  *out = res;
  return SONAR_OK;
}

}  // extern "C"
