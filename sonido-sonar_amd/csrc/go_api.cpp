// go_api.cpp -- C++ restatement of the Go orchestration above the GPU seams.
//
//   sonar_generate_fingerprint      FingerprintGenerator.GenerateFingerprint
//                                   (fingerprint/fingerprint.go:137-236) with the
//                                   ContentAwareConfigManager tables (content_config.go:54-278)
//   sonar_extract_speech_features   SpeechFeatureExtractor.ExtractFeatures
//                                   (fingerprint/extractors/speech.go:135-550)
//   sonar_align_features            AlignmentExtractor.ExtractAlignmentFeatures
//                                   (fingerprint/extractors/alignment.go:139-476)
//
// Every per-frame / per-cell array is produced by a HIP kernel (sonar_fingerprint,
// YIN, NCC, DTW, energy, tilt, stats); this file only runs what the Go code runs
// sequentially on O(frames) data: YIN temporal tracking, percentile thresholds,
// onset peak picking, scorer formulas.  Formants (lpc_kernels.hip), voice quality
// (voice_api.cpp) and content detection (content_api.cpp) run on their own kernels;
// fingerprint ID/timestamp metadata is not produced.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
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

enum ContentType { CT_MUSIC = 0, CT_NEWS, CT_SPORTS, CT_TALK, CT_MIXED, CT_UNKNOWN };

int to_content_type(const char* s) {   // config.ToContentType (fingerprint/config/config.go:50-65)
  if (!s) return CT_UNKNOWN;
  const std::string v(s);
  if (v == "music") return CT_MUSIC;
  if (v == "news") return CT_NEWS;
  if (v == "sports") return CT_SPORTS;
  if (v == "talk") return CT_TALK;
  if (v == "mixed") return CT_MIXED;
  return CT_UNKNOWN;
}

struct Settings { bool mfcc, speech, temporal; };
// content_config.go:104-278 (sports has no entry -> unknown settings, :68-72)
Settings settings_for(int ct) {
  switch (ct) {
    case CT_MUSIC: return {true, false, false};
    case CT_NEWS: return {true, true, true};
    case CT_TALK: return {true, true, true};
    case CT_MIXED: return {true, true, true};
    default: return {true, false, true};
  }
}

template <typename T>
int d2h(sonar_ctx* c, std::vector<T>& v, const void* d, size_t n) {
  v.resize(n);
  if (n) HIP_TRY(c, hipMemcpyAsync(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, c->stream));
  return SONAR_OK;
}

double percentile10_threshold(std::vector<double> e) {            // speech.go:594-604 (bubble sort)
  // the element at index n/10 of the sorted order; a selection gives the same value in O(n)
  std::nth_element(e.begin(), e.begin() + e.size() / 10, e.end());
  return e[e.size() / 10];
}

// speech_analysis.go:165-202 on the first 1024 samples
bool check_periodicity(const std::vector<double>& fr) {
  if (fr.size() < 1024) return false;
  double mc = 0.0;
  for (int lag = 20; lag < 400 && lag < 512; lag++) {
    double corr = 0.0; int cnt = 0;
    for (int i = 0; i < 1024 - lag; i++) { corr += fr[i] * fr[i + lag]; cnt++; }
    if (cnt > 0) { corr /= (double)cnt; if (corr > mc) mc = corr; }
  }
  double en = 0.0;
  for (int i = 0; i < 1024; i++) en += fr[i] * fr[i];
  en /= 1024.0;
  if (en > 0) mc /= en;
  return mc > 0.1;
}

}  // namespace

extern "C" {

void sonar_fingerprint_config_default(sonar_fingerprint_config* c) {   // fingerprint.go:70-98
  std::memset(c, 0, sizeof(*c));
  c->window_size = 2048;
  c->hop_size = 512;
  c->feature_window_size = 0;    // FeatureConfig.WindowSize is unset in the default config (F13)
  c->feature_hop_size = 0;
  c->enable_content_detect = 1;
  c->window_type = SONAR_WIN_HANN;
  c->precision = SONAR_F64;
  c->acoustic_detection = 1;     // ContentConfig (fingerprint.go:92-96)
  c->default_content_type = SONAR_CT_UNKNOWN;
  c->auto_detect_threshold = 2.0;
}

void sonar_feature_config_default(sonar_feature_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->stft_window_size = 1024;
  c->stft_hop_size = 256;
  c->window_type = SONAR_WIN_HANN;
  c->enable_mfcc = 1;
  c->mfcc_coefficients = 13;
  c->is_news = 1;
  c->precision = SONAR_F64;
}

// ------------------------------------------------ SpeechFeatureExtractor ----
int sonar_extract_speech_features(sonar_ctx* c, const double* pcm, int64_t n, int32_t sample_rate,
                                  const sonar_feature_config* fc, sonar_result** out) {
  if (!c || !fc || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  if (n <= 0 || !pcm) return fail(c, SONAR_ERR_EMPTY, "PCM data cannot be empty");
  if (sample_rate <= 0) return fail(c, SONAR_ERR_INVALID, "sample rate must be positive");
  const int W = fc->stft_window_size, H = fc->stft_hop_size;
  const int64_t F = sonar_stft_frames(n, W, H);
  if (F == SONAR_ERR_EMPTY) return fail(c, SONAR_ERR_EMPTY, "empty signal");
  if (F == SONAR_ERR_INVALID) return fail(c, SONAR_ERR_INVALID, W <= 0 ? "window size must be positive" : "hop size must be positive");
  if (F < 0) return fail(c, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int csr = fc->sample_rate;                                // FeatureConfig.SampleRate (0 under F1)
  const int K = W / 2 + 1;
  const int nm = fc->mfcc_coefficients > 0 ? fc->mfcc_coefficients : 13;
  const int64_t Fe = sonar_energy_frames(n, fc->window_size, fc->hop_size);
  const int64_t Fp = sonar_pitch_frames(n);
  (void)K;

  // ---- device buffers ------------------------------------------------------------
  double* dpcm = (double*)dbuf(c, "sx.pcm", n * 8);
  double* dy = (double*)dbuf(c, "sx.pre", n * 8);
  if (!dpcm || !dy) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (pcm)");
  const size_t fsz = (size_t)std::max<int64_t>(F, 1);
  double* dmfcc = (double*)dbuf(c, "sx.mfcc", fsz * nm * 8);
  double* dspec = (double*)dbuf(c, "sx.spec", fsz * 9 * 8);
  double* dzcr = (double*)dbuf(c, "sx.zcr", fsz * 8);
  double* den = (double*)dbuf(c, "sx.energy", std::max<int64_t>(Fe, 1) * 8);
  if (!dmfcc || !dspec || !dzcr || !den) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (features)");
  double* dpit = (double*)dbuf(c, "sx.pitch", std::max<int64_t>(Fp, 1) * 8);
  double* dcon = (double*)dbuf(c, "sx.conf", std::max<int64_t>(Fp, 1) * 8);
  if (!dpit || !dcon) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (pitch)");
  // extractSimpleEnvelope (speech.go:752-777): RMS 512/256 of the pre-emphasised PCM
  const int64_t Fenv = sonar_energy_frames(n, 512, 256);
  double* denv = (double*)dbuf(c, "sx.env", std::max<int64_t>(Fenv, 1) * 8);
  // ComputeLoudnessRange (energy.go:145-178): 400 ms / 100 ms RMS frames when sr > 0
  const int lw = (int)(0.4 * (double)csr);
  const int lh = std::max(1, lw / 4);
  const int64_t Fl = csr > 0 ? sonar_energy_frames(n, lw, lh) : 0;
  double* dld = (double*)dbuf(c, "sx.loud", std::max<int64_t>(Fl, 1) * 8);
  if (!denv || !dld) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (envelope)");

  // the fused STFT kernel: MFCC + descriptors + ZCR (the energy frames are launched beside it)
  sonar_fp_cfg cfg;
  sonar_fp_cfg_default(&cfg);
  cfg.window_size = W; cfg.hop_size = H; cfg.window_type = fc->window_type;
  cfg.sample_rate = csr;                                          // NewMFCC(config.SampleRate, ...) etc.
  cfg.n_mfcc = nm; cfg.n_filters = 26; cfg.use_lifter = 1; cfg.lifter = 22.0;   // NewMFCC defaults (mfcc.go:44-54)
  cfg.low_freq = 0.0; cfg.high_freq = (double)csr / 2.0;
  cfg.preemph_alpha = 0.97;
  cfg.flags = SONAR_FP_SPECTRAL | SONAR_FP_ZCR | (fc->enable_mfcc ? SONAR_FP_MFCC : 0);
  cfg.precision = fc->precision; cfg.pcm_dtype = SONAR_F64; cfg.out_dtype = SONAR_F64; cfg.device_ptrs = 1;
  sonar_fp_out fo;
  std::memset(&fo, 0, sizeof(fo));
  fo.mfcc = dmfcc;
  const size_t Fz = (size_t)F;
  fo.centroid = dspec; fo.rolloff = dspec + Fz; fo.bandwidth = dspec + 2 * Fz; fo.flatness = dspec + 3 * Fz;
  fo.crest = dspec + 4 * Fz; fo.slope = dspec + 5 * Fz; fo.flux = dspec + 6 * Fz; fo.low_ratio = dspec + 7 * Fz;
  fo.high_ratio = dspec + 8 * Fz; fo.zcr = dzcr;
  if (!c->side) {
    HIP_TRY(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    for (auto& e : c->side_ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }

  // ---- results: ONE pinned block from the pool, every array copied into it by DMA; the result's
  // large arrays point into the block (no host copy, no page faults on fresh vectors).  The
  // per-frame arrays travel chunk by chunk during the pipeline below, the rest after it ----
  const size_t Fe_z = (size_t)std::max<int64_t>(Fe, 0), Fp_z = (size_t)std::max<int64_t>(Fp, 0);
  const size_t Fenv_z = (size_t)std::max<int64_t>(Fenv, 0), Fl_z = (size_t)std::max<int64_t>(Fl, 0);
  const bool lohi_copy = (int64_t)Fe_z > F;                       // Go pads the ratios past the spectrogram
  const int SB = 256;
  size_t off = 0;
  auto take = [&](size_t cnt) { const size_t o = off; off += (cnt + 7) & ~size_t(7); return o; };
  const size_t o_mfcc = take(fc->enable_mfcc ? Fz * nm : 0), o_spec = take(Fz * 9), o_zcr = take(Fz);
  const size_t o_en = take(Fe_z), o_ent = take(Fe_z), o_praw = take(Fp_z), o_craw = take(Fp_z);
  const size_t o_part = take(SB * 4), o_env = take(Fenv_z), o_loud = take(Fl_z);
  const size_t o_tilt = take(fc->enable_speech_features ? Fp_z : 0), o_head = take((size_t)std::min<int64_t>(n, 1024));
  const size_t o_trk = take(6 * Fp_z), o_lohi = take(lohi_copy ? 2 * Fe_z : 0);
  std::shared_ptr<void> blk = sonar::detail::pinned_block(off * 8);
  if (!blk) return fail(c, SONAR_ERR_NOMEM, "pinned host allocation failed (results)");
  double* B = (double*)blk.get();

  // ---- the host PCM crosses PCIe in chunks on the copy stream; once chunk k has landed, every
  // frame whose samples lie in [0, end of chunk k) is computed while the next chunk is in flight:
  // pre-emphasis of the chunk, the fused STFT kernel + descriptors + ZCR over the frames it
  // completes, the energy / envelope / loudness frames, and YIN (1024 / 512) on the side stream.
  // Frames are independent (the flux reads the previous frame's |X| row, already written in stream
  // order), so the results equal the one-shot schedule's.  The fused kernel takes frame ranges on
  // the per-frame path (W = 128 .. 2048); other W run it once after the last chunk.
  int64_t CH = n > ((int64_t)24 << 20) ? ((int64_t)8 << 20) : n;         // 8 M samples (64 MB) per chunk
  if (const char* e = std::getenv("SONAR_PCM_CHUNK")) {                   // samples per chunk (tests)
    const long long v = std::atoll(e);
    if (v > 0) CH = std::min<int64_t>(n, v);
  }
  const int64_t NCH = (n + CH - 1) / CH;
  auto grow_ev = [&](std::vector<hipEvent_t>& v, int64_t cnt) -> int {
    while ((int64_t)v.size() < cnt) {
      hipEvent_t e;
      HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      v.push_back(e);
    }
    return SONAR_OK;
  };
  if (grow_ev(c->back_ev, NCH)) return SONAR_ERR_DEVICE;
  if (NCH > 1) {
    if (!c->copy) HIP_TRY(c, hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
    if (grow_ev(c->chunk_ev, NCH)) return SONAR_ERR_DEVICE;
    HIP_TRY(c, hipEventRecord(c->side_ev[0], s));                // the buffers' previous readers
    HIP_TRY(c, hipStreamWaitEvent(c->copy, c->side_ev[0], 0));
  }
  const bool fp_chunks = sonar::fingerprint_supported(W);
  // frames t < total whose samples [t hop, t hop + win) lie below sample b (all of them at the end)
  auto ready = [&](int64_t b, int64_t total, int64_t win, int64_t hop) -> int64_t {
    if (b >= n) return total;
    if (b < win || hop <= 0) return 0;
    return std::min<int64_t>(total, (b - win) / hop + 1);
  };
  // the harmonic features' tracker runs chunk by chunk during the pipeline (below) when the speech
  // block does not need the pitch rows first (SONAR_GF_EARLY=0: after the last chunk)
  const char* gf_env = std::getenv("SONAR_GF_EARLY");
  const int gf_early = gf_env ? std::atoi(gf_env) : 1;
  // the device's address of the block's pitch rows (mapped pinned memory); none -> the late order
  double *hpit = nullptr, *hcon = nullptr;
  if (!fc->enable_speech_features && gf_early != 0 && Fp_z) {
    void* dB = nullptr;
    if (hipHostGetDevicePointer(&dB, B, 0) == hipSuccess && dB) {
      hpit = (double*)dB + o_praw;
      hcon = (double*)dB + o_craw;
    } else {
      (void)hipGetLastError();
    }
  }
  const bool trk_early = hpit != nullptr;
  // YIN writes into the pinned block: on any early return the side stream is drained before the
  // block goes back to the pool (declared after `blk`, so it runs first)
  struct SideDrain {
    hipStream_t st;
    ~SideDrain() { if (st) (void)hipStreamSynchronize(st); }
  } side_drain{trk_early ? c->side : nullptr};
  int64_t done_fp = 0, done_e = 0, done_p = 0, done_env = 0, done_l = 0;
  std::vector<int64_t> p_end(NCH, 0);                              // pitch frames complete after chunk k
  for (int64_t k = 0; k < NCH; ++k) {
    const int64_t a = k * CH, b = std::min<int64_t>(n, a + CH);
    if (NCH > 1) {
      HIP_TRY(c, hipMemcpyAsync(dpcm + a, pcm + a, (size_t)(b - a) * 8, hipMemcpyHostToDevice, c->copy));
      HIP_TRY(c, hipEventRecord(c->chunk_ev[k], c->copy));
      HIP_TRY(c, hipStreamWaitEvent(s, c->chunk_ev[k], 0));
    } else {
      HIP_TRY(c, hipMemcpyAsync(dpcm, pcm, (size_t)n * 8, hipMemcpyHostToDevice, s));
    }
    // preprocessForSpeech: PreEmphasis("speech") alpha 0.97, fresh state (speech.go:238-245)
    if (sonar::launch_preemph(dpcm, 1, n, 0.97, dy, s, a, b) != 0) return fail(c, SONAR_ERR_DEVICE, "preemph launch failed");
    // YIN raw results on the pre-emphasised PCM (extractHarmonicFeatures :464), side stream
    const int64_t pk = ready(b, Fp, 1024, 512);
    if (pk > done_p) {
      HIP_TRY(c, hipEventRecord(c->side_ev[0], s));
      HIP_TRY(c, hipStreamWaitEvent(c->side, c->side_ev[0], 0));
      if (sonar::launch_yin(dy, n, Fp, 512, csr, trk_early ? hpit : dpit, trk_early ? hcon : dcon, nullptr,
                            c->side, done_p, pk) != 0)
        return fail(c, SONAR_ERR_DEVICE, "yin launch failed");
      done_p = pk;
    }
    const int64_t fk = fp_chunks ? ready(b, F, W, H) : (b >= n ? F : 0);
    if (fk > done_fp) {
      const int rc = sonar::detail::fingerprint_impl(c, dpcm, n, &cfg, &fo, true, done_fp, fk);
      if (rc != SONAR_OK) return rc;
      done_fp = fk;
    }
    const int64_t ek = ready(b, Fe, fc->window_size, fc->hop_size);
    if (ek > done_e && sonar::launch_energy(dpcm, 1, n, Fe, fc->window_size, fc->hop_size, 0.97, den, 1, s, done_e, ek) != 0)
      return fail(c, SONAR_ERR_DEVICE, "energy launch failed");
    done_e = std::max(done_e, ek);
    const int64_t vk = ready(b, Fenv, 512, 256);
    if (vk > done_env && sonar::launch_energy(dpcm, 1, n, Fenv, 512, 256, 0.97, denv, 1, s, done_env, vk) != 0)
      return fail(c, SONAR_ERR_DEVICE, "envelope launch failed");
    done_env = std::max(done_env, vk);
    const int64_t lk = ready(b, Fl, lw, lh);
    if (lk > done_l && sonar::launch_energy(dpcm, 1, n, Fl, lw, lh, 0.97, dld, 1, s, done_l, lk) != 0)
      return fail(c, SONAR_ERR_DEVICE, "loudness launch failed");
    // the tracker's input: with trk_early, YIN writes this chunk's pitch rows straight into the
    // pinned result block (mapped host memory) and the event marks them complete.  A DMA copy per
    // chunk instead queues behind the next chunk's H2D on the copy engine and serialises the
    // pipeline: 41-42 against 30 ms per hour (profiles/r06r_gf_early_ab.log)
    if (trk_early) HIP_TRY(c, hipEventRecord(c->back_ev[k], c->side));
    p_end[k] = done_p;
    done_l = std::max(done_l, lk);
  }
  HIP_TRY(c, hipEventRecord(c->side_ev[1], c->side));
  HIP_TRY(c, hipStreamWaitEvent(s, c->side_ev[1], 0));
  // whole-signal statistics of the pre-emphasised PCM: read by detectSpeech and the temporal
  // block only (the music generation config enables neither, content_config.go:108-140)
  double* dpart = (double*)dbuf(c, "sx.stats", SB * 4 * 8);
  if (!dpart) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (stats)");
  if (fc->enable_speech_features || fc->enable_temporal_features) {
    if (sonar::launch_stats(dy, n, dpart, SB, s) != 0) return fail(c, SONAR_ERR_DEVICE, "stats launch failed");
  } else {
    HIP_TRY(c, hipMemsetAsync(dpart, 0, SB * 4 * 8, s));
  }
  double* dtilt = (double*)dbuf(c, "sx.tilt", std::max<int64_t>(Fp, 1) * 8);
  if (fc->enable_speech_features && sonar::launch_tilt(dy, n, Fp, dtilt, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "tilt launch failed");

  double* dent = (double*)dbuf(c, "sx.ent", std::max<size_t>(Fe_z, 1) * 8);
  if (!dent) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (entropy)");
  if (Fe_z && sonar::launch_energy_entropy(den, (int64_t)Fe_z, dent, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "entropy launch failed");
  auto d2h = [&](size_t o, const void* d, size_t cnt) -> int {
    if (cnt) HIP_TRY(c, hipMemcpyAsync(B + o, d, cnt * 8, hipMemcpyDeviceToHost, s));
    return SONAR_OK;
  };
  // everything but the pitch rows
  if ((!trk_early && (d2h(o_praw, dpit, Fp_z) || d2h(o_craw, dcon, Fp_z))) ||
      d2h(o_mfcc, dmfcc, fc->enable_mfcc ? Fz * nm : 0) || d2h(o_spec, dspec, Fz * 9) || d2h(o_zcr, dzcr, Fz) ||
      d2h(o_en, den, Fe_z) || d2h(o_env, denv, Fenv_z) || d2h(o_loud, dld, Fl_z))
    return SONAR_ERR_DEVICE;
  if (d2h(o_ent, dent, Fe_z) || d2h(o_part, dpart, SB * 4) ||
      d2h(o_tilt, dtilt, fc->enable_speech_features ? Fp_z : 0) ||
      d2h(o_head, dy, (size_t)std::min<int64_t>(n, 1024)))
    return SONAR_ERR_DEVICE;
  // Without the speech block (the GenerateFingerprint content configs for music / news / sports,
  // content_config.go:108-140) the harmonic features' sequential tracker is the only consumer of the
  // pitch frames before the end: it runs chunk by chunk as each chunk's pitch rows land, while the
  // device and PCIe work on (the speech block's voicing pass must see the tracker first, so with it
  // the tracker runs after the sync, below)
  int64_t trk_done = 0;
  sonar::host::YinTracker tracker;
  const double* praw = B + o_praw;
  const double* craw = B + o_craw;
  double* pe = B + o_trk;
  double* pc = pe + Fp_z;
  double* vs = pc + Fp_z;
  double* hr = vs + Fp_z;
  double* ih = hr + Fp_z;
  double* tcen = ih + Fp_z;
  auto track = [&](int64_t hi) {                                  // extractHarmonicFeatures :464-509
    for (int64_t i = trk_done; i < hi; i++) {
      double p = 0.0, q = 0.0, v = 0.0;
      if (i * 512 + 1024 <= n) {                                  // DetectPitch size check (pitch_detection.go:226)
        p = praw[i]; q = craw[i];
        tracker.step(p, q, v);
      }
      pe[i] = p; pc[i] = q; vs[i] = v;
      hr[i] = v * 10.0;
      ih[i] = 1.0 - v;
      tcen[i] = p > 0 ? p : 0.0;
    }
    trk_done = std::max(trk_done, hi);
  };
  if (trk_early) {
    for (int64_t k = 0; k < NCH; ++k) {
      HIP_TRY(c, hipEventSynchronize(c->back_ev[k]));
      track(p_end[k]);
    }
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  const double* energy = B + o_en;
  const double* spec = B + o_spec;
  const double* part = B + o_part;

  auto* res = new sonar_result();
  res->hold(blk);
  if (fc->enable_mfcc) res->put_ext("mfcc", B + o_mfcc, F, nm);
  static const char* spec_names[9] = {"spectral_centroid", "spectral_rolloff", "spectral_bandwidth",
                                      "spectral_flatness", "spectral_crest", "spectral_slope", "spectral_flux",
                                      "", ""};
  for (int d = 0; d < 7; d++) {
    const int64_t cnt = d == 6 ? (F > 1 ? F - 1 : 0) : F;
    if (d == 6 && F <= 1) continue;                               // flux only when TimeFrames > 1 (:362-365)
    res->put_ext(spec_names[d], spec + d * Fz, cnt, 1);
  }
  res->put_ext("zero_crossing_rate", B + o_zcr, (int64_t)Fz, 1);

  // whole-signal stats: partials reduced in block order
  double peak = 0, sabs = 0, ssq = 0, cross = 0;
  for (int b = 0; b < SB; b++) {
    peak = std::max(peak, part[4 * b]); sabs += part[4 * b + 1]; ssq += part[4 * b + 2]; cross += part[4 * b + 3];
  }
  // cross-block sign changes at block boundaries are counted inside each block (i > 0 uses y[i-1])

  // ---- speech features (extractSpeechFeatures :272-313) -------------------------
  bool is_speech = false;
  double thr10 = 0.0;                                             // percentile10_threshold(energy), once
  bool have_thr10 = false;
  auto energy_thr10 = [&]() {
    if (!have_thr10) { thr10 = percentile10_threshold(std::vector<double>(energy, energy + Fe_z)); have_thr10 = true; }
    return thr10;
  };
  if (fc->enable_speech_features) {
    // detectSpeech (speech_analysis.go:105-132), sample rate = FeatureConfig.SampleRate
    bool sp = !(n < (int64_t)(csr / 4));
    const double z = n <= 1 ? 0.0 : cross / (double)(n - 1);
    if (sp && (z < 0.01 || z > 0.3)) sp = false;
    if (sp && std::sqrt(ssq / (double)n) < 0.001) sp = false;
    if (sp) sp = check_periodicity(std::vector<double>(B + o_head, B + o_head + std::min<int64_t>(n, 1024)));
    is_speech = sp;
    res->scalar("is_speech", sp ? 1.0 : 0.0);
    // AnalyzeSpeech -> FormantAnalyzer.AnalyzeFormants(preprocessed PCM) (speech_analysis.go:70-74,
    // format.go:85-124); a failed analysis leaves FormantResult nil (speech.go:297-303)
    std::vector<double> formants;
    double vtl = 17.5;
    if (sp) {
      const int W = csr >= 16000 ? 2048 : 1024, p = 12 + csr / 1000;
      sonar_formant_frame* dfm = (sonar_formant_frame*)dbuf(c, "sx.formant", sizeof(sonar_formant_frame));
      double* dham = (double*)dbuf(c, "sx.ham", W * 8);
      if (!dfm || !dham) { delete res; return fail(c, SONAR_ERR_NOMEM, "device allocation failed"); }
      std::vector<double> ham(W);
      for (int i = 0; i < W; i++) ham[i] = 0.54 - 0.46 * std::cos(2.0 * M_PI * (double)i / (double)(W - 1));
      sonar_formant_frame fm;
      if (hipMemcpyAsync(dham, ham.data(), W * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
          p > 64 || sonar::launch_formants(dy, 1, 0, W, p, csr, n >= W ? 1 : 0, dham, dfm, nullptr, nullptr, s) != 0 ||
          hipMemcpyAsync(&fm, dfm, sizeof(fm), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess) {
        delete res;
        return fail(c, SONAR_ERR_DEVICE, "formant launch failed");
      }
      if (fm.status == 0) {
        formants.assign(fm.frequency, fm.frequency + fm.n_formants);
        vtl = fm.vocal_tract_length;
      }
    }
    res->put("formant_frequencies", formants, formants.empty() ? 0 : 1, (int64_t)formants.size());   // convertFormantData
    res->scalar("vocal_tract_length", vtl);
    // AnalyzeSpeech -> VoiceQualityAnalyzer.AnalyzeVoiceQuality(preprocessed PCM) (speech_analysis.go:76-80);
    // a failed analysis leaves VoiceQualityResult nil and Jitter/Shimmer 0 (speech.go:287-288, 306-309)
    double jitter = 0.0, shimmer = 0.0;
    if (sp) {
      sonar_voice_quality_result vq;
      const int rc = sonar::detail::voice_quality(c, dy, n, csr, &vq);
      if (rc == SONAR_ERR_DEVICE || rc == SONAR_ERR_NOMEM) { delete res; return rc; }
      if (rc == SONAR_OK) { jitter = vq.jitter; shimmer = vq.shimmer; }
    }
    res->scalar("jitter", jitter);
    res->scalar("shimmer", shimmer);
    if (sp) {
      // estimateSpeechRate (speech.go:779-797) on the energy frames of the pre-emphasised PCM
      const double dur = (double)n / (double)csr;
      double sil = 0.0;
      if (Fe_z) {
        const double thr = energy_thr10();
        int64_t k = 0;
        for (size_t i = 0; i < Fe_z; i++) if (energy[i] <= thr) k++;
        sil = (double)k / (double)Fe_z;
      }
      const double speech_time = dur * (1.0 - sil);
      res->scalar("speech_rate", speech_time > 0 ? 4.0 * speech_time / dur : 3.0);
    } else {
      res->scalar("speech_rate", 0.0);
    }
    if (sp) {
      std::vector<double> voicing(Fp_z);                           // extractVoicingProbability (:530-550)
      for (int64_t i = 0; i < Fp; i++) {
        double p = praw[i], q = craw[i], v = 0;
        if (i * 512 + 1024 <= n) { tracker.step(p, q, v); voicing[i] = v; }
      }
      res->vec("voicing_probability", voicing);
      res->put_ext("spectral_tilt", B + o_tilt, (int64_t)Fp_z, 1);
      // extractPauseDurations (:587-637)
      std::vector<double> pauses;
      if (Fe_z) {
        const double thr = energy_thr10();
        const double fts = (double)fc->hop_size / (double)csr;
        bool in = false; int64_t st = 0;
        for (int64_t i = 0; i < (int64_t)Fe_z; i++) {
          if (energy[i] <= thr) { if (!in) { in = true; st = i; } }
          else if (in) { const double d = (double)(i - st) * fts; if (d > 0.1) pauses.push_back(d); in = false; }
        }
        if (in) { const double d = (double)((int64_t)Fe_z - st) * fts; if (d > 0.1) pauses.push_back(d); }
      }
      res->vec("pause_duration", pauses);
    }
  }

  // ---- temporal features (extractTemporalFeatures :370-409) ---------------------
  const double lrange = csr > 0 ? sonar::host::loudness_range_from_rms(std::vector<double>(B + o_loud, B + o_loud + Fl_z)) : 0.0;
  if (fc->enable_temporal_features) {
    res->put_ext("rms_energy", energy, (int64_t)Fe_z, 1);
    res->scalar("dynamic_range", lrange);
    double sil = 0.0;
    if (Fe_z) {                                                   // calculateSilenceRatio (:639-665)
      const double thr = energy_thr10();
      int64_t k = 0;
      for (size_t i = 0; i < Fe_z; i++) if (energy[i] <= thr) k++;
      sil = (double)k / (double)Fe_z;
    }
    res->scalar("silence_ratio", sil);
    res->scalar("peak_amplitude", peak);
    res->scalar("average_amplitude", n > 0 ? sabs / (double)n : 0.0);
    // detectOnsets (:668-693) + calculateAdaptiveThreshold (:695-716)
    std::vector<int64_t> onsets;
    if (Fe_z >= 3) {
      std::vector<double> der(Fe_z - 1);
      for (size_t i = 0; i + 1 < Fe_z; i++) der[i] = energy[i + 1] - energy[i];
      double sum = 0; for (double v : der) sum += v;
      const double mean = sum / (double)der.size();
      double var = 0; for (double v : der) { const double d = v - mean; var += d * d; }
      const double thr = mean + 2 * std::sqrt(var / (double)der.size());
      for (size_t i = 1; i + 1 < der.size(); i++)
        if (der[i] > der[i - 1] && der[i] > der[i + 1] && der[i] > thr) onsets.push_back((int64_t)i);
    }
    res->scalar("onset_density", (double)onsets.size() / ((double)n / (double)sample_rate));
    std::vector<double> att(onsets.size());                       // calculateAttackTimes (:718-749)
    const double fts = (double)fc->hop_size / (double)csr;
    for (size_t i = 0; i < onsets.size(); i++) {
      const int64_t on = onsets[i];
      const double pk = energy[on];
      int64_t st = on;
      for (int64_t j = on - 1; j >= 0 && j > on - 10; j--) if (energy[j] < 0.1 * pk) { st = j; break; }
      att[i] = (double)(on - st) * fts;
      if (att[i] > 0.1) att[i] = 0.1;
    }
    res->vec("attack_time", att);
    res->put_ext("envelope_shape", B + o_env, (int64_t)Fenv_z, 1);
  }

  // ---- energy features (extractEnergyFeatures :411-461) -------------------------
  res->put_ext("short_time_energy", energy, (int64_t)Fe_z, 1);
  res->scalar("energy_variance", sonar::host::energy_variance(energy, Fe_z));
  res->scalar("loudness_range", lrange);
  res->put_ext("energy_entropy", B + o_ent, (int64_t)Fe_z, 1);
  if (!lohi_copy) {                                               // every energy frame has a spectrogram row
    res->put_ext("low_energy_ratio", spec + 7 * Fz, (int64_t)Fe_z, 1);
    res->put_ext("high_energy_ratio", spec + 8 * Fz, (int64_t)Fe_z, 1);
  } else {
    double* lo = B + o_lohi;
    double* hi = lo + Fe_z;
    for (size_t i = 0; i < Fe_z; i++) {
      lo[i] = (int64_t)i < F ? spec[7 * Fz + i] : 0.0;
      hi[i] = (int64_t)i < F ? spec[8 * Fz + i] : 0.0;
    }
    res->put_ext("low_energy_ratio", lo, (int64_t)Fe_z, 1);
    res->put_ext("high_energy_ratio", hi, (int64_t)Fe_z, 1);
  }

  // ---- harmonic features (extractHarmonicFeatures :464-509) --------------------
  {
    track(Fp);                                                    // the rest (all of it after the speech block)
    res->put_ext("pitch_estimate", pe, (int64_t)Fp_z, 1);
    res->put_ext("pitch_confidence", pc, (int64_t)Fp_z, 1);
    res->put_ext("voicing_strength", vs, (int64_t)Fp_z, 1);
    res->put_ext("harmonic_ratio", hr, (int64_t)Fp_z, 1);
    res->put_ext("inharmonicity_ratio", ih, (int64_t)Fp_z, 1);
    res->put_ext("tonal_centroid", tcen, (int64_t)Fp_z, 1);
  }
  (void)is_speech;
  *out = res;
  return SONAR_OK;
}

// ------------------------------------------ FingerprintGenerator ------------
int sonar_generate_fingerprint(sonar_ctx* c, const double* pcm, int64_t n, int32_t sample_rate, const char* content_type,
                               const sonar_fingerprint_config* cfg, sonar_result** out) {
  if (!c || !cfg || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  int ct = to_content_type(content_type);                         // fingerprint.go:155
  if (ct == CT_UNKNOWN && cfg->enable_content_detect) {           // fingerprint.go:156-158
    int32_t d = CT_UNKNOWN;
    const int rc = sonar::detail::detect_content_type(c, pcm, n, sample_rate, 1, content_type, cfg->genre,
                                                      cfg->station, cfg->url, cfg->acoustic_detection,
                                                      cfg->default_content_type, cfg->auto_detect_threshold, &d);
    if (rc != SONAR_OK) return rc;
    ct = d;
  }
  const Settings st = settings_for(ct);                           // GetGenerationConfig -> buildFeatureConfig
  sonar_feature_config fc;
  sonar_feature_config_default(&fc);
  fc.sample_rate = 0;                                             // F1: SampleRate is never copied (content_config.go:87-103)
  fc.window_size = cfg->feature_window_size;                      // base FeatureConfig.WindowSize/HopSize
  fc.hop_size = cfg->feature_hop_size;
  fc.stft_window_size = cfg->window_size;                         // generationConfig.WindowSize/HopSize (:174-179)
  fc.stft_hop_size = cfg->hop_size;
  fc.window_type = cfg->window_type;
  fc.enable_mfcc = st.mfcc; fc.enable_speech_features = st.speech; fc.enable_temporal_features = st.temporal;
  fc.mfcc_coefficients = 13;
  fc.is_news = ct != CT_TALK;                                     // CreateExtractor (feature_extractor.go:38-62)
  fc.precision = cfg->precision;
  const int rc = sonar_extract_speech_features(c, pcm, n, sample_rate, &fc, out);
  if (rc != SONAR_OK) return rc;
  (*out)->scalar("content_type", (double)ct);
  (*out)->scalar("sample_rate", (double)sample_rate);
  (*out)->scalar("hop_size", (double)cfg->feature_hop_size);       // AudioFingerprint.HopSize (fingerprint.go:215)
  (*out)->scalar("duration_seconds", (double)n / (double)sample_rate);
  return SONAR_OK;
}

// ------------------------------------------ AlignmentExtractor --------------
}  // extern "C"

namespace {
// MusicFeatureExtractor energy + chroma (music.go:245-259, :327-376, :460-466) on c->stream; `tag`
// names this call's scratch, so two calls on different streams do not share it
int music_features_impl(sonar_ctx* c, const double* pcm, int64_t n, int32_t sr, int32_t stft_w, int32_t stft_h,
                        int32_t fw, int32_t fh, double* energy, double* chroma, int32_t device_ptrs,
                        const std::string& tag) {
  if (!c) return SONAR_ERR_INVALID;
  if (!pcm || n <= 0) return fail(c, SONAR_ERR_INVALID, "invalid input data");        // music.go:179-181
  if (stft_w <= 0 || stft_h <= 0) return fail(c, SONAR_ERR_INVALID, "window and hop size must be positive");
  const int64_t F = sonar_stft_frames(n, stft_w, stft_h);
  if (F <= 0) return fail(c, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
  if (fh <= 0) return fail(c, SONAR_ERR_INVALID, "hop size must be positive");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const double* dp = pcm;
  if (!device_ptrs) {
    void* b = dbuf(c, "mf.pcm" + tag, n * 8);
    if (!b) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    HIP_TRY(c, hipMemcpyAsync(b, pcm, n * 8, hipMemcpyHostToDevice, s));
    dp = (const double*)b;
  }
  double* y = (double*)dbuf(c, "mf.pre" + tag, n * 8);           // processedPCM
  if (!y) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  double* dcs = (double*)dbuf(c, "mf.dcscratch" + tag, sonar::dc_preemph_scratch_bytes(n));
  if (!dcs) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  if (sonar::launch_dc_preemph(dp, n, 0.995, 0.95, y, dcs, s) != 0) return fail(c, SONAR_ERR_DEVICE, "dc launch failed");
  const int64_t Fe = sonar_energy_frames(n, fw, fh);
  double* de = device_ptrs ? energy : (double*)dbuf(c, "mf.energy" + tag, std::max<int64_t>(Fe, 1) * 8);
  // ShortTimeEnergy of the already pre-emphasised signal: alpha 0 makes the kernel's
  // pre-emphasis the identity (x - 0 * x[n-1] == x exactly)
  if (Fe > 0 && sonar::launch_energy(y, 1, n, Fe, fw, fh, 0.0, de, 1, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "energy launch failed");
  double* dc = device_ptrs ? chroma : (double*)dbuf(c, "mf.chroma" + tag, F * 12 * 8);
  if (!de || !dc) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  const int rc = sonar_chroma_stft(c, y, n, F, fh, sr, 0, dc, 1);
  if (rc != SONAR_OK) return rc;
  if (!device_ptrs) {
    if (Fe > 0) HIP_TRY(c, hipMemcpyAsync(energy, de, Fe * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(chroma, dc, F * 12 * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SONAR_OK;
}
}  // namespace

extern "C" {

int sonar_music_alignment_features(sonar_ctx* c, const double* pcm, int64_t n, int32_t sr, int32_t stft_w,
                                   int32_t stft_h, int32_t fw, int32_t fh, double* energy, double* chroma,
                                   int32_t device_ptrs) {
  return music_features_impl(c, pcm, n, sr, stft_w, stft_h, fw, fh, energy, chroma, device_ptrs, "");
}

}  // extern "C"

namespace sonar {
namespace detail {

// ExtractAlignmentFeatures after the GPU work (alignment.go:139-476): the candidates' scorers,
// selectBestAlignment (:412-446) and estimateTimeStretch (:448-476)
void align_finish(const AlignIn& in, sonar_result* res, sonar_pair_record* rec) {
  const double qlen = (double)in.q_pcm_len / (double)in.sample_rate, rlen = (double)in.r_pcm_len / (double)in.sample_rate;
  if (res) {
    res->scalar("query_length", qlen);
    res->scalar("reference_length", rlen);
  }
  if (rec) {
    std::memset(rec, 0, sizeof(*rec));
    rec->temporal_offset = rec->offset_confidence = rec->alignment_similarity = rec->alignment_quality = NAN;
    rec->corr_offset_seconds = rec->dtw_distance = rec->peak_lag = NAN;
  }
  struct Cand { bool ok = false; int type = 0; sonar::host::AlignScores s; bool dtw = false;
                int64_t p0q = 0, p0r = 0, p1q = 0, p1r = 0, plen = 0; };
  Cand corr, chroma;
  if (in.corr || in.corr_sums) {   // alignWithFeatures (:357-410) on the energy correlation
    const auto m = in.corr_sums ? sonar::host::ncc_metrics(*in.corr_sums, in.L, in.nqe, in.nre)
                                : sonar::host::ncc_metrics(in.corr, 2 * in.L + 1, in.L, in.nqe, in.nre);
    corr.ok = true; corr.type = 1;
    corr.s = sonar::host::xcorr_scores(m, in.hop, in.sample_rate, (int)in.mlf);
    if (rec) { rec->peak_lag = (double)m.peak_lag; rec->corr_offset_seconds = corr.s.offset_seconds; }
    if (res && in.corr) {
      res->vec("correlations", std::vector<double>(in.corr, in.corr + 2 * in.L + 1));
      res->scalar("peak_lag", (double)m.peak_lag);
      res->scalar("peak_correlation", m.peak_corr);
      res->scalar("corr_snr", m.snr);
      res->scalar("corr_sharpness", m.sharpness);
      res->scalar("corr_peak_to_sidelobe", m.psl);
      res->scalar("corr_offset", (double)corr.s.offset);
      res->scalar("corr_offset_seconds", corr.s.offset_seconds);
      res->scalar("corr_similarity", corr.s.similarity);
      res->scalar("corr_confidence", corr.s.confidence);
      res->scalar("corr_quality", corr.s.quality);
      res->scalar("corr_noise_level", corr.s.noise_level);
    }
  }
  if (in.has_dtw) {  // alignWithDTW (:129-148)
    const int64_t P = in.P;
    chroma.ok = true; chroma.type = 2; chroma.dtw = true;
    const sonar::host::PathSums ps = in.path_sums ? *in.path_sums : sonar::host::path_sums(in.pq, in.pr, in.pc, P);
    chroma.s = sonar::host::dtw_scores(ps, in.nqc, in.nrc, in.dist, in.sample_rate);
    chroma.plen = P;
    if (P > 0) { chroma.p0q = ps.p0q; chroma.p0r = ps.p0r; chroma.p1q = ps.p1q; chroma.p1r = ps.p1r; }
    if (rec) rec->dtw_distance = in.dist;
    if (res && in.pq) {
      std::vector<double> vq(P), vr(P), vc(P);
      for (int64_t i = 0; i < P; i++) { vq[i] = in.pq[i]; vr[i] = in.pr[i]; vc[i] = in.pc[i]; }
      res->scalar("dtw_distance", in.dist);
      res->vec("dtw_path_query", vq);
      res->vec("dtw_path_reference", vr);
      res->vec("dtw_path_cost", vc);
      res->scalar("dtw_offset", (double)chroma.s.offset);
      res->scalar("dtw_offset_seconds", chroma.s.offset_seconds);
      res->scalar("dtw_similarity", chroma.s.similarity);
      res->scalar("dtw_confidence", chroma.s.confidence);
      res->scalar("dtw_quality", chroma.s.quality);
      res->scalar("dtw_stability", chroma.s.stability);
    }
  }
  // selectBestAlignment (:412-446); Go iterates a map (random order) with strict >:
  // here corr_energy is visited first, so exact ties go to it deterministically
  const Cand* best = nullptr;
  double best_score = 0.0;
  for (const Cand* cd : {&corr, &chroma}) {
    if (!cd->ok) continue;
    const double w = cd->type == 1 ? 1.0 : 0.7;
    const double sc = w * (0.4 * cd->s.confidence + 0.4 * cd->s.similarity + 0.2 * cd->s.quality);
    if (sc > best_score) { best_score = sc; best = cd; }
  }
  double stretch = 1.0;                                           // estimateTimeStretch (:448-476)
  if (best) {
    if (res) {
      res->scalar("temporal_offset", best->s.offset_seconds);
      res->scalar("offset_confidence", best->s.confidence);
      res->scalar("alignment_similarity", best->s.similarity);
      res->scalar("alignment_quality", best->s.quality);
      res->scalar("method", (double)best->type);
    }
    if (rec) {
      rec->temporal_offset = best->s.offset_seconds;
      rec->offset_confidence = best->s.confidence;
      rec->alignment_similarity = best->s.similarity;
      rec->alignment_quality = best->s.quality;
      rec->method = (double)best->type;
    }
    if (qlen > 0 && rlen > 0) {
      const double lr = qlen / rlen;
      stretch = lr;
      if (best->dtw && best->plen > 1) {
        const double qs = (double)(best->p1q - best->p0q + 1), rs = (double)(best->p1r - best->p0r + 1);
        if (rs > 0) stretch = 0.7 * (qs / rs) + 0.3 * lr;
      }
    }
  } else if (res) {
    res->scalar("method", 0.0);
  }
  if (res) {
    if (corr.ok) res->scalar("feature_similarity_corr_energy", corr.s.similarity);
    if (chroma.ok) res->scalar("feature_similarity_dtw_chroma", chroma.s.similarity);
    res->scalar("time_stretch", stretch);
  }
}

}  // namespace detail
}  // namespace sonar

namespace {

// AlignmentExtractor.ExtractAlignmentFeatures body; dev = the four feature arrays are device
// pointers on the ctx's device (no H2D), else host arrays
int align_impl(sonar_ctx* c, const double* qe, int64_t nqe, const double* re, int64_t nre, const double* qc,
               int64_t nqc, const double* rc_, int64_t nrc, int64_t q_pcm_len, int64_t r_pcm_len,
               int32_t sample_rate, int32_t feature_sample_rate, int32_t hop, int32_t win,
               double max_lag_seconds, int32_t dev, sonar_result** out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  if (hop <= 0) return fail(c, SONAR_ERR_INVALID, "hop size must be positive (NewAlignmentExtractor divides by it)");
  (void)win;
  const int64_t max_lag_samples = (int64_t)(max_lag_seconds * (double)feature_sample_rate);   // alignment.go:104
  const bool want_corr = qe && re && nqe > 0 && nre > 0, want_dtw = qc && rc_ && nqc > 0 && nrc > 0;
  const int64_t mlf = want_corr ? std::min(max_lag_samples / hop, std::min(nqe, nre) - 1) : 0;
  // device arrays: the NCC and the DTW are both queued before one stream synchronisation; their
  // small results (correlation, path length, status words) arrive in pinned host memory
  double* hcorr = nullptr;
  int64_t hL = 0;
  sonar::detail::DtwPending pend;
  if (dev) {
    HIP_TRY(c, hipSetDevice(c->device));
    int st = SONAR_OK;
    if (want_corr && want_dtw) {
      // the NCC (energies) and the DTW (chroma) are independent: the NCC runs on the side stream
      // beside the band kernel (which leaves LDS and wave slots free on every CU), and the main
      // stream waits for it, so the one synchronisation below still covers both
      if (!c->side) {
        HIP_TRY(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        for (auto& e : c->side_ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      }
      HIP_TRY(c, hipEventRecord(c->side_ev[0], c->stream));
      HIP_TRY(c, hipStreamWaitEvent(c->side, c->side_ev[0], 0));
      hipStream_t main_stream = c->stream;
      c->stream = c->side;
      st = sonar::detail::ncc_enqueue(c, qe, nqe, re, nre, (int32_t)mlf, &hcorr, &hL);
      c->stream = main_stream;
      if (st != SONAR_OK) return st;
      HIP_TRY(c, hipEventRecord(c->side_ev[1], c->side));
      st = sonar::detail::dtw_enqueue(c, qc, nqc, rc_, nrc, 12, -1, &pend);
      if (st != SONAR_OK) return st;
      HIP_TRY(c, hipStreamWaitEvent(c->stream, c->side_ev[1], 0));
    } else {
      if (want_corr) st = sonar::detail::ncc_enqueue(c, qe, nqe, re, nre, (int32_t)mlf, &hcorr, &hL);
      if (st == SONAR_OK && want_dtw) st = sonar::detail::dtw_enqueue(c, qc, nqc, rc_, nrc, 12, -1, &pend);
      if (st != SONAR_OK) return st;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  sonar::detail::AlignIn in;
  in.q_pcm_len = q_pcm_len; in.r_pcm_len = r_pcm_len; in.sample_rate = sample_rate; in.hop = hop;
  std::vector<double> cr;
  if (want_corr) {   // 2. energy cross-correlation (performMultiFeatureAlignment :320-333)
    const int64_t L = std::max<int64_t>(0, std::min({mlf, nqe - 1, nre - 1}));
    if (dev) {
      cr.assign(hcorr, hcorr + 2 * hL + 1);
    } else {
      cr.resize(2 * L + 1);
      const int rc = sonar_ncc(c, qe, nqe, re, nre, (int32_t)mlf, cr.data(), nullptr, 0);
      if (rc != SONAR_OK) return rc;
    }
    in.corr = cr.data(); in.L = L; in.nqe = nqe; in.nre = nre; in.mlf = mlf;
  }
  std::vector<int32_t> vpq, vpr;
  std::vector<double> vpc;
  if (want_dtw) {    // 4. chroma DTW (:346-351)
    int rc;
    if (dev) {
      rc = sonar::detail::dtw_finish(c, &pend, &in.pq, &in.pr, &in.pc, &in.P, &in.dist);
    } else {
      const int64_t cap = nqc + nrc + 1;
      vpq.resize(cap); vpr.resize(cap); vpc.resize(cap);
      rc = sonar_dtw(c, qc, nqc, rc_, nrc, 12, -1, &in.dist, vpq.data(), vpr.data(), vpc.data(), &in.P, nullptr, 0);
      in.pq = vpq.data(); in.pr = vpr.data(); in.pc = vpc.data();
    }
    if (rc != SONAR_OK) return rc;
    in.has_dtw = true; in.nqc = nqc; in.nrc = nrc;
  }
  auto* res = new sonar_result();
  sonar::detail::align_finish(in, res, nullptr);
  *out = res;
  return SONAR_OK;
}

}  // namespace

extern "C" {

int sonar_align_features(sonar_ctx* c, const double* qe, int64_t nqe, const double* re, int64_t nre, const double* qc,
                         int64_t nqc, const double* rc_, int64_t nrc, int64_t q_pcm_len, int64_t r_pcm_len,
                         int32_t sample_rate, int32_t feature_sample_rate, int32_t hop, int32_t win,
                         double max_lag_seconds, sonar_result** out) {
  return align_impl(c, qe, nqe, re, nre, qc, nqc, rc_, nrc, q_pcm_len, r_pcm_len, sample_rate, feature_sample_rate,
                    hop, win, max_lag_seconds, 0, out);
}

// One stream pair end to end from device-resident PCM: MusicFeatureExtractor energy + chroma of
// both streams (music.go:245-259, :327-376, :460-466) into ctx buffers, then
// ExtractAlignmentFeatures on those device arrays -- no feature round trip through the host.
int sonar_align_pair_device(sonar_ctx* c, const double* q_pcm, int64_t nq, const double* r_pcm, int64_t nr,
                            int32_t sample_rate, int32_t stft_window, int32_t hop, int32_t feature_window,
                            double max_lag_seconds, sonar_result** out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  if (stft_window <= 0 || hop <= 0) return fail(c, SONAR_ERR_INVALID, "window and hop size must be positive");
  const int64_t Fq = sonar_stft_frames(nq, stft_window, hop), Fr = sonar_stft_frames(nr, stft_window, hop);
  if (Fq <= 0 || Fr <= 0) return fail(c, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
  const int64_t Eq = sonar_energy_frames(nq, feature_window, hop), Er = sonar_energy_frames(nr, feature_window, hop);
  double* qe = (double*)dbuf(c, "ap.qe", std::max<int64_t>(Eq, 1) * 8);
  double* re = (double*)dbuf(c, "ap.re", std::max<int64_t>(Er, 1) * 8);
  double* qc = (double*)dbuf(c, "ap.qc", Fq * 12 * 8);
  double* rc = (double*)dbuf(c, "ap.rc", Fr * 12 * 8);
  if (!qe || !re || !qc || !rc) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  // the two streams' features are independent: r's on the side stream (its own scratch) beside q's
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->side) {
    HIP_TRY(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    for (auto& e : c->side_ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  HIP_TRY(c, hipEventRecord(c->side_ev[0], c->stream));        // the caller's PCM is ready on c->stream
  HIP_TRY(c, hipStreamWaitEvent(c->side, c->side_ev[0], 0));
  int st = music_features_impl(c, q_pcm, nq, sample_rate, stft_window, hop, feature_window, hop, qe, qc, 1, "");
  if (st != SONAR_OK) return st;
  hipStream_t main_stream = c->stream;
  c->stream = c->side;
  st = music_features_impl(c, r_pcm, nr, sample_rate, stft_window, hop, feature_window, hop, re, rc, 1, ".r");
  c->stream = main_stream;
  if (st != SONAR_OK) return st;
  HIP_TRY(c, hipEventRecord(c->side_ev[1], c->side));
  HIP_TRY(c, hipStreamWaitEvent(c->stream, c->side_ev[1], 0));
  return align_impl(c, Eq > 0 ? qe : nullptr, Eq, Er > 0 ? re : nullptr, Er, qc, Fq, rc, Fr, nq, nr, sample_rate,
                    sample_rate, hop, feature_window, max_lag_seconds, 1, out);
}

}  // extern "C"
