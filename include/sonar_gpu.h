/*
 * sonar_gpu.h -- C ABI of the MI355X (gfx950) implementation of the
 * sonido-sonar per-frame DSP + alignment hot path.
 *
 * Library: sonido-sonar_amd/lib/libsonar_gpu.so (HIP kernels + C++ host code).
 * Plain C types only: pointers, sizes, POD structs.  No torch, no HIP types.
 *
 * Every entry replaces one seam of the Go reference (RyanBlaney/sonido-sonar,
 * paths relative to the repo root); INTEGRATION.md shows the cgo binding.
 *
 *   sonar_fingerprint          <- SpectralAnalyzer.ComputeSTFTWithWindow
 *                                 (fingerprint/analyzers/spectral.go:385) fused with
 *                                 MFCC.ComputeFrames (algorithms/spectral/mfcc.go:167),
 *                                 the per-frame descriptors of
 *                                 SpeechFeatureExtractor.extractSpectralFeatures
 *                                 (fingerprint/extractors/speech.go:320) and
 *                                 Energy.ComputeShortTimeEnergy (algorithms/temporal/energy.go:25)
 *   sonar_fingerprint_batch    <- SpectralAnalyzer.ComputeSTFTBatch (fingerprint/analyzers/spectral.go:234)
 *   sonar_pitch_yin            <- PitchDetector.DetectPitch per-frame YIN core
 *                                 (algorithms/tonal/pitch_detection.go:225-420)
 *   sonar_chroma_stft          <- MusicFeatureExtractor.extractChromaFeatures
 *                                 (fingerprint/extractors/music.go:327) ->
 *                                 ChromaSTFT.ComputeChroma (algorithms/chroma/chroma_stft.go:45)
 *   sonar_ncc                  <- CrossCorrelation.Compute, NormalizedCrossCorrelation /
 *                                 TimeDomain (algorithms/stats/correlation.go:131)
 *   sonar_dtw                  <- DTWAlignment.Align (algorithms/stats/dtw.go:55)
 *   sonar_formants             <- FormantAnalyzer.AnalyzeMultipleFrames / AnalyzeFormants
 *                                 (algorithms/speech/format.go:85-449) over LPCAnalyzer.Analyze
 *                                 (algorithms/speech/lpc.go:44-265)
 *   sonar_voice_quality        <- VoiceQualityAnalyzer.AnalyzeVoiceQuality
 *                                 (algorithms/speech/voice_quality.go:56-111)
 *   sonar_generate_fingerprint <- FingerprintGenerator.GenerateFingerprint
 *                                 (fingerprint/fingerprint.go:137)
 *   sonar_extract_speech_features <- SpeechFeatureExtractor.ExtractFeatures
 *                                 (fingerprint/extractors/speech.go:135), the extractor
 *                                 GenerateFingerprint builds for every content type
 *   sonar_align_features       <- AlignmentExtractor.ExtractAlignmentFeatures
 *                                 (fingerprint/extractors/alignment.go:139)
 *   sonar_music_alignment_features <- MusicFeatureExtractor energy + chroma
 *                                 (fingerprint/extractors/music.go:178-376)
 *   sonar_detect_from_audio / sonar_detect_content_type
 *                              <- ContentDetector.DetectFromAudio / DetectContentType
 *                                 (fingerprint/content_detector.go:31-101)
 *   sonar_gallery_* / sonar_compare / sonar_find_best_matches
 *                              <- FingerprintComparator.Compare / BatchCompare /
 *                                 FindBestMatches (fingerprint/comparison.go:133-263, 1107)
 *
 * Conventions
 *  - Every call returns SONAR_OK (0) or a negative SONAR_ERR_*; the message
 *    (same text as the Go error where one exists) is in sonar_last_error(ctx).
 *  - Buffers are owned by the caller.  With cfg->device_ptrs == 0 they are
 *    host memory and the call is synchronous; with device_ptrs == 1 they are
 *    device pointers on the ctx's device and the call is asynchronous on the
 *    ctx stream (sonar_synchronize() waits).
 *  - One ctx per OS thread / goroutine (the Go objects are not goroutine-safe
 *    either).  Several ctxs may share one device.
 */
#ifndef SONAR_GPU_H
#define SONAR_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SONAR_ABI_VERSION 4

enum {
  SONAR_OK = 0,
  SONAR_ERR_INVALID = -1,      /* bad argument (message says which)            */
  SONAR_ERR_TOO_SHORT = -2,    /* "signal too short for given window size ..."  */
  SONAR_ERR_EMPTY = -3,        /* "empty signal" / "empty sequences provided"   */
  SONAR_ERR_UNSUPPORTED = -4,  /* configuration not implemented on the GPU path */
  SONAR_ERR_DEVICE = -5,       /* HIP runtime error                             */
  SONAR_ERR_NOMEM = -6,        /* device allocation failed                      */
  SONAR_ERR_PANIC = -7         /* the Go reference panics on this input (message: Go's runtime
                                  error text); see the entry for what *out then holds */
};

/* window types: analyzers.WindowType (fingerprint/analyzers/windowing.go:13-23) */
enum {
  SONAR_WIN_HANN = 0, SONAR_WIN_HAMMING, SONAR_WIN_BLACKMAN, SONAR_WIN_BLACKMAN_HARRIS,
  SONAR_WIN_KAISER, SONAR_WIN_TUKEY, SONAR_WIN_RECTANGULAR, SONAR_WIN_BARTLETT, SONAR_WIN_WELCH
};

enum { SONAR_F32 = 0, SONAR_F64 = 1 };              /* arithmetic / element types */
enum { SONAR_FB_MEL = 0, SONAR_FB_BARK = 1 };       /* mel_scale.go / bark_scale.go */

/* sonar_fp_cfg.flags: which outputs sonar_fingerprint produces */
enum {
  SONAR_FP_MFCC = 1u << 0,      /* out->mfcc       F x n_mfcc                        */
  SONAR_FP_MAGNITUDE = 1u << 1, /* out->magnitude  F x (W/2+1)  (SpectrogramResult)  */
  SONAR_FP_SPECTRAL = 1u << 2,  /* centroid..slope, flux (F-1), low/high energy ratio */
  SONAR_FP_ZCR = 1u << 3,       /* out->zcr        F, on the pre-emphasised PCM       */
  SONAR_FP_ENERGY = 1u << 4,    /* out->energy     sonar_energy_frames(), pre-emphasised */
  SONAR_FP_COMPLEX = 1u << 5,   /* out->complex    F x (W/2+1) x 2 (re, im)  SpectrogramResult.Complex */
  SONAR_FP_PHASE = 1u << 6,     /* out->phase      F x (W/2+1), atan2(im, re) SpectrogramResult.Phase */
  SONAR_FP_GENERIC = 1u << 30   /* force the general fused kernel (A/B checks of the f32 MFCC path) */
};

typedef struct sonar_ctx sonar_ctx;

/* ---- context ---------------------------------------------------------- */
int sonar_create(int device, sonar_ctx** out);
void sonar_destroy(sonar_ctx* ctx);
const char* sonar_last_error(const sonar_ctx* ctx);
int sonar_abi_version(void);
/* Run on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the ctx-owned stream. */
int sonar_set_stream(sonar_ctx* ctx, void* hip_stream);
int sonar_synchronize(sonar_ctx* ctx);
/* Average duration (ms) of the last `n` launches of the dominant kernel of
 * the last call, measured with HIP events on the stream it ran on (bench). */
int sonar_last_kernel_ms(sonar_ctx* ctx, double* ms);
int sonar_enable_kernel_timing(sonar_ctx* ctx, int on);
/* Name of the fused path-A kernel the last sonar_fingerprint call launched
 * ("mfcc_pair_kernel" or "fp_wave_kernel"; "" if none) -- diagnostics. */
const char* sonar_last_fp_kernel(sonar_ctx* ctx);
/* HIP-event durations (ms) of the kernels of the last sonar_dtw call on this
 * context: ms3[0] the band sweep (dtw_band_kernel), ms3[1] the backtrack walk,
 * ms3[2] the path decode -- diagnostics and the bench's DTW roofline. */
int sonar_dtw_last_timing(sonar_ctx* ctx, double* ms3);
/* Liveness counters of the DTW band pipeline accumulated on this context (and
 * the worker contexts of sonar_align_pairs) since the last reset: out4[0]
 * edge-poll refresh fences (an agent-scope acquire issued after 1 ms without
 * a new value from the band above), out4[1] those after which the next poll
 * found new values, out4[2] DTWs whose pipeline timed out (the call returned
 * SONAR_ERR_DEVICE with a diagnostic text in sonar_last_error), out4[3] waves
 * that timed out.  reset != 0 zeroes them after reading -- diagnostics. */
int sonar_dtw_counters(sonar_ctx* ctx, int64_t* out4, int32_t reset);
/* Frees the device and pinned host buffers this context (and its sonar_align_pairs
 * worker contexts) cache between calls; the tables and streams stay.  The next call
 * allocates what it needs again.  sonar_align_pairs' workers keep up to ~70 % of the
 * device memory that was free when it ran: trim releases it.  No Go counterpart
 * (memory management of this library). */
int sonar_trim(sonar_ctx* ctx);

/* ---- sizes (same integer rules as the Go code) ------------------------ */
/* (n - W)/H + 1, Go truncating division; <= 0 -> SONAR_ERR_TOO_SHORT
 * (fingerprint/analyzers/spectral.go:409-412) */
int64_t sonar_stft_frames(int64_t n, int32_t window_size, int32_t hop_size);
/* Energy.ComputeShortTimeEnergy frame count, 0 when n < W or W,H <= 0 (energy.go:25-31) */
int64_t sonar_energy_frames(int64_t n, int32_t window_size, int32_t hop_size);
/* extractHarmonicFeatures frame count (1024/512), speech.go:469-471 */
int64_t sonar_pitch_frames(int64_t n);

/* ---- path A: fused STFT -> |X| -> filterbank -> ln -> DCT (+ descriptors) */
typedef struct {
  int32_t window_size;     /* STFT W (FFT size)                                     */
  int32_t hop_size;        /* STFT H                                                */
  int32_t window_type;     /* SONAR_WIN_*; always {Normalize, Symmetric} like spectral.go:415 */
  int32_t sample_rate;     /* rate the algorithms see (0 reproduces GenerateFingerprint, F1) */
  /* MFCCParams (mfcc.go:27-34); <=0 fields take the Go defaults of NewMFCCWithParams */
  int32_t n_mfcc;
  int32_t n_filters;
  int32_t filterbank;      /* SONAR_FB_MEL / SONAR_FB_BARK                          */
  int32_t use_lifter;
  double low_freq;
  double high_freq;
  double lifter;
  int32_t mfcc_input_power;/* 0: Compute() is fed |X| (speech.go:257); 1: fed |X|^2 (music.go:311, F5) */
  int32_t energy_window;   /* ShortTimeEnergy frame size (extractor FeatureConfig.WindowSize) */
  int32_t energy_hop;      /* ShortTimeEnergy hop                                   */
  double preemph_alpha;    /* pre-emphasis for ZCR/energy (0.97 speech, pre_emphasis.go:116) */
  uint32_t flags;          /* SONAR_FP_*                                            */
  int32_t precision;       /* SONAR_F32 (throughput) / SONAR_F64 (parity); calls with
                              SONAR_FP_SPECTRAL always run the f64 transform          */
  int32_t pcm_dtype;       /* SONAR_F32 / SONAR_F64                                 */
  int32_t out_dtype;       /* SONAR_F32 / SONAR_F64 element type of every output    */
  int32_t device_ptrs;     /* 0: host buffers (sync); 1: device buffers (async)     */
} sonar_fp_cfg;

typedef struct {
  void* mfcc;       /* F x n_mfcc                     */
  void* magnitude;  /* F x (W/2+1)                    */
  void* centroid;   /* F each ...                     */
  void* rolloff;
  void* bandwidth;
  void* flatness;
  void* crest;
  void* slope;
  void* flux;       /* F-1                            */
  void* low_ratio;  /* F (per STFT frame)             */
  void* high_ratio; /* F                              */
  void* zcr;        /* F                              */
  void* energy;     /* sonar_energy_frames(n, ew, eh) */
  void* complex;    /* F x (W/2+1) x 2, interleaved (re, im)   (spectral.go:491) */
  void* phase;      /* F x (W/2+1)                             (spectral.go:493) */
} sonar_fp_out;

void sonar_fp_cfg_default(sonar_fp_cfg* cfg);
/* Window sizes: 128, 256, 512, 1024 and 2048 run the fused kernels (every flag); any other W up
 * to 8192 runs the generic float64 DFT path (MFCC, magnitude, complex, phase, ZCR, energy; the
 * spectral descriptors -> SONAR_ERR_UNSUPPORTED), as go-dsp's FFTReal takes any length. */
int sonar_fingerprint(sonar_ctx* ctx, const void* pcm, int64_t n, const sonar_fp_cfg* cfg,
                      sonar_fp_out* out);
/* Which transform kernel sonar_fingerprint runs for (cfg, n): pure host logic, the decision the
 * call itself makes (no device needed).  SONAR_PLAN_PAIR: mfcc_pair_kernel (float32 MFCC only,
 * W = 1024, at most SONAR_PAIR_MAX_FRAMES frames -- its frame indices are 32-bit -- and a
 * filterbank that fits its lane chunks, else the call takes fp_wave_kernel); SONAR_PLAN_WAVE:
 * fp_wave_kernel; SONAR_PLAN_DFT: stft_dft_kernel (other W); SONAR_PLAN_NONE: no transform
 * requested (ZCR / energy only).  < 0: the error code the call would return for (cfg, n). */
enum { SONAR_PLAN_NONE = 0, SONAR_PLAN_PAIR = 1, SONAR_PLAN_WAVE = 2, SONAR_PLAN_DFT = 3 };
#define SONAR_PAIR_MAX_FRAMES 2147483646LL
int32_t sonar_fp_kernel_plan(const sonar_fp_cfg* cfg, int64_t n);
/* SpectralAnalyzer.ComputeSTFTBatch (fingerprint/analyzers/spectral.go:234-285): sonar_fingerprint
 * of `count` signals with one configuration; out[i] receives signal i's outputs (sizes as for
 * sonar_fingerprint with n[i]).  count <= 0 -> SONAR_ERR_EMPTY "no signals provided"; the first
 * failing signal by index -> its code with "error processing signal i: <message>" (:276-281), and
 * nothing is launched when a signal fails ComputeSTFTWithWindow's argument checks.  The f32 MFCC
 * configuration at W = 1024 (flags == SONAR_FP_MFCC, precision / pcm_dtype / out_dtype F32) runs
 * every signal's frames in ONE mfcc_pair_kernel launch; other configurations run sonar_fingerprint
 * per signal on the ctx stream.  cfg->device_ptrs applies to every pcm[i] and out[i] buffer. */
int sonar_fingerprint_batch(sonar_ctx* ctx, const void* const* pcm, const int64_t* n, int32_t count,
                            const sonar_fp_cfg* cfg, sonar_fp_out* out);

/* ---- STFTStreamer (fingerprint/analyzers/spectral.go:287-374) ---------------------------------
 * SpectralAnalyzer.ComputeSTFTStreaming(W, H, windowType) + STFTStreamer.ProcessChunk.  The stream
 * keeps Go's buffer (the samples not yet consumed, < W for H <= W) on the device; each push appends
 * a chunk and emits every complete frame in ONE fused STFT launch over [buffer | chunk].  Rows are
 * bit-identical to one sonar_fingerprint call over the concatenated stream with the same cfg plus
 * SONAR_FP_GENERIC (the per-frame kernel; the headline pair kernel's bits depend on a frame's
 * partner, which a push may not have yet).  Frame placement is Go's, including its quirk for
 * H > W: a frame whose hop reaches past the buffered samples clears the buffer (:355-362), so the
 * rest of that skip is not carried into the next chunk. */
typedef struct sonar_stft_stream sonar_stft_stream;
/* cfg: window_size, hop_size, window_type ({Normalize, Symmetric} and Go's zero Beta / Alpha, as
 * :290-295), flags (SONAR_FP_MAGNITUDE / _PHASE / _COMPLEX -- SpectrogramFrame -- and SONAR_FP_MFCC
 * with cfg's MFCC parameters), precision, pcm_dtype, out_dtype, device_ptrs (for every push's chunk
 * and outputs).  Errors: "failed to generate window: window size must be positive: W" / "... too
 * large: W" (windowing.go:180-187); other flags -> SONAR_ERR_UNSUPPORTED. */
int sonar_stft_stream_create(sonar_ctx* ctx, const sonar_fp_cfg* cfg, sonar_stft_stream** out);
/* Frames the next push of n samples will emit: 0 for n <= 0 or while fewer than W samples are held,
 * else (buffered + n - W) / H + 1 (host arithmetic; size the outputs of the push with it). */
int64_t sonar_stft_stream_frames(const sonar_stft_stream* st, int64_t n);
/* STFTStreamer.ProcessChunk(chunk) (:322-366): n <= 0 emits nothing (Go returns nil, nil).  out's
 * requested arrays receive *frames rows (laid out as sonar_fingerprint's for that many frames).
 * H == 0 with a frame due -> SONAR_ERR_INVALID (Go's loop never advances); H < 0 -> SONAR_ERR_PANIC
 * "runtime error: slice bounds out of range [H:]" (:359).  Host buffers: synchronous; device buffers:
 * asynchronous on the ctx stream (the chunk may be reused once the stream has passed the push). */
int sonar_stft_stream_push(sonar_stft_stream* st, const void* chunk, int64_t n, sonar_fp_out* out,
                           int64_t* frames);
int64_t sonar_stft_stream_buffered(const sonar_stft_stream* st);   /* len(s.buffer) */
void sonar_stft_stream_destroy(sonar_stft_stream* st);

/* ---- PCM ingest: the decoder's f64le byte stream -> device samples.
 * Replaces Decoder.bytesToFloat64 + processFFmpegOutput's empty check (transcode/decoder.go:850-871,
 * :782-787; ffmpeg "-f f64le" at :709): nbytes is trimmed to a multiple of 8, zero samples fail with
 * SONAR_ERR_EMPTY "no audio samples decoded".  Samples keep the stream's (interleaved) order, as
 * AudioData.PCM does.  The bytes go through a ring of pinned host slots filled by host_threads
 * threads (0 = OMP_NUM_THREADS or min(16, cores)) while earlier slots DMA on the ctx stream:
 *   SONAR_INGEST_DEVICE_CONVERT  f64 crosses PCIe, a kernel rounds to f32 (if out_dtype F32)
 *   SONAR_INGEST_HOST_CONVERT    the filling threads round to f32 (half the PCIe bytes)
 * Rounding is round-to-nearest-even in both (Go float32(x)).  d_out: device buffer of
 * n_samples * (out_dtype F64 ? 8 : 4) bytes, 16-B aligned; NULL only reports *n_samples.
 * Returns once the host bytes are consumed; the device writes complete in ctx-stream order. */
#define SONAR_INGEST_DEVICE_CONVERT 0
#define SONAR_INGEST_HOST_CONVERT 1
int sonar_ingest_f64le(sonar_ctx* ctx, const void* bytes, int64_t nbytes, int32_t out_dtype, int32_t mode,
                       int32_t host_threads, void* d_out, int64_t* n_samples);
/* Decoder output straight into path A: sonar_ingest_f64le (in cfg->pcm_dtype, `mode`) into a
 * ctx-owned device buffer, then sonar_fingerprint on it; pcm_dtype F64 (the default) keeps Go's
 * []float64 samples end to end, F32 rounds them to nearest even; outputs are host buffers
 * (cfg->device_ptrs must be 0).  Replaces bytesToFloat64 + ComputeSTFTWithWindow's upload of
 * AudioData.PCM (decoder.go:850-871 -> analyzers/spectral.go:385) with one call. */
int sonar_fingerprint_f64le(sonar_ctx* ctx, const void* bytes, int64_t nbytes, int32_t mode,
                            const sonar_fp_cfg* cfg, sonar_fp_out* out);

/* ---- YIN per-frame core (frames of 1024 at hop 512, PitchDetector defaults).
 * Writes the raw YIN result per frame (pitch Hz or 0, confidence 1-cmndf or 0)
 * before the sequential octave-correction / median tracking, which the host
 * layer (sonar_generate_fingerprint) applies.  pcm is float64. ----------- */
int sonar_pitch_yin(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                    double* pitch_raw, double* conf_raw, int32_t* tau, int32_t device_ptrs);

/* ---- chroma (music extractor): DC removal + pre-emphasis 0.95, frames of
 * frame_size = n / n_frames at hop, normalised symmetric Hann, |DFT|^2 folded
 * to 12 pitch classes over [80, 8000] Hz, unit-sum normalised. ----------- */
int sonar_chroma_stft(sonar_ctx* ctx, const double* pcm, int64_t n, int64_t n_frames, int32_t hop,
                      int32_t sample_rate, int32_t preprocess, double* chroma /* n_frames x 12 */,
                      int32_t device_ptrs);

/* ---- path B: normalized cross-correlation (float64) --------------------
 * corr has 2L+1 entries, L = max(0, min(max_lag, na-1, nb-1)); metrics[10] =
 * {peak_corr, peak_lag, peak_index, p_value, snr, sharpness, second_peak,
 *  peak_to_sidelobe, overlap_length, num_lags} (correlation.go:131-200). */
int sonar_ncc(sonar_ctx* ctx, const double* a, int64_t na, const double* b, int64_t nb,
              int32_t max_lag, double* corr, double* metrics, int32_t device_ptrs);

/* ---- path B: DTW (float64, Euclidean, symmetric2, optional Sakoe-Chiba band)
 * q: nq x dim, r: nr x dim row-major.  path_* capacity >= nq + nr.  cost
 * (nullable) receives costMatrix[1:] = nq x (nr+1) (dtw.go:96).  Path points
 * are in forward order with cost = C[i][j] - C[i-1][j-1] (dtw.go:165-188). */
int sonar_dtw(sonar_ctx* ctx, const double* q, int64_t nq, const double* r, int64_t nr, int32_t dim,
              int32_t band, double* distance, int32_t* path_q, int32_t* path_r, double* path_cost,
              int64_t* path_len, double* cost, int32_t device_ptrs);

/* ---- LPC formants: FormantAnalyzer.AnalyzeMultipleFrames (algorithms/speech/format.go:427-449)
 * over FormantAnalyzer.AnalyzeFormants (:85-124) + LPCAnalyzer.Analyze (lpc.go:44-82).
 * Analysis window W = 2048 if sample_rate >= 16000 else 1024, LPC order 12 + sr/1000,
 * pre-emphasis 0.97, symmetric Hamming (format.go:48-69).  Frames start at 0, hop, ...
 * while start < n - frame_size (frame_size <= 0 -> W, hop <= 0 -> frame_size/2).  Every
 * attempted frame gets a record; status != 0 marks the frames Go skips. ------------ */
typedef struct {
  int32_t status;          /* 0 ok; 1 frame shorter than W; 3 "zero energy signal";
                              4 "prediction error energy became zero" (lpc.go:93-113)   */
  int32_t n_formants;      /* validated formants, <= 4 (ascending frequency)            */
  double frequency[4];
  double bandwidth[4];
  double amplitude[4];
  double confidence[4];
  double vocal_tract_length;   /* cm, 17.5 when no formant qualifies                    */
  double quality;              /* calculateAnalysisQuality                               */
  double gain;                 /* sqrt(residual energy)                                  */
  double residual_energy;
  int32_t stable;              /* checkStability: every |a_i| < 1                        */
  int32_t lpc_order;
} sonar_formant_frame;

int64_t sonar_formant_frame_count(int64_t n, int32_t sample_rate, int32_t frame_size, int32_t hop_size);
/* lpc_coeffs (nullable): frames x (order+1) a[0..p], a[0] = 1; reflection (nullable): frames x order */
int sonar_formants(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate, int32_t frame_size,
                   int32_t hop_size, sonar_formant_frame* out, double* lpc_coeffs, double* reflection,
                   int32_t device_ptrs);

/* ---- VoiceQualityAnalyzer.AnalyzeVoiceQuality (algorithms/speech/voice_quality.go:56-111),
 * the analysis AnalyzeSpeech runs on the speech extractor's pre-emphasised PCM
 * (speech_analysis.go:77-80) and whose Jitter / Shimmer land in SpeechFeatures
 * (extractors/speech.go:306-309).  Pitch periods come from a YIN scan of 1024-sample frames at
 * hop 256 with a fresh PitchDetector (:114-157); voicing_strength is DetectPitch on the whole
 * signal, which Go only accepts for exactly 1024 samples (else 0).  Errors, as Go:
 * SONAR_ERR_TOO_SHORT "signal too short for voice quality analysis (need at least 1 second)"
 * and "insufficient pitch periods for analysis (found k, need at least 3)". ------------------ */
typedef struct {                     /* speech.VoiceQualityResult (voice_quality.go:21-43) */
  double jitter, shimmer, hnr, noise_measure, f0_stability, amplitude_stability;
  double voicing_strength, overall_quality;
  int64_t num_periods;
  double mean_f0, f0_range, analysis_quality;
} sonar_voice_quality_result;

int sonar_voice_quality(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                        sonar_voice_quality_result* out);

/* ---- host mirror of the Go API (C++ above the kernels) ------------------ */
typedef struct sonar_result sonar_result;   /* named float64 arrays + scalars */

typedef struct {              /* fingerprint.FingerprintConfig (fingerprint.go:29-35) */
  int32_t window_size;        /* FingerprintConfig.WindowSize (STFT)                 */
  int32_t hop_size;           /* FingerprintConfig.HopSize                            */
  int32_t feature_window_size;/* FingerprintConfig.FeatureConfig.WindowSize (energy)  */
  int32_t feature_hop_size;   /* FingerprintConfig.FeatureConfig.HopSize              */
  int32_t enable_content_detect;
  int32_t window_type;        /* content settings WindowType (all Hann in the tables) */
  int32_t precision;          /* SONAR_F32 / SONAR_F64                                */
  /* ContentConfig (config.ContentAwareConfig, config/config.go:5-10) and the rest of
   * AudioData.Metadata, used by ContentDetector.DetectContentType when the content type
   * is unknown and enable_content_detect is set (fingerprint.go:155-158) */
  int32_t acoustic_detection;     /* ContentConfig.EnableContentDetection               */
  int32_t default_content_type;   /* ContentConfig.DefaultContentType (SONAR_CT_*)      */
  double auto_detect_threshold;   /* ContentConfig.AutoDetectThreshold                  */
  const char* genre;              /* Metadata.Genre   (NULL = "")                       */
  const char* station;            /* Metadata.Station (NULL = "")                       */
  const char* url;                /* Metadata.URL     (NULL = "")                       */
} sonar_fingerprint_config;

void sonar_fingerprint_config_default(sonar_fingerprint_config* cfg);  /* fingerprint.go:70-98 */

typedef struct {              /* config.FeatureConfig fields the speech extractor reads (config/config.go:13-38) */
  int32_t sample_rate;        /* FeatureConfig.SampleRate (0 under GenerateFingerprint, F1)           */
  int32_t window_size;        /* FeatureConfig.WindowSize: ShortTimeEnergy frames                     */
  int32_t hop_size;           /* FeatureConfig.HopSize                                                */
  int32_t stft_window_size;   /* spectrogram handed to ExtractFeatures (ComputeSTFTWithWindow W)     */
  int32_t stft_hop_size;      /* ... and H                                                            */
  int32_t window_type;
  int32_t enable_mfcc;
  int32_t enable_speech_features;
  int32_t enable_temporal_features;
  int32_t mfcc_coefficients;
  int32_t is_news;
  int32_t precision;          /* SONAR_F64 (parity, default) / SONAR_F32                              */
} sonar_feature_config;

void sonar_feature_config_default(sonar_feature_config* cfg);

/* NewSpeechFeatureExtractor(cfg, is_news) + ExtractFeatures(STFT(pcm, W, H), pcm, sample_rate).
 * Result arrays: "mfcc", "spectral_centroid" ... "spectral_flux", "zero_crossing_rate",
 * "short_time_energy", "energy_variance", "loudness_range", "energy_entropy",
 * "low_energy_ratio", "high_energy_ratio", "pitch_estimate", "pitch_confidence",
 * "voicing_strength", "harmonic_ratio", "inharmonicity_ratio", "tonal_centroid",
 * temporal ("rms_energy", "dynamic_range", "silence_ratio", "peak_amplitude",
 * "average_amplitude", "onset_density", "attack_time", "envelope_shape") and speech
 * ("is_speech", "voicing_probability", "spectral_tilt", "pause_duration") groups when enabled. */
int sonar_extract_speech_features(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                                  const sonar_feature_config* cfg, sonar_result** out);

/* NewMusicFeatureExtractor(cfg) + ExtractFeatures(STFT(pcm, W, H), pcm, sample_rate)
 * (fingerprint/extractors/music.go:70-583).  cfg: sample_rate = FeatureConfig.SampleRate (the
 * analyzers' and MFCC's rate), window_size / hop_size = FeatureConfig (ShortTimeEnergy frames,
 * chroma hop), stft_window_size / stft_hop_size / window_type = the spectrogram; sample_rate
 * (the argument) = SpectrogramResult.SampleRate.  Result arrays: "spectral_centroid" ..
 * "spectral_slope", "spectral_flux" (F, [0] = 0), "zero_crossing_rate" (F zeros, never filled in
 * Go), "spectral_contrast" (F x 6), "mfcc" (F x 13 of |X|^4 over 26 mels, F5), "chroma" (F x 12),
 * "rms_energy", "envelope_shape", "peak_amplitude", "average_amplitude", then "dynamic_range",
 * "onset_density", "attack_time", "crest_factor", "silence_ratio", "activity_level",
 * "short_time_energy", "energy_variance", "energy_entropy", "loudness_range",
 * "low_energy_ratio", "high_energy_ratio" and the harmonic block "pitch_estimate",
 * "pitch_confidence", "voicing_strength", "harmonic_ratio", "inharmonicity_ratio",
 * "tonal_centroid" (zero by F7 unless the chroma frame is exactly 1024 samples).
 * The reference panics in extractTemporalFeatures for every signal of >= 1536 samples
 * (music.go:403 passes percentiles 10 and 90 where fractions are expected:
 * "index out of range [10 (L-1)] with length L") and for a signal with no energy frame
 * (music.go:383: "integer divide by zero").  Then the call returns SONAR_ERR_PANIC with that
 * text and *out holds the arrays computed before the panic (the spectral group, "mfcc",
 * "chroma", "rms_energy", and after the division also "envelope_shape" and the amplitudes);
 * the caller frees it.  float64. */
int sonar_extract_music_features(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                                 const sonar_feature_config* cfg, sonar_result** out);

/* AudioData{PCM, SampleRate, Metadata.ContentType}.  content_type is the raw
 * metadata string ("music", "news", "talk", ... ; unknown strings -> content
 * detection, F12).  Returns arrays named like ExtractedFeatures fields:
 * "mfcc", "spectral_centroid", ..., "short_time_energy", "pitch_estimate", ... */
int sonar_generate_fingerprint(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                               const char* content_type, const sonar_fingerprint_config* cfg,
                               sonar_result** out);

/* AlignmentExtractor.ExtractAlignmentFeatures on the energy (+ optional chroma)
 * features of two fingerprints.  feature_sample_rate / hop / window are the
 * extractor's FeatureConfig; max_lag_seconds as NewAlignmentExtractorWithMaxLag. */
int sonar_align_features(sonar_ctx* ctx,
                         const double* q_energy, int64_t nq_energy, const double* r_energy, int64_t nr_energy,
                         const double* q_chroma, int64_t nq_chroma, const double* r_chroma, int64_t nr_chroma,
                         int64_t q_pcm_len, int64_t r_pcm_len, int32_t sample_rate,
                         int32_t feature_sample_rate, int32_t hop_size, int32_t window_size,
                         double max_lag_seconds, sonar_result** out);

/* One stream pair end to end (the C5 unit): sonar_music_alignment_features of both device-resident
 * float64 PCM streams into ctx buffers (stft_window / hop; energy frames feature_window / hop), then
 * sonar_align_features on those device arrays with feature_sample_rate = sample_rate.  Same result
 * arrays as sonar_align_features; only the feature round trip through the host is gone. */
int sonar_align_pair_device(sonar_ctx* ctx, const double* q_pcm, int64_t nq, const double* r_pcm, int64_t nr,
                            int32_t sample_rate, int32_t stft_window, int32_t hop, int32_t feature_window,
                            double max_lag_seconds, sonar_result** out);

/* ---- many stream pairs (the C5 workload) -----------------------------------------
 * The fixed-size record a caller of ExtractAlignmentFeatures keeps per pair
 * (extractors/alignment.go:139-219: TemporalOffset, OffsetConfidence, AlignmentSimilarity,
 * AlignmentQuality, Method; the NCC candidate's offset and peak lag; the chroma DTW distance). */
typedef struct {
  double temporal_offset;        /* seconds                                       */
  double offset_confidence;
  double alignment_similarity;
  double alignment_quality;
  double method;                 /* SONAR_ALIGN_* of the chosen candidate          */
  double corr_offset_seconds;    /* the energy-NCC candidate (NaN if none)         */
  double dtw_distance;           /* the chroma-DTW candidate (NaN if none)         */
  double peak_lag;               /* NCC peak lag in feature frames (NaN if none)   */
  int32_t status;                /* SONAR_OK or this pair's error code             */
  int32_t flags;                 /* SONAR_PAIR_REDONE_* bits (0: the batched path) */
} sonar_pair_record;

/* sonar_pair_record.flags: the pair's record came from the single-pair path instead of its batch */
#define SONAR_PAIR_REDONE_TIMEOUT 1    /* its batched band pipeline timed out (retry on)  */
#define SONAR_PAIR_REDONE_NONFINITE 2  /* its chroma is not finite (exact math.Min path)  */

/* sonar_align_pair_device over npairs pairs: q_pcm[k] / r_pcm[k] float64 streams of nq[k] / nr[k]
 * samples (device pointers on ctx's device if device_ptrs, else host arrays).  `workers` is the
 * number of pairs in flight (<= 0: 128).  They are split over SONAR_PAIR_STREAMS worker contexts
 * (environment, default 16; each one HIP stream and one host thread) in batches of
 * ceil(workers / streams) pairs, each batch's chroma DTWs in ONE band-kernel launch, so the pairs'
 * latency-bound kernels (the DC-removal scan, the Go-order NCC sums, the DTW band pipeline and
 * walk) overlap on the GPU.  HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues
 * (4 by default, at most 32): set GPU_MAX_HW_QUEUES >= SONAR_PAIR_STREAMS in the environment
 * before the first HIP call of the process, or the streams share queues and serialise.  out[k] is
 * filled for every pair; the return is SONAR_OK or the first error.  A pair whose batched band
 * pipeline timed out is redone once on the single-pair path (exact; counted in
 * sonar_dtw_counters and flagged SONAR_PAIR_REDONE_TIMEOUT in its record); with
 * SONAR_PAIR_RETRY=0 it is an error instead, naming the pair and carrying its diagnostic record in
 * sonar_last_error. */
int sonar_align_pairs(sonar_ctx* ctx, int64_t npairs, const double* const* q_pcm, const int64_t* nq,
                      const double* const* r_pcm, const int64_t* nr, int32_t sample_rate, int32_t stft_window,
                      int32_t hop, int32_t feature_window, double max_lag_seconds, int32_t workers,
                      int32_t device_ptrs, sonar_pair_record* out);

/* ---- one process, several GPUs: a context per device plus an RCCL communicator
 * over them (ncclCommInitAll; collectives run over xGMI). ------------------------------------- */
typedef struct sonar_multi sonar_multi;
int sonar_multi_create(const int32_t* devices, int32_t n_devices, sonar_multi** out);
void sonar_multi_destroy(sonar_multi* m);
const char* sonar_multi_last_error(const sonar_multi* m);
int32_t sonar_multi_size(const sonar_multi* m);
sonar_ctx* sonar_multi_ctx(sonar_multi* m, int32_t rank);   /* the rank's context (do not destroy) */

/* Frame shard g of G over n samples at W/H: frames [f0, f1) = [e(g), e(g+1)) with
 * e(k) = floor(k F / G) rounded down to even (e(G) = F), F = sonar_stft_frames(n, W, H), and the
 * samples they read [s0, s1) = [f0 H, (f1-1) H + W) (empty shard: f0 == f1, s0 == s1).  Even
 * boundaries keep the headline kernel's frame pairs, so the shards reassemble bit-identically to
 * the unsharded call.  Pure arithmetic, the same on every host. */
int sonar_multi_shard(int64_t n, int32_t window_size, int32_t hop_size, int32_t n_shards, int32_t shard,
                      int64_t* f0, int64_t* f1, int64_t* s0, int64_t* s1);

/* sonar_fingerprint with the STFT frames sharded over the devices: device g runs frames [f0, f1)
 * of sonar_multi_shard on its sample slice (host pcm, cfg->device_ptrs must be 0) and writes its
 * rows of every requested output straight into the host arrays.  Frames are independent, so the
 * result equals the single-device call.  Supported flags: SONAR_FP_MFCC, SONAR_FP_MAGNITUDE,
 * SONAR_FP_COMPLEX, SONAR_FP_PHASE and SONAR_FP_SPECTRAL without flux (out->flux must be NULL: frame f0's flux needs frame f0-1); the
 * pre-emphasised outputs (ZCR, energy) read the sample before the slice -> SONAR_ERR_UNSUPPORTED. */
int sonar_fingerprint_multi(sonar_multi* m, const void* pcm, int64_t n, const sonar_fp_cfg* cfg,
                            sonar_fp_out* out);

/* The MFCC timeline assembled on EVERY device over RCCL: device g holds its shard's sample slice
 * pcm_dev[g] (samples [s0, s1) of sonar_multi_shard, cfg->pcm_dtype), computes its frames, and one
 * ncclAllGather (shards padded to the largest) fills mfcc_dev[g] (F x n_mfcc, cfg->out_dtype) on
 * every device -- the device-resident timeline a comparator on any GPU can read.  Synchronous. */
int sonar_fingerprint_multi_gather(sonar_multi* m, const void* const* pcm_dev, int64_t n, const sonar_fp_cfg* cfg,
                                   void* const* mfcc_dev);

/* sonar_align_pairs with the pairs split into contiguous ranges over the devices (host PCM; each
 * device aligns its range as sonar_align_pairs, `workers` pairs in flight); the per-device records are then
 * all-gathered over RCCL and device 0's gathered copy is returned in out[npairs]. */
int sonar_align_pairs_multi(sonar_multi* m, int64_t npairs, const double* const* q_pcm, const int64_t* nq,
                            const double* const* r_pcm, const int64_t* nr, int32_t sample_rate,
                            int32_t stft_window, int32_t hop, int32_t feature_window, double max_lag_seconds,
                            int32_t workers, sonar_pair_record* out);

/* ---- AlignmentAnalyzer.AnalyzeAlignmentConsistency (algorithms/stats/alignment.go:709-800) -----
 * num_trials (< 2 -> 5) alignments of addNoise(query, 0.01) (:737-749: q[i][j] += sin(i*j+i+j)
 * * 0.01 * q[i][j]) against reference with AlignFeatures (:84-106) for `method`, then the offset
 * statistics (:751-800).  The perturbation is deterministic, so every trial aligns the same
 * perturbed query: the alignment runs once and its offset is counted num_trials times (the
 * statistics are those of num_trials equal offsets, as in Go).  query / reference: host
 * row-major nq x dim / nr x dim float64.  method: SONAR_ALIGN_*; max_lag and hop as
 * NewAlignmentAnalyzer (:60-81).  Errors: "no successful alignments" (empty input or an
 * unsupported method, where every Go trial fails). */
enum { SONAR_ALIGN_DTW = 0, SONAR_ALIGN_XCORR = 1, SONAR_ALIGN_PHASE = 2, SONAR_ALIGN_HYBRID = 3 };
typedef struct {                     /* stats.AlignmentStats (alignment.go:700-707) */
  double mean_offset, stddev_offset, median_offset, offset_range, consistency;
  int64_t offset;                    /* the (single) AlignFeatures offset, samples or frames per method */
  int32_t trials;
} sonar_alignment_stats;

int sonar_alignment_consistency(sonar_ctx* ctx, const double* query, int64_t nq, const double* reference, int64_t nr,
                                int32_t dim, int32_t method, int32_t max_lag, int32_t hop, int32_t sample_rate,
                                int32_t num_trials, sonar_alignment_stats* out);

/* ---- AlignmentAnalyzer.AlignFeatures / AlignAudio and AlignmentExtractor.AlignAudioFiles --------
 * The analyzer's own entry (algorithms/stats/alignment.go:84-106) for method SONAR_ALIGN_DTW,
 * SONAR_ALIGN_XCORR or SONAR_ALIGN_HYBRID (alignWithHybrid :308-337: the cross-correlation of the
 * features' first component; when its confidence is <= 0.7 the DTW of the full rows, with Go's
 * result aliasing F8: Confidence = 0.6 c + 0.4 c and Similarity = 0.7 s + 0.3 s of the DTW values,
 * Offset / AlignmentQuality / Stability the DTW's, NoiseLevel the correlation's).  query /
 * reference: row-major nq x dim / nr x dim float64 (device pointers if device_ptrs).  max_lag and
 * hop as NewAlignmentAnalyzer (:60-81).  *out: scalars "method", "offset" (samples for the
 * correlation, frames for the DTW, F9), "offset_seconds", "confidence", "similarity",
 * "alignment_quality", "noise_level", "stability", "query_length", "reference_length",
 * "sample_rate", "dtw_ran"; with the correlation "correlations" (2L+1) and its metrics
 * ("peak_correlation", "peak_lag", ... as sonar_ncc); with the DTW "dtw_distance",
 * "dtw_path_query", "dtw_path_reference", "dtw_path_cost".  Errors as Go: "empty feature sequences
 * provided", "unsupported alignment method: N". */
int sonar_analyzer_align_features(sonar_ctx* ctx, const double* query, int64_t nq, const double* reference,
                                  int64_t nr, int32_t dim, int32_t method, int32_t max_lag, int32_t hop,
                                  int32_t sample_rate, int32_t device_ptrs, sonar_result** out);

/* AlignmentAnalyzer.AlignAudio (:108-126): extractEnergyFeatures (:341-361) of both float64 PCM
 * streams -- numFrames = (len - window) / hop + 1 (truncating), RMS over [i hop, min(i hop + window,
 * len)) -- then sonar_analyzer_align_features with dim 1.  Go panics are SONAR_ERR_PANIC with
 * Go's text (hop 0: "integer divide by zero"; a negative frame count: "makeslice: len out of
 * range"); window <= 0, hop < 0 or an empty stream: SONAR_ERR_UNSUPPORTED (Go divides 0 by 0). */
int sonar_align_audio(sonar_ctx* ctx, const double* q_pcm, int64_t nq, const double* r_pcm, int64_t nr,
                      int32_t method, int32_t max_lag, int32_t hop, int32_t window, int32_t sample_rate,
                      int32_t device_ptrs, sonar_result** out);

/* AlignmentExtractor.AlignAudioFiles (extractors/alignment.go:489-553) of an extractor built by
 * NewAlignmentExtractorWithMaxLag (:99-136) from FeatureConfig{feature_sample_rate, hop, window}:
 * ShortTimeEnergy (algorithms/temporal/energy.go:25-50) of both streams, then the Hybrid
 * AlignFeatures at maxLagFrames = int(max_lag_seconds * feature_sample_rate) / hop.  *out: the
 * sonar_analyzer_align_features keys (BestAlignment) plus the AlignmentFeatures fields
 * "temporal_offset", "offset_confidence", "alignment_similarity", "alignment_quality",
 * "feature_similarity_energy", "query_length_seconds", "reference_length_seconds", "time_stretch"
 * (never set by Go: 0) and "max_lag_frames"; Method is always "energy_correlation".  Errors as Go:
 * "alignment failed: empty feature sequences provided"; hop 0 panics ("integer divide by zero"). */
int sonar_align_audio_files(sonar_ctx* ctx, const double* q_pcm, int64_t nq, const double* r_pcm, int64_t nr,
                            int32_t sample_rate, int32_t feature_sample_rate, int32_t hop, int32_t window,
                            double max_lag_seconds, int32_t device_ptrs, sonar_result** out);

/* AlignmentExtractor.TruncateToAlignmentPCM (extractors/alignment.go:223-297) as sample indices:
 * the aligned segments are pcm1[start1 : start1+length] and pcm2[start2 : start2+length] (the
 * PCM stays where it is, e.g. in HBM).  Errors as Go: "offset too large ...", "no overlapping
 * audio after alignment". */
int sonar_truncate_to_alignment(sonar_ctx* ctx, int64_t n1, int64_t n2, int32_t sample_rate, double temporal_offset,
                                int64_t* start1, int64_t* start2, int64_t* length);

/* The two MusicFeatureExtractor.ExtractFeatures outputs that the alignment extractor consumes
 * (fingerprint/extractors/music.go:178-245): preprocessAudio (DC removal R = 0.995, then
 * pre-emphasis 0.95, :245-259) -> extractEnergyFeatures' ShortTimeEnergy with the extractor's
 * FeatureConfig WindowSize/HopSize (:460-466, temporal/energy.go:25-50) and
 * extractChromaFeatures (:327-376): spectrogram frames F = sonar_stft_frames(n, stft_window,
 * stft_hop), frame length n / F, hop = FeatureConfig.HopSize.  energy has
 * sonar_energy_frames(n, feature_window, feature_hop) entries, chroma F x 12.  float64. */
int sonar_music_alignment_features(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                                   int32_t stft_window, int32_t stft_hop, int32_t feature_window,
                                   int32_t feature_hop, double* energy, double* chroma, int32_t device_ptrs);

/* ---- ContentDetector (fingerprint/content_detector.go) -----------------------------
 * DetectFromAudio (:72-101): zero-crossing rate, energy variance, silence ratio, dynamic range
 * and temporal stability over the whole PCM, the spectral centroid / frequency split /
 * harmonic ratio of a direct DFT of the first min(2048, n) samples, then classifyFromFeatures
 * (:153-217).  Go picks among equal best scores in map order (random); here the order is
 * music, news, talk, sports. */
typedef struct {                     /* AcousticFeatures (:104-115) */
  double zero_crossing_rate, spectral_centroid, energy_variance, silence_ratio, harmonic_ratio;
  double low_freq_energy, high_freq_energy, dynamic_range, temporal_stability;
  double classification_confidence;
} sonar_acoustic_features;

/* content_type <- SONAR_CT_* (SONAR_CT_UNKNOWN when no score beats the threshold).
 * sample_rate < 10 -> SONAR_ERR_INVALID (the 100 ms frame loop never ends in Go). */
int sonar_detect_from_audio(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                            double auto_detect_threshold, int32_t* content_type,
                            sonar_acoustic_features* features);

/* DetectContentType (:31-69): metadata first (parseContentType of Metadata.ContentType, else
 * inferFromGenre, else inferFromStation on station + URL), then DetectFromAudio when
 * acoustic_detection is set and n > 0, else default_content_type.  has_metadata = 0 is a nil
 * Metadata; NULL strings are "". */
int sonar_detect_content_type(sonar_ctx* ctx, const double* pcm, int64_t n, int32_t sample_rate,
                              int32_t has_metadata, const char* content_type, const char* genre,
                              const char* station, const char* url, int32_t acoustic_detection,
                              int32_t default_content_type, double auto_detect_threshold,
                              int32_t* out_content_type);

/* ---- FingerprintComparator (fingerprint/comparison.go) ------------------------------
 * The comparator's candidate set lives on the device as a gallery of per-fingerprint
 * summary records (MFCC column mean/std, chroma column means, mean/std of the compared
 * sequences, the scalars and weights).  Compare() in the reference rebuilds those
 * statistics from the full feature arrays on every call (comparison.go:344-402,
 * 646-770, 774-842); they depend on one fingerprint only, so they are reduced once per
 * fingerprint when it is added, and every comparison reads two records.  Results are the
 * reference's formulas on the same statistics. */

/* config.ContentType (fingerprint/config/config.go:39-48).  Any other content-type string
 * is given its own code >= SONAR_CT_UNKNOWN by the caller, so ContentTypeMatch (string
 * equality, comparison.go:157) keeps distinct unknown strings apart. */
enum { SONAR_CT_MUSIC = 0, SONAR_CT_NEWS, SONAR_CT_SPORTS, SONAR_CT_TALK, SONAR_CT_MIXED,
       SONAR_CT_UNKNOWN };

/* sonar_fp_features.present: which members of AudioFingerprint.Features are non-nil */
enum {
  SONAR_FEAT_FEATURES = 1u << 0,   /* Features != nil                                    */
  SONAR_FEAT_MFCC = 1u << 1,       /* Features.MFCC != nil                               */
  SONAR_FEAT_SPECTRAL = 1u << 2,   /* Features.SpectralFeatures != nil                   */
  SONAR_FEAT_CHROMA = 1u << 3,     /* Features.ChromaFeatures != nil                     */
  SONAR_FEAT_TEMPORAL = 1u << 4,   /* Features.TemporalFeatures != nil                   */
  SONAR_FEAT_SPEECH = 1u << 5,     /* Features.SpeechFeatures != nil                     */
  SONAR_FEAT_HARMONIC = 1u << 6,   /* Features.HarmonicFeatures != nil                   */
  SONAR_FEAT_WEIGHTS = 1u << 7     /* Metadata["feature_weights"] is a map[string]float64 */
};

/* FeatureDistances keys (comparison.go:284-330), bit i of sonar_similarity.distance_mask */
enum { SONAR_FD_MFCC = 0, SONAR_FD_SPECTRAL, SONAR_FD_CHROMA, SONAR_FD_TEMPORAL, SONAR_FD_SPEECH,
       SONAR_FD_HARMONIC };

/* One AudioFingerprint as the comparator reads it (fingerprint.go:15-26,
 * extractors/features.go).  Matrices are row-major float64; MFCC rows are len(mfcc[0])
 * wide -- a shorter Go row is padded with 0 (the value extractMFCCStatistics uses for a
 * missing coefficient, comparison.go:784-789).  A sequence with n_* = 0 is empty. */
typedef struct {
  int64_t id;                      /* AudioFingerprint.ID, interned (self-skip, comparison.go:218) */
  uint32_t present;                /* SONAR_FEAT_*                                        */
  int32_t content_type;            /* SONAR_CT_* (or a distinct code >= SONAR_CT_UNKNOWN)  */
  double duration_seconds;         /* Duration.Seconds()                                  */
  const double* mfcc; int64_t mfcc_frames; int32_t mfcc_coeffs;
  const double* chroma; int64_t chroma_frames; int32_t chroma_bins;
  const double* spectral_centroid; int64_t n_spectral_centroid;
  const double* spectral_rolloff; int64_t n_spectral_rolloff;
  const double* spectral_flux; int64_t n_spectral_flux;
  double dynamic_range, silence_ratio, onset_density;          /* TemporalFeatures     */
  const double* rms_energy; int64_t n_rms_energy;
  double speech_rate, vocal_tract_length;                      /* SpeechFeatures       */
  const double* voicing_probability; int64_t n_voicing_probability;
  const double* harmonic_ratio; int64_t n_harmonic_ratio;      /* HarmonicFeatures     */
  const double* pitch_estimate; int64_t n_pitch_estimate;
  double feature_weights[6];       /* Metadata weights by SONAR_FD_* (absent key = 0)     */
} sonar_fp_features;

/* config.ComparisonConfig (fingerprint/config/config.go:68-80) */
typedef struct {
  double similarity_threshold;
  int32_t max_candidates;
  int32_t enable_detailed_metrics;
  int32_t enable_content_filter;
  int32_t method;                  /* 0 auto, 1 fast, 2 precise (Compare ignores it, :133-194) */
} sonar_compare_cfg;

/* SimilarityResult (comparison.go:28-39) */
typedef struct {
  double overall_similarity;
  double feature_similarity;
  double confidence;
  double feature_distances[6];     /* by SONAR_FD_*, where distance_mask has the bit      */
  double data_availability, feature_coverage, temporal_alignment;   /* QualityMetrics,   */
  double noise_level, dynamic_range_match, spectral_coherence;      /* when has_quality  */
  uint32_t distance_mask;
  int32_t content_type_match;
  int32_t has_quality;
  int32_t status;                  /* 0 compared, 1 skipped (same ID), 2 calculateFeatureSimilarity
                                      returned an error (nil features / nothing comparable) */
} sonar_similarity;

enum { SONAR_MATCH_EXACT = 0, SONAR_MATCH_VERY_SIMILAR, SONAR_MATCH_SIMILAR,
       SONAR_MATCH_SOMEWHAT_SIMILAR, SONAR_MATCH_WEAK };   /* classifyMatch, comparison.go:1040-1052 */

typedef struct {                   /* Match (comparison.go:52-58) */
  int64_t candidate;               /* position in the candidates list of the call          */
  int32_t rank;                    /* 1-based                                              */
  int32_t match_type;              /* SONAR_MATCH_*                                        */
  sonar_similarity similarity;
} sonar_match;

typedef struct sonar_gallery sonar_gallery;
int sonar_gallery_create(sonar_ctx* ctx, sonar_gallery** out);
void sonar_gallery_destroy(sonar_gallery* g);
int64_t sonar_gallery_size(const sonar_gallery* g);
/* Append `count` fingerprints: their statistics are reduced on the device and only the
 * records stay resident.  keep_sequences keeps SpectralCentroid / SpectralRolloff on the
 * device for EnableDetailedMetrics' spectral coherence (comparison.go:977-1008).
 * device_ptrs: the feature arrays are device pointers.  Index of the first -> *first. */
int sonar_gallery_add(sonar_gallery* g, const sonar_fp_features* fps, int32_t count,
                      int32_t keep_sequences, int32_t device_ptrs, int64_t* first);
/* FingerprintComparator.Compare / BatchCompare (comparison.go:133-194, 1107-1151) for every
 * (query, candidate) pair: out[q * nc + c].  candidates NULL -> the whole gallery
 * (nc = sonar_gallery_size).  A pair with equal IDs gets status 1 (BatchCompare drops it).
 * Detailed metrics need SpectralCentroid / SpectralRolloff of equal length on both sides
 * when both are non-empty (gonum stat.Correlation panics otherwise) -> SONAR_ERR_INVALID.
 * device_ptrs: out is a device pointer. */
int sonar_compare(sonar_gallery* g, const int64_t* queries, int64_t nq, const int64_t* candidates,
                  int64_t nc, const sonar_compare_cfg* cfg, sonar_similarity* out, int32_t device_ptrs);
/* FingerprintComparator.FindBestMatches (comparison.go:197-263) per query: matches with
 * OverallSimilarity >= threshold, descending, at most max_candidates, ranked from 1.
 * out[q * max_candidates + k], n_matches[q].  Equal similarities keep candidate order. */
int sonar_find_best_matches(sonar_gallery* g, const int64_t* queries, int64_t nq,
                            const int64_t* candidates, int64_t nc, const sonar_compare_cfg* cfg,
                            sonar_match* out, int64_t* n_matches);

/* FindBestMatches over candidates split across ranks: lists[r] holds rank r's
 * sonar_find_best_matches output (nq x max_candidates, row q at q * max_candidates) with
 * counts[r * nq + q] valid entries and its candidates numbered from cand_base[r].  out / n_out:
 * the result of ONE call over all ranks' candidates -- similarity descending (the single call's
 * radix order), equal similarities in global candidate order, at most max_candidates, ranked
 * from 1, candidate = cand_base[r] + local position.  Host-only (no device); the rank-local lists
 * can come from other processes (torch.distributed all-gather) or sonar_find_best_matches_multi. */
int sonar_merge_matches(const sonar_match* const* lists, const int64_t* counts, const int64_t* cand_base,
                        int32_t nlists, int64_t nq, int32_t max_candidates, sonar_match* out, int64_t* n_out);

/* FingerprintComparator.FindBestMatches (fingerprint/comparison.go:197-263) over rank-local
 * galleries: galleries[g] lives on rank g's context (sonar_multi_ctx); queries[g] are the query
 * fingerprints' indices in galleries[g] (every rank holds the queries); candidates[g] / nc[g] rank
 * g's candidates (candidates NULL: every gallery whole, nc ignored).  Each rank ranks its own
 * candidates, the per-rank top max_candidates travel through one RCCL all-gather, and
 * sonar_merge_matches gives out[q * max_candidates + k] / n_matches[q] equal to one call over the
 * concatenated candidates (rank g's numbered after those of ranks 0..g-1).  Synchronous. */
int sonar_find_best_matches_multi(sonar_multi* m, sonar_gallery* const* galleries, const int64_t* const* queries,
                                  int64_t nq, const int64_t* const* candidates, const int64_t* nc,
                                  const sonar_compare_cfg* cfg, sonar_match* out, int64_t* n_matches);

/* result accessors: rows*cols float64 values, row-major; scalars are 1x1 */
int sonar_result_get(const sonar_result* res, const char* name, const double** data, int64_t* rows,
                     int64_t* cols);
int sonar_result_count(const sonar_result* res);
const char* sonar_result_name(const sonar_result* res, int index);
void sonar_result_free(sonar_result* res);

#ifdef __cplusplus
}
#endif
#endif /* SONAR_GPU_H */
