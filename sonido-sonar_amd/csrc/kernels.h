// kernels.h -- launch interfaces between the C-ABI host layer (sonar_api.cpp)
// and the HIP kernels (*.hip).  Device pointers only; all launches are async
// on the given stream.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/sonar_gpu.h"
#include "host_dsp.h"

namespace sonar {

// Issue priority of the latency-bound kernels of a pair's feature phase (DC / pre-emphasis passes,
// energy, chroma, NCC) against the DTW waves sharing their SIMDs in a batched C5 run
// (-DSONAR_FEAT_PRIO=<0..3>, A/B knob; 0 = the hardware default, no instruction)
#ifndef SONAR_FEAT_PRIO_LEVEL
#define SONAR_FEAT_PRIO_LEVEL 0
#endif
#if SONAR_FEAT_PRIO_LEVEL > 0
#define SONAR_FEAT_PRIO() __builtin_amdgcn_s_setprio(SONAR_FEAT_PRIO_LEVEL)
#else
#define SONAR_FEAT_PRIO() ((void)0)
#endif

// Fused per-frame kernel (fp_kernel.hip).  Every wave owns a contiguous range
// of STFT frames and processes it in batches of NB frames: whole-frame FFTs
// (W = 128 * R real points as a 64*R-point complex FFT + real split) into
// wave-private LDS rows, then the batch epilogue with lane = (frame, group)
// -- filterbank + ln + DCT (MFCC) and the spectral descriptors -- with no
// block-level barrier after the twiddle tables are built.
struct FpParams {
  const void* pcm;      // device, f32 or f64
  int64_t n;            // samples
  int pcm_f64;
  int64_t F;            // STFT frames
  int W, H;             // window / hop
  int64_t frames_per_wave;   // multiple of the batch size
  int64_t f_first, f_last;   // the frames this launch computes: [f_first, f_last) of F
  const void* window;   // W coefficients, precision T
  uint32_t flags;       // SONAR_FP_* bits (see sonar_gpu.h); bit 31: debug FFT-only
  // filterbank + MFCC
  int n_mels, n_mfcc;
  int input_power;      // MFCC.Compute fed |X|^2 (F5) -> uses |X|^4
  int n_groups;         // epilogue groups per frame (64 / NB)
  const int* mel_lo;    // [n_mels] first nonzero bin
  const int* mel_hi;    // [n_mels] one past last nonzero bin
  const int* mel_woff;  // [n_mels] offset into mel_w
  const void* mel_w;    // packed nonzero weights (T)
  const int* grp_off;   // [n_groups+1] ranges into grp_mels
  const int* grp_mels;  // mel indices per group (balanced by nnz)
  const void* dct;      // [n_mfcc][n_mels] (T)
  const void* lift;     // [n_mfcc] lifter multipliers (T)
  int sample_rate;
  // outputs (device); element type double if out_f64 else float
  int out_f64;
  void* out_mfcc;
  void* out_mag;
  int mag_f64;          // element type of out_mag (the SPEC scratch rows are float64 whatever out_f64 says)
  void* out_spec[9];    // centroid, rolloff, bandwidth, flatness, crest, slope, flux(F-1), low, high
  void* out_cplx;       // F x K x 2 (re, im) straight from the FFT's real split (nullable)
  void* out_phase;      // F x K atan2(im, re) (nullable)
  // LDS carve (bytes): shared twiddle tables, then one region per wave
  int lds_tab_t1, lds_tab_t2, lds_tab_t3, lds_tab_mel, lds_tab_w, lds_tab_dct, lds_wave0, lds_wave_stride;
  int nnz;              // packed filterbank weights
  int lds_logmel, lds_stage;   // offsets inside a wave region (rows start at 0)
  int lds_bytes;
  int waves_per_block;
};

int launch_fingerprint(const FpParams& p, int precision_f64, hipStream_t s);

// The per-frame spectral descriptors of SpeechFeatureExtractor.extractSpectralFeatures
// (extractors/speech.go:320-367, :438-458) from float64 |X| rows already in HBM (the fused kernel's
// magnitude output, or the DFT path's scratch): spec_rows_kernel (fp_kernel.hip), one wave per
// frame at a time over a contiguous frame run, every lane a contiguous bin chunk.
struct SpecParams {
  const double* mag;    // [F][K] |X| rows
  int64_t F;            // frames
  int K;                // bins per row (W/2 + 1)
  int sample_rate;
  int64_t frames_per_wave;
  int64_t f_first, f_last;   // the frames this launch reduces: [f_first, f_last) of F (flux reads row f_first - 1)
  int out_f64;
  void* out_spec[9];    // centroid, rolloff, bandwidth, flatness, crest, slope, flux(F-1), low, high
};
int launch_spec_rows(const SpecParams& p, hipStream_t s);

// Headline fused kernel (mfcc_pair.hip): W = 1024, MFCC output only, float32 (the headline) or
// float64 arithmetic (f64 = 1: float64 tables and output, PCM float32 or float64 per pcm_f64).
// One wave transforms two consecutive frames as one 1024-point complex FFT.  Table element type
// T = float or double per f64; "complex" = {T re, T im}.
struct MfccPairParams {
  const void* pcm;      // device PCM (float, or double when pcm_f64)
  int64_t n;            // samples
  int64_t F;            // STFT frames
  int H;                // hop
  int64_t pairs_per_block;   // contiguous pairs per block (one block per CU), claimed pair by pair by its waves
  const void* window;   // [1024] T
  const void* tw1;      // [64][16] complex  w_1024^{b k1}
  const void* tw2;      // [8][8]   complex  w_64^{b0 c0}
  const int* chunk_ks;  // [64] first bin of each lane's filterbank chunk
  const void* chunk_w;  // [64][JS] complex (weight of slot a, weight of slot b), 1/4 (or 1/16) folded
  const uint16_t* mel_src; // [16][64] partial-sum pair index (2 lane + slot), bit 15 = unused
  const void* dct;      // [16][NMP + mfcc_pair_dct_pad] T: DCT-II rows with the lifter folded in
  const void* zeros;    // [1024] zero PCM samples (8 KB): the samples of frames past the signal
  int J;                // bins per chunk (<= 16)
  int JS;               // chunk_w row stride = J | 1 (odd: conflict-free reads)
  int max_src;          // most partial sums of one filter (<= 16)
  int NMP;              // n_mels padded to a multiple of 8 (<= 64)
  int n_mels, n_mfcc;   // n_mfcc <= 16
  int pow2;             // F5: MFCC.Compute fed |X|^2 -> filterbank of |X|^4
  void* out;            // [F][n_mfcc] T
  int lds_src, lds_dct, lds_ctr, lds_tw2, lds_wave0, lds_bytes;   // lds_tw2: float64 only ([8][kPairTw2Row] complex)
  int waves_per_block;  // mfcc_pair_waves_per_block(f64)
  // sonar_fingerprint_batch (float32 only): nseg > 0 signals, F = 2 x the batch's pairs, pcm / n /
  // out unused; seg (device) = {pcm address[nseg], frames inside the signal[nseg], F[nseg], out
  // address[nseg], first pair[nseg + 1]}
  const int64_t* seg;
  int nseg;
  int f64, pcm_f64;
  uint64_t* stamp;      // HL_STAMP diagnostics builds only: per wave {start, end, pairs}
};
int launch_mfcc_pair(const MfccPairParams& p, hipStream_t s);
int mfcc_pair_wave_bytes(int f64);
int mfcc_pair_waves_per_block(int f64);   // waves per block of mfcc_pair_kernel (its LDS carve: tables + waves x wave bytes)
int mfcc_pair_waves_per_cu(int f64);      // resident waves per CU it is sized for
int mfcc_pair_rows();
// Per-instance LDS layout of mfcc_pair_kernel, shared with the host tables (bank-conflict-free
// strides for its 8-B float32 and 16-B float64 accesses: tools/pair_lds_model.py):
//   pad rows after every 16 power rows: float32 2 (18 rows x 8 B = 36 dwords per 16 bins), float64
//   1 (17 x 16 B = 68 dwords: 8-lane ds_write_b128 groups of rows 18 apart collide mod 32);
//   DCT row stride NMP + 4 (float32) / NMP + 2 (float64), stage-2 twiddle rows of 9 complex (float64).
constexpr int mfcc_pair_pad_rows(int f64) { return f64 ? 1 : 2; }
constexpr int mfcc_pair_dct_pad(int f64) { return f64 ? 2 : 4; }
constexpr int kPairTw2Row = 9;
bool fingerprint_supported(int W);
int fp_batch_frames(int W, int f64, int spec);
int fp_pre_rows(int W, int spec);

// STFT for window lengths outside the fused kernels (any W <= 8192, misc_kernels.hip): direct
// float64 DFT per frame -> |X| scratch (F x (W/2+1)) + optional Magnitude / Complex / Phase
// outputs; trig = (cos, -sin) of 2 pi m / W, m < W
int launch_stft_dft(const void* pcm, int pcm_f64, int64_t n, int64_t F, int W, int H, const double* win,
                    const double* trig, double* mag, void* out_mag, void* out_cplx, void* out_phase, int out_f64,
                    hipStream_t s);
// MFCC.ComputeFrames from |X| rows (float64 tables of host::make_mfcc_tables)
int launch_mfcc_rows(const double* mag, int64_t F, int K, const int* lo, const int* hi, const int* woff,
                     const double* w, int n_mels, const double* dct, const double* lift, int n_mfcc, int input_power,
                     void* out, int out_f64, hipStream_t s);
// ZCR + short-time energy on the pre-emphasised PCM (misc_kernels.hip)
// [f0, f1): only those frames (f1 < 0: to the end) -- the chunked host-PCM pipeline
int launch_zcr(const void* pcm, int pcm_f64, int64_t n, int64_t F, int W, int H, double alpha, int sample_rate,
               void* out, int out_f64, hipStream_t s, int64_t f0 = 0, int64_t f1 = -1);
int launch_energy(const void* pcm, int pcm_f64, int64_t n, int64_t Fe, int W, int H, double alpha,
                  void* out, int out_f64, hipStream_t s, int64_t f0 = 0, int64_t f1 = -1);
// EnergyEntropy (extractors/speech.go:429-433) of the short-time energy frames (misc_kernels.hip)
int launch_energy_entropy(const double* e, int64_t n, double* out, hipStream_t s);
// YIN raw per-frame results (misc_kernels.hip); frames start at 0, hop, 2 hop, ...
int launch_yin(const double* pcm, int64_t n, int64_t frames, int64_t hop, int sample_rate, double* pitch,
               double* conf, int32_t* tau, hipStream_t s, int64_t f0 = 0, int64_t f1 = -1);
// VoiceQualityAnalyzer helpers (misc_kernels.hip): per-period RMS, 2048-lag HNR autocorrelation
int launch_period_rms(const double* y, const int64_t* start, const int64_t* len, int64_t np, double* amp,
                      hipStream_t s);
int launch_hnr_autocorr(const double* frame2048, double* ac, hipStream_t s);
// Chroma STFT (misc_kernels.hip)
// cls (nullable): [13 class offsets][bins ascending per class] -> wave-per-frame FFT kernel (fs 256 / 512)
int launch_chroma(const double* y, int64_t n, int64_t frames, int hop, int fs, const double* window,
                  const double* trig, const int* chroma_map, const int* cls, double* out, hipStream_t s);
int launch_dc_preemph(const double* x, int64_t n, double R, double alpha, double* y, double* scratch, hipStream_t s);
size_t dc_preemph_scratch_bytes(int64_t n);
// speech-extractor helpers (misc_kernels.hip)
int launch_preemph(const void* pcm, int pcm_f64, int64_t n, double alpha, double* y, hipStream_t s, int64_t i0 = 0,
                   int64_t i1 = -1);
int launch_stats(const double* y, int64_t n, double* part, int blocks, hipStream_t s);
int launch_tilt(const double* y, int64_t n, int64_t frames, double* tilt, hipStream_t s);
// PCM ingest: f64 -> f32 (RNE); both pointers 16-B aligned (misc_kernels.hip)
int launch_f64_to_f32(const double* in, float* out, int64_t n, hipStream_t s);
// NCC (align_kernels.hip)
// One signal of a batched music-feature launch (launch_music_features_batch): its PCM, the
// pre-emphasised output, the DC chunk scratch (T chunks), energy (Fe frames) and chroma (F frames)
struct MfJob {
  const double* x;
  int64_t n;
  double* y;
  double* ends;
  double* ystart;
  int64_t T;
  double* energy;
  int64_t Fe;
  double* chroma;
  int64_t F;
};
int launch_music_features_batch(const MfJob* hjobs, const MfJob* djobs, int nj, int W, int H, int fs,
                                const double* window, const double* trig, const int* cls, hipStream_t s);
// DC chunk length of launch_dc_preemph (MfJob::T = ceil(n / chunk))
int64_t dc_chunks(int64_t n);
// One pair of a batched NCC launch (launch_ncc_batch): as launch_ncc's arguments
struct NccJob {
  const double* a;
  int64_t na;
  const double* b;
  int64_t nb;
  int64_t L;
  double* xa;
  double* xb;
  double* stats;
  double* corr;
};
int launch_ncc_batch(const NccJob* hjobs, const NccJob* djobs, int nj, hipStream_t s);
int launch_ncc(const double* a, int64_t na, const double* b, int64_t nb, int64_t L, double* norm_a,
               double* norm_b, double* stats, double* corr, hipStream_t s);
// AlignmentAnalyzer.addNoise and flatten2DFeatures (align_kernels.hip)
int launch_perturb(const double* q, int64_t nq, int dim, double level, double* out, hipStream_t s);
int launch_first_column(const double* x, int64_t n, int dim, double* out, hipStream_t s);
// DTW (dtw.go:55-217).  Band-pipelined persistent kernel; see align_kernels.hip.
struct DtwGeom {
  int64_t nq, nr;   // sequence lengths
  int64_t nb;       // 64-row bands = ceil(nq / 64)
  int64_t S;        // sweep steps per band = nr + 63
  int64_t SW;       // 16-step direction words per band = ceil(S / 16)
};
DtwGeom dtw_geom(int64_t nq, int64_t nr);
// bytes of the band-skewed cost store Cn, direction store Dn and edge buffer E
size_t dtw_cn_bytes(const DtwGeom& g);
size_t dtw_dn_bytes(const DtwGeom& g);
size_t dtw_edge_bytes(const DtwGeom& g);
// offset (elements) of C[i][j] (1-based, i,j >= 1) inside Cn
int64_t dtw_cn_index(const DtwGeom& g, int64_t i, int64_t j);
// forward sweep + backtrack; `fast` = every input finite (no NaN path in math.Min)
int launch_dtw(const double* q, const double* r, int dim, int band, bool fast, const DtwGeom& g, double* Cn,
               uint32_t* Dn, uint64_t* E, int32_t* sync_words /* [0] ticket, [1] error */,
               uint32_t* codes /* walk moves, 2 bits each */, int64_t* plen,
               uint64_t* trace /* nullable, [nb][8] diagnostics */, hipStream_t s,
               hipEvent_t mid = nullptr /* recorded between the sweep and the walk */,
               double* CK = nullptr /* Cn null: dtw_ck_bytes of checkpoint columns instead */);
// wstart: scratch of (P + 15) / 16 int2 (each code word's starting cell).  Cn null: only the
// points (and the zero cost of border points) are written; launch_dtw_path_tiles adds the costs
int launch_dtw_path_cost(const double* Cn, const DtwGeom& g, const uint32_t* codes, int64_t P, int2* wstart,
                         int32_t* pq, int32_t* pr, double* pc, hipStream_t s);
// costMatrix[1:] (nq x (nr+1), column 0 = +Inf) from the band-skewed store
int launch_dtw_cost_rowmajor(const double* Cn, const DtwGeom& g, double* out, hipStream_t s);
// One DTW's arguments (the band kernel's parameter; an array of them for launch_dtw_batch)
struct DtwArgs {
  const double* q;
  const double* r;
  int dim, band;
  int64_t nq, nr, nb, S, SW;
  double* Cn;
  uint32_t* Dn;
  uint64_t* E;
  int32_t* sync;   // [0] band ticket, [1] error flag, [2] non-finite input flag
  uint64_t* trace; // optional [nb][8]: t_start, t_first_edge, t_end, sweep wait ticks (s_memrealtime, 100 MHz),
                   // the sweep's wait ticks on its distance waves and on the band above's edge,
                   // distance-wave-0 and code-wave wait ticks
  // batched launches only (launch_dtw_batch): the walk / path-decode outputs of this DTW
  uint32_t* codes;
  int64_t* plen;
  int2* wstart;
  int32_t *pq, *pr;
  double* pc;
  double* cnm;     // C[nq][nr]
  // Cn null: the band kernel keeps only every 64th column of C (CK, dtw_ck_bytes), and the path
  // costs are recomputed per 64 x 64 tile the path visits (launch_dtw_path_tiles); runs holds
  // [0] the tile count, then each tile's first path index (dtw_run_words ints)
  double* CK;
  int32_t* runs;
  // nullable: the DTW's 16-word diagnostic record (zeroed before the launch).  The first band-kernel
  // wave of this DTW whose wait makes no progress for DTW_STALL_TICKS writes it:
  //  [0]  bit 63 valid, bits 56-62 role (DtwRole), bits 32-55 block ticket, bits 0-31 band
  //  [1]  prog | cprog << 32        [2] efill | rdy << 32        [3] dchunk[0..3], 16 bits each
  //  [4]  edge target column (min(prog, cprog) + 64, <= nr) | nr << 32
  //  [5]  E[efill+1] of the band above by an agent-scope (sc1) load, [6] the same after an
  //       agent-scope acquire (buffer_inv sc1), [7] by a system-scope load, [8] by an agent-scope
  //       atomic fetch_or(0), [9] by a system-scope fetch_or(0)
  //  [10] the first column of that E row still holding the sentinel (sc1 scan; -1: none)
  //  [11] s_memrealtime ticks (10 ns) of the failed wait (low 40 bits) | polls / 1024 << 40
  //  [12] XCC id | HW_ID << 32 of the reporting wave
  //  [13] edge-poll refresh fences issued by any band of this DTW (an agent acquire after 1 ms
  //       without a new edge value), [14] those after which the next poll found new values,
  //  [15] waves of this DTW that timed out
  uint64_t* diag;
  // tests only (SONAR_DTW_DBG_STALL=<band>): the sweep of that 64-row band stops after 1,024 steps
  // without publishing more, so the
  // pipeline's bounded waits and its diagnostic record can be exercised; -1: off
  int32_t dbg_stall = -1;
  int32_t pad_;
};
constexpr int DTW_DIAG_WORDS = 16;
// bytes of a single DTW's sync block (launch_dtw): 4 status words + the diagnostic record
constexpr int DTW_SYNC_BYTES = 16 + 8 * DTW_DIAG_WORDS;
enum DtwRole : int { DTW_ROLE_EDGE = 1, DTW_ROLE_FEEDER = 2, DTW_ROLE_SWEEP = 3, DTW_ROLE_CODE = 4,
                     DTW_ROLE_DIST = 5, DTW_ROLE_LOADER = 6 };
// checkpoint columns C[64b+1 .. 64b+64][64c] (c = 1 .. nr/64) of every band, and the run words of
// the path-tile pass
size_t dtw_ck_bytes(const DtwGeom& g);
int64_t dtw_run_words(const DtwGeom& g);
// path costs and C[nq][nr] from CK + E (the band kernel's checkpoint columns and band edges), for
// a path whose points (pq, pr) are already written: one wave per 64 x 64 tile the path visits
// recomputes the tile's cells in the band kernel's arithmetic (bit-identical).  Needs a.q, r, dim,
// band, nq, nr, nb, E, CK, pq, pr, pc, runs, cnm.
int launch_dtw_path_tiles(const DtwArgs& a, int64_t P, hipStream_t s);
// n DTWs of 12-dim finite sequences, unbanded (the chroma DTWs of sonar_align_pairs), from a
// device array of DtwArgs: the band kernel over all of them (block tickets run through DTW k's
// bands at dstart[k] .. dstart[k+1]-1; dstart[n] = total_bands), the walks (one block each), the
// path scans (which also save C[nq][nr]) and the path points, in four launches and no host
// round trip.  The caller zeroes each DTW's sync words and *ticket and fills each E with the
// sentinel words 0x7FF00001 first; max_cap >= every nq + nr + 1.
// (hargs: the same array on the host)
// dmap (nullable): ticket -> (DTW, band) order, e.g. band-major across the batch so a band waits
// about one hand-off for its predecessor instead of b of them
int32_t dtw_dbg_stall_band(bool batch);   // SONAR_DTW_DBG_STALL (tests only), -1 when unset
int launch_dtw_batch(const DtwArgs* hargs, const DtwArgs* dargs, const int64_t* dstart, int n, int64_t total_bands,
                     int64_t max_cap, int32_t* ticket, hipStream_t s, const int2* dmap = nullptr);
// One pair of sonar_align_pairs' device-side scorer reductions (pair_score_kernel): the warping
// path (length at *plen) and the energy correlation (nl lags, null: none) in, PathSums / CorrSums
// (host_dsp.h) out
struct ScoreJob {
  const int32_t *pq, *pr;
  const double* pc;
  const int64_t* plen;
  const double* corr;
  int64_t nl;
  host::PathSums* path;
  host::CorrSums* corr_out;
};
int launch_pair_scores(const ScoreJob* djobs, int n, hipStream_t s);
// sets *flag = 1 if any of the n values is not finite
int launch_nonfinite(const double* x, int64_t n, int32_t* flag, hipStream_t s);
// the same probe over q and r of every DTW of a batch (sets args[k].sync[2]); max_elems >= every
// (nq + nr) * dim
int launch_nonfinite_batch(const DtwArgs* dargs, int n, int64_t max_elems, hipStream_t s);

// MusicFeatureExtractor per-frame parts (music_kernels.hip): spectral contrast over the
// nbands bands [edges[b], edges[b+1]) of each magnitude row (contrast F x nbands) and the music
// low / high band energy ratios (nullable); maxband = the widest band
int launch_music_frames(const double* mag, int64_t F, int K, const int* edges, int nbands, int maxband,
                        double* contrast, double* lo_ratio, double* hi_ratio, hipStream_t s);
// out[0] = max |y|, out[1] = sum |y| in sample order (one wave)
int launch_abs_stats(const double* y, int64_t n, double* out, hipStream_t s);
// out[i] = max |y| over frame i = [i fs, min(i fs + fs, n))
int launch_frame_peak(const double* y, int64_t n, int64_t frames, int64_t fs, double* out, hipStream_t s);

// LPC formants (lpc_kernels.hip): one block per frame; out is sonar_formant_frame[frames]
int launch_formants(const double* pcm, int64_t frames, int64_t hop, int W, int p, int sr, int frame_ok_len,
                    const double* ham, sonar_formant_frame* out, double* coeffs, double* refl, hipStream_t s);

// ---- ContentDetector (content_kernels.hip) ------------------------------------------
// words[0] zero crossings, words[1] bits of max |x|, words[2] bits of min |x| > 1e-10 (+Inf)
int launch_detect_scan(const double* x, int64_t n, unsigned long long* words, hipStream_t s);
int launch_frame_sums(const double* x, int64_t n, int64_t frames, int64_t hop, int64_t fs, double* out,
                      hipStream_t s);
int launch_dft_mag(const double* x, int N, double* mag, hipStream_t s);

// ---- FingerprintComparator (compare_kernels.hip) -------------------------------------
// sequences summarised per fingerprint (mean, std), in compare order (comparison.go:646-770)
enum { SEQ_CENTROID = 0, SEQ_ROLLOFF, SEQ_FLUX, SEQ_RMS, SEQ_VOICING, SEQ_HARMONIC, SEQ_PITCH, SEQ_COUNT };
// One gallery record: everything Compare reads from one fingerprint.
struct FpRec {
  int64_t id;
  uint32_t present;            // SONAR_FEAT_*
  int32_t ct;
  double duration;
  double w[6];                 // getEffectiveWeights(fp) by SONAR_FD_* (comparison.go:1055-1104)
  int64_t mfcc_frames, chroma_frames;
  int32_t mfcc_C, chroma_B;
  int64_t mfcc_off;            // pool: column means [C] then stds [C] (extractMFCCStatistics order)
  int64_t chroma_off;          // pool: column means [B]
  double seq_mean[SEQ_COUNT], seq_std[SEQ_COUNT];
  int64_t seq_len[SEQ_COUNT];
  double dynamic_range, silence_ratio, onset_density, speech_rate, vtl;
  const double* centroid;      // kept sequences (device) for the spectral coherence, or null
  const double* rolloff;
};
// column statistics of one row-major matrix (a sequence is cols = 1): gonum stat.Mean and
// stat.Variance, one pass over row chunks + a chunk merge
struct StatJob {
  const double* src;
  int64_t rows;
  int32_t cols;
  int32_t nchunks;
  int64_t chunk_rows;
  int64_t part_off;            // first partial of this job: part[part_off + k * cols + c]
  double* out_mean;            // [cols]
  double* out_std;             // [cols] or null (mean only)
};
int64_t colstats_chunk_rows_for(int cols);   // rows per block (the kernel's register tile)
int launch_colstats(const StatJob* jobs, int njobs, const int* chunk_job, const int* chunk_k, int nchunks,
                    double* part_sum, double* part_m2, hipStream_t s);
// gonum stat.Correlation of SpectralCentroid / SpectralRolloff per pair -> coh[pair][2] (NaN = skip)
int launch_coherence(const FpRec* recs, const int64_t* q_idx, int64_t nq, const int64_t* c_idx, int64_t nc,
                     double* coh, hipStream_t s);
struct CompareArgs {
  const FpRec* recs;
  const double* pool;
  const int64_t* q_idx;        // [nq]
  const int64_t* c_idx;        // [nc] or null (identity)
  int64_t nq, nc;
  const double* coh;           // [nq * nc][2] when detailed
  int detailed, content_filter;
  sonar_similarity* out;       // [nq * nc]
};
int launch_compare(const CompareArgs& a, hipStream_t s);
// FindBestMatches: keys (overall or -inf), per-query counts, two stable sorts, gather
int launch_match_keys(const sonar_similarity* sims, int64_t nq, int64_t nc, double threshold, double* keys,
                      int64_t* vals, uint8_t* pass_flag, int64_t* counts, hipStream_t s);
int sort_match_keys(const double* keys, double* keys2, const int64_t* vals, int64_t* vals2, int64_t* vals3,
                    int32_t* qk, int32_t* qk2, int64_t nq, int64_t nc, void* temp, size_t* temp_bytes,
                    hipStream_t s);
int launch_match_gather(const sonar_similarity* sims, const int64_t* vals_sorted, const int64_t* counts,
                        int64_t nq, int64_t nc, int K, sonar_match* out, hipStream_t s);

}  // namespace sonar
