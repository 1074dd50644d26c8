/*
 * sonar_oracle.h -- CPU fp64 restatement of the sonido-sonar hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (sonido-sonar_amd/) links,
 * loads or calls this library.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker / the timed CPU
 * baseline ("port" of the Go code, kind="port").
 *
 * Every function restates the Go reference (read as text from
 * /root/reference, RyanBlaney/sonido-sonar) and cites file:line.
 * The Go reference cannot be compiled or run here (no Go toolchain, no module
 * cache for github.com/mjibson/go-dsp v0.0.0-20180508042940-11479a337f12 or
 * gonum v0.16.0, no network), so parity to Go is UNPINNED: the oracle is pinned
 * only by analytic known-answer tests and by numpy.
 *
 * Arithmetic follows Go on amd64 (GOAMD64=v1): float64 everywhere, no fused
 * multiply-add (this file is compiled with -ffp-contract=off), sequential
 * summation order exactly as in the Go loops.
 */
#ifndef SONAR_ORACLE_H
#define SONAR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* window types, same order as analyzers/windowing.go:14-22 */
enum { OR_WIN_HANN = 0, OR_WIN_HAMMING, OR_WIN_BLACKMAN, OR_WIN_BLACKMAN_HARRIS,
       OR_WIN_KAISER, OR_WIN_TUKEY, OR_WIN_RECTANGULAR, OR_WIN_BARTLETT, OR_WIN_WELCH };

int    or_window(int type, int size, int symmetric, int normalize, double beta, double alpha, double* out);
void   or_fft(const double* re_in, const double* im_in, int n, double* re_out, double* im_out);
int64_t or_stft_frames(int64_t n, int W, int H);
int    or_stft_mag(const double* pcm, int64_t n, int W, int H, int window_type, int nthreads, double* mag);
int    or_stft_mag_window(const double* pcm, int64_t n, int W, int H, const double* window, int nthreads, double* mag);
int    or_filterbank(int kind, int n_filters, int fft_size, int sample_rate, double low, double high, double* out);
void   or_mfcc_params(int sample_rate, int* n_coef, int* n_mels, double* low, double* high, double* lifter);
int    or_mfcc_frames(const double* mag, int64_t F, int K, int sample_rate, int n_coef, int n_mels,
                      double low, double high, int use_lifter, double lifter, int fb_kind,
                      int input_is_power, double* out);
void   or_spectral_descriptors(const double* mag, int64_t F, int K, int sample_rate,
                               double* centroid, double* rolloff, double* bandwidth, double* flatness,
                               double* crest, double* slope, double* flux, double* low_ratio, double* high_ratio);
void   or_preemphasis(const double* x, int64_t n, double alpha, double* out);
void   or_zcr_frames(const double* pcm, int64_t n, int64_t F, int W, int H, int sample_rate, double* out);
int64_t or_short_time_energy(const double* x, int64_t n, int W, int H, double* out);
int64_t or_pitch_frames(int64_t n);
void   or_yin_raw(const double* frame1024, int sample_rate, double* pitch, double* conf, int* tau);
int64_t or_pitch_track(const double* pcm, int64_t n, int sample_rate, int passes, double* pitch, double* conf, double* voicing);
int    or_voice_quality(const double* sig, int64_t n, int sample_rate, double* out12);
int    or_chroma_music(const double* pcm, int64_t n, int64_t F, int H, int sample_rate, double* out);
int    or_chroma_frames(const double* y, int64_t n, int64_t F, int H, int fs, int sample_rate, double* out);
void   or_dc_removal(const double* x, int64_t n, double R, double* out);
int    or_ncc(const double* a, int64_t na, const double* b, int64_t nb, int max_lag, double* corr, double* metrics);
int    or_dtw(const double* q, int64_t nq, const double* r, int64_t nr, int dim, int band,
              double* cost, int32_t* path_q, int32_t* path_r, double* path_cost, int64_t* path_len, double* dist);
void   or_align_dtw_metrics(const int32_t* pq, const int32_t* pr, const double* pc, int64_t P,
                            int64_t nq, int64_t nr, double dist, int sample_rate, double* out);
void   or_align_xcorr_metrics(const double* metrics, int hop, int sample_rate, int max_lag, double* out);
int    or_autocorr_fft(const double* x, int n, int max_lag, double* corr);
int    or_formant_frame(const double* sig, int64_t len, int sample_rate, double* rec24, double* coeffs, double* refl);
int    or_detect_from_audio(const double* pcm, int64_t n, int sr, double thr, double* out10, int* content_type);
int64_t or_formant_frames(const double* sig, int64_t n, int sample_rate, int frame_size, int hop, double* recs,
                          double* coeffs, double* refl);

/* SpectralContrast.Compute per row (spectral_contrast.go:26-185), F x nb */
void or_spectral_contrast(const double* mag, int64_t F, int K, int sr, int nb, double* out);
#ifdef __cplusplus
}
#endif
#endif
