/*
 * sonar_oracle.c -- fp64 CPU restatement of the sonido-sonar hot path.
 * TEST INFRASTRUCTURE ONLY (see sonar_oracle.h).  Compiled with
 * -O2 -ffp-contract=off so that a*b+c is rounded twice, like Go on amd64.
 * Citations are /root/reference paths (RyanBlaney/sonido-sonar).
 */
#include "sonar_oracle.h"
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------ */
/* Go helpers                                                          */
/* ------------------------------------------------------------------ */

/* math.Hypot (Go src/math/hypot.go): used by cmplx.Abs at
 * fingerprint/analyzers/spectral.go:492 and algorithms/spectral/stft.go:131 */
static double go_hypot(double p, double q) {
    if (isinf(p) || isinf(q)) return INFINITY;
    if (isnan(p) || isnan(q)) return NAN;
    p = fabs(p); q = fabs(q);
    if (p < q) { double t = p; p = q; q = t; }
    if (p == 0) return 0;
    q = q / p;
    return p * sqrt(1 + q * q);
}

/* Go int(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> MinInt64 */
static int64_t go_f2i(double x) {
    if (!(x >= -9.2233720368547758e18 && x < 9.2233720368547758e18)) return INT64_MIN;
    return (int64_t)x;
}

/* math.Min (Go): NaN-propagating, -0 < +0 */
static double go_min(double x, double y) {
    if (isinf(x) && x < 0) return x;
    if (isinf(y) && y < 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? x : y;
    return x < y ? x : y;
}
static double go_max(double x, double y) {
    if (isinf(x) && x > 0) return x;
    if (isinf(y) && y > 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? y : x;
    return x > y ? x : y;
}

static int cmp_dbl(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

/* ------------------------------------------------------------------ */
/* Window generation: fingerprint/analyzers/windowing.go:77-136,       */
/* 228-437 (generate*, calculateWindowProperties, normalizeWindow)     */
/* ------------------------------------------------------------------ */
static double bessel_i0(double x) {           /* windowing.go:425-441 */
    double sum = 1.0, term = 1.0;
    for (int k = 1; k < 50; k++) {
        double t = x / (2.0 * (double)k);
        term *= t * t;
        sum += term;
        if (term < 1e-12) break;
    }
    return sum;
}

int or_window(int type, int size, int symmetric, int normalize, double beta, double alpha, double* c) {
    if (size <= 0 || size > 1048576) return -1;                    /* validateConfig :177-199 */
    int N = size;
    double den = symmetric ? (double)(N - 1) : (double)N;
    switch (type) {
    case OR_WIN_HANN:                                              /* :246-256 */
        for (int i = 0; i < N; i++) c[i] = 0.5 * (1.0 - cos(2 * M_PI * (double)i / den));
        break;
    case OR_WIN_HAMMING:                                           /* :259-269 */
        for (int i = 0; i < N; i++) c[i] = 0.54 - 0.46 * cos(2 * M_PI * (double)i / den);
        break;
    case OR_WIN_BLACKMAN:                                          /* :272-285 */
        for (int i = 0; i < N; i++) { double a = 2 * M_PI * (double)i / den;
            c[i] = 0.42 - 0.5 * cos(a) + 0.08 * cos(2 * a); }
        break;
    case OR_WIN_BLACKMAN_HARRIS:                                   /* :288-301 */
        for (int i = 0; i < N; i++) { double a = 2 * M_PI * (double)i / den;
            c[i] = 0.35875 - 0.48829 * cos(a) + 0.14128 * cos(2 * a) - 0.01168 * cos(3 * a); }
        break;
    case OR_WIN_KAISER: {                                          /* :304-318 */
        if (beta < 0) return -1;
        double i0b = bessel_i0(beta);
        for (int i = 0; i < N; i++) { double a = 2.0 * (double)i / den - 1.0;
            c[i] = bessel_i0(beta * sqrt(1 - a * a)) / i0b; }
        break; }
    case OR_WIN_TUKEY: {                                           /* :321-340 */
        if (alpha < 0 || alpha > 1) return -1;
        int taper = (int)(alpha * (double)N / 2.0);
        for (int i = 0; i < N; i++) {
            if (i < taper) c[i] = 0.5 * (1 + cos(M_PI * (double)i / (double)taper - M_PI));
            else if (i >= N - taper) c[i] = 0.5 * (1 + cos(M_PI * (double)(i - (N - taper)) / (double)taper));
            else c[i] = 1.0;
        }
        break; }
    case OR_WIN_RECTANGULAR:
        for (int i = 0; i < N; i++) c[i] = 1.0;
        break;
    case OR_WIN_BARTLETT:                                          /* :350-360 */
        for (int i = 0; i < N; i++)
            c[i] = (i <= N / 2) ? 2.0 * (double)i / (double)(N - 1) : 2.0 - 2.0 * (double)i / (double)(N - 1);
        break;
    case OR_WIN_WELCH:                                             /* :363-371 */
        for (int i = 0; i < N; i++) { double a = ((double)i - (double)(N - 1) / 2.0) / ((double)(N - 1) / 2.0);
            c[i] = 1.0 - a * a; }
        break;
    default: return -1;
    }
    if (normalize) {                                               /* :393-437 */
        double energy = 0.0;
        for (int i = 0; i < N; i++) energy += c[i] * c[i];
        double power_gain = energy / (double)N;
        double nf = 1.0 / sqrt(power_gain);
        for (int i = 0; i < N; i++) c[i] *= nf;
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* FFT (stand-in for github.com/mjibson/go-dsp fft.FFTReal; parity     */
/* UNPINNED: only the DFT definition X_k = sum x_n e^{-2 pi i kn/N} is  */
/* relied on).  Radix-2 for powers of two, Bluestein otherwise.        */
/* ------------------------------------------------------------------ */
/* twiddles e^{-2 pi i k/n}, k < n/2, cached per thread (go-dsp also caches its factors) */
static __thread double* tw_re = NULL;
static __thread double* tw_im = NULL;
static __thread int tw_n = 0;

static void fft_pow2(double* re, double* im, int n, int inverse) {
    if (n != tw_n) {
        free(tw_re); free(tw_im);
        tw_re = malloc(sizeof(double) * (n / 2 + 1)); tw_im = malloc(sizeof(double) * (n / 2 + 1));
        for (int k = 0; k < n / 2; k++) { double a = -2.0 * M_PI * (double)k / (double)n; tw_re[k] = cos(a); tw_im[k] = sin(a); }
        tw_n = n;
    }
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { double t = re[i]; re[i] = re[j]; re[j] = t; t = im[i]; im[i] = im[j]; im[j] = t; }
    }
    for (int len = 2; len <= n; len <<= 1) {
        int half = len >> 1, step = n / len;
        for (int k = 0; k < half; k++) {
            double wr = tw_re[k * step], wi = inverse ? -tw_im[k * step] : tw_im[k * step];
            for (int i = k; i < n; i += len) {
                int j = i + half;
                double xr = re[j] * wr - im[j] * wi;
                double xi = re[j] * wi + im[j] * wr;
                re[j] = re[i] - xr; im[j] = im[i] - xi;
                re[i] += xr; im[i] += xi;
            }
        }
    }
}

void or_fft(const double* re_in, const double* im_in, int n, double* re, double* im) {
    if (n <= 0) return;
    if ((n & (n - 1)) == 0) {
        for (int i = 0; i < n; i++) { re[i] = re_in[i]; im[i] = im_in ? im_in[i] : 0.0; }
        fft_pow2(re, im, n, 0);
        return;
    }
    /* Bluestein */
    int m = 1; while (m < 2 * n - 1) m <<= 1;
    double* wr = malloc(sizeof(double) * n); double* wi = malloc(sizeof(double) * n);
    double* ar = calloc(m, sizeof(double)); double* ai = calloc(m, sizeof(double));
    double* br = calloc(m, sizeof(double)); double* bi = calloc(m, sizeof(double));
    for (int k = 0; k < n; k++) {
        long long kk = ((long long)k * k) % (2LL * n);
        double ang = M_PI * (double)kk / (double)n;
        wr[k] = cos(ang); wi[k] = -sin(ang);                     /* w_k = e^{-i pi k^2/n} */
    }
    for (int k = 0; k < n; k++) {
        double xr = re_in[k], xi = im_in ? im_in[k] : 0.0;
        ar[k] = xr * wr[k] - xi * wi[k]; ai[k] = xr * wi[k] + xi * wr[k];
    }
    br[0] = wr[0]; bi[0] = -wi[0];
    for (int k = 1; k < n; k++) { br[k] = br[m - k] = wr[k]; bi[k] = bi[m - k] = -wi[k]; }
    fft_pow2(ar, ai, m, 0); fft_pow2(br, bi, m, 0);
    for (int k = 0; k < m; k++) {
        double r = ar[k] * br[k] - ai[k] * bi[k], i = ar[k] * bi[k] + ai[k] * br[k];
        ar[k] = r; ai[k] = i;
    }
    fft_pow2(ar, ai, m, 1);
    for (int k = 0; k < n; k++) {
        double r = ar[k] / m, i = ai[k] / m;
        re[k] = r * wr[k] - i * wi[k]; im[k] = r * wi[k] + i * wr[k];
    }
    free(wr); free(wi); free(ar); free(ai); free(br); free(bi);
}

/* ------------------------------------------------------------------ */
/* STFT magnitude: fingerprint/analyzers/spectral.go:385-545            */
/* (same math as algorithms/spectral/stft.go:45-160 with a caller window)*/
/* ------------------------------------------------------------------ */
int64_t or_stft_frames(int64_t n, int W, int H) {                /* spectral.go:409-412 */
    if (n <= 0 || W <= 0 || H <= 0) return -1;
    int64_t F = (n - W) / H + 1;                                  /* Go truncating division */
    return F <= 0 ? -1 : F;
}

typedef struct { const double* pcm; int64_t n; int W, H, K; const double* win; double* mag;
                 int64_t f0, f1; } stft_job;

static void* stft_worker(void* arg) {                             /* worker body :470-497 */
    stft_job* j = (stft_job*)arg;
    double* buf = malloc(sizeof(double) * j->W);
    double* re = malloc(sizeof(double) * j->W); double* im = malloc(sizeof(double) * j->W);
    for (int64_t t = j->f0; t < j->f1; t++) {
        int64_t s = t * j->H;
        double* row = j->mag + t * j->K;
        if (s + j->W > j->n) { memset(row, 0, sizeof(double) * j->K); continue; } /* job skipped :524-534 */
        for (int i = 0; i < j->W; i++) buf[i] = j->pcm[s + i] * j->win[i];     /* ApplyInPlace :152-160 */
        or_fft(buf, NULL, j->W, re, im);
        for (int k = 0; k < j->K; k++) row[k] = go_hypot(re[k], im[k]);          /* cmplx.Abs :492 */
    }
    free(buf); free(re); free(im);
    return NULL;
}

int or_stft_mag_window(const double* pcm, int64_t n, int W, int H, const double* win, int nthreads, double* mag) {
    int64_t F = or_stft_frames(n, W, H);
    if (F < 0) return -1;
    int K = W / 2 + 1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > F) nthreads = (int)F;
    pthread_t* th = malloc(sizeof(pthread_t) * nthreads);
    stft_job* jobs = malloc(sizeof(stft_job) * nthreads);
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = (stft_job){pcm, n, W, H, K, win, mag, F * i / nthreads, F * (i + 1) / nthreads};
        if (nthreads == 1) stft_worker(&jobs[i]);
        else pthread_create(&th[i], NULL, stft_worker, &jobs[i]);
    }
    if (nthreads > 1) for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th); free(jobs);
    return 0;
}

int or_stft_mag(const double* pcm, int64_t n, int W, int H, int window_type, int nthreads, double* mag) {
    double* win = malloc(sizeof(double) * W);
    /* SpectralAnalyzer always asks for {Normalize:true, Symmetric:true} (spectral.go:415-420); the
     * literal leaves Beta and Alpha at Go's zero value (not DefaultWindowConfig's 8.6 / 0.5,
     * windowing.go:66-73): Kaiser is I0(0)/I0(0) = 1, Tukey has no taper -- both rectangular */
    if (or_window(window_type, W, 1, 1, 0.0, 0.0, win) != 0) { free(win); return -2; }
    int rc = or_stft_mag_window(pcm, n, W, H, win, nthreads, mag);
    free(win);
    return rc;
}

/* SpectrogramResult.Complex / .Phase rows (spectral.go:490-494): fftResult[i] for the positive
 * bins and cmplx.Phase = atan2(imag, real); skipped frames (:524-534) stay zero. */
int or_stft_complex(const double* pcm, int64_t n, int W, int H, int window_type, double* re_out, double* im_out,
                    double* phase) {
    int64_t F = or_stft_frames(n, W, H);
    if (F < 0) return -1;
    int K = W / 2 + 1;
    double* win = malloc(sizeof(double) * W);
    if (or_window(window_type, W, 1, 1, 0.0, 0.0, win) != 0) { free(win); return -2; }   /* as or_stft_mag */
    double* buf = malloc(sizeof(double) * W);
    double* re = malloc(sizeof(double) * W); double* im = malloc(sizeof(double) * W);
    for (int64_t t = 0; t < F; t++) {
        int64_t s = t * H;
        double *ro = re_out + t * K, *io = im_out + t * K, *po = phase + t * K;
        if (s + W > n) { memset(ro, 0, sizeof(double) * K); memset(io, 0, sizeof(double) * K);
                         memset(po, 0, sizeof(double) * K); continue; }
        for (int i = 0; i < W; i++) buf[i] = pcm[s + i] * win[i];
        or_fft(buf, NULL, W, re, im);
        for (int k = 0; k < K; k++) { ro[k] = re[k]; io[k] = im[k]; po[k] = atan2(im[k], re[k]); }
    }
    free(buf); free(re); free(im); free(win);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Filterbanks: algorithms/spectral/mel_scale.go:19-86 and              */
/* algorithms/spectral/bark_scale.go:20-93 (kind 0 = mel, 1 = bark)     */
/* ------------------------------------------------------------------ */
static double hz_to_mel(double hz) { return 2595.0 * log10(1.0 + hz / 700.0); }
static double mel_to_hz(double m) { return 700.0 * (pow(10.0, m / 2595.0) - 1.0); }
static double hz_to_bark(double hz) { return (26.81 * hz / (1960.0 + hz)) - 0.53; }
static double bark_to_hz(double b) { return 1960.0 * (b + 0.53) / (26.28 - b); }

int or_filterbank(int kind, int nf, int fft_size, int sr, double low, double high, double* fb) {
    if (nf <= 0 || fft_size <= 0) return -1;
    int K = fft_size / 2 + 1;
    memset(fb, 0, sizeof(double) * (size_t)nf * K);
    double lo = kind ? hz_to_bark(low) : hz_to_mel(low);
    double hi = kind ? hz_to_bark(high) : hz_to_mel(high);
    double step = (hi - lo) / (double)(nf + 1);
    int64_t* bins = malloc(sizeof(int64_t) * (nf + 2));
    for (int i = 0; i < nf + 2; i++) {
        double p = lo + (double)i * step;
        double hz = kind ? bark_to_hz(p) : mel_to_hz(p);
        int64_t b = go_f2i(floor(((double)fft_size + 1.0) * hz / (double)sr + 0.5));
        if (b > fft_size / 2) b = fft_size / 2;
        bins[i] = b;
    }
    for (int m = 1; m <= nf; m++) {
        int64_t l = bins[m - 1], c = bins[m], r = bins[m + 1];
        double* row = fb + (size_t)(m - 1) * K;
        for (int64_t k = l; k < c && k < K; k++)
            if (c != l && k >= 0) row[k] = (double)(k - l) / (double)(c - l);
        for (int64_t k = c; k < r && k < K; k++)
            if (r != c && k >= 0) row[k] = (double)(r - k) / (double)(r - c);
    }
    free(bins);
    return 0;
}

/* ------------------------------------------------------------------ */
/* MFCC: algorithms/spectral/mfcc.go:44-245                              */
/* ------------------------------------------------------------------ */
void or_mfcc_params(int sr, int* n_coef, int* n_mels, double* low, double* high, double* lifter) {
    /* NewMFCCWithParams defaults (mfcc.go:58-84) */
    if (*n_coef <= 0) *n_coef = 13;
    if (*n_mels <= 0) *n_mels = 26;
    if (*high <= 0) *high = (double)sr / 2.0;
    if (*lifter <= 0) *lifter = 22.0;
    (void)low;
}

int or_mfcc_frames(const double* mag, int64_t F, int K, int sr, int n_coef, int n_mels,
                   double low, double high, int use_lifter, double lifter, int fb_kind,
                   int input_is_power, double* out) {
    or_mfcc_params(sr, &n_coef, &n_mels, &low, &high, &lifter);
    int fft_size = (K - 1) * 2;                                   /* ComputeFrames :173-178 */
    double* fb = malloc(sizeof(double) * (size_t)n_mels * K);
    if (or_filterbank(fb_kind, n_mels, fft_size, sr, low, high, fb) != 0) { free(fb); return -1; }
    double* dct = malloc(sizeof(double) * (size_t)n_coef * n_mels); /* createDCTMatrix :194-212 */
    for (int k = 0; k < n_coef; k++)
        for (int n = 0; n < n_mels; n++) {
            double v = cos(M_PI * (double)k * ((double)n + 0.5) / (double)n_mels);
            v *= (k == 0) ? sqrt(1.0 / (double)n_mels) : sqrt(2.0 / (double)n_mels);
            dct[k * n_mels + n] = v;
        }
    double* p = malloc(sizeof(double) * K);
    double* lm = malloc(sizeof(double) * n_mels);
    for (int64_t t = 0; t < F; t++) {
        const double* m = mag + t * K;
        for (int k = 0; k < K; k++) p[k] = m[k] * m[k];           /* Compute :126-130 */
        (void)input_is_power; /* music path passes |X|^2 here -> |X|^4 (F5): caller squares first */
        for (int f = 0; f < n_mels; f++) {                        /* ApplyFilterBank mel_scale.go:89-105 */
            double s = 0.0;
            const double* w = fb + (size_t)f * K;
            for (int k = 0; k < K; k++) s += p[k] * w[k];
            lm[f] = s > 0 ? log(s) : log(1e-10);                  /* :135-143 */
        }
        double* o = out + t * n_coef;
        for (int k = 0; k < n_coef; k++) {                        /* applyDCT :215-227 */
            double s = 0.0;
            for (int n = 0; n < n_mels; n++) s += lm[n] * dct[k * n_mels + n];
            o[k] = s;
        }
        if (use_lifter)                                           /* applyLiftering :230-245 */
            for (int i = 1; i < n_coef; i++)
                o[i] = o[i] * (1.0 + (lifter / 2.0) * sin(M_PI * (double)i / lifter));
    }
    free(fb); free(dct); free(p); free(lm);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Per-frame spectral descriptors, SpeechFeatureExtractor.              */
/* extractSpectralFeatures (fingerprint/extractors/speech.go:320-367)   */
/* and extractEnergyFeatures ratios (:438-458)                           */
/* ------------------------------------------------------------------ */
void or_spectral_descriptors(const double* mag, int64_t F, int K, int sr,
                             double* centroid, double* rolloff, double* bandwidth, double* flatness,
                             double* crest, double* slope, double* flux, double* low_ratio, double* high_ratio) {
    double* fb = malloc(sizeof(double) * K);
    for (int i = 0; i < K; i++) fb[i] = (double)i * (double)sr / (double)((K - 1) * 2); /* initializeFreqBins */
    for (int64_t t = 0; t < F; t++) {
        const double* s = mag + t * K;
        /* spectral_centroid.go:18-41 */
        double num = 0, den = 0;
        for (int i = 0; i < K; i++) { num += fb[i] * s[i]; den += s[i]; }
        double c = den == 0 ? 0 : num / den;
        centroid[t] = c;
        /* spectral_rolloff.go:18-52, threshold 0.85 */
        double tot = 0;
        for (int i = 0; i < K; i++) tot += s[i] * s[i];
        double ro = 0;
        if (tot != 0) {
            double target = 0.85 * tot, cum = 0;
            int found = 0;
            for (int i = 0; i < K; i++) { cum += s[i] * s[i]; if (cum >= target) { ro = fb[i]; found = 1; break; } }
            if (!found) ro = fb[K - 1];
        }
        rolloff[t] = ro;
        /* spectral_bandwidth.go:22-47 */
        num = 0; den = 0;
        for (int i = 0; i < K; i++) { double d = fb[i] - c; num += d * d * s[i]; den += s[i]; }
        bandwidth[t] = den == 0 ? 0 : sqrt(num / den);
        /* spectral_flatness.go:31-73 */
        double ls = 0; int vc = 0;
        for (int i = 0; i < K; i++) if (s[i] > 1e-10) { ls += log(s[i]); vc++; }
        double fl = 0;
        if (vc > 0) {
            double geo = exp(ls / (double)vc), am = 0;
            for (int i = 0; i < K; i++) am += s[i];
            am /= (double)K;
            if (am > 1e-10) { fl = geo / am; if (fl > 1.0) fl = 1.0; }
        }
        flatness[t] = fl;
        /* spectral_crest.go:18-38 */
        double mx = 0, ss = 0;
        for (int i = 0; i < K; i++) { if (s[i] > mx) mx = s[i]; ss += s[i] * s[i]; }
        double rms = sqrt(ss / (double)K);
        crest[t] = rms == 0 ? 0 : mx / rms;
        /* spectral_slope.go:23-63 */
        double sl = 0;
        if (K >= 2) {
            int nn = 0; double sx = 0, sy = 0, sxy = 0, sxx = 0;
            for (int i = 0; i < K; i++)
                if (s[i] > 1e-10 && fb[i] > 0) {
                    double x = log10(fb[i]), y = log10(s[i]);
                    sx += x; sy += y; sxy += x * y; sxx += x * x; nn++;
                }
            if (nn >= 2) {
                double d = (double)nn * sxx - sx * sx;
                if (d != 0) sl = ((double)nn * sxy - sx * sy) / d;
            }
        }
        slope[t] = sl;
        /* energy band ratios, speech.go:438-458 */
        if (low_ratio) {
            double lo = 0, hi = 0, tt = 0; int split = K / 4;
            for (int j = 0; j < K; j++) { double e = s[j] * s[j]; tt += e; if (j < split) lo += e; else hi += e; }
            low_ratio[t] = tt > 0 ? lo / tt : 0;
            high_ratio[t] = tt > 0 ? hi / tt : 0;
        }
        /* spectral_flux.go:17-36 (F-1 values) */
        if (flux && t > 0) {
            const double* pv = mag + (t - 1) * K;
            double sm = 0;
            for (int f = 0; f < K; f++) { double d = s[f] - pv[f]; if (d > 0) sm += d * d; }
            flux[t - 1] = sqrt(sm);
        }
    }
    free(fb);
}

/* pre_emphasis.go:135-190 (fresh filter: x[-1] = 0) */
void or_preemphasis(const double* x, int64_t n, double alpha, double* out) {
    double last = 0.0;
    for (int64_t i = 0; i < n; i++) { out[i] = x[i] - alpha * last; last = x[i]; }
}

/* dc_removal.go:101-115 (fresh filter) */
void or_dc_removal(const double* x, int64_t n, double R, double* out) {
    double x1 = 0.0, y1 = 0.0;
    for (int64_t i = 0; i < n; i++) { double y = x[i] - x1 + R * y1; x1 = x[i]; y1 = y; out[i] = y; }
}

/* ZCR per STFT frame on the pre-emphasised PCM: speech.go:351-358 ->
 * zero_crossing_rate.go:37-52 */
void or_zcr_frames(const double* pcm, int64_t n, int64_t F, int W, int H, int sr, double* out) {
    for (int64_t t = 0; t < F; t++) {
        int64_t s = t * H, e = s + W;
        if (e > n) e = n;
        out[t] = 0.0;
        if (s >= n) continue;
        int64_t len = e - s;
        if (len < 2) continue;
        int64_t cr = 0;
        for (int64_t i = s + 1; i < e; i++) {
            double a = pcm[i - 1], b = pcm[i];
            if ((a >= 0 && b < 0) || (a < 0 && b >= 0)) cr++;
        }
        double dur = (double)len / (double)sr;
        out[t] = (double)cr / dur;
    }
}

/* temporal/energy.go:25-50 */
int64_t or_short_time_energy(const double* x, int64_t n, int W, int H, double* out) {
    if (n < W || H <= 0 || W <= 0) return 0;
    int64_t F = (n - W) / H + 1;
    for (int64_t i = 0; i < F; i++) {
        int64_t s = i * H, e = s + W;
        if (e > n) return i;
        double ss = 0;
        for (int64_t j = s; j < e; j++) ss += x[j] * x[j];
        if (out) out[i] = sqrt(ss / (double)W);
    }
    return F;
}

/* ------------------------------------------------------------------ */
/* YIN: algorithms/tonal/pitch_detection.go:225-420, 743-921            */
/* ------------------------------------------------------------------ */
#define YIN_N 1024
void or_yin_raw(const double* fr, int sr, double* pitch, double* conf, int* tau_out) {
    double x[YIN_N], w[YIN_N];
    for (int i = 0; i < YIN_N; i++) w[i] = 0.5 * (1.0 - cos(2.0 * M_PI * (double)i / (double)(YIN_N - 1))); /* :314-318 */
    x[0] = fr[0];                                                 /* applyPreEmphasis :296-310 */
    for (int i = 1; i < YIN_N; i++) x[i] = fr[i] - 0.97 * fr[i - 1];
    for (int i = 0; i < YIN_N; i++) x[i] *= w[i];                 /* preprocessFrame :282-293 */
    const int half = YIN_N / 2;
    double diff[YIN_N / 2], cm[YIN_N / 2];
    for (int tau = 0; tau < half; tau++) {                        /* detectPitchYin :349-362 */
        double s = 0.0;
        for (int j = 0; j < half; j++) { double d = x[j] - x[j + tau]; s += d * d; }
        diff[tau] = s;
    }
    cm[0] = 1.0; double run = 0.0;
    for (int tau = 1; tau < half; tau++) { run += diff[tau]; cm[tau] = diff[tau] / (run / (double)tau); }
    int mt = -1;
    for (int tau = 1; tau < half; tau++)
        if (cm[tau] < 0.15) if (tau + 1 < half && cm[tau] < cm[tau + 1]) { mt = tau; break; }
    *pitch = 0; *conf = 0; if (tau_out) *tau_out = mt;
    if (mt > 0) {
        double period = (double)mt;                               /* parabolicInterpolation :743-764 */
        if (!(mt <= 0 || mt >= half - 1)) {
            double y1 = cm[mt - 1], y2 = cm[mt], y3 = cm[mt + 1];
            double a = (y1 - 2 * y2 + y3) / 2, b = (y3 - y1) / 2;
            if (a != 0) period = (double)mt + (-b / (2 * a));
        }
        double f = (double)sr / period, c = 1.0 - cm[mt];
        if (f >= 80.0 && f <= 1000.0) { *pitch = f; *conf = c; }
    }
}

static double median_pos(const double* v, int n) {                 /* calculateMedian :975-1004 */
    double tmp[32]; int m = 0;
    for (int i = 0; i < n; i++) if (v[i] > 0) tmp[m++] = v[i];
    if (m == 0) return 0.0;
    qsort(tmp, m, sizeof(double), cmp_dbl);
    return (m % 2 == 0) ? (tmp[m / 2 - 1] + tmp[m / 2]) / 2.0 : tmp[m / 2];
}

typedef struct { double hist[20]; int nh; double prev; } yin_track;

/* postProcessResult + updateTemporalTracking (:767-921) for one frame */
static void yin_track_step(yin_track* st, double* pitch, double* conf, double* voicing) {
    double p = *pitch, c = *conf, v = *conf;
    if (p != 0.0 && st->nh > 0) {                                 /* applyOctaveCorrection :789-827 */
        int cnt = st->nh < 5 ? st->nh : 5;
        if (cnt >= 3) {
            double med = median_pos(st->hist + st->nh - cnt, cnt);
            const double ratios[4] = {0.5, 2.0, 1.0 / 3.0, 3.0};
            for (int r = 0; r < 4; r++) {
                double ex = med * ratios[r];
                if (fabs(p - ex) / ex < 0.1) {
                    if (fabs(p - med) > fabs(ex - med)) p = ex;
                    break;
                }
            }
        }
    }
    if (c < 0.5) { p = 0; c = 0; v = 0; }                         /* MinConfidence gate :781-785 */
    if (st->nh == 20) { memmove(st->hist, st->hist + 1, sizeof(double) * 19); st->nh = 19; }
    st->hist[st->nh++] = p;                                       /* updateTemporalTracking :876-891 */
    if (st->nh > 1) {                                             /* applyTemporalSmoothing :903-921 */
        int cnt = st->nh < 3 ? st->nh : 3;
        if (cnt >= 3) p = median_pos(st->hist + st->nh - cnt, cnt);
        else p = 0.3 * p + (1 - 0.3) * st->prev;
    }
    st->prev = p;
    *pitch = p; *conf = c; *voicing = v;
}

int64_t or_pitch_frames(int64_t n) {                              /* speech.go:469-471 */
    int64_t F = (n - 1024) / 512 + 1;
    return F < 0 ? 0 : F;
}

int64_t or_pitch_track(const double* pcm, int64_t n, int sr, int passes, double* pitch, double* conf, double* voicing) {
    int64_t F = or_pitch_frames(n);
    yin_track st; memset(&st, 0, sizeof(st));
    for (int ps = 0; ps < passes; ps++)
        for (int64_t i = 0; i < F; i++) {
            int64_t s = i * 512, e = s + 1024;
            if (e > n) e = n;
            pitch[i] = conf[i] = voicing[i] = 0;
            if (e - s != 1024) continue;                           /* DetectPitch size check :226-228 */
            double p, c;
            or_yin_raw(pcm + s, sr, &p, &c, NULL);
            double v;
            yin_track_step(&st, &p, &c, &v);
            pitch[i] = p; conf[i] = c; voicing[i] = v;
        }
    return F;
}

/* ------------------------------------------------------------------ */
/* VoiceQualityAnalyzer.AnalyzeVoiceQuality                              */
/* (algorithms/speech/voice_quality.go:56-111) on the signal the speech  */
/* extractor hands AnalyzeSpeech (the pre-emphasised PCM,                */
/* speech_analysis.go:77).  out[12] = jitter, shimmer, hnr,              */
/* noise_measure, f0_stability, amplitude_stability, voicing_strength,   */
/* overall_quality, num_periods, mean_f0, f0_range, analysis_quality.    */
/* Returns 0, -1 (shorter than one second, :57-59) or -2 (fewer than 3   */
/* periods, :67-69); on error out[] is left zero (the Go result is nil). */
/* ------------------------------------------------------------------ */
int or_voice_quality(const double* sig, int64_t n, int sr, double* out) {
    for (int k = 0; k < 12; k++) out[k] = 0.0;
    if (n < (int64_t)sr) return -1;
    /* extractPitchPeriodsAndF0 :114-157: fresh PitchDetector (NewVoiceQualityAnalyzer :51),
     * frames of 1024 at hop 256 while i < len-1024 */
    int64_t cap = n > 1024 ? (n - 1025) / 256 + 1 : 0;
    int64_t* ps = (int64_t*)malloc(sizeof(int64_t) * (cap + 1));
    int64_t* pl = (int64_t*)malloc(sizeof(int64_t) * (cap + 1));
    double* f0v = (double*)malloc(sizeof(double) * (cap + 1));
    int64_t np_ = 0, last_end = 0;
    yin_track st; memset(&st, 0, sizeof(st));
    for (int64_t i = 0; i < n - 1024; i += 256) {
        double p, c, v;
        or_yin_raw(sig + i, sr, &p, &c, NULL);
        yin_track_step(&st, &p, &c, &v);
        if (v > 0.5 && c > 0.5 && p >= 50.0 && p <= 500.0) {
            int64_t len = go_f2i((double)sr / p);
            int64_t s0 = i > last_end ? i : last_end;
            int64_t e0 = s0 + len;
            if (e0 < n) { ps[np_] = s0; pl[np_] = len; f0v[np_] = p; np_++; last_end = e0; }
        }
    }
    /* calculateVoicingStrength :363-371: DetectPitch on the whole signal, which only accepts
     * exactly 1024 samples (pitch_detection.go:226); the tracker state carries over */
    double vstr = 0.0;
    if (n == 1024) { double p, c; or_yin_raw(sig, sr, &p, &c, NULL); yin_track_step(&st, &p, &c, &vstr); }
    int rc = 0;
    if (np_ < 3) { rc = -2; goto done; }
    {
        double* amp = (double*)malloc(sizeof(double) * np_);
        for (int64_t k = 0; k < np_; k++) {                       /* RMS per period :200-207 */
            double r = 0.0;
            for (int64_t j = 0; j < pl[k]; j++) r += sig[ps[k] + j] * sig[ps[k] + j];
            amp[k] = sqrt(r / (double)pl[k]);
        }
        /* calculateJitter :160-191 */
        double avg = 0.0, js = 0.0;
        for (int64_t k = 0; k < np_; k++) avg += (double)pl[k];
        avg /= (double)np_;
        for (int64_t k = 1; k < np_; k++) js += fabs((double)pl[k] - (double)pl[k - 1]);
        double jitter = avg == 0 ? 0.0 : (js / (double)(np_ - 1)) / avg * 100.0;
        /* calculateShimmer :194-229 */
        double aavg = 0.0, ss = 0.0;
        for (int64_t k = 0; k < np_; k++) aavg += amp[k];
        aavg /= (double)np_;
        for (int64_t k = 1; k < np_; k++) ss += fabs(amp[k] - amp[k - 1]);
        double shimmer = aavg == 0 ? 0.0 : (ss / (double)(np_ - 1)) / aavg * 100.0;
        /* calculateHNR :232-294 (mean F0, 2048-sample frame at the middle) */
        double hnr = 0.0, mf = 0.0;
        for (int64_t k = 0; k < np_; k++) mf += f0v[k];
        mf /= (double)np_;
        if (n >= 2048) {
            int64_t s0 = n / 2 - 1024; if (s0 < 0) s0 = 0;
            const double* fr = sig + s0;
            double* ac = (double*)malloc(sizeof(double) * 2048);
            for (int lag = 0; lag < 2048; lag++) {
                double s = 0.0; int cnt = 0;
                for (int i = 0; i < 2048 - lag; i++) { s += fr[i] * fr[i + lag]; cnt++; }
                ac[lag] = cnt > 0 ? s / (double)cnt : 0.0;
            }
            int64_t el = go_f2i((double)sr / mf);
            if (el < 2048) {
                double mc = 0.0;
                int64_t sr_ = el / 4, a = el - sr_ > 1 ? el - sr_ : 1, b = el + sr_ < 2047 ? el + sr_ : 2047;
                for (int64_t i = a; i <= b; i++) if (ac[i] > mc) mc = ac[i];
                if (mc > 0 && mc < ac[0]) hnr = 10.0 * log10(mc / (ac[0] - mc));
            }
            free(ac);
        }
        /* calculateF0Stability :297-322 */
        double var = 0.0;
        for (int64_t k = 0; k < np_; k++) { double d = f0v[k] - mf; var += d * d; }
        var /= (double)np_;
        double f0s = mf == 0 ? 0.0 : go_max(0.0, 1.0 - sqrt(var) / mf);
        /* calculateAmplitudeStability :325-360 */
        double av = 0.0;
        for (int64_t k = 0; k < np_; k++) { double d = amp[k] - aavg; av += d * d; }
        av /= (double)np_;
        double ams = aavg == 0 ? 0.0 : go_max(0.0, 1.0 - sqrt(av) / aavg);
        /* calculateNoiseMeasure :374-398 */
        double nm = 0.0;
        if (n >= 1024) {
            double hf = 0.0, te = 0.0;
            for (int i = 1; i < 1024; i++) { double d = sig[i] - sig[i - 1]; hf += d * d; te += sig[i] * sig[i]; }
            nm = te == 0 ? 0.0 : hf / te;
        }
        /* calculateF0Statistics :401-426 */
        double lo = f0v[0], hi = f0v[0];
        for (int64_t k = 0; k < np_; k++) { if (f0v[k] < lo) lo = f0v[k]; if (f0v[k] > hi) hi = f0v[k]; }
        /* calculateOverallQuality :429-437, calculateAnalysisQuality :440-451 */
        double oq = (go_max(0, 1.0 - jitter / 5.0) + go_max(0, 1.0 - shimmer / 10.0) +
                     go_min(1.0, go_max(0, hnr / 20.0)) + f0s) / 4.0;
        double aq = (go_min(1.0, (double)np_ / 10.0) + f0s + go_min(1.0, go_max(0, hnr / 15.0))) / 3.0;
        out[0] = jitter; out[1] = shimmer; out[2] = hnr; out[3] = nm; out[4] = f0s; out[5] = ams;
        out[6] = vstr; out[7] = oq; out[8] = (double)np_; out[9] = mf; out[10] = hi - lo; out[11] = aq;
        free(amp);
    }
done:
    free(ps); free(pl); free(f0v);
    return rc;
}

/* ------------------------------------------------------------------ */
/* Chroma: MusicFeatureExtractor.extractChromaFeatures                   */
/* (fingerprint/extractors/music.go:327-376) -> ChromaSTFT.ComputeChroma */
/* (algorithms/chroma/chroma_stft.go:45-138)                             */
/* ------------------------------------------------------------------ */
int or_chroma_frames(const double* y, int64_t n, int64_t F, int H, int fs, int sr, double* out) {
    if (fs <= 0) return -1;
    double* win = malloc(sizeof(double) * fs);
    or_window(OR_WIN_HANN, fs, 1, 1, 0.0, 0.0, win);     /* music.go:335-340 literal (Hann: no parameter) */
    int K = fs / 2 + 1;
    int* map = malloc(sizeof(int) * K);
    double res = (double)sr / (double)fs;                         /* FreqResolution stft.go:158 */
    for (int f = 0; f < K; f++) {                                 /* calculateChromaMapping :95-117 */
        double fr = (double)f * res;
        if (fr < 80.0 || fr > 8000.0) { map[f] = -1; continue; }
        double midi = fr <= 0 ? 0 : 69.0 + 12.0 * log2(fr / 440.0);
        map[f] = (int)(go_f2i(round(midi)) % 12);
    }
    double* buf = malloc(sizeof(double) * fs);
    double* re = malloc(sizeof(double) * fs); double* im = malloc(sizeof(double) * fs);
    for (int64_t t = 0; t < F; t++) {
        int64_t s = t * H, e = s + fs;
        if (e > n) e = n;
        for (int i = 0; i < fs; i++) buf[i] = (s + i < e) ? y[s + i] : 0.0;   /* zero pad :351-357 */
        for (int i = 0; i < fs; i++) buf[i] *= win[i];
        or_fft(buf, NULL, fs, re, im);
        double* c = out + t * 12;
        for (int b = 0; b < 12; b++) c[b] = 0;
        for (int f = 0; f < K; f++) {
            double m = go_hypot(re[f], im[f]);
            int b = map[f];
            if (b >= 0 && b < 12) c[b] += m * m;
        }
        double tot = 0;                                           /* normalizeChromaFrame :125-138 */
        for (int b = 0; b < 12; b++) tot += c[b];
        if (tot > 1e-10) for (int b = 0; b < 12; b++) c[b] /= tot;
    }
    free(win); free(map); free(buf); free(re); free(im);
    return 0;
}

int or_chroma_music(const double* pcm, int64_t n, int64_t F, int H, int sr, double* out) {
    if (F <= 0) return -1;
    double* d = malloc(sizeof(double) * n); double* y = malloc(sizeof(double) * n);
    or_dc_removal(pcm, n, 0.995, d);                              /* preprocessAudio music.go:245-259 */
    or_preemphasis(d, n, 0.95, y);
    int fs = (int)(n / F);                                        /* frameSize = len/numFrames :331 */
    int rc = or_chroma_frames(y, n, F, H, fs, sr, out);
    free(d); free(y);
    return rc;
}

/* ------------------------------------------------------------------ */
/* Normalized cross-correlation, time domain:                           */
/* algorithms/stats/correlation.go:131-200, 203-228, 373-501, 526-667   */
/* metrics[] = {peak_corr, peak_lag, peak_idx, p_value, snr, sharpness, */
/*              second_peak, psl, overlap_len, num_lags}                */
/* ------------------------------------------------------------------ */
static double* ncc_normalize(const double* s, int64_t n) {        /* :464-501 */
    double* o = malloc(sizeof(double) * (n > 0 ? n : 1));
    double mean = 0; for (int64_t i = 0; i < n; i++) mean += s[i];
    mean /= (double)n;
    double var = 0; for (int64_t i = 0; i < n; i++) { double d = s[i] - mean; var += d * d; }
    var /= (double)n;
    double sd = sqrt(var);
    if (sd < 1e-10) for (int64_t i = 0; i < n; i++) o[i] = s[i] - mean;
    else for (int64_t i = 0; i < n; i++) o[i] = (s[i] - mean) / sd;
    return o;
}

static void overlap_region(int64_t l1, int64_t l2, int64_t lag, int64_t* s1, int64_t* e1, int64_t* s2, int64_t* e2) {
    if (lag >= 0) { *s1 = 0; *e1 = l1; *s2 = lag; *e2 = l2; if (*e1 > l2 - lag) *e1 = l2 - lag; if (*e2 > l2) *e2 = l2; }
    else { *s1 = -lag; *e1 = l1; *s2 = 0; *e2 = l2; if (*e1 > l1) *e1 = l1; if (*e2 > l1 + lag) *e2 = l1 + lag; }
}

int or_ncc(const double* a, int64_t na, const double* b, int64_t nb, int max_lag, double* corr, double* met) {
    if (na == 0 || nb == 0) return -1;                            /* "empty signals provided" */
    double* x = ncc_normalize(a, na); double* y = ncc_normalize(b, nb);
    int64_t L = max_lag;                                          /* calculateActualMaxLag :452-461 */
    if (L > na - 1) L = na - 1;
    if (L > nb - 1) L = nb - 1;
    if (L < 0) L = 0;
    int64_t nl = 2 * L + 1;
    for (int64_t i = 0; i < nl; i++) {                            /* normalizedCrossCorrelation :373-409 */
        int64_t lag = i - L, s1, e1, s2, e2;
        overlap_region(na, nb, lag, &s1, &e1, &s2, &e2);
        int64_t ov = (e1 - s1) < (e2 - s2) ? (e1 - s1) : (e2 - s2);
        double c = 0.0;
        if (ov > 0) {
            double sm = 0, q1 = 0, q2 = 0;
            for (int64_t k = 0; k < ov; k++) {
                double v1 = x[s1 + k], v2 = y[s2 + k];
                sm += v1 * v2; q1 += v1 * v1; q2 += v2 * v2;
            }
            double dn = sqrt(q1 * q2);
            c = dn < 1e-10 ? 0.0 : sm / dn;
        }
        corr[i] = c;
    }
    free(x); free(y);
    /* findPeak :526-544 */
    double pk = corr[0]; int64_t pidx = 0;
    for (int64_t i = 0; i < nl; i++) if (fabs(corr[i]) > fabs(pk)) { pk = corr[i]; pidx = i; }
    int64_t plag = pidx - L;
    /* calculatePValue :547-569 */
    int64_t nmin = na < nb ? na : nb; double pv = 1.0;
    if (nmin > 2) {
        double t = fabs(pk) * sqrt((double)(nmin - 2)) / sqrt(1.0 - pk * pk);
        pv = t > 2.0 ? 0.01 : t > 1.5 ? 0.05 : t > 1.0 ? 0.1 : 0.5;
    }
    /* calculateSNR :572-601 */
    double snr = 0.0;
    { double pv2 = fabs(corr[pidx]), ns = 0; int64_t nc = 0;
      for (int64_t i = 0; i < nl; i++) if (llabs(i - pidx) > 5) { ns += corr[i] * corr[i]; nc++; }
      if (nc > 0) { double nlv = sqrt(ns / (double)nc); snr = nlv < 1e-10 ? INFINITY : 20.0 * log10(pv2 / nlv); } }
    /* calculateSharpness :611-619 */
    double sharp = 0.0;
    if (nl >= 3 && pidx > 0 && pidx < nl - 1) sharp = -(corr[pidx + 1] - 2 * corr[pidx] + corr[pidx - 1]);
    /* findSecondPeak :622-636 */
    double sp = 0.0;
    for (int64_t i = 0; i < nl; i++) if (i != pidx && fabs(corr[i]) > fabs(sp)) sp = corr[i];
    /* calculatePeakToSidelobe :639-661 */
    double psl; { double pv2 = fabs(corr[pidx]), ms = 0;
      for (int64_t i = 0; i < nl; i++) if (llabs(i - pidx) > 10 && fabs(corr[i]) > ms) ms = fabs(corr[i]);
      psl = ms < 1e-10 ? INFINITY : 20.0 * log10(pv2 / ms); }
    int64_t s1, e1, s2, e2; overlap_region(na, nb, plag, &s1, &e1, &s2, &e2);
    int64_t ovl = (e1 - s1) < (e2 - s2) ? (e1 - s1) : (e2 - s2);
    met[0] = pk; met[1] = (double)plag; met[2] = (double)pidx; met[3] = pv; met[4] = snr;
    met[5] = sharp; met[6] = sp; met[7] = psl; met[8] = (double)ovl; met[9] = (double)nl;
    return 0;
}

/* ------------------------------------------------------------------ */
/* DTW: algorithms/stats/dtw.go:55-217 + distance.go:29-36               */
/* cost (nullable) = costMatrix[1:], nq rows x (nr+1) cols               */
/* path arrays sized >= nq+nr; points in forward order                   */
/* ------------------------------------------------------------------ */
int or_dtw(const double* q, int64_t nq, const double* r, int64_t nr, int dim, int band,
           double* cost, int32_t* pq, int32_t* pr, double* pc, int64_t* plen, double* dist) {
    if (nq == 0 || nr == 0) return -1;                            /* "empty sequences provided" */
    int64_t C = nr + 1;
    double* M = malloc(sizeof(double) * (size_t)(nq + 1) * C);
    if (!M) return -3;
    for (int64_t i = 0; i < (nq + 1) * C; i++) M[i] = INFINITY;
    M[0] = 0;
    for (int64_t i = 1; i <= nq; i++)                              /* fillCostMatrix :106-135 */
        for (int64_t j = 1; j <= nr; j++) {
            if (band > 0 && fabs((double)(i - j)) > (double)band) continue;
            const double* a = q + (i - 1) * dim; const double* b = r + (j - 1) * dim;
            double s = 0.0;
            for (int d = 0; d < dim; d++) { double df = a[d] - b[d]; s += df * df; }
            double ld = sqrt(s);
            double mn = go_min(go_min(M[(i - 1) * C + j], M[i * C + j - 1]), M[(i - 1) * C + j - 1]);
            M[i * C + j] = ld + mn;
        }
    /* backtrack :165-188 (collected in reverse, then flipped) */
    int64_t i = nq, j = nr, P = 0;
    while (i > 0 || j > 0) {
        double c = 0.0;
        if (i > 0 && j > 0) c = M[i * C + j] - M[(i - 1) * C + j - 1];
        pq[P] = (int32_t)(i - 1); pr[P] = (int32_t)(j - 1); pc[P] = c; P++;
        if (i == 0) { j--; continue; }                            /* findPreviousStep :191-217 */
        if (j == 0) { i--; continue; }
        double cv = M[(i - 1) * C + j], ch = M[i * C + j - 1], cd = M[(i - 1) * C + j - 1];
        int mi = 0; double best = cv;
        if (ch < best) { mi = 1; best = ch; }
        if (cd < best) { mi = 2; }
        if (mi == 0) i--; else if (mi == 1) j--; else { i--; j--; }
    }
    for (int64_t k = 0; k < P / 2; k++) {
        int32_t t = pq[k]; pq[k] = pq[P - 1 - k]; pq[P - 1 - k] = t;
        t = pr[k]; pr[k] = pr[P - 1 - k]; pr[P - 1 - k] = t;
        double u = pc[k]; pc[k] = pc[P - 1 - k]; pc[P - 1 - k] = u;
    }
    *plen = P;
    *dist = M[nq * C + nr] / (double)P;
    if (cost) memcpy(cost, M + C, sizeof(double) * (size_t)nq * C);
    free(M);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Alignment scoring epilogues: algorithms/stats/alignment.go            */
/* ------------------------------------------------------------------ */
static double cost_consistency(const double* pc, int64_t P) {     /* :466-512 */
    if (P <= 1) return 0.0;
    int64_t w = P / 4 < 5 ? P / 4 : 5; if (w < 2) w = 2;
    double* sm = malloc(sizeof(double) * P);
    for (int64_t i = 0; i < P; i++) {
        double s = 0; int64_t c = 0;
        int64_t lo = i - w / 2 < 0 ? 0 : i - w / 2, hi = i + w / 2 > P - 1 ? P - 1 : i + w / 2;
        for (int64_t j = lo; j <= hi; j++) { s += pc[j]; c++; }
        sm[i] = s / (double)c;
    }
    double mean = 0; for (int64_t i = 0; i < P; i++) mean += sm[i];
    mean /= (double)P;
    if (mean <= 1e-10) { free(sm); return 1.0; }
    double var = 0; for (int64_t i = 0; i < P; i++) { double d = sm[i] - mean; var += d * d; }
    var /= (double)P;
    free(sm);
    return 1.0 / (1.0 + sqrt(var) / mean);
}
static double diagonal_bias(const int32_t* pq, const int32_t* pr, int64_t P) {   /* :514-540 */
    if (P <= 1) return 1.0;
    int64_t dg = 0;
    for (int64_t i = 1; i < P; i++) if (pq[i] - pq[i - 1] > 0 && pr[i] - pr[i - 1] > 0) dg++;
    double ratio = (double)dg / (double)(P - 1);
    return 1.0 / (1.0 + exp(-10.0 * (ratio - 0.3)));
}
static double path_smoothness(const int32_t* pq, const int32_t* pr, int64_t P) { /* :569-603 */
    if (P <= 2) return 1.0;
    int64_t ch = 0; int pdq = 0, pdr = 0;
    for (int64_t i = 1; i < P; i++) {
        int dq = pq[i] - pq[i - 1], dr = pr[i] - pr[i - 1];
        if (i > 1 && (dq != pdq || dr != pdr)) ch++;
        pdq = dq; pdr = dr;
    }
    double r = 1.0 - (double)ch / (double)(P - 1);
    return r > 0 ? r : 0.0;
}
static double dtw_quality(const int32_t* pq, const int32_t* pr, const double* pc, int64_t P, int64_t nq, int64_t nr) {
    if (P == 0) return 0.0;                                       /* calculateDTWQuality :543-566 */
    double ex = (double)(nq > nr ? nq : nr);
    double eff = ex / (double)P; if (eff > 1.0) eff = 1.0;
    double q = 0.3 * eff + 0.3 * diagonal_bias(pq, pr, P) + 0.2 * path_smoothness(pq, pr, P) + 0.2 * cost_consistency(pc, P);
    return go_min(1.0, go_max(0.0, q));
}

/* out = {similarity, confidence, offset(int), offset_seconds, quality, stability} : alignWithDTW :129-148 */
void or_align_dtw_metrics(const int32_t* pq, const int32_t* pr, const double* pc, int64_t P,
                          int64_t nq, int64_t nr, double dist, int sr, double* out) {
    double avg = (double)(nq + nr) / 2.0;
    /* calculateSimilarityFromDTW :380-406 */
    double sim = 0.0;
    if (avg != 0) {
        double ds = 1.0 / (1.0 + dist / avg);
        double pq_ = dtw_quality(pq, pr, pc, P, nq, nr);
        double mc = 0; if (P > 0) { for (int64_t i = 0; i < P; i++) mc += pc[i]; mc /= (double)P; }
        sim = go_min(1.0, go_max(0.0, 0.5 * ds + 0.3 * pq_ + 0.2 * (1.0 / (1.0 + mc))));
    }
    /* calculateDTWConfidence :420-463 */
    double conf = 0.0;
    if (P > 0 && avg != 0) {
        double c1 = exp(-(dist / avg) * 2.0);
        double ex = (double)(nq > nr ? nq : nr);
        double pe = ex / (double)P; pe = go_min(1.0, pe);
        conf = go_min(1.0, go_max(0.0, 0.4 * c1 + 0.25 * pe + 0.2 * cost_consistency(pc, P) + 0.15 * diagonal_bias(pq, pr, P)));
    }
    /* calculateAverageOffset :530-541 */
    int64_t off = 0;
    if (P > 0) { int64_t s = 0; for (int64_t i = 0; i < P; i++) s += pr[i] - pq[i]; off = s / P; }
    /* calculatePathStability :620-643 */
    double stab = 0.0;
    if (P >= 3) {
        int64_t ch = 0; int pd0 = 0, pd1 = 0;
        for (int64_t i = 1; i < P; i++) {
            int d0 = pq[i] - pq[i - 1], d1 = pr[i] - pr[i - 1];
            if (i > 1 && (d0 != pd0 || d1 != pd1)) ch++;
            pd0 = d0; pd1 = d1;
        }
        stab = go_max(0.0, 1.0 - (double)ch / (double)(P - 1));
    }
    out[0] = sim; out[1] = conf; out[2] = (double)off; out[3] = (double)off / (double)sr;
    out[4] = dtw_quality(pq, pr, pc, P, nq, nr); out[5] = stab;
}

/* metrics from or_ncc -> out = {offset, offset_seconds, similarity, confidence, quality, noise_level}
 * alignWithCrossCorrelation :151-181, calculateCorrelationConfidence :183-243,
 * calculateCorrelationQuality :245-305 */
void or_align_xcorr_metrics(const double* m, int hop, int sr, int max_lag, double* out) {
    double pk = m[0]; int64_t plag = (int64_t)m[1];
    double snr = m[4], sharp = m[5], sp = m[6], psl = m[7];
    int64_t off = plag * hop;
    double sim = go_min(1.0, go_max(0.0, fabs(pk)));
    double pm = fabs(pk), conf = 0.0, qual = 0.0;
    if (pm >= 0.1) {
        double ps = pm; if (pm >= 0.6) ps = pm + (pm - 0.6) * 0.5;
        double ss = go_min(0.9, sharp * 8.0);
        double sl = 0.0; if (psl > 0 && !isinf(psl)) sl = go_min(0.8, psl / 15.0);
        double sn = 0.0; if (snr > 0) sn = go_min(0.7, snr / 25.0);
        double pen = 0.0; if (sp != 0 && pm > 0) { double r = fabs(sp) / pm; if (r > 0.7) pen = (r - 0.7) * 0.25; }
        double bonus = pm >= 0.75 ? 0.12 : pm >= 0.6 ? 0.08 : 0.0;
        double c = 0.55 * ps + 0.22 * ss + 0.12 * sl + 0.06 * sn + 0.05 * 0.15 + bonus - pen;
        conf = go_min(0.95, go_max(0.0, c));
    }
    if (pm >= 0.08) {
        double pq = pm; if (pm >= 0.6) pq = pm + (pm - 0.6) * 0.4;
        double sq = go_min(0.85, sharp * 5.0);
        double slq = 0.0; if (psl > 0 && !isinf(psl)) slq = go_min(0.7, psl / 20.0);
        double snq = 0.0; if (snr > 0) snq = go_min(0.6, snr / 30.0);
        double lp = 0.0;
        if (max_lag > 0 && plag < 0) { double nr_ = fabs((double)plag) / (double)max_lag; if (nr_ > 0.90) lp = (nr_ - 0.90) * 4.0; }
        double qb = pm >= 0.7 ? 0.10 : pm >= 0.55 ? 0.06 : 0.0;
        double q = 0.50 * pq + 0.25 * sq + 0.15 * slq + 0.10 * snq + qb - lp;
        qual = go_min(1.0, go_max(0.0, q));
    }
    out[0] = (double)off; out[1] = (double)off / (double)sr; out[2] = sim; out[3] = conf;
    out[4] = qual; out[5] = 1.0 - snr / 20.0;
}

/* ======================================================== LPC / formants ====
 * FormantAnalyzer.AnalyzeFormants (algorithms/speech/format.go:85-124) with
 * LPCAnalyzer.Analyze (algorithms/speech/lpc.go:44-82).  The autocorrelation
 * is AutoCorrelation(1024) = CrossCorrelation{maxLag 1024, useFFT, threshold
 * 1000}.Compute(x, x) (stats/correlation.go:103-114, 131-200, 231-297): the
 * z-scored frame, nextPowerOf2(2n-1)-point recursive radix-2 FFT (:726-774),
 * |X|^2 via Go's complex multiply, conj-FFT-conj inverse.  R = Correlations[:p+1]
 * i.e. lags -L .. -L+p (F11). */

static void go_rec_fft(double* re, double* im, int n) {           /* correlation.go:727-755 */
  if (n <= 1) return;
  const int h = n / 2;
  double* er = (double*)malloc(sizeof(double) * 4 * h);
  double *ei = er + h, *odr = er + 2 * h, *odi = er + 3 * h;
  for (int i = 0; i < h; i++) { er[i] = re[2 * i]; ei[i] = im[2 * i]; odr[i] = re[2 * i + 1]; odi[i] = im[2 * i + 1]; }
  go_rec_fft(er, ei, h);
  go_rec_fft(odr, odi, h);
  for (int i = 0; i < h; i++) {
    const double th = -2.0 * M_PI * (double)i / (double)n;
    const double c = cos(th), s = sin(th);                        /* cmplx.Exp(0 + i*th) = (cos, sin) */
    const double tr = c * odr[i] - s * odi[i], ti = c * odi[i] + s * odr[i];
    re[i] = er[i] + tr; im[i] = ei[i] + ti;
    re[i + h] = er[i] - tr; im[i + h] = ei[i] - ti;
  }
  free(er);
}

/* Correlations of AutoCorrelation(maxLag).Compute on the FFT path; fills corr[0..2L] */
int or_autocorr_fft(const double* x, int n, int max_lag, double* corr) {
  double mean = 0.0;                                               /* normalize :464-501 */
  for (int i = 0; i < n; i++) mean += x[i];
  mean /= (double)n;
  double var = 0.0;
  for (int i = 0; i < n; i++) { const double d = x[i] - mean; var += d * d; }
  var /= (double)n;
  const double sd = sqrt(var);
  int N = 1;
  while (N < 2 * n - 1) N <<= 1;                                   /* nextPowerOf2 */
  double* re = (double*)calloc((size_t)4 * N, sizeof(double));
  double *im = re + N, *re2 = re + 2 * N, *im2 = re + 3 * N;
  for (int i = 0; i < n; i++) re[i] = sd < 1e-10 ? x[i] - mean : (x[i] - mean) / sd;
  memcpy(re2, re, sizeof(double) * N);
  go_rec_fft(re, im, N);
  go_rec_fft(re2, im2, N);
  for (int i = 0; i < N; i++) {                                    /* fft1 * conj(fft2), then conj for ifft */
    const double a = re[i], b = im[i], c = re2[i], d = -im2[i];
    re[i] = a * c - b * d;
    im[i] = -(a * d + b * c);
  }
  go_rec_fft(re, im, N);
  int L = max_lag < n - 1 ? max_lag : n - 1;
  if (L < 0) L = 0;
  for (int k = 0; k <= 2 * L; k++) {
    const int lag = k - L;
    const int idx = lag >= 0 ? lag : N + lag;
    corr[k] = re[idx] / (double)N;                                 /* real(conj(y) / N) */
  }
  free(re);
  return L;
}

static void go_envelope(const double* a, int p, int nfft, double* env) {   /* lpc.go:233-265 */
  for (int k = 0; k <= nfft / 2; k++) {
    const double w = 2.0 * M_PI * (double)k / (double)nfft;
    double rp = 1.0, ip = 0.0;
    for (int i = 1; i <= p; i++) {
      const double ang = -(double)i * w;
      rp += a[i] * cos(ang);
      ip += a[i] * sin(ang);
    }
    const double m = sqrt(rp * rp + ip * ip);
    env[k] = m > 0 ? 1.0 / m : 0.0;
  }
}

/* rec[24]: status, n_formants, freq[4], bw[4], amp[4], conf[4], vtl, quality, gain,
 * residual_energy, stable, order.  status: 0 ok, 1 too short, 2 LPC too short,
 * 3 zero energy, 4 prediction error became zero. */
int or_formant_frame(const double* sig, int64_t len, int sr, double* rec, double* coeffs, double* refl) {
  const int W = sr >= 16000 ? 2048 : 1024;                         /* NewFormantAnalyzer format.go:48-69 */
  const int p = 12 + sr / 1000;
  memset(rec, 0, sizeof(double) * 24);
  rec[23] = p;
  if (len < W) { rec[0] = 1; return 1; }
  double* x = (double*)malloc(sizeof(double) * W);                 /* preprocessSignal :127-146 */
  x[0] = sig[0];
  for (int i = 1; i < W; i++) x[i] = sig[i] - 0.97 * sig[i - 1];
  for (int i = 0; i < W; i++) x[i] *= 0.54 - 0.46 * cos(2.0 * M_PI * (double)i / (double)(W - 1));
  if (W < 2 * p) { free(x); rec[0] = 2; return 2; }                /* lpc.go:45-47 */
  double* corr = (double*)malloc(sizeof(double) * (2 * 1024 + 1));
  or_autocorr_fft(x, W, 1024, corr);
  double R[128];
  for (int i = 0; i <= p; i++) R[i] = corr[i];                     /* F11 */
  free(corr);
  free(x);
  if (R[0] == 0) { rec[0] = 3; return 3; }
  double a[128] = {0}, k[128] = {0};                               /* levinsonDurbin lpc.go:85-135 */
  double E = R[0];
  a[0] = 1.0;
  for (int i = 1; i <= p; i++) {
    double num = R[i];
    for (int j = 1; j < i; j++) num -= a[j] * R[i - j];
    if (E == 0) { rec[0] = 4; return 4; }
    k[i - 1] = num / E;
    a[i] = k[i - 1];
    for (int j = 1; j < i; j++) a[j] = a[j] - k[i - 1] * a[i - j];   /* in place, as written */
    E *= (1 - k[i - 1] * k[i - 1]);
    if (E <= 0) break;
  }
  const double gain = sqrt(E);
  int stable = 1;                                                  /* checkStability :155-166 */
  for (int i = 1; i <= p; i++) if (fabs(a[i]) >= 1.0) stable = 0;
  if (coeffs) memcpy(coeffs, a, sizeof(double) * (p + 1));
  if (refl) memcpy(refl, k, sizeof(double) * p);

  double env[513];                                                 /* findFormantsFromLPC format.go:148-190 */
  go_envelope(a, p, 1024, env);
  const double res = (double)sr / 1024.0;
  double maxv = 0.0;
  for (int i = 0; i < 513; i++) if (env[i] > maxv) maxv = env[i];
  double fq[513], bw[513], am[513], cf[513];
  int nf = 0;
  if (maxv != 0) {
    for (int i = 1; i < 512; i++) {                                /* findSpectralPeaks :193-222 */
      if (!(env[i] > env[i - 1] && env[i] > env[i + 1])) continue;
      if (!(env[i] / maxv > 0.1)) continue;
      const double f = (double)i * res;
      if (f < 50.0 || f > (double)sr / 2.0) continue;
      const double hh = env[i] / 2.0;                              /* estimateFormantBandwidth :225-262 */
      int li = i, ri = i;
      for (int t = i - 1; t >= 0; t--) if (env[t] <= hh) { li = t; break; }
      for (int t = i + 1; t < 513; t++) if (env[t] <= hh) { ri = t; break; }
      double b = (double)(ri - li) * res;
      if (b < 50.0) b = 50.0; else if (b > 500.0) b = 500.0;
      double c = 1.0;                                              /* calculateFormantConfidence :265-289 */
      if (f >= 300 && f <= 3500) c *= 1.0;
      else if (f >= 100 && f <= 5000) c *= 0.7;
      else c *= 0.3;
      c *= go_min(env[i], 1.0);
      if (b >= 50 && b <= 300) c *= 1.0;
      else if (b >= 30 && b <= 500) c *= 0.8;
      else c *= 0.5;
      c = go_max(0.0, go_min(1.0, c));
      fq[nf] = f; bw[nf] = b; am[nf] = env[i]; cf[nf] = c; nf++;
    }
  }
  if (nf > 4) nf = 4;                                              /* already ascending; maxFormants */
  double vf[4], vb[4], va[4], vc[4];                               /* validateFormants :292-315 */
  int nv = 0;
  for (int i = 0; i < nf; i++) {
    if (fq[i] < 50.0 || fq[i] > (double)sr / 2.0) continue;
    if (cf[i] < 0.2) continue;
    if (bw[i] <= 0 || bw[i] > 1000) continue;
    vf[nv] = fq[i]; vb[nv] = bw[i]; va[nv] = am[i]; vc[nv] = cf[i]; nv++;
  }
  if (nv > 1) {                                                    /* ensureProperSpacing :318-343 */
    int ns = 1;
    for (int i = 1; i < nv; i++) {
      if (vf[i] - vf[ns - 1] >= 200.0) { vf[ns] = vf[i]; vb[ns] = vb[i]; va[ns] = va[i]; vc[ns] = vc[i]; ns++; }
      else if (vc[i] > vc[ns - 1]) { vf[ns - 1] = vf[i]; vb[ns - 1] = vb[i]; va[ns - 1] = va[i]; vc[ns - 1] = vc[i]; }
    }
    nv = ns;
  }
  double vtl = 17.5;                                               /* estimateVocalTractLength :346-377 */
  if (nv > 0) {
    double tot = 0.0;
    int cnt = 0;
    for (int i = 0; i < nv; i++) {
      if (vf[i] > 0 && vc[i] > 0.3) {
        const double v = (2.0 * (i + 1) - 1.0) * 35000.0 / (4.0 * vf[i]);
        if (v >= 10.0 && v <= 25.0) { tot += v; cnt++; }
      }
    }
    if (cnt > 0) vtl = tot / (double)cnt;
  }
  double quality = 0.0;                                            /* calculateAnalysisQuality :380-411 */
  if (nv > 0) {
    const double q1 = go_min((double)nv / 3.0, 1.0);
    double ac = 0.0;
    for (int i = 0; i < nv; i++) ac += vc[i];
    ac /= (double)nv;
    double lq = 1.0;
    if (E > 0) lq = go_max(0.0, 1.0 - go_min(1.0, E));
    quality = (q1 + ac + lq + (stable ? 1.0 : 0.0)) / 4.0;
  }
  rec[0] = 0; rec[1] = nv;
  for (int i = 0; i < nv; i++) { rec[2 + i] = vf[i]; rec[6 + i] = vb[i]; rec[10 + i] = va[i]; rec[14 + i] = vc[i]; }
  rec[18] = vtl; rec[19] = quality; rec[20] = gain; rec[21] = E; rec[22] = stable;
  return 0;
}

/* AnalyzeMultipleFrames (format.go:427-449): frames i = 0, hop, ... while i < n - frame_size;
 * every attempted frame gets a record (status != 0 frames are the ones Go skips). */
int64_t or_formant_frames(const double* sig, int64_t n, int sr, int frame_size, int hop, double* recs,
                          double* coeffs, double* refl) {
  const int W = sr >= 16000 ? 2048 : 1024;
  const int p = 12 + sr / 1000;
  if (frame_size <= 0) frame_size = W;
  if (hop <= 0) hop = frame_size / 2;
  int64_t f = 0;
  for (int64_t i = 0; i < n - frame_size; i += hop, f++)
    or_formant_frame(sig + i, frame_size, sr, recs + 24 * f, coeffs ? coeffs + (p + 1) * f : NULL,
                     refl ? refl + p * f : NULL);
  return f;
}

/* SpectralContrast(sample_rate, num_bands).Compute per row (algorithms/spectral/spectral_contrast.go:
 * 26-137, initializeBands :140-185): log-spaced band edges from 200 Hz to Nyquist, per band |X|^2,
 * insertion sort ascending, mean of the bottom and top 20 % (at least one value each) in sorted
 * order, 10 log10(peak / valley) (valley <= 0 -> 1e-10, peak <= 0 -> 0).  out is F x num_bands. */
static int64_t or_go_int(double x) {   /* Go int(float64) on amd64: NaN / out of range -> MinInt64 */
    if (!(x >= -9.2233720368547758e18 && x < 9.2233720368547758e18)) return INT64_MIN;
    return (int64_t)x;
}
void or_spectral_contrast(const double* mag, int64_t F, int K, int sr, int nb, double* out) {
    int* edges = malloc(sizeof(int) * (nb + 1));
    const double nyq = (double)sr / 2.0;
    double maxf = nyq;
    if (maxf <= 200.0) maxf = 400.0;
    const double lmin = log10(200.0), lmax = log10(maxf), step = (lmax - lmin) / (double)nb;
    for (int i = 0; i <= nb; i++) {
        int64_t b = or_go_int(pow(10.0, lmin + (double)i * step) * (double)(K - 1) / nyq);
        if (b >= K) b = K - 1;
        if (b < 0) b = 0;
        edges[i] = (int)b;
    }
    for (int i = 1; i <= nb; i++) if (edges[i] <= edges[i - 1]) edges[i] = edges[i - 1] + 1;
    double* buf = malloc(sizeof(double) * (K > 0 ? K : 1));
    for (int64_t t = 0; t < F; t++) {
        const double* s = mag + t * K;
        for (int b = 0; b < nb; b++) {
            const int st = edges[b];
            int en = edges[b + 1];
            if (en > K) en = K;
            double c = 0.0;
            if (st < en) {
                const int L = en - st;
                for (int i = 0; i < L; i++) buf[i] = s[st + i] * s[st + i];
                for (int i = 1; i < L; i++) {                 /* insertion sort, :83-92 */
                    const double key = buf[i];
                    int j = i - 1;
                    while (j >= 0 && buf[j] > key) { buf[j + 1] = buf[j]; j--; }
                    buf[j + 1] = key;
                }
                int vc = (int)(0.2 * (double)L), pc = (int)(0.2 * (double)L);
                if (vc == 0) vc = 1;
                if (pc == 0) pc = 1;
                double valley = 0.0, peak = 0.0;
                for (int i = 0; i < vc; i++) valley += buf[i];
                valley /= (double)vc;
                for (int i = L - pc; i < L; i++) peak += buf[i];
                peak /= (double)pc;
                if (valley <= 0) valley = 1e-10;
                c = peak <= 0 ? 0.0 : 10.0 * log10(peak / valley);
            }
            out[t * nb + b] = c;
        }
    }
    free(buf);
    free(edges);
}
