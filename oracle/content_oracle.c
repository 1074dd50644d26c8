/*
 * content_oracle.c -- CPU fp64 restatement of ContentDetector.DetectFromAudio
 * (fingerprint/content_detector.go:72-467).  TEST INFRASTRUCTURE ONLY (see sonar_oracle.h).
 * Follows the Go loops literally: sequential sums, the direct O(N^2) DFT with libm cos/sin
 * (Go's math.Cos/Sin agree to an ulp or two: parity unpinned at that level), and the
 * classification scores visited in the order music, news, talk, sports (Go visits a map in
 * random order; ties between equal best scores are therefore not reproducible in Go).
 */
#include "sonar_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* out[10]: AcousticFeatures in struct order; *ct: 0 music, 1 news, 2 sports, 3 talk, 5 unknown */
int or_detect_from_audio(const double* pcm, int64_t n, int sr, double thr, double* out, int* ct) {
    memset(out, 0, 10 * sizeof(double));
    *ct = 5;
    if (n == 0) return 0;
    if (sr < 10) return -1;
    double zcr = 0, cent = 0, ev = 0, sil = 0, hr = 0, lo = 0, hi = 0, dr = 0, stab = 0;
    if (n > 1) {                                                        /* :220-233 */
        int64_t c = 0;
        for (int64_t i = 1; i < n; i++)
            if ((pcm[i - 1] >= 0 && pcm[i] < 0) || (pcm[i - 1] < 0 && pcm[i] >= 0)) c++;
        zcr = (double)c / (double)(n - 1);
    }
    const int N = n < 2048 ? (int)n : 2048, K = N / 2 + 1;             /* :128-133 */
    double* spec = malloc(sizeof(double) * K);
    for (int k = 0; k < K; k++) {                                       /* computeBasicSpectrum :452-467 */
        double re = 0, im = 0;
        for (int t = 0; t < N; t++) {
            const double ang = -2 * M_PI * (double)k * (double)t / (double)N;
            re += pcm[t] * cos(ang);
            im += pcm[t] * sin(ang);
        }
        spec[k] = sqrt(re * re + im * im);
    }
    {                                                                   /* :236-252 */
        double ws = 0, ms = 0;
        for (int i = 0; i < K; i++) {
            const double f = (double)i * (double)sr / (double)(K * 2);
            ws += f * spec[i];
            ms += spec[i];
        }
        cent = ms == 0 ? 0 : ws / ms;
    }
    if (n >= 2048) {                                                    /* :255-290 */
        int64_t m = 0;
        double mean = 0;
        for (int64_t i = 0; i < n - 1024; i += 512) {
            double e = 0;
            for (int64_t j = 0; j < 1024 && i + j < n; j++) e += pcm[i + j] * pcm[i + j];
            mean += e / 1024.0;
            m++;
        }
        if (m > 1) {
            mean /= (double)m;
            double var = 0;
            for (int64_t i = 0; i < n - 1024; i += 512) {
                double e = 0;
                for (int64_t j = 0; j < 1024 && i + j < n; j++) e += pcm[i + j] * pcm[i + j];
                const double d = e / 1024.0 - mean;
                var += d * d;
            }
            ev = var / (double)m;
        }
    }
    {                                                                   /* :293-317 */
        int64_t s = 0, t = 0;
        for (int64_t i = 0; i < n - 1024; i += 512) {
            double r = 0;
            for (int64_t j = 0; j < 1024 && i + j < n; j++) r += pcm[i + j] * pcm[i + j];
            r = sqrt(r / 1024.0);
            if (r < 0.01) s++;
            t++;
        }
        sil = t ? (double)s / (double)t : 0;
    }
    {                                                                   /* :320-343 */
        double mx = 0, mn = INFINITY;
        for (int64_t i = 0; i < n; i++) {
            const double a = fabs(pcm[i]);
            if (a > mx) mx = a;
            if (a < mn && a > 1e-10) mn = a;
        }
        dr = (mn == 0 || isinf(mn)) ? 0 : 20 * log10(mx / mn);
    }
    {                                                                   /* :346-369 */
        const int sp = K / 4;
        double l = 0, h = 0;
        for (int i = 0; i < sp && i < K; i++) l += spec[i] * spec[i];
        for (int i = sp; i < K; i++) h += spec[i] * spec[i];
        if (l + h != 0) { lo = l / (l + h); hi = h / (l + h); }
    }
    if (K >= 10) {                                                      /* :372-401 */
        int* pk = malloc(sizeof(int) * K);
        int np = 0;
        for (int i = 2; i < K - 2; i++)
            if (spec[i] > spec[i - 1] && spec[i] > spec[i + 1] && spec[i] > spec[i - 2] && spec[i] > spec[i + 2])
                pk[np++] = i;
        if (np >= 2) {
            int h = 0;
            for (int q = 1; q < np; q++) {
                const double r = (double)pk[q] / (double)pk[0];
                if (fabs(r - round(r)) < 0.1) h++;
            }
            hr = (double)h / (double)(np - 1);
        }
        free(pk);
    }
    {                                                                   /* :404-447 */
        const int64_t fs = sr / 10;
        if (n >= fs * 3) {
            int64_t m = 0;
            for (int64_t i = 0; i < n - fs; i += fs) m++;
            if (m > 1) {
                double* e = malloc(sizeof(double) * m);
                int64_t q = 0;
                for (int64_t i = 0; i < n - fs; i += fs) {
                    double s = 0;
                    for (int64_t j = 0; j < fs && i + j < n; j++) s += pcm[i + j] * pcm[i + j];
                    e[q++] = s;
                }
                double mean = 0;
                for (int64_t i = 0; i < m; i++) mean += e[i];
                mean /= (double)m;
                if (mean != 0) {
                    double var = 0;
                    for (int64_t i = 0; i < m; i++) var += (e[i] - mean) * (e[i] - mean);
                    var /= (double)m;
                    const double cv = sqrt(var) / mean;
                    stab = 1 - cv > 0 ? 1 - cv : 0;
                }
                free(e);
            }
        }
    }
    free(spec);
    /* classifyFromFeatures :153-217 */
    double music = 0, speech = 0, sports = 0;
    if (zcr < 0.1) music += 2.0;
    if (hr > 0.3) music += 2.0;
    if (stab > 0.5) music += 1.0;
    if (dr > 20) music += 1.0;
    if (zcr > 0.05 && zcr < 0.3) speech += 2.0;
    if (cent > 800 && cent < 3000) speech += 2.0;
    if (hr < 0.2) speech += 1.0;
    if (sil > 0.1 && sil < 0.4) speech += 1.0;
    if (ev > 0.3) sports += 2.0;
    if (dr > 30) sports += 1.5;
    if (stab < 0.4) sports += 1.0;
    const int types[4] = {0, 1, 3, 2};
    const double sc[4] = {music, speech, speech * 0.9, sports};
    double best = thr;
    for (int i = 0; i < 4; i++)
        if (sc[i] > best) { best = sc[i]; *ct = types[i]; }
    const double f[10] = {zcr, cent, ev, sil, hr, lo, hi, dr, stab, best / 6.0};
    memcpy(out, f, sizeof(f));
    return 0;
}
