/*
 * compare_oracle.c -- CPU fp64 restatement of FingerprintComparator
 * (fingerprint/comparison.go).  TEST INFRASTRUCTURE ONLY (see sonar_oracle.h):
 * tests/, smoke() and bench.py's cpu_baseline use it as the checker.
 *
 * Follows the Go code call by call: every Compare rebuilds the statistics from the
 * full feature arrays (extractMFCCStatistics, calculateMeanChromaVector,
 * compareSequenceStats), as the reference does.  gonum v0.16.0 (go.mod:7) is absent
 * from /root/reference; its published algorithms are restated: stat.Mean = floats.Sum/n
 * (summed sequentially here; gonum's SSE2 kernel pairs the terms, so the two agree to
 * rounding), stat.Variance = corrected two-pass (sum of squared deviations minus the
 * squared sum of deviations / n, over n - 1), stat.Correlation = the same corrected
 * co-moments, floats.Norm(x, 2) = f64.L2NormUnitary (scaled sum of squares).
 * Parity to Go is UNPINNED (no reference tests; gonum not available).
 */
#include "sonar_oracle.h"
#include "../include/sonar_gpu.h"   /* struct layouts only (sonar_fp_features, sonar_similarity, ...) */

#include <math.h>
#include <stdlib.h>
#include <string.h>

static double cmin(double x, double y) {   /* math.Min */
    if (isinf(x) && x < 0) return x;
    if (isinf(y) && y < 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? x : y;
    return x < y ? x : y;
}
static double cmax(double x, double y) {   /* math.Max */
    if (isinf(x) && x > 0) return x;
    if (isinf(y) && y > 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? y : x;
    return x > y ? x : y;
}

static double g_mean(const double* x, int64_t n, int64_t stride) {   /* stat.Mean(x, nil) */
    double s = 0.0;
    for (int64_t i = 0; i < n; i++) s += x[i * stride];
    return s / (double)n;
}
static double g_variance(const double* x, int64_t n, int64_t stride) {   /* stat.Variance(x, nil) */
    const double mu = g_mean(x, n, stride);
    double ss = 0.0, comp = 0.0;
    for (int64_t i = 0; i < n; i++) {
        const double d = x[i * stride] - mu;
        ss += d * d;
        comp += d;
    }
    return (ss - comp * comp / (double)n) / (double)(n - 1);
}
static double g_norm2(const double* x, int n) {   /* floats.Norm(x, 2) */
    double scale = 0.0, ss = 1.0;
    for (int i = 0; i < n; i++) {
        if (x[i] == 0) continue;
        const double a = fabs(x[i]);
        if (isnan(a)) return NAN;
        if (scale < a) {
            const double s = scale / a;
            ss = 1 + ss * s * s;
            scale = a;
        } else {
            const double s = a / scale;
            ss += s * s;
        }
    }
    if (isinf(scale)) return INFINITY;
    return scale * sqrt(ss);
}
static double g_correlation(const double* x, const double* y, int64_t n) {   /* stat.Correlation */
    const double xu = g_mean(x, n, 1), yu = g_mean(y, n, 1);
    double sxx = 0, syy = 0, sxy = 0, xc = 0, yc = 0;
    for (int64_t i = 0; i < n; i++) {
        const double xd = x[i] - xu, yd = y[i] - yu;
        sxx += xd * xd;
        syy += yd * yd;
        sxy += xd * yd;
        xc += xd;
        yc += yd;
    }
    sxx -= xc * xc / (double)n;
    syy -= yc * yc / (double)n;
    sxy -= xc * yc / (double)n;
    return sxy / sqrt(sxx * syy);
}

/* cosineSimilarity (comparison.go:858-873) */
static double cosine(const double* a, int na, const double* b, int nb) {
    if (na != nb || na == 0) return 0.0;
    double dot = 0.0;
    for (int i = 0; i < na; i++) dot += a[i] * b[i];
    const double n1 = g_norm2(a, na), n2 = g_norm2(b, nb);
    if (n1 == 0 || n2 == 0) return 0.0;
    return dot / (n1 * n2);
}

/* compareSequenceStats (:827-842) */
static double seq_stats(const double* s1, int64_t n1, const double* s2, int64_t n2) {
    if (n1 == 0 || n2 == 0) return 0.0;
    const double f1[2] = {g_mean(s1, n1, 1), sqrt(g_variance(s1, n1, 1))};
    const double f2[2] = {g_mean(s2, n2, 1), sqrt(g_variance(s2, n2, 1))};
    return cosine(f1, 2, f2, 2);
}

/* compareScalarFeatures (:844-856) */
static double scalar_sim(double v1, double v2) {
    if (v1 == 0 && v2 == 0) return 1.0;
    const double mx = cmax(fabs(v1), fabs(v2));
    if (mx == 0) return 1.0;
    return cmax(0.0, 1.0 - fabs(v1 - v2) / mx);
}

static double list_mean(const double* v, int n) { return g_mean(v, n, 1); }

/* extractMFCCStatistics (:774-800): [means..., stds...]; returns length (0 = nil) */
static int mfcc_stats(const sonar_fp_features* f, double* out) {
    if (f->mfcc_frames == 0 || f->mfcc_coeffs == 0) return 0;
    const int C = f->mfcc_coeffs;
    for (int c = 0; c < C; c++) {
        out[c] = g_mean(f->mfcc + c, f->mfcc_frames, C);
        out[c + C] = sqrt(g_variance(f->mfcc + c, f->mfcc_frames, C));
    }
    return 2 * C;
}

/* calculateMeanChromaVector (:802-825) */
static int chroma_means(const sonar_fp_features* f, double* out) {
    if (f->chroma_frames == 0 || f->chroma_bins == 0) return 0;
    for (int b = 0; b < f->chroma_bins; b++) out[b] = g_mean(f->chroma + b, f->chroma_frames, f->chroma_bins);
    return f->chroma_bins;
}

static const double W_NEWS[6] = {0.50, 0.25, 0.05, 0.15, 0.10, 0.05};
static const double W_MUSIC[6] = {0.30, 0.20, 0.25, 0.10, 0.05, 0.15};
static const double W_SPORTS[6] = {0.25, 0.20, 0.05, 0.25, 0.10, 0.05};
static const double W_DEFAULT[6] = {0.35, 0.25, 0.10, 0.20, 0.10, 0.10};

/* getEffectiveWeights (:1055-1104), by SONAR_FD_* */
static const double* weights_of(const sonar_fp_features* f) {
    if (f->present & SONAR_FEAT_WEIGHTS) return f->feature_weights;
    switch (f->content_type) {
        case SONAR_CT_NEWS: case SONAR_CT_TALK: return W_NEWS;
        case SONAR_CT_MUSIC: return W_MUSIC;
        case SONAR_CT_SPORTS: return W_SPORTS;
        default: return W_DEFAULT;
    }
}

static int64_t nrows(const sonar_fp_features* f, uint32_t bit, int64_t n) {   /* len(nil slice) = 0 */
    return (f->present & bit) ? n : 0;
}

int or_fp_compare(const sonar_fp_features* a, const sonar_fp_features* b, const sonar_compare_cfg* cfg,
                  sonar_similarity* r) {
    memset(r, 0, sizeof(*r));
    r->content_type_match = a->content_type == b->content_type;
    r->status = a->id == b->id ? 1 : 0;
    if (cfg->enable_content_filter && !r->content_type_match) {          /* :160-166 */
        r->confidence = 0.25;
        return 0;
    }
    const int feat = (a->present & SONAR_FEAT_FEATURES) && (b->present & SONAR_FEAT_FEATURES);
    double fs = 0.0;
    if (!feat) {                                                         /* :267-273 */
        if (!r->status) r->status = 2;
    } else {
        double sims[6], ws[6];
        int n = 0;
        const double* W = weights_of(a);
        const uint32_t both = a->present & b->present;
#define ADD(key, sim) do { sims[n] = (sim); ws[n] = W[key]; n++; \
        r->feature_distances[key] = 1.0 - sims[n - 1]; r->distance_mask |= 1u << (key); } while (0)
        const int64_t fa = nrows(a, SONAR_FEAT_MFCC, a->mfcc_frames), fb = nrows(b, SONAR_FEAT_MFCC, b->mfcc_frames);
        if (fa > 0 && fb > 0) {                                          /* compareMFCC :344-402 */
            double* s1 = malloc(sizeof(double) * (2 * (size_t)a->mfcc_coeffs + 1));
            double* s2 = malloc(sizeof(double) * (2 * (size_t)b->mfcc_coeffs + 1));
            const int l1 = mfcc_stats(a, s1), l2 = mfcc_stats(b, s2);
            double sim = 0.0;
            if (l1 > 0 && l2 > 0) sim = cosine(s1, l1, s2, l2);
            free(s1);
            free(s2);
            ADD(SONAR_FD_MFCC, sim);
        }
        if (both & SONAR_FEAT_SPECTRAL) {                                /* :646-671 */
            double v[3];
            int m = 0;
            if (a->n_spectral_centroid > 0 && b->n_spectral_centroid > 0)
                v[m++] = seq_stats(a->spectral_centroid, a->n_spectral_centroid, b->spectral_centroid,
                                   b->n_spectral_centroid);
            if (a->n_spectral_rolloff > 0 && b->n_spectral_rolloff > 0)
                v[m++] = seq_stats(a->spectral_rolloff, a->n_spectral_rolloff, b->spectral_rolloff,
                                   b->n_spectral_rolloff);
            if (a->n_spectral_flux > 0 && b->n_spectral_flux > 0)
                v[m++] = seq_stats(a->spectral_flux, a->n_spectral_flux, b->spectral_flux, b->n_spectral_flux);
            ADD(SONAR_FD_SPECTRAL, m ? list_mean(v, m) : 0.0);
        }
        const int64_t ca = nrows(a, SONAR_FEAT_CHROMA, a->chroma_frames), cb = nrows(b, SONAR_FEAT_CHROMA, b->chroma_frames);
        if (ca > 0 && cb > 0) {                                          /* :673-688 */
            double* m1 = malloc(sizeof(double) * ((size_t)a->chroma_bins + 1));
            double* m2 = malloc(sizeof(double) * ((size_t)b->chroma_bins + 1));
            const int l1 = chroma_means(a, m1), l2 = chroma_means(b, m2);
            const double sim = (l1 == 0 || l2 == 0) ? 0.0 : cosine(m1, l1, m2, l2);
            free(m1);
            free(m2);
            ADD(SONAR_FD_CHROMA, sim);
        }
        if (both & SONAR_FEAT_TEMPORAL) {                                /* :690-719 */
            double v[4];
            int m = 0;
            if (a->dynamic_range > 0 && b->dynamic_range > 0) v[m++] = scalar_sim(a->dynamic_range, b->dynamic_range);
            v[m++] = scalar_sim(a->silence_ratio, b->silence_ratio);
            if (a->onset_density > 0 && b->onset_density > 0) v[m++] = scalar_sim(a->onset_density, b->onset_density);
            if (a->n_rms_energy > 0 && b->n_rms_energy > 0)
                v[m++] = seq_stats(a->rms_energy, a->n_rms_energy, b->rms_energy, b->n_rms_energy);
            ADD(SONAR_FD_TEMPORAL, list_mean(v, m));
        }
        if (both & SONAR_FEAT_SPEECH) {                                  /* :721-747 */
            double v[3];
            int m = 0;
            if (a->speech_rate > 0 && b->speech_rate > 0) v[m++] = scalar_sim(a->speech_rate, b->speech_rate);
            if (a->vocal_tract_length > 0 && b->vocal_tract_length > 0)
                v[m++] = scalar_sim(a->vocal_tract_length, b->vocal_tract_length);
            if (a->n_voicing_probability > 0 && b->n_voicing_probability > 0)
                v[m++] = seq_stats(a->voicing_probability, a->n_voicing_probability, b->voicing_probability,
                                   b->n_voicing_probability);
            ADD(SONAR_FD_SPEECH, m ? list_mean(v, m) : 0.0);
        }
        if (both & SONAR_FEAT_HARMONIC) {                                /* :749-770 */
            double v[2];
            int m = 0;
            if (a->n_harmonic_ratio > 0 && b->n_harmonic_ratio > 0)
                v[m++] = seq_stats(a->harmonic_ratio, a->n_harmonic_ratio, b->harmonic_ratio, b->n_harmonic_ratio);
            if (a->n_pitch_estimate > 0 && b->n_pitch_estimate > 0)
                v[m++] = seq_stats(a->pitch_estimate, a->n_pitch_estimate, b->pitch_estimate, b->n_pitch_estimate);
            ADD(SONAR_FD_HARMONIC, m ? list_mean(v, m) : 0.0);
        }
#undef ADD
        if (n == 0) {                                                    /* :332-338 */
            if (!r->status) r->status = 2;
        } else {                                                         /* calculateWeightedMean */
            double sv = 0.0, sw = 0.0;
            for (int i = 0; i < n; i++) { sv += ws[i] * sims[i]; sw += ws[i]; }
            fs = sv / sw;
        }
    }
    r->feature_similarity = fs;
    r->overall_similarity = fs;
    int nd = 0;
    for (int k = 0; k < 6; k++) nd += (r->distance_mask >> k) & 1;
    if (cfg->enable_detailed_metrics) {                                  /* :892-936 */
        if (!feat) return -1;                                            /* Go: nil dereference panic */
        r->has_quality = 1;
        const uint32_t both = a->present & b->present;
        int avail = 0;
        const uint32_t bits[6] = {SONAR_FEAT_MFCC, SONAR_FEAT_SPECTRAL, SONAR_FEAT_CHROMA, SONAR_FEAT_TEMPORAL,
                                  SONAR_FEAT_SPEECH, SONAR_FEAT_HARMONIC};
        for (int k = 0; k < 6; k++) avail += (both & bits[k]) != 0;
        r->data_availability = (double)avail / 6.0;
        r->feature_coverage = (double)nd / 6.0;
        const double dd = fabs(a->duration_seconds - b->duration_seconds);
        const double md = cmax(a->duration_seconds, b->duration_seconds);
        r->temporal_alignment = md > 0 ? 1.0 - cmin(1.0, dd / md) : 1.0;
        if (nd == 0) r->noise_level = 0.5;                               /* estimateNoiseLevel :939-958 */
        else if (nd <= 1) r->noise_level = 0.0;
        else {
            double v[6];
            int m = 0;
            for (int k = 0; k < 6; k++)
                if (r->distance_mask & (1u << k)) v[m++] = 1.0 - r->feature_distances[k];
            r->noise_level = cmin(1.0, sqrt(g_variance(v, m, 1)));
        }
        if (!(both & SONAR_FEAT_TEMPORAL) || a->dynamic_range <= 0 || b->dynamic_range <= 0)   /* :961-974 */
            r->dynamic_range_match = 0.5;
        else
            r->dynamic_range_match = scalar_sim(a->dynamic_range, b->dynamic_range);
        if (!(both & SONAR_FEAT_SPECTRAL)) {                             /* :977-1008 */
            r->spectral_coherence = 0.5;
        } else {
            double v[2];
            int m = 0;
            if (a->n_spectral_centroid > 0 && b->n_spectral_centroid > 0) {
                if (a->n_spectral_centroid != b->n_spectral_centroid) return -2;   /* gonum panics */
                const double c = g_correlation(a->spectral_centroid, b->spectral_centroid, a->n_spectral_centroid);
                if (!isnan(c)) v[m++] = fabs(c);
            }
            if (a->n_spectral_rolloff > 0 && b->n_spectral_rolloff > 0) {
                if (a->n_spectral_rolloff != b->n_spectral_rolloff) return -2;
                const double c = g_correlation(a->spectral_rolloff, b->spectral_rolloff, a->n_spectral_rolloff);
                if (!isnan(c)) v[m++] = fabs(c);
            }
            r->spectral_coherence = m ? list_mean(v, m) : 0.5;
        }
    }
    double conf = 0.5;                                                   /* calculateConfidence :1011-1037 */
    if (r->overall_similarity > 0.8) conf += 0.3;
    else if (r->overall_similarity > 0.6) conf += 0.2;
    if (r->content_type_match) conf += 0.1;
    conf += (double)nd * 0.05;
    if (r->has_quality) {
        conf += r->data_availability * 0.1;
        conf -= r->noise_level * 0.1;
    }
    r->confidence = cmax(0.0, cmin(1.0, conf));
    return 0;
}

static int classify(double s) {   /* classifyMatch :1040-1052 */
    if (s >= 0.95) return SONAR_MATCH_EXACT;
    if (s >= 0.85) return SONAR_MATCH_VERY_SIMILAR;
    if (s >= 0.75) return SONAR_MATCH_SIMILAR;
    if (s >= 0.6) return SONAR_MATCH_SOMEWHAT_SIMILAR;
    return SONAR_MATCH_WEAK;
}

/* FindBestMatches (:197-263).  sort.Slice is not stable; equal similarities are kept in
 * candidate order here (insertion sort), which is one of the orders Go may produce. */
int or_find_best_matches(const sonar_fp_features* query, const sonar_fp_features* cands, int64_t n,
                         const sonar_compare_cfg* cfg, sonar_match* out, int64_t* n_out) {
    sonar_match* m = malloc(sizeof(sonar_match) * (size_t)(n > 0 ? n : 1));
    int64_t k = 0;
    for (int64_t i = 0; i < n; i++) {
        if (query->id == cands[i].id) continue;
        sonar_similarity s;
        const int rc = or_fp_compare(query, &cands[i], cfg, &s);
        if (rc) { free(m); return rc; }
        if (s.overall_similarity >= cfg->similarity_threshold) {
            m[k].candidate = i;
            m[k].similarity = s;
            m[k].match_type = classify(s.overall_similarity);
            k++;
        }
    }
    for (int64_t i = 1; i < k; i++) {
        const sonar_match x = m[i];
        int64_t j = i - 1;
        while (j >= 0 && m[j].similarity.overall_similarity < x.similarity.overall_similarity) { m[j + 1] = m[j]; j--; }
        m[j + 1] = x;
    }
    if (cfg->max_candidates < 0) { free(m); return -3; }
    if (k > cfg->max_candidates) k = cfg->max_candidates;
    for (int64_t i = 0; i < k; i++) { out[i] = m[i]; out[i].rank = (int32_t)i + 1; }
    *n_out = k;
    free(m);
    return 0;
}
