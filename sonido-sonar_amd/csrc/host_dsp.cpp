// host_dsp.cpp -- see host_dsp.h.  Go semantics restated (file:line cited per
// function); float64 throughout, evaluation order as in the Go source.
#include "host_dsp.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace sonar {
namespace host {

namespace {
constexpr double kPi = 3.14159265358979323846;

// Go int(float64) on amd64: NaN / out-of-range -> MinInt64 (CVTTSD2SQ)
int64_t go_trunc(double x) {
  if (!(x >= -9.2233720368547758e18 && x < 9.2233720368547758e18)) return std::numeric_limits<int64_t>::min();
  return static_cast<int64_t>(x);
}
double go_min(double x, double y) {
  if (std::isinf(x) && x < 0) return x;
  if (std::isinf(y) && y < 0) return y;
  if (std::isnan(x) || std::isnan(y)) return std::numeric_limits<double>::quiet_NaN();
  if (x == 0 && x == y) return std::signbit(x) ? x : y;
  return x < y ? x : y;
}
double go_max(double x, double y) {
  if (std::isinf(x) && x > 0) return x;
  if (std::isinf(y) && y > 0) return y;
  if (std::isnan(x) || std::isnan(y)) return std::numeric_limits<double>::quiet_NaN();
  if (x == 0 && x == y) return std::signbit(x) ? y : x;
  return x > y ? x : y;
}
double bessel_i0(double x) {   // windowing.go:425-441
  double sum = 1.0, term = 1.0;
  for (int k = 1; k < 50; k++) {
    const double t = x / (2.0 * (double)k);
    term *= t * t;
    sum += term;
    if (term < 1e-12) break;
  }
  return sum;
}
}  // namespace

bool make_window(int type, int size, bool symmetric, bool normalize, double beta, double alpha,
                 std::vector<double>& c) {
  if (size <= 0 || size > 1048576) return false;                 // validateConfig :177-199
  const int N = size;
  c.assign(N, 0.0);
  const double den = symmetric ? (double)(N - 1) : (double)N;
  switch (type) {
    case 0: for (int i = 0; i < N; i++) c[i] = 0.5 * (1.0 - std::cos(2 * kPi * (double)i / den)); break;   // :246
    case 1: for (int i = 0; i < N; i++) c[i] = 0.54 - 0.46 * std::cos(2 * kPi * (double)i / den); break;   // :259
    case 2: for (int i = 0; i < N; i++) {                                                                  // :272
        const double a = 2 * kPi * (double)i / den; c[i] = 0.42 - 0.5 * std::cos(a) + 0.08 * std::cos(2 * a); }
      break;
    case 3: for (int i = 0; i < N; i++) {                                                                  // :288
        const double a = 2 * kPi * (double)i / den;
        c[i] = 0.35875 - 0.48829 * std::cos(a) + 0.14128 * std::cos(2 * a) - 0.01168 * std::cos(3 * a); }
      break;
    case 4: {                                                                                              // :304
      if (beta < 0) return false;
      const double i0b = bessel_i0(beta);
      for (int i = 0; i < N; i++) { const double a = 2.0 * (double)i / den - 1.0;
        c[i] = bessel_i0(beta * std::sqrt(1 - a * a)) / i0b; }
      break; }
    case 5: {                                                                                              // :321
      if (alpha < 0 || alpha > 1) return false;
      const int taper = (int)(alpha * (double)N / 2.0);
      for (int i = 0; i < N; i++) {
        if (i < taper) c[i] = 0.5 * (1 + std::cos(kPi * (double)i / (double)taper - kPi));
        else if (i >= N - taper) c[i] = 0.5 * (1 + std::cos(kPi * (double)(i - (N - taper)) / (double)taper));
        else c[i] = 1.0;
      }
      break; }
    case 6: for (int i = 0; i < N; i++) c[i] = 1.0; break;
    case 7: for (int i = 0; i < N; i++)                                                                    // :350
        c[i] = (i <= N / 2) ? 2.0 * (double)i / (double)(N - 1) : 2.0 - 2.0 * (double)i / (double)(N - 1);
      break;
    case 8: for (int i = 0; i < N; i++) {                                                                  // :363
        const double a = ((double)i - (double)(N - 1) / 2.0) / ((double)(N - 1) / 2.0); c[i] = 1.0 - a * a; }
      break;
    default: return false;
  }
  if (normalize) {                                                // calculateWindowProperties + normalizeWindow :393-437
    double energy = 0.0;
    for (double v : c) energy += v * v;
    const double nf = 1.0 / std::sqrt(energy / (double)N);
    for (double& v : c) v *= nf;
  }
  return true;
}

bool make_filterbank(int kind, int nf, int fft_size, int sr, double low, double high, std::vector<double>& fb) {
  if (nf <= 0 || fft_size <= 0) return false;
  const int K = fft_size / 2 + 1;
  fb.assign((size_t)nf * K, 0.0);
  auto fwd = [kind](double hz) {
    return kind ? (26.81 * hz / (1960.0 + hz)) - 0.53 : 2595.0 * std::log10(1.0 + hz / 700.0);
  };
  auto inv = [kind](double v) {
    return kind ? 1960.0 * (v + 0.53) / (26.28 - v) : 700.0 * (std::pow(10.0, v / 2595.0) - 1.0);
  };
  const double lo = fwd(low), hi = fwd(high);
  const double step = (hi - lo) / (double)(nf + 1);
  std::vector<int64_t> bins(nf + 2);
  for (int i = 0; i < nf + 2; i++) {
    const double hz = inv(lo + (double)i * step);
    int64_t b = go_trunc(std::floor(((double)fft_size + 1.0) * hz / (double)sr + 0.5));
    bins[i] = std::min<int64_t>(b, fft_size / 2);
  }
  for (int m = 1; m <= nf; m++) {
    const int64_t l = bins[m - 1], c = bins[m], r = bins[m + 1];
    double* row = fb.data() + (size_t)(m - 1) * K;
    for (int64_t k = l; k < c && k < K; k++)
      if (c != l && k >= 0) row[k] = (double)(k - l) / (double)(c - l);
    for (int64_t k = c; k < r && k < K; k++)
      if (r != c && k >= 0) row[k] = (double)(r - k) / (double)(r - c);
  }
  return true;
}

bool make_mfcc_tables(int sr, int n_mfcc, int n_filters, int fb_kind, double low, double high, bool use_lifter,
                      double lifter, int fft_size, MfccTables& t) {
  if (n_mfcc <= 0) n_mfcc = 13;                                   // NewMFCCWithParams :58-70
  if (n_filters <= 0) n_filters = 26;
  if (high <= 0) high = (double)sr / 2.0;
  if (lifter <= 0) lifter = 22.0;
  std::vector<double> fb;
  if (!make_filterbank(fb_kind, n_filters, fft_size, sr, low, high, fb)) return false;
  t.n_mfcc = n_mfcc; t.n_mels = n_filters; t.K = fft_size / 2 + 1;
  t.lo.assign(n_filters, 0); t.hi.assign(n_filters, 0); t.woff.assign(n_filters, 0); t.w.clear();
  for (int m = 0; m < n_filters; m++) {
    const double* row = fb.data() + (size_t)m * t.K;
    int lo = -1, hi = -1;
    for (int k = 0; k < t.K; k++) if (row[k] != 0.0) { if (lo < 0) lo = k; hi = k + 1; }
    if (lo < 0) { lo = 0; hi = 0; }
    t.lo[m] = lo; t.hi[m] = hi; t.woff[m] = (int)t.w.size();
    for (int k = lo; k < hi; k++) t.w.push_back(row[k]);    // zeros inside the range kept: same sum order
  }
  t.dct.assign((size_t)n_mfcc * n_filters, 0.0);
  for (int k = 0; k < n_mfcc; k++)
    for (int n = 0; n < n_filters; n++) {
      double v = std::cos(kPi * (double)k * ((double)n + 0.5) / (double)n_filters);
      v *= (k == 0) ? std::sqrt(1.0 / (double)n_filters) : std::sqrt(2.0 / (double)n_filters);
      t.dct[(size_t)k * n_filters + n] = v;
    }
  t.lift.assign(n_mfcc, 1.0);
  if (use_lifter)
    for (int i = 1; i < n_mfcc; i++) t.lift[i] = 1.0 + (lifter / 2.0) * std::sin(kPi * (double)i / lifter);
  return true;
}

void balance_groups(const MfccTables& t, int groups, std::vector<int>& off, std::vector<int>& mels) {
  std::vector<std::vector<int>> g(groups);
  std::vector<long> load(groups, 0);
  std::vector<int> order(t.n_mels);
  for (int m = 0; m < t.n_mels; m++) order[m] = m;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return (t.hi[a] - t.lo[a]) > (t.hi[b] - t.lo[b]); });
  for (int m : order) {   // longest-processing-time first
    int best = 0;
    for (int k = 1; k < groups; k++) if (load[k] < load[best]) best = k;
    g[best].push_back(m);
    load[best] += (t.hi[m] - t.lo[m]) + 8;
  }
  off.assign(groups + 1, 0); mels.clear();
  for (int k = 0; k < groups; k++) { off[k] = (int)mels.size(); for (int m : g[k]) mels.push_back(m); }
  off[groups] = (int)mels.size();
}

std::vector<int> chroma_map(int fs, int sr) {
  const int K = fs / 2 + 1;
  std::vector<int> map(K, -1);
  const double res = (double)sr / (double)fs;                    // stft.go:158
  for (int f = 0; f < K; f++) {
    const double fr = (double)f * res;
    if (fr < 80.0 || fr > 8000.0) continue;
    const double midi = fr <= 0 ? 0.0 : 69.0 + 12.0 * std::log2(fr / 440.0);
    map[f] = (int)(go_trunc(std::round(midi)) % 12);
  }
  return map;
}

static double median_positive(const double* v, int n) {           // calculateMedian :975-1004
  double tmp[8];                                                  // n <= 5
  int m = 0;
  for (int i = 0; i < n; i++)
    if (v[i] > 0) {                                               // insertion sort of the positives
      int j = m++;
      while (j > 0 && tmp[j - 1] > v[i]) { tmp[j] = tmp[j - 1]; --j; }
      tmp[j] = v[i];
    }
  if (m == 0) return 0.0;
  return (m % 2 == 0) ? (tmp[m / 2 - 1] + tmp[m / 2]) / 2.0 : tmp[m / 2];
}

void YinTracker::step(double& pitch, double& conf, double& voicing) {
  double p = pitch, c = conf, v = conf;
  if (p != 0.0 && count > 0) {                                    // applyOctaveCorrection :789-827
    const int cnt = std::min(count, 5);
    if (cnt >= 3) {
      const double med = median_positive(hist + count - cnt, cnt);
      const double ratios[4] = {0.5, 2.0, 1.0 / 3.0, 3.0};
      for (double r : ratios) {
        const double ex = med * r;
        if (std::fabs(p - ex) / ex < 0.1) {
          if (std::fabs(p - med) > std::fabs(ex - med)) p = ex;
          break;
        }
      }
    }
  }
  if (c < 0.5) { p = 0; c = 0; v = 0; }                          // MinConfidence :781-785
  if (count == 20) {                                              // updateTemporalTracking :876-899
    for (int i = 1; i < 20; i++) hist[i - 1] = hist[i];
    hist[19] = p;
  } else {
    hist[count++] = p;
  }
  if (count > 1) {                                                // applyTemporalSmoothing :903-921
    const int cnt = std::min(count, 3);
    if (cnt >= 3) p = median_positive(hist + count - cnt, cnt);
    else p = 0.3 * p + (1 - 0.3) * prev;
  }
  prev = p;
  pitch = p; conf = c; voicing = v;
}

CorrSums corr_sums(const double* corr, int64_t nl) {
  CorrSums c;
  c.num_lags = nl;
  if (nl <= 0) return c;
  double pk = corr[0]; int64_t pidx = 0;                          // findPeak :526-544
  for (int64_t i = 0; i < nl; i++) if (std::fabs(corr[i]) > std::fabs(pk)) { pk = corr[i]; pidx = i; }
  c.peak = pk; c.peak_index = pidx;
  for (int64_t i = 0; i < nl; i++)                                // calculateSNR :572-601
    if (std::llabs(i - pidx) > 5) { c.noise_sum += corr[i] * corr[i]; c.noise_count++; }
  if (nl >= 3 && pidx > 0 && pidx < nl - 1)                        // calculateSharpness :611-619
    c.sharpness = -(corr[pidx + 1] - 2 * corr[pidx] + corr[pidx - 1]);
  for (int64_t i = 0; i < nl; i++)                                // findSecondPeak :622-636
    if (i != pidx && std::fabs(corr[i]) > std::fabs(c.second_peak)) c.second_peak = corr[i];
  for (int64_t i = 0; i < nl; i++)                                // calculatePeakToSidelobe :639-661
    if (std::llabs(i - pidx) > 10 && std::fabs(corr[i]) > c.max_sidelobe) c.max_sidelobe = std::fabs(corr[i]);
  return c;
}

NccMetrics ncc_metrics(const CorrSums& c, int64_t L, int64_t na, int64_t nb) {
  NccMetrics m;
  m.num_lags = c.num_lags;
  if (c.num_lags <= 0) return m;
  const double pk = c.peak;
  const int64_t pidx = c.peak_index;
  m.peak_corr = pk; m.peak_index = pidx; m.peak_lag = pidx - L;
  const int64_t n = std::min(na, nb);                              // calculatePValue :547-569
  m.p_value = 1.0;
  if (n > 2) {
    const double t = std::fabs(pk) * std::sqrt((double)(n - 2)) / std::sqrt(1.0 - pk * pk);
    m.p_value = t > 2.0 ? 0.01 : t > 1.5 ? 0.05 : t > 1.0 ? 0.1 : 0.5;
  }
  {                                                               // calculateSNR :572-601
    const double pv = std::fabs(pk);
    if (c.noise_count > 0) {
      const double lvl = std::sqrt(c.noise_sum / (double)c.noise_count);
      m.snr = lvl < 1e-10 ? INFINITY : 20.0 * std::log10(pv / lvl);
    }
  }
  m.sharpness = c.sharpness;
  m.second_peak = c.second_peak;
  {                                                               // calculatePeakToSidelobe :639-661
    const double pv = std::fabs(pk), ms = c.max_sidelobe;
    m.psl = ms < 1e-10 ? INFINITY : 20.0 * std::log10(pv / ms);
  }
  const int64_t lag = m.peak_lag;                                  // calculateOverlapLength :664-667
  int64_t s1, e1, s2, e2;
  if (lag >= 0) { s1 = 0; e1 = na; s2 = lag; e2 = nb; if (e1 > nb - lag) e1 = nb - lag; if (e2 > nb) e2 = nb; }
  else { s1 = -lag; e1 = na; s2 = 0; e2 = nb; if (e1 > na) e1 = na; if (e2 > na + lag) e2 = na + lag; }
  m.overlap = std::min(e1 - s1, e2 - s2);
  return m;
}

NccMetrics ncc_metrics(const double* corr, int64_t nl, int64_t L, int64_t na, int64_t nb) {
  return ncc_metrics(corr_sums(corr, nl), L, na, nb);
}

AlignScores xcorr_scores(const NccMetrics& m, int hop, int sr, int max_lag) {
  AlignScores s;                                                  // alignWithCrossCorrelation :151-181
  s.offset = m.peak_lag * hop;
  s.offset_seconds = (double)s.offset / (double)sr;
  s.similarity = go_min(1.0, go_max(0.0, std::fabs(m.peak_corr)));
  const double pm = std::fabs(m.peak_corr);
  if (pm >= 0.1) {                                                // calculateCorrelationConfidence :183-243
    double ps = pm; if (pm >= 0.6) ps = pm + (pm - 0.6) * 0.5;
    const double ss = go_min(0.9, m.sharpness * 8.0);
    double sl = 0.0; if (m.psl > 0 && !std::isinf(m.psl)) sl = go_min(0.8, m.psl / 15.0);
    double sn = 0.0; if (m.snr > 0) sn = go_min(0.7, m.snr / 25.0);
    double pen = 0.0;
    if (m.second_peak != 0 && pm > 0) { const double r = std::fabs(m.second_peak) / pm; if (r > 0.7) pen = (r - 0.7) * 0.25; }
    const double bonus = pm >= 0.75 ? 0.12 : pm >= 0.6 ? 0.08 : 0.0;
    const double c = 0.55 * ps + 0.22 * ss + 0.12 * sl + 0.06 * sn + 0.05 * 0.15 + bonus - pen;
    s.confidence = go_min(0.95, go_max(0.0, c));
  }
  if (pm >= 0.08) {                                               // calculateCorrelationQuality :245-305
    double pq = pm; if (pm >= 0.6) pq = pm + (pm - 0.6) * 0.4;
    const double sq = go_min(0.85, m.sharpness * 5.0);
    double slq = 0.0; if (m.psl > 0 && !std::isinf(m.psl)) slq = go_min(0.7, m.psl / 20.0);
    double snq = 0.0; if (m.snr > 0) snq = go_min(0.6, m.snr / 30.0);
    double lp = 0.0;
    if (max_lag > 0 && m.peak_lag < 0) {
      const double nr = std::fabs((double)m.peak_lag) / (double)max_lag;
      if (nr > 0.90) lp = (nr - 0.90) * 4.0;
    }
    const double qb = pm >= 0.7 ? 0.10 : pm >= 0.55 ? 0.06 : 0.0;
    s.quality = go_min(1.0, go_max(0.0, 0.50 * pq + 0.25 * sq + 0.15 * slq + 0.10 * snq + qb - lp));
  }
  s.noise_level = 1.0 - m.snr / 20.0;
  return s;
}

PathSums path_sums(const int32_t* pq, const int32_t* pr, const double* pc, int64_t P) {
  PathSums s;
  s.P = P;
  if (P <= 0) return s;
  s.p0q = pq[0]; s.p0r = pr[0]; s.p1q = pq[P - 1]; s.p1r = pr[P - 1];
  for (int64_t i = 0; i < P; i++) { s.offset_sum += pr[i] - pq[i]; s.sum_cost += pc[i]; }   // :530-541, :380-406
  int pd0 = 0, pd1 = 0;
  for (int64_t i = 1; i < P; i++) {
    const int d0 = pq[i] - pq[i - 1], d1 = pr[i] - pr[i - 1];
    if (d0 > 0 && d1 > 0) s.diag_steps++;                         // calculateDiagonalBias :514-540
    if (i > 1 && (d0 != pd0 || d1 != pd1)) s.changes++;           // calculatePathChanges :569-603
    pd0 = d0; pd1 = d1;
  }
  if (P > 1) {                                                    // calculateCostConsistency :466-512
    int64_t w = std::min<int64_t>(5, P / 4);
    w = std::max<int64_t>(w, 2);
    std::vector<double> sm(P);
    for (int64_t i = 0; i < P; i++) {
      double t = 0; int64_t c = 0;
      for (int64_t j = std::max<int64_t>(0, i - w / 2); j <= std::min<int64_t>(P - 1, i + w / 2); j++) { t += pc[j]; c++; }
      sm[i] = t / (double)c;
    }
    for (double v : sm) s.sum_smooth += v;
    const double mean = s.sum_smooth / (double)P;
    for (double v : sm) { const double d = v - mean; s.var_smooth += d * d; }
  }
  return s;
}

namespace {
double cost_consistency(const PathSums& s) {                      // alignment.go:466-512
  if (s.P <= 1) return 0.0;
  const double mean = s.sum_smooth / (double)s.P;
  if (mean <= 1e-10) return 1.0;
  const double var = s.var_smooth / (double)s.P;
  return 1.0 / (1.0 + std::sqrt(var) / mean);
}
double diagonal_bias(const PathSums& s) {                         // :514-540
  if (s.P <= 1) return 1.0;
  const double ratio = (double)s.diag_steps / (double)(s.P - 1);
  return 1.0 / (1.0 + std::exp(-10.0 * (ratio - 0.3)));
}
double path_changes_ratio(const PathSums& s) {                    // :569-603 / :620-643
  return (double)s.changes / (double)(s.P - 1);
}
double dtw_quality(const PathSums& s, int64_t nq, int64_t nr) {
  if (s.P == 0) return 0.0;                                       // calculateDTWQuality :543-566
  double eff = (double)std::max(nq, nr) / (double)s.P;
  eff = go_min(1.0, eff);
  const double smooth = s.P <= 2 ? 1.0 : go_max(0.0, 1.0 - path_changes_ratio(s));
  const double q = 0.3 * eff + 0.3 * diagonal_bias(s) + 0.2 * smooth + 0.2 * cost_consistency(s);
  return go_min(1.0, go_max(0.0, q));
}
}  // namespace

AlignScores dtw_scores(const PathSums& ps, int64_t nq, int64_t nr, double dist, int sr) {
  AlignScores s;                                                  // alignWithDTW :129-148
  const int64_t P = ps.P;
  const double avg = (double)(nq + nr) / 2.0;
  if (avg != 0) {                                                 // calculateSimilarityFromDTW :380-406
    const double ds = 1.0 / (1.0 + dist / avg);
    double mc = 0; if (P > 0) mc = ps.sum_cost / (double)P;
    s.similarity = go_min(1.0, go_max(0.0, 0.5 * ds + 0.3 * dtw_quality(ps, nq, nr) + 0.2 * (1.0 / (1.0 + mc))));
  }
  if (P > 0 && avg != 0) {                                        // calculateDTWConfidence :420-463
    const double c1 = std::exp(-(dist / avg) * 2.0);
    const double pe = go_min(1.0, (double)std::max(nq, nr) / (double)P);
    s.confidence = go_min(1.0, go_max(0.0, 0.4 * c1 + 0.25 * pe + 0.2 * cost_consistency(ps) +
                                               0.15 * diagonal_bias(ps)));
  }
  if (P > 0) s.offset = ps.offset_sum / P;                        // calculateAverageOffset :530-541
  s.offset_seconds = (double)s.offset / (double)sr;               // F9: frames / sample rate
  s.quality = dtw_quality(ps, nq, nr);
  if (P >= 3) s.stability = go_max(0.0, 1.0 - path_changes_ratio(ps));   // :620-643
  return s;
}

AlignScores dtw_scores(const int32_t* pq, const int32_t* pr, const double* pc, int64_t P, int64_t nq, int64_t nr,
                       double dist, int sr) {
  return dtw_scores(path_sums(pq, pr, pc, P), nq, nr, dist, sr);
}

double energy_variance(const double* e, size_t n) {               // energy.go:96-117
  if (n < 2) return 0.0;
  double mean = 0.0;
  for (size_t i = 0; i < n; i++) mean += e[i];
  mean /= (double)n;
  double var = 0.0;
  for (size_t i = 0; i < n; i++) { const double d = e[i] - mean; var += d * d; }
  return var / (double)(n - 1);
}

double loudness_range_from_rms(std::vector<double> v) {           // energy.go:145-205
  if (v.empty()) return 0.0;
  for (double& x : v) x = x > 0 ? -0.691 + 10.0 * std::log10(x * x) : -70.0;
  std::sort(v.begin(), v.end());
  const int64_t lo = (int64_t)(0.10 * (double)(v.size() - 1));
  const int64_t hi = (int64_t)(0.95 * (double)(v.size() - 1));
  double lv = v[lo], hv = v[hi];
  if (lv <= 0.0) lv = 1e-10;
  if (hv <= 0.0) return 0.0;
  return 20.0 * std::log10(hv / lv);
}

}  // namespace host
}  // namespace sonar
