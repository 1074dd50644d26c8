// host_dsp.h -- host-side parts of the hot path that are O(table) or O(path):
// window / filterbank / DCT tables built once per configuration, and the
// sequential scalar epilogues of the Go API (YIN temporal tracking, NCC peak
// metrics, alignment scorers).  Pure C++17, float64, Go evaluation order.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace sonar {
namespace host {

// analyzers.WindowGenerator.Generate (fingerprint/analyzers/windowing.go:77-136)
bool make_window(int type, int size, bool symmetric, bool normalize, double beta, double alpha,
                 std::vector<double>& out);

// MelScale / BarkScale.CreateXFilterBank (algorithms/spectral/mel_scale.go:29-86,
// bark_scale.go:36-93) as dense rows [n_filters][fft_size/2+1]
bool make_filterbank(int kind, int n_filters, int fft_size, int sample_rate, double low, double high,
                     std::vector<double>& fb);

struct MfccTables {
  int n_mfcc = 13, n_mels = 26, K = 0;
  std::vector<int> lo, hi, woff;   // per filter nonzero range [lo, hi)
  std::vector<double> w;           // packed weights
  std::vector<double> dct;         // [n_mfcc][n_mels] (mfcc.go:194-212)
  std::vector<double> lift;        // [n_mfcc] lifter multipliers (mfcc.go:230-245)
};
// NewMFCCWithParams defaults + Initialize (mfcc.go:58-110)
bool make_mfcc_tables(int sample_rate, int n_mfcc, int n_filters, int fb_kind, double low, double high,
                      bool use_lifter, double lifter, int fft_size, MfccTables& t);
// balanced assignment of filter rows to `groups` epilogue groups (by nonzeros)
void balance_groups(const MfccTables& t, int groups, std::vector<int>& off, std::vector<int>& mels);

// ChromaSTFT.calculateChromaMapping (algorithms/chroma/chroma_stft.go:95-117)
std::vector<int> chroma_map(int fs, int sample_rate);

// PitchDetector post-processing + temporal tracking (pitch_detection.go:767-921)
// The history is Go's pitchHistory capped at 20 entries (only its last 5 are ever read), kept in a
// fixed array: one step allocates nothing (a 1-hour call runs 310,000 steps).
struct YinTracker {
  double hist[20] = {0};
  int count = 0;                   // entries held (<= 20), oldest first
  double prev = 0.0;
  void step(double& pitch, double& conf, double& voicing);
};

// CrossCorrelation metrics from the correlation array (correlation.go:526-667)
struct NccMetrics {
  double peak_corr = 0, p_value = 1, snr = 0, sharpness = 0, second_peak = 0, psl = 0;
  int64_t peak_lag = 0, peak_index = 0, overlap = 0, num_lags = 0;
};
// The O(lags) part of those metrics: findPeak's index and value, calculateSNR's noise sum and count
// (|i - peak| > 5), findSecondPeak's value, calculatePeakToSidelobe's sidelobe maximum (|i - peak|
// > 10) and calculateSharpness's second difference (0 at the ends).  corr_sums runs Go's loops; the
// batched pair path computes the same on the device (pair_score_kernel, align_kernels.hip), every
// sum in Go's index order with masked terms added as exact zeros, so the two are bit-identical
// (test_device_scorer_equals_host_scorer).  Plain data, shared with the kernels.
struct CorrSums {
  int64_t num_lags = 0, peak_index = 0, noise_count = 0;
  double peak = 0, noise_sum = 0, second_peak = 0, max_sidelobe = 0, sharpness = 0;
};
CorrSums corr_sums(const double* corr, int64_t nl);
NccMetrics ncc_metrics(const CorrSums& c, int64_t L, int64_t na, int64_t nb);
NccMetrics ncc_metrics(const double* corr, int64_t nl, int64_t L, int64_t na, int64_t nb);
// The O(path) part of the DTW scorers (alignment.go:380-643): the path length and end points,
// diagonal steps and direction changes (calculateDiagonalBias, calculatePathChanges), the offset
// sum (calculateAverageOffset), the cost sum (calculateSimilarityFromDTW's mean cost) and
// calculateCostConsistency's smoothed-cost sum and squared deviations from their mean
struct PathSums {
  int64_t P = 0, diag_steps = 0, changes = 0, offset_sum = 0;
  int32_t p0q = 0, p0r = 0, p1q = 0, p1r = 0;
  double sum_cost = 0, sum_smooth = 0, var_smooth = 0;
};
PathSums path_sums(const int32_t* pq, const int32_t* pr, const double* pc, int64_t P);

// AlignmentAnalyzer scorers (algorithms/stats/alignment.go)
struct AlignScores {
  double similarity = 0, confidence = 0, offset_seconds = 0, quality = 0, stability = 0, noise_level = 0;
  int64_t offset = 0;
};
AlignScores xcorr_scores(const NccMetrics& m, int hop, int sample_rate, int max_lag);
AlignScores dtw_scores(const int32_t* pq, const int32_t* pr, const double* pc, int64_t P, int64_t nq, int64_t nr,
                       double distance, int sample_rate);
AlignScores dtw_scores(const PathSums& s, int64_t nq, int64_t nr, double distance, int sample_rate);

// Energy helpers used by extractEnergyFeatures (algorithms/temporal/energy.go:96-178)
double energy_variance(const double* e, size_t n);
// ComputeLoudnessRange tail: RMS of 400 ms / 100 ms frames -> LU -> 10th..95th percentile range
double loudness_range_from_rms(std::vector<double> rms);

}  // namespace host
}  // namespace sonar
