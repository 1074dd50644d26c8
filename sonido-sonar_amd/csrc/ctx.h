// ctx.h -- internal state behind the opaque sonar_ctx / sonar_result handles,
// shared by sonar_api.cpp (kernel-level entries) and go_api.cpp (Go-API mirror).
#pragma once
#include "../../include/sonar_gpu.h"

#include <hip/hip_runtime.h>

#include "kernels.h"

#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

struct DevBuf {
  void* ptr = nullptr;
  size_t cap = 0;
};

struct FpTables {
  void* window = nullptr;
  int *mel_lo = nullptr, *mel_hi = nullptr, *mel_woff = nullptr, *grp_off = nullptr, *grp_mels = nullptr;
  void *mel_w = nullptr, *dct = nullptr, *lift = nullptr;
  void* trig = nullptr;   // generic-W path: (cos, -sin) of 2 pi m / W
  int n_mels = 0, n_mfcc = 0, nnz = 0;
};

// tables of the headline kernel (mfcc_pair.hip); ok = false -> configuration unsupported there
struct PairTables {
  bool ok = false;
  // [0] float32 tables (the headline), [1] float64 (the same bank at the reference's precision; its
  // own chunk lane order, searched for its 16-byte power-row reads)
  void *window[2] = {}, *tw1[2] = {}, *tw2[2] = {}, *chunk_w[2] = {}, *dct[2] = {};
  int* chunk_ks[2] = {};
  uint16_t* mel_src[2] = {};
  void* zeros = nullptr;    // 1024 zero samples of either PCM type (8 KB)
  int J = 0, JS = 0, NMP = 0, n_mels = 0, n_mfcc = 0, max_src = 0;
};

struct IngestState;  // pinned slots + host pool of sonar_ingest_f64le (ingest_api.cpp)

struct sonar_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  std::map<std::string, DevBuf> bufs;
  std::map<std::string, DevBuf> hbufs;   // pinned host staging (hipHostMalloc)
  std::map<std::string, FpTables> fp_tables;
  std::map<std::string, PairTables> pair_tables;
  struct ChromaT { void* win; void* trig; void* map; void* cls; };
  std::map<std::string, ChromaT> chroma_tables;
  bool timing = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;   // spare pair (kept for ABI simplicity)
  // one event pair per timed launch since the last sonar_last_kernel_ms query
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  size_t ev_used = 0;
  double last_ms = 0.0;
  const char* last_fp_kernel = "";
  hipEvent_t dtw_ev[4] = {nullptr, nullptr, nullptr, nullptr};   // band | walk | decode boundaries
  double dtw_ms[3] = {0.0, 0.0, 0.0};
  IngestState* ingest = nullptr;
  std::vector<sonar_ctx*> workers;   // sonar_align_pairs' worker contexts (multi_api.cpp)
  // a second stream for the NCC while the chroma DTW runs on `stream` (align_impl), and the two
  // events that order it: features done -> side, NCC done -> stream
  hipStream_t side = nullptr;
  hipEvent_t side_ev[2] = {nullptr, nullptr};
  // the host-PCM pipeline of sonar_extract_speech_features: H2D chunks on `copy`, one event per
  // chunk the compute streams wait on (go_api.cpp)
  hipStream_t copy = nullptr;
  std::vector<hipEvent_t> chunk_ev;
  // ... and chunk k's pitch rows on the host (side stream), for the early tracker
  std::vector<hipEvent_t> back_ev;
  // band-kernel liveness counters (sonar_dtw_counters): edge refresh fences, those followed by new
  // edge values, DTWs that timed out, waves that timed out
  long long dtw_ctr[4] = {0, 0, 0, 0};
  // sonar_fingerprint_batch: its segment table's pinned staging is rewritten only after the previous
  // call's upload of it has completed (this event)
  hipEvent_t fpb_ev = nullptr;
};

// Named float64 arrays + scalars.  An array either owns its values (v) or points into a block the
// result holds a reference to (ext + owners: pinned host memory the device copied into directly,
// sonar::detail::pinned_block), so large outputs reach the caller without a host copy.
struct sonar_result {
  struct Arr {
    std::string name;
    std::vector<double> v;
    int64_t rows = 0, cols = 0;
    const double* ext = nullptr;
    const double* data() const { return ext ? ext : v.data(); }
  };
  std::vector<Arr> arrays;
  std::vector<std::shared_ptr<void>> owners;
  Arr& slot(const std::string& name) {
    for (auto& a : arrays)
      if (a.name == name) return a;
    arrays.push_back({name, {}, 0, 0, nullptr});
    return arrays.back();
  }
  void put(const std::string& name, std::vector<double> v, int64_t rows, int64_t cols) {
    Arr& a = slot(name);
    a.v = std::move(v); a.rows = rows; a.cols = cols; a.ext = nullptr;
  }
  // rows x cols values at p, inside a block this result holds (see hold)
  void put_ext(const std::string& name, const double* p, int64_t rows, int64_t cols) {
    Arr& a = slot(name);
    a.v.clear(); a.rows = rows; a.cols = cols; a.ext = p;
  }
  void hold(std::shared_ptr<void> block) { owners.push_back(std::move(block)); }
  void scalar(const std::string& name, double x) { put(name, {x}, 1, 1); }
  void vec(const std::string& name, const std::vector<double>& v) { put(name, v, (int64_t)v.size(), 1); }
  double get(const std::string& name, double dflt = 0.0) const {
    for (auto& a : arrays)
      if (a.name == name && a.rows * a.cols > 0) return a.data()[0];
    return dflt;
  }
};

namespace sonar {
namespace detail {
int fail(sonar_ctx* c, int code, const std::string& msg);
void* dbuf(sonar_ctx* c, const std::string& name, size_t bytes);
// frees every cached device / pinned host buffer of c (sonar_trim; the batch path's NOMEM retry)
void trim_buffers(sonar_ctx* c);
void* hbuf(sonar_ctx* c, const std::string& name, size_t bytes);
// A block of `bytes` of pinned host memory from a process-wide pool (hipHostMalloc'd once, reused):
// device-to-host copies land in it at DMA speed and result arrays can point into it; the block
// returns to the pool when the last shared_ptr to it goes.  Null on allocation failure.
std::shared_ptr<void> pinned_block(size_t bytes);
// frees the pool's idle blocks (sonar_trim)
void pinned_pool_trim();
// chroma tables of frame size fs at sample rate sr, built once per context (sonar_api.cpp); null on
// allocation failure
const sonar_ctx::ChromaT* chroma_tables_for(sonar_ctx* c, int fs, int sr);
// NCC + chroma DTW of one stream pair with two stream synchronisations (align_impl's device
// path, sonar_api.cpp): ncc_enqueue and dtw_enqueue only launch and queue their small results
// into pinned host memory; after one hipStreamSynchronize, ncc_metrics_host reads the
// correlation and dtw_finish decodes the warping path into pinned host arrays (second sync).
struct DtwPending {
  const double *dq = nullptr, *dr = nullptr;
  int64_t nq = 0, nr = 0;
  int32_t dim = 0, band = -1;
  int64_t* st = nullptr;   // pinned: [0] path length, [1] sync words 0..1, [2] non-finite flag
};
int ncc_enqueue(sonar_ctx* c, const double* da, int64_t na, const double* db, int64_t nb, int32_t max_lag,
                double** hcorr, int64_t* L);
void ncc_metrics_host(const double* corr, int64_t L, int64_t na, int64_t nb, double* metrics);
// the path-tile pass's arguments (launch_dtw_path_tiles) of one DTW in checkpoint mode
sonar::DtwArgs tile_args(const double* q, const double* r, int dim, int band, const sonar::DtwGeom& g, uint64_t* E,
                         double* CK, int32_t* runs, int32_t* pq, int32_t* pr, double* pc, int64_t* plen, double* cnm);
// the band kernel's status block of one DTW (int32 sync[4] + the DtwArgs::diag record): adds its
// counters to c->dtw_ctr and, when the DTW timed out, returns the failure text with the record
std::string dtw_status(sonar_ctx* c, const void* sync_block);
int dtw_enqueue(sonar_ctx* c, const double* dq, int64_t nq, const double* dr, int64_t nr, int32_t dim, int32_t band,
                DtwPending* p);
int dtw_finish(sonar_ctx* c, DtwPending* p, const int32_t** hq, const int32_t** hr, const double** hc, int64_t* P,
               double* distance);
// ExtractAlignmentFeatures' host tail over the GPU results of one pair (go_api.cpp): the scorers,
// selectBestAlignment and the time-stretch estimate, into a result handle and/or a pair record
struct AlignIn {
  const double* corr = nullptr;   // energy correlation, 2L+1 lags (null: no correlation candidate)
  const host::CorrSums* corr_sums = nullptr;   // or its reductions (the device scorer's), no array
  int64_t L = 0, nqe = 0, nre = 0, mlf = 0;
  bool has_dtw = false;           // chroma DTW candidate
  const int32_t *pq = nullptr, *pr = nullptr;
  const double* pc = nullptr;
  const host::PathSums* path_sums = nullptr;   // or the path's reductions, no arrays
  int64_t P = 0, nqc = 0, nrc = 0;
  double dist = 0.0;
  int64_t q_pcm_len = 0, r_pcm_len = 0;
  int32_t sample_rate = 0, hop = 0;
};
void align_finish(const AlignIn& in, sonar_result* res, sonar_pair_record* rec);
hipEvent_t timed_begin(sonar_ctx* c, hipStream_t s);
// the context a comparator gallery lives on (compare_api.cpp)
sonar_ctx* gallery_ctx(const sonar_gallery* g);
// ContentDetector (content_api.cpp)
int detect_from_audio(sonar_ctx* c, const double* pcm, int64_t n, int32_t sr, double thr, int32_t* out,
                      sonar_acoustic_features* feat);
int detect_content_type(sonar_ctx* c, const double* pcm, int64_t n, int32_t sr, int32_t has_md, const char* ct,
                        const char* genre, const char* station, const char* url, int32_t acoustic,
                        int32_t dflt, double thr, int32_t* out);
void timed_end(sonar_ctx* c, hipStream_t s, hipEvent_t end);
// frees the ingest ring and joins its host threads (ingest_api.cpp)
void ingest_release(sonar_ctx* c);
// sonar_fingerprint with the PCM already on the device and host outputs (sonar_api.cpp)
// [f_lo, f_hi): only those frames of the whole signal's STFT (device outputs, per-frame kernel)
int fingerprint_impl(sonar_ctx* c, const void* pcm, int64_t n, const sonar_fp_cfg* cfg, sonar_fp_out* out,
                     bool pcm_dev, int64_t f_lo = 0, int64_t f_hi = -1);
// VoiceQualityAnalyzer.AnalyzeVoiceQuality on device-resident float64 samples (voice_api.cpp)
int voice_quality(sonar_ctx* c, const double* dsig, int64_t n, int32_t sr, sonar_voice_quality_result* out);
}  // namespace detail
}  // namespace sonar

#define HIP_TRY(ctx, call)                                                                   \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return ::sonar::detail::fail(ctx, SONAR_ERR_DEVICE, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)
