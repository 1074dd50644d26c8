// compare_api.cpp -- FingerprintComparator (fingerprint/comparison.go) behind the C ABI:
// the device gallery of fingerprint records, Compare / BatchCompare and FindBestMatches.
// Kernels: compare_kernels.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "ctx.h"
#include "kernels.h"

using sonar::FpRec;
using sonar::StatJob;
using sonar::detail::dbuf;
using sonar::detail::fail;

struct sonar_gallery {
  sonar_ctx* c = nullptr;
  std::vector<FpRec> host;            // mirror of the device records (host-side checks)
  FpRec* recs = nullptr;
  int64_t cap = 0;
  double* pool = nullptr;             // MFCC column mean/std and chroma column means
  int64_t pool_cap = 0, pool_used = 0;
  std::vector<void*> seqs;            // kept SpectralCentroid / SpectralRolloff copies
};

namespace sonar {
namespace detail {
sonar_ctx* gallery_ctx(const sonar_gallery* g) { return g ? g->c : nullptr; }
}  // namespace detail
}  // namespace sonar

namespace {

constexpr double kNaN = std::numeric_limits<double>::quiet_NaN();

// getEffectiveWeights (comparison.go:1055-1104), by SONAR_FD_* (mfcc, spectral, chroma,
// temporal, speech, harmonic); "energy" is never looked up by calculateFeatureSimilarity
void effective_weights(const sonar_fp_features& f, double* w) {
  static const double news[6] = {0.50, 0.25, 0.05, 0.15, 0.10, 0.05};
  static const double music[6] = {0.30, 0.20, 0.25, 0.10, 0.05, 0.15};
  static const double sports[6] = {0.25, 0.20, 0.05, 0.25, 0.10, 0.05};
  static const double dflt[6] = {0.35, 0.25, 0.10, 0.20, 0.10, 0.10};
  const double* src = dflt;
  if (f.present & SONAR_FEAT_WEIGHTS) src = f.feature_weights;
  else if (f.content_type == SONAR_CT_NEWS || f.content_type == SONAR_CT_TALK) src = news;
  else if (f.content_type == SONAR_CT_MUSIC) src = music;
  else if (f.content_type == SONAR_CT_SPORTS) src = sports;
  std::memcpy(w, src, 6 * sizeof(double));
}

template <typename T>
int grow(sonar_ctx* c, T** p, int64_t* cap, int64_t used, int64_t need) {
  if (need <= *cap) return 0;
  int64_t nc = std::max<int64_t>(need, std::max<int64_t>(64, *cap * 2));
  T* q = nullptr;
  if (hipMalloc(&q, nc * sizeof(T)) != hipSuccess) return fail(c, SONAR_ERR_NOMEM, "gallery allocation failed");
  if (*p) {
    if (used > 0 && hipMemcpyAsync(q, *p, used * sizeof(T), hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
      return fail(c, SONAR_ERR_DEVICE, "gallery copy failed");
    hipStreamSynchronize(c->stream);
    hipFree(*p);
  }
  *p = q;
  *cap = nc;
  return 0;
}

struct SeqRef { const double* p; int64_t n; };

SeqRef seq_of(const sonar_fp_features& f, int s) {
  switch (s) {
    case sonar::SEQ_CENTROID: return {f.spectral_centroid, f.n_spectral_centroid};
    case sonar::SEQ_ROLLOFF: return {f.spectral_rolloff, f.n_spectral_rolloff};
    case sonar::SEQ_FLUX: return {f.spectral_flux, f.n_spectral_flux};
    case sonar::SEQ_RMS: return {f.rms_energy, f.n_rms_energy};
    case sonar::SEQ_VOICING: return {f.voicing_probability, f.n_voicing_probability};
    case sonar::SEQ_HARMONIC: return {f.harmonic_ratio, f.n_harmonic_ratio};
    default: return {f.pitch_estimate, f.n_pitch_estimate};
  }
}

// a sequence is read only when its parent struct is non-nil (comparison.go:293, 309, 317, 325)
bool seq_used(const sonar_fp_features& f, int s) {
  const uint32_t need = s <= sonar::SEQ_FLUX ? SONAR_FEAT_SPECTRAL
                        : s == sonar::SEQ_RMS ? SONAR_FEAT_TEMPORAL
                        : s == sonar::SEQ_VOICING ? SONAR_FEAT_SPEECH : SONAR_FEAT_HARMONIC;
  return (f.present & SONAR_FEAT_FEATURES) && (f.present & need);
}

}  // namespace

extern "C" {

int sonar_gallery_create(sonar_ctx* c, sonar_gallery** out) {
  if (!c || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = new sonar_gallery();
  (*out)->c = c;
  return SONAR_OK;
}

void sonar_gallery_destroy(sonar_gallery* g) {
  if (!g) return;
  if (g->c) hipStreamSynchronize(g->c->stream);
  hipFree(g->recs);
  hipFree(g->pool);
  for (void* p : g->seqs) hipFree(p);
  delete g;
}

int64_t sonar_gallery_size(const sonar_gallery* g) { return g ? (int64_t)g->host.size() : 0; }

int sonar_gallery_add(sonar_gallery* g, const sonar_fp_features* fps, int32_t count, int32_t keep_sequences,
                      int32_t device_ptrs, int64_t* first) {
  if (!g) return SONAR_ERR_INVALID;
  sonar_ctx* c = g->c;
  if (count < 0 || (count > 0 && !fps)) return fail(c, SONAR_ERR_INVALID, "invalid fingerprint list");
  const int64_t base = (int64_t)g->host.size();
  if (first) *first = base;
  if (count == 0) return SONAR_OK;
  // ---- validate, size the pool and the staging area ----------------------------------
  int64_t pool_need = 0, stage = 0;
  for (int i = 0; i < count; i++) {
    const sonar_fp_features& f = fps[i];
    if (f.mfcc_frames < 0 || f.mfcc_coeffs < 0 || f.chroma_frames < 0 || f.chroma_bins < 0)
      return fail(c, SONAR_ERR_INVALID, "negative feature size");
    const bool feat = f.present & SONAR_FEAT_FEATURES;
    if (feat && (f.present & SONAR_FEAT_MFCC) && f.mfcc_frames > 0 && f.mfcc_coeffs > 0) {
      if (!f.mfcc) return fail(c, SONAR_ERR_INVALID, "mfcc pointer is null");
      pool_need += 2 * (int64_t)f.mfcc_coeffs;
      stage += f.mfcc_frames * f.mfcc_coeffs;
    }
    if (feat && (f.present & SONAR_FEAT_CHROMA) && f.chroma_frames > 0 && f.chroma_bins > 0) {
      if (!f.chroma) return fail(c, SONAR_ERR_INVALID, "chroma pointer is null");
      pool_need += f.chroma_bins;
      stage += f.chroma_frames * f.chroma_bins;
    }
    for (int s = 0; s < sonar::SEQ_COUNT; s++) {
      const SeqRef q = seq_of(f, s);
      if (!seq_used(f, s) || q.n <= 0) continue;
      if (!q.p) return fail(c, SONAR_ERR_INVALID, "sequence pointer is null");
      stage += q.n;
    }
  }
  int rc;
  if ((rc = grow(c, &g->recs, &g->cap, base, base + count))) return rc;
  if ((rc = grow(c, &g->pool, &g->pool_cap, g->pool_used, g->pool_used + pool_need))) return rc;
  hipStream_t s = c->stream;
  double* st = nullptr;
  if (!device_ptrs && stage > 0) {
    st = static_cast<double*>(dbuf(c, "cmp.stage", stage * sizeof(double)));
    if (!st) return fail(c, SONAR_ERR_NOMEM, "staging allocation failed");
  }
  int64_t st_used = 0;
  auto on_device = [&](const double* p, int64_t n) -> const double* {   // H2D into staging
    if (device_ptrs) return p;
    double* d = st + st_used;
    st_used += n;
    if (hipMemcpyAsync(d, p, n * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess) return nullptr;
    return d;
  };
  // ---- records and statistics jobs ---------------------------------------------------
  std::vector<FpRec> recs(count);
  std::vector<StatJob> jobs;
  for (int i = 0; i < count; i++) {
    const sonar_fp_features& f = fps[i];
    FpRec& r = recs[i];
    std::memset(&r, 0, sizeof(r));
    r.id = f.id;
    r.present = f.present;
    r.ct = f.content_type;
    r.duration = f.duration_seconds;
    effective_weights(f, r.w);
    const bool feat = f.present & SONAR_FEAT_FEATURES;
    // a nil MFCC / ChromaFeatures slice has no rows
    r.mfcc_frames = feat && (f.present & SONAR_FEAT_MFCC) ? f.mfcc_frames : 0;
    r.mfcc_C = r.mfcc_frames > 0 ? f.mfcc_coeffs : 0;
    r.chroma_frames = feat && (f.present & SONAR_FEAT_CHROMA) ? f.chroma_frames : 0;
    r.chroma_B = r.chroma_frames > 0 ? f.chroma_bins : 0;
    r.dynamic_range = f.dynamic_range;
    r.silence_ratio = f.silence_ratio;
    r.onset_density = f.onset_density;
    r.speech_rate = f.speech_rate;
    r.vtl = f.vocal_tract_length;
    FpRec* dr = g->recs + base + i;
    if (r.mfcc_C > 0) {
      r.mfcc_off = g->pool_used;
      g->pool_used += 2 * (int64_t)r.mfcc_C;
      const double* src = on_device(f.mfcc, f.mfcc_frames * f.mfcc_coeffs);
      if (!src) return fail(c, SONAR_ERR_DEVICE, "mfcc upload failed");
      jobs.push_back({src, f.mfcc_frames, r.mfcc_C, 0, 0, 0, g->pool + r.mfcc_off, g->pool + r.mfcc_off + r.mfcc_C});
    }
    if (r.chroma_B > 0) {
      r.chroma_off = g->pool_used;
      g->pool_used += r.chroma_B;
      const double* src = on_device(f.chroma, f.chroma_frames * f.chroma_bins);
      if (!src) return fail(c, SONAR_ERR_DEVICE, "chroma upload failed");
      jobs.push_back({src, f.chroma_frames, r.chroma_B, 0, 0, 0, g->pool + r.chroma_off, nullptr});
    }
    for (int q = 0; q < sonar::SEQ_COUNT; q++) {
      r.seq_mean[q] = r.seq_std[q] = kNaN;
      const SeqRef sq = seq_of(f, q);
      if (!seq_used(f, q) || sq.n <= 0) continue;
      r.seq_len[q] = sq.n;
      const double* src = nullptr;
      if (keep_sequences && (q == sonar::SEQ_CENTROID || q == sonar::SEQ_ROLLOFF)) {
        double* keep = nullptr;
        if (hipMalloc(&keep, sq.n * sizeof(double)) != hipSuccess)
          return fail(c, SONAR_ERR_NOMEM, "sequence allocation failed");
        g->seqs.push_back(keep);
        if (hipMemcpyAsync(keep, sq.p, sq.n * sizeof(double),
                           device_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s) != hipSuccess)
          return fail(c, SONAR_ERR_DEVICE, "sequence copy failed");
        (q == sonar::SEQ_CENTROID ? r.centroid : r.rolloff) = keep;
        src = keep;
      } else {
        src = on_device(sq.p, sq.n);
        if (!src) return fail(c, SONAR_ERR_DEVICE, "sequence upload failed");
      }
      jobs.push_back({src, sq.n, 1, 0, 0, 0, &dr->seq_mean[q], &dr->seq_std[q]});
    }
  }
  // NaN placeholders of the statistics are overwritten by the jobs below
  HIP_TRY(c, hipMemcpyAsync(g->recs + base, recs.data(), count * sizeof(FpRec), hipMemcpyHostToDevice, s));
  std::vector<int> chunk_job, chunk_k;
  int64_t parts = 0;
  for (size_t j = 0; j < jobs.size(); j++) {
    StatJob& J = jobs[j];
    J.chunk_rows = sonar::colstats_chunk_rows_for(J.cols);
    const int64_t nch = (J.rows + J.chunk_rows - 1) / J.chunk_rows;
    if (nch > 0x7fffffff) return fail(c, SONAR_ERR_UNSUPPORTED, "feature matrix too large");
    J.nchunks = (int32_t)nch;
    J.part_off = parts;
    parts += nch * J.cols;
    for (int64_t k = 0; k < nch; k++) { chunk_job.push_back((int)j); chunk_k.push_back((int)k); }
  }
  if (!jobs.empty()) {
    const size_t jb = jobs.size() * sizeof(StatJob), cb = chunk_job.size() * sizeof(int);
    char* meta = static_cast<char*>(dbuf(c, "cmp.jobs", jb + 2 * cb + 64));
    double* part = static_cast<double*>(dbuf(c, "cmp.part", 2 * parts * sizeof(double)));
    if (!meta || !part) return fail(c, SONAR_ERR_NOMEM, "statistics allocation failed");
    StatJob* djobs = reinterpret_cast<StatJob*>(meta);
    int* dcj = reinterpret_cast<int*>(meta + ((jb + 15) & ~size_t(15)));
    int* dck = dcj + chunk_job.size();
    HIP_TRY(c, hipMemcpyAsync(djobs, jobs.data(), jb, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(dcj, chunk_job.data(), cb, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(dck, chunk_k.data(), cb, hipMemcpyHostToDevice, s));
    hipEvent_t tend = sonar::detail::timed_begin(c, s);
    if (sonar::launch_colstats(djobs, (int)jobs.size(), dcj, dck, (int)chunk_job.size(), part, part + parts, s))
      return fail(c, SONAR_ERR_DEVICE, "colstats launch failed");
    sonar::detail::timed_end(c, s, tend);
  }
  HIP_TRY(c, hipStreamSynchronize(s));   // staging and the host job list are reused next call
  // host mirror with the device statistics (checks and diagnostics)
  std::vector<FpRec> back(count);
  HIP_TRY(c, hipMemcpy(back.data(), g->recs + base, count * sizeof(FpRec), hipMemcpyDeviceToHost));
  g->host.insert(g->host.end(), back.begin(), back.end());
  return SONAR_OK;
}

static int compare_core(sonar_gallery* g, const int64_t* queries, int64_t nq, const int64_t* candidates,
                        int64_t* nc_io, const sonar_compare_cfg* cfg, sonar_similarity** dout) {
  sonar_ctx* c = g->c;
  const int64_t size = (int64_t)g->host.size();
  if (!cfg || nq < 0 || (nq > 0 && !queries)) return fail(c, SONAR_ERR_INVALID, "invalid arguments");
  int64_t nc = candidates ? *nc_io : size;
  *nc_io = nc;
  if (nc < 0) return fail(c, SONAR_ERR_INVALID, "invalid candidate count");
  for (int64_t i = 0; i < nq; i++)
    if (queries[i] < 0 || queries[i] >= size) return fail(c, SONAR_ERR_INVALID, "query index out of range");
  if (candidates)
    for (int64_t i = 0; i < nc; i++)
      if (candidates[i] < 0 || candidates[i] >= size)
        return fail(c, SONAR_ERR_INVALID, "candidate index out of range");
  const int64_t n = nq * nc;
  hipStream_t s = c->stream;
  if (cfg->enable_detailed_metrics) {
    // calculateQualityMetrics dereferences Features (panics when nil); stat.Correlation
    // panics on a length mismatch (comparison.go:899, 989, 997)
    for (int64_t a = 0; a < nq; a++) {
      const FpRec& A = g->host[queries[a]];
      for (int64_t b = 0; b < nc; b++) {
        const FpRec& B = g->host[candidates ? candidates[b] : b];
        if (!(A.present & B.present & SONAR_FEAT_FEATURES))
          return fail(c, SONAR_ERR_INVALID, "features cannot be nil (detailed metrics)");
        if (!(A.present & B.present & SONAR_FEAT_SPECTRAL)) continue;
        for (int q = sonar::SEQ_CENTROID; q <= sonar::SEQ_ROLLOFF; q++) {
          if (A.seq_len[q] == 0 || B.seq_len[q] == 0) continue;
          if (A.seq_len[q] != B.seq_len[q]) return fail(c, SONAR_ERR_INVALID, "stat: slice length mismatch");
          const bool kept = q == sonar::SEQ_CENTROID ? (A.centroid && B.centroid) : (A.rolloff && B.rolloff);
          if (!kept) return fail(c, SONAR_ERR_INVALID, "detailed metrics need keep_sequences in sonar_gallery_add");
        }
      }
    }
  }
  const size_t ib = (size_t)(nq + (candidates ? nc : 0)) * sizeof(int64_t);
  int64_t* didx = static_cast<int64_t*>(dbuf(c, "cmp.idx", ib));
  sonar_similarity* out = static_cast<sonar_similarity*>(dbuf(c, "cmp.out", n * sizeof(sonar_similarity)));
  double* coh = cfg->enable_detailed_metrics ? static_cast<double*>(dbuf(c, "cmp.coh", 2 * n * sizeof(double)))
                                             : nullptr;
  if (!didx || !out || (cfg->enable_detailed_metrics && !coh)) return fail(c, SONAR_ERR_NOMEM, "allocation failed");
  HIP_TRY(c, hipMemcpyAsync(didx, queries, nq * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (candidates) HIP_TRY(c, hipMemcpyAsync(didx + nq, candidates, nc * sizeof(int64_t), hipMemcpyHostToDevice, s));
  const int64_t* dc = candidates ? didx + nq : nullptr;
  if (coh && sonar::launch_coherence(g->recs, didx, nq, dc, nc, coh, s))
    return fail(c, SONAR_ERR_DEVICE, "coherence launch failed");
  sonar::CompareArgs a;
  a.recs = g->recs;
  a.pool = g->pool;
  a.q_idx = didx;
  a.c_idx = dc;
  a.nq = nq;
  a.nc = nc;
  a.coh = coh;
  a.detailed = cfg->enable_detailed_metrics != 0;
  a.content_filter = cfg->enable_content_filter != 0;
  a.out = out;
  hipEvent_t tend = sonar::detail::timed_begin(c, s);
  if (sonar::launch_compare(a, s)) return fail(c, SONAR_ERR_DEVICE, "compare launch failed");
  sonar::detail::timed_end(c, s, tend);
  *dout = out;
  return SONAR_OK;
}

int sonar_compare(sonar_gallery* g, const int64_t* queries, int64_t nq, const int64_t* candidates, int64_t nc,
                  const sonar_compare_cfg* cfg, sonar_similarity* out, int32_t device_ptrs) {
  if (!g) return SONAR_ERR_INVALID;
  sonar_ctx* c = g->c;
  sonar_similarity* d = nullptr;
  int rc = compare_core(g, queries, nq, candidates, &nc, cfg, &d);
  if (rc) return rc;
  const size_t bytes = (size_t)(nq * nc) * sizeof(sonar_similarity);
  if (bytes == 0) return SONAR_OK;
  if (!out) return fail(c, SONAR_ERR_INVALID, "out is null");
  if (device_ptrs) {
    HIP_TRY(c, hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToDevice, c->stream));
  } else {
    HIP_TRY(c, hipMemcpyAsync(out, d, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  return SONAR_OK;
}

int sonar_find_best_matches(sonar_gallery* g, const int64_t* queries, int64_t nq, const int64_t* candidates,
                            int64_t nc, const sonar_compare_cfg* cfg, sonar_match* out, int64_t* n_matches) {
  if (!g) return SONAR_ERR_INVALID;
  sonar_ctx* c = g->c;
  if (!cfg) return fail(c, SONAR_ERR_INVALID, "cfg is null");
  if (cfg->max_candidates < 0)   // matches[:maxResults] with a negative bound panics in Go
    return fail(c, SONAR_ERR_INVALID, "max candidates must not be negative");
  if (nq > 0 && !n_matches) return fail(c, SONAR_ERR_INVALID, "n_matches is null");
  sonar_similarity* sims = nullptr;
  int rc = compare_core(g, queries, nq, candidates, &nc, cfg, &sims);
  if (rc) return rc;
  const int64_t n = nq * nc, K = cfg->max_candidates;
  if (n > 0x7fffffff) return fail(c, SONAR_ERR_UNSUPPORTED, "too many pairs for one call");
  hipStream_t s = c->stream;
  char* w = static_cast<char*>(dbuf(c, "cmp.match", (size_t)n * 49 + nq * 8 + 256));
  if (!w) return fail(c, SONAR_ERR_NOMEM, "allocation failed");
  double* keys = reinterpret_cast<double*>(w);
  double* keys2 = keys + n;
  int64_t* vals = reinterpret_cast<int64_t*>(keys2 + n);
  int64_t* vals2 = vals + n;
  int64_t* vals3 = vals2 + n;
  int32_t* qk = reinterpret_cast<int32_t*>(vals3 + n);
  int32_t* qk2 = qk + n;
  int64_t* counts = reinterpret_cast<int64_t*>(qk2 + n + (n & 1));
  uint8_t* pass = reinterpret_cast<uint8_t*>(counts + nq);
  if (sonar::launch_match_keys(sims, nq, nc, cfg->similarity_threshold, keys, vals, pass, counts, s))
    return fail(c, SONAR_ERR_DEVICE, "match key launch failed");
  if (n > 0) {
    size_t tb = 0;
    if (sonar::sort_match_keys(keys, keys2, vals, vals2, vals3, qk, qk2, nq, nc, nullptr, &tb, s))
      return fail(c, SONAR_ERR_DEVICE, "sort sizing failed");
    void* tmp = dbuf(c, "cmp.sorttmp", tb);
    if (!tmp) return fail(c, SONAR_ERR_NOMEM, "allocation failed");
    if (sonar::sort_match_keys(keys, keys2, vals, vals2, vals3, qk, qk2, nq, nc, tmp, &tb, s))
      return fail(c, SONAR_ERR_DEVICE, "sort failed");
  }
  std::vector<int64_t> cnt(nq);
  if (nq > 0) HIP_TRY(c, hipMemcpyAsync(cnt.data(), counts, nq * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  if (K > 0 && nq > 0) {
    sonar_match* dm = static_cast<sonar_match*>(dbuf(c, "cmp.matches", (size_t)(nq * K) * sizeof(sonar_match)));
    if (!dm) return fail(c, SONAR_ERR_NOMEM, "allocation failed");
    HIP_TRY(c, hipMemsetAsync(dm, 0, (size_t)(nq * K) * sizeof(sonar_match), s));
    if (sonar::launch_match_gather(sims, vals3, counts, nq, nc, (int)K, dm, s))
      return fail(c, SONAR_ERR_DEVICE, "gather launch failed");
    if (!out) return fail(c, SONAR_ERR_INVALID, "out is null");
    HIP_TRY(c, hipMemcpyAsync(out, dm, (size_t)(nq * K) * sizeof(sonar_match), hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  for (int64_t q = 0; q < nq; q++) n_matches[q] = std::min<int64_t>(cnt[q], K);
  return SONAR_OK;
}

// FindBestMatches over candidates split across ranks (comparison.go:197-263): the single call's
// order is similarity descending -- in the radix order of its device sort, i.e. the doubles'
// order-preserving 64-bit keys -- with ties in candidate order; a rank's top max_candidates hold
// every match of the global top max_candidates that lies in that rank, so merging the per-rank
// lists under the same order (candidates renumbered by their rank's base) is exact.
int sonar_merge_matches(const sonar_match* const* lists, const int64_t* counts, const int64_t* cand_base,
                        int32_t nlists, int64_t nq, int32_t max_candidates, sonar_match* out, int64_t* n_out) {
  if (nlists < 0 || nq < 0 || max_candidates < 0) return SONAR_ERR_INVALID;
  if (nq > 0 && (!n_out || (nlists > 0 && (!lists || !counts || !cand_base)))) return SONAR_ERR_INVALID;
  const int64_t K = max_candidates;
  if (K > 0 && nq > 0 && !out) return SONAR_ERR_INVALID;
  auto key = [](double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return (u >> 63) ? ~u : (u | (uint64_t(1) << 63));
  };
  struct Item { uint64_t k; int64_t cand; const sonar_match* m; };
  std::vector<Item> items;
  for (int64_t q = 0; q < nq; ++q) {
    items.clear();
    for (int32_t r = 0; r < nlists; ++r) {
      const int64_t cnt = std::min<int64_t>(counts[(int64_t)r * nq + q], K);
      for (int64_t k = 0; k < cnt; ++k) {
        const sonar_match* m = lists[r] + q * K + k;
        items.push_back({key(m->similarity.overall_similarity), cand_base[r] + m->candidate, m});
      }
    }
    std::sort(items.begin(), items.end(), [](const Item& a, const Item& b) {
      return a.k != b.k ? a.k > b.k : a.cand < b.cand;
    });
    const int64_t take = std::min<int64_t>((int64_t)items.size(), K);
    for (int64_t k = 0; k < take; ++k) {
      sonar_match m = *items[k].m;
      m.candidate = items[k].cand;
      m.rank = (int32_t)(k + 1);
      out[q * K + k] = m;
    }
    n_out[q] = take;
  }
  return SONAR_OK;
}

}  // extern "C"
