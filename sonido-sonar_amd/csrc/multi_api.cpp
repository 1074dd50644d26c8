// multi_api.cpp -- many stream pairs on one device, and one process driving several GPUs
// (SURVEY.md 8(e)).
//
//  sonar_align_pairs        the C5 unit (sonar_align_pair_device) over many pairs: worker
//                           contexts on the caller's device, one HIP stream + host thread each,
//                           taking pairs in order (pairs are independent; the per-pair kernels are
//                           latency-bound, so concurrent streams keep the GPU busy)
//  sonar_multi_*            a context per device and one RCCL communicator over them
//                           (ncclCommInitAll: collectives over xGMI, no MPI/torchrun needed)
//  sonar_fingerprint_multi  path A frame-sharded: frames [gF/G, (g+1)F/G) on device g from its
//                           sample slice (+ the W-H halo); rows land straight in the host arrays
//  sonar_fingerprint_multi_gather
//                           the same from device-resident slices, the MFCC timeline
//                           all-gathered over RCCL into every device
//  sonar_align_pairs_multi  contiguous pair ranges per device, records all-gathered over RCCL
//
// The reference is single-process Go with no GPU; these entries are the MI355X-side scaling of
// the same functions (fingerprint/fingerprint.go:137, extractors/alignment.go:139), and results
// equal the single-device calls (frames and pairs are independent).
#include "../../include/sonar_gpu.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "ctx.h"
#include "kernels.h"

using sonar::detail::dbuf;
using sonar::detail::fail;

struct sonar_multi {
  std::vector<int> dev;
  std::vector<sonar_ctx*> ctx;
  std::vector<ncclComm_t> comm;
  std::string err;
};

namespace {

int mfail(sonar_multi* m, int code, const std::string& msg) {
  if (m) m->err = msg;
  return code;
}

double scalar_of(const sonar_result* r, const char* name) {
  const double* d = nullptr;
  int64_t rows = 0, cols = 0;
  if (sonar_result_get(r, name, &d, &rows, &cols) != SONAR_OK || !d || rows * cols < 1) return NAN;
  return d[0];
}

// worker contexts of sonar_align_pairs, created once per parent context and kept
std::vector<sonar_ctx*>& workers_of(sonar_ctx* c, int n, int* rc) {
  *rc = SONAR_OK;
  while ((int)c->workers.size() < n) {
    sonar_ctx* w = nullptr;
    const int r = sonar_create(c->device, &w);
    if (r != SONAR_OK) { *rc = r; break; }
    c->workers.push_back(w);
  }
  return c->workers;
}

int align_one(sonar_ctx* w, const double* q, int64_t nq, const double* r, int64_t nr, int32_t sr, int32_t sw,
              int32_t hop, int32_t fw, double max_lag, int32_t device_ptrs, sonar_pair_record* out) {
  std::memset(out, 0, sizeof(*out));
  out->temporal_offset = out->offset_confidence = out->alignment_similarity = out->alignment_quality = NAN;
  out->method = out->corr_offset_seconds = out->dtw_distance = out->peak_lag = NAN;
  const double *dq = q, *dr = r;
  if (!device_ptrs) {
    if (!q || !r || nq <= 0 || nr <= 0) return out->status = fail(w, SONAR_ERR_EMPTY, "empty signal");
    double* bq = (double*)dbuf(w, "pairs.q", (size_t)nq * 8);
    double* br = (double*)dbuf(w, "pairs.r", (size_t)nr * 8);
    if (!bq || !br) return out->status = fail(w, SONAR_ERR_NOMEM, "device allocation failed");
    if (hipSetDevice(w->device) != hipSuccess ||
        hipMemcpyAsync(bq, q, (size_t)nq * 8, hipMemcpyHostToDevice, w->stream) != hipSuccess ||
        hipMemcpyAsync(br, r, (size_t)nr * 8, hipMemcpyHostToDevice, w->stream) != hipSuccess)
      return out->status = fail(w, SONAR_ERR_DEVICE, "pair upload failed");
    dq = bq; dr = br;
  }
  sonar_result* res = nullptr;
  const int rc = sonar_align_pair_device(w, dq, nq, dr, nr, sr, sw, hop, fw, max_lag, &res);
  out->status = rc;
  if (rc != SONAR_OK) return rc;
  out->temporal_offset = scalar_of(res, "temporal_offset");
  out->offset_confidence = scalar_of(res, "offset_confidence");
  out->alignment_similarity = scalar_of(res, "alignment_similarity");
  out->alignment_quality = scalar_of(res, "alignment_quality");
  out->method = scalar_of(res, "method");
  out->corr_offset_seconds = scalar_of(res, "corr_offset_seconds");
  out->dtw_distance = scalar_of(res, "dtw_distance");
  out->peak_lag = scalar_of(res, "peak_lag");
  sonar_result_free(res);
  return SONAR_OK;
}

int elt_size(int32_t dtype) { return dtype == SONAR_F32 ? 4 : 8; }

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct PairGeo {
  int64_t k = 0, nq = 0, nr = 0, Fq = 0, Fr = 0, Eq = 0, Er = 0, L = 0, mlf = 0, cap = 0;
  bool corr = false;
  sonar::DtwGeom g{};
  size_t chroma = 0, ck = 0, runs = 0, dn = 0, e = 0, codes = 0, wst = 0, path = 0, corr_off = 0;   // region offsets
};

// device bytes one pair of a batch holds (chroma, the DTW stores, the path)
size_t pair_bytes(const PairGeo& p) {
  return al256((size_t)(p.Fq + p.Fr) * 96) +
         al256(sonar::dtw_ck_bytes(p.g)) + al256((size_t)sonar::dtw_run_words(p.g) * 4) + al256(sonar::dtw_dn_bytes(p.g)) +
         al256(sonar::dtw_edge_bytes(p.g)) + al256((size_t)((p.cap + 1023) / 1024) * 256) +
         al256((size_t)((p.cap + 15) / 16 + 1) * 8) + al256((size_t)p.cap * 16) + al256((size_t)(2 * p.L + 1) * 8) +
         // batched features (feat_batch): pre-emphasised signals, DC scratch, energies, NCC inputs
         al256((size_t)p.nq * 8) + al256((size_t)p.nr * 8) + al256(sonar::dc_preemph_scratch_bytes(p.nq)) +
         al256(sonar::dc_preemph_scratch_bytes(p.nr)) + 2 * al256((size_t)(p.Eq + p.Er + 2) * 8) + 256;
}

// SONAR_FEAT_BATCH=0: the pair-by-pair feature launches inside a batch (A/B)
bool feat_batch_enabled() {
  const char* e = std::getenv("SONAR_FEAT_BATCH");
  return !(e && e[0] == '0');
}

// The batch's music features (music.go:245-376 per signal: DC removal + pre-emphasis, energy,
// chroma) and energy NCCs (correlation.go:131-409 per pair) in eight launches instead of
// 13 per pair: per-signal and per-pair regions of the worker's scratch, job tables staged through
// pinned memory.  Each signal / pair runs the same kernels' arithmetic in the same order as the
// per-pair path, so the outputs are bit-identical.  Under C5 the per-pair launches were the
// stream's serial phase: each small latency-bound kernel also waited for room beside the other
// streams' DTW waves (r03 kernel trace: ~65 % of every worker stream's time in feature kernels).
// Returns false (nothing launched) when the batch does not fit: signals of different chroma frame
// sizes or outside the batched kernels' shapes; on an allocation failure it also sets w->err to
// "batch features: ..." (the caller's NOMEM retry path).
bool feat_batch(sonar_ctx* w, const std::vector<PairGeo>& pg, int32_t sr, int32_t sw, int32_t hop, int32_t fw,
                const double* const* q_pcm, const double* const* r_pcm, char* chroma, char* corr, hipStream_t s,
                bool dry = false) {
  w->err.clear();
  if (!feat_batch_enabled() || pg.empty() || fw <= 0 || hop <= 0) return false;
  const int n = (int)pg.size();
  int fs = -1;
  size_t ysz = 0, dsz = 0, esz = 0, xsz = 0;
  int ncorr = 0;
  for (const auto& p : pg) {
    for (int side = 0; side < 2; ++side) {
      const int64_t ns = side ? p.nr : p.nq, F = side ? p.Fr : p.Fq;
      const int f = (int)(ns / F);                                    // music.go:331
      if (fs < 0) fs = f;
      if (f != fs) return false;
      ysz += al256((size_t)ns * 8);
      dsz += al256((size_t)sonar::dc_preemph_scratch_bytes(ns));
      esz += al256((size_t)std::max<int64_t>(side ? p.Er : p.Eq, 1) * 8);
    }
    if (p.corr) { xsz += al256((size_t)(p.Eq + p.Er) * 8) + 256; ++ncorr; }
  }
  if (fs != 256 && fs != 512) return false;
  const sonar_ctx::ChromaT* ct = sonar::detail::chroma_tables_for(w, fs, sr);
  char* y = (char*)dbuf(w, "fb.y", ysz);
  char* dcs = (char*)dbuf(w, "fb.dc", dsz);
  char* en = (char*)dbuf(w, "fb.energy", esz);
  char* nx = (char*)dbuf(w, "fb.ncc", std::max<size_t>(xsz, 256));
  const size_t jb = al256((size_t)2 * n * sizeof(sonar::MfJob)), nb = al256((size_t)std::max(ncorr, 1) * sizeof(sonar::NccJob));
  char* dj = (char*)dbuf(w, "fb.jobs", jb + nb);
  char* hj = (char*)sonar::detail::hbuf(w, "fb.hjobs", jb + nb);
  if (!ct || !y || !dcs || !en || !nx || !dj || !hj) {
    fail(w, SONAR_ERR_NOMEM, "batch features: allocation failed");
    return false;
  }
  if (dry) return true;                          // buffers reserved, nothing launched
  auto* mj = (sonar::MfJob*)hj;
  auto* nj = (sonar::NccJob*)(hj + jb);
  size_t yo = 0, doff = 0, eo = 0, xo = 0;
  int k = 0, m = 0;
  for (const auto& p : pg) {
    double* e2[2];
    for (int side = 0; side < 2; ++side) {
      const int64_t ns = side ? p.nr : p.nq;
      sonar::MfJob& j = mj[k++];
      j.x = side ? r_pcm[p.k] : q_pcm[p.k];
      j.n = ns;
      j.y = (double*)(y + yo); yo += al256((size_t)ns * 8);
      j.T = sonar::dc_chunks(ns);
      j.ends = (double*)(dcs + doff);
      j.ystart = j.ends + j.T;
      doff += al256((size_t)sonar::dc_preemph_scratch_bytes(ns));
      j.Fe = side ? p.Er : p.Eq;
      j.energy = (double*)(en + eo); eo += al256((size_t)std::max<int64_t>(j.Fe, 1) * 8);
      j.F = side ? p.Fr : p.Fq;
      j.chroma = (double*)(chroma + p.chroma) + (side ? p.Fq * 12 : 0);
      e2[side] = j.energy;
    }
    if (p.corr) {
      sonar::NccJob& j = nj[m++];
      j.a = e2[0]; j.na = p.Eq; j.b = e2[1]; j.nb = p.Er; j.L = p.L;
      j.xa = (double*)(nx + xo);
      j.xb = j.xa + p.Eq;
      j.stats = (double*)(nx + xo + al256((size_t)(p.Eq + p.Er) * 8));
      xo += al256((size_t)(p.Eq + p.Er) * 8) + 256;
      j.corr = (double*)(corr + p.corr_off);
    }
  }
  (void)sw;
  if (hipMemcpyAsync(dj, hj, jb + nb, hipMemcpyHostToDevice, s) != hipSuccess) return false;
  if (sonar::launch_music_features_batch(mj, (const sonar::MfJob*)dj, 2 * n, fw, hop, fs, (const double*)ct->win,
                                         (const double*)ct->trig, (const int*)ct->cls, s) != 0)
    return false;
  if (ncorr && sonar::launch_ncc_batch(nj, (const sonar::NccJob*)(dj + jb), ncorr, s) != 0) return false;
  return true;
}

// A batch of pairs on worker w's stream with one host synchronisation: every pair's music
// features and energy NCC (batched launches, feat_batch), then ONE launch_dtw_batch over all their
// chroma DTWs, then the correlations, path arrays and status words in three copies.  Pairs to be
// redone on the single-pair path (align_one) are appended to `redo` with the record flag that says
// why: SONAR_PAIR_REDONE_NONFINITE (the chroma is not finite: the batch ran the finite-input
// kernel, the exact math.Min rules are on the single-pair path) or SONAR_PAIR_REDONE_TIMEOUT (the
// band pipeline timed out and the retry is on).  dry: reserve the buffers only.
int align_batch(sonar_ctx* w, const std::vector<PairGeo>& in, const double* const* q_pcm, const double* const* r_pcm,
                int32_t sr, int32_t sw, int32_t hop, int32_t fw, int32_t device_ptrs, bool retry_timeouts,
                sonar_pair_record* out, std::vector<std::pair<int64_t, int32_t>>* redo,
                std::vector<std::pair<int64_t, std::string>>* errs, bool dry = false) {
  const int n = (int)in.size();
  if (n == 0) return SONAR_OK;
  HIP_TRY(w, hipSetDevice(w->device));
  hipStream_t s = w->stream;
  std::vector<PairGeo> pg = in;
  size_t chroma_b = 0, ck_b = 0, runs_b = 0, dn_b = 0, e_b = 0, codes_b = 0, wst_b = 0, path_b = 0, corr_b = 0;
  int64_t maxE = 1, maxn = 1, max_cap = 1, total_bands = 0, maxnb = 0;
  for (auto& p : pg) {
    p.chroma = chroma_b; chroma_b += al256((size_t)(p.Fq + p.Fr) * 96);
    p.ck = ck_b; ck_b += al256(sonar::dtw_ck_bytes(p.g));
    p.runs = runs_b; runs_b += al256((size_t)sonar::dtw_run_words(p.g) * 4);
    p.dn = dn_b; dn_b += al256(sonar::dtw_dn_bytes(p.g));
    p.e = e_b; e_b += al256(sonar::dtw_edge_bytes(p.g));
    p.codes = codes_b; codes_b += al256((size_t)((p.cap + 1023) / 1024) * 256);
    p.wst = wst_b; wst_b += al256((size_t)((p.cap + 15) / 16 + 1) * 8);
    p.path = path_b; path_b += al256((size_t)p.cap * 16);
    p.corr_off = corr_b; corr_b += al256((size_t)(2 * p.L + 1) * 8);
    maxE = std::max({maxE, p.Eq, p.Er});
    maxn = std::max({maxn, p.nq, p.nr});
    max_cap = std::max(max_cap, p.cap);
    maxnb = std::max(maxnb, p.g.nb);
    total_bands += p.g.nb;   // band-kernel tickets
  }
  // small (device) and the head of h (pinned host) share one layout: per-pair status words + the
  // batch ticket, the per-pair band-kernel diagnostic records, then the DTW arguments, ticket
  // starts and the band-major ticket map
  const size_t stat_b = al256((size_t)n * 32 + 16), diag_b = al256((size_t)n * 8 * sonar::DTW_DIAG_WORDS),
               ps_b = al256((size_t)n * sizeof(sonar::host::PathSums)),
               cs_b = al256((size_t)n * sizeof(sonar::host::CorrSums)),
               args_b = al256((size_t)n * sizeof(sonar::DtwArgs)), start_b = al256((size_t)(n + 1) * 8),
               map_b = al256((size_t)total_bands * 8), sj_b = al256((size_t)n * sizeof(sonar::ScoreJob));
  char* chroma = (char*)dbuf(w, "pb.chroma", chroma_b);
  char* CK = (char*)dbuf(w, "pb.CK", ck_b);
  char* runs = (char*)dbuf(w, "pb.runs", runs_b);
  char* Dn = (char*)dbuf(w, "pb.Dn", dn_b);
  char* E = (char*)dbuf(w, "pb.E", e_b);
  char* codes = (char*)dbuf(w, "pb.codes", codes_b);
  char* wst = (char*)dbuf(w, "pb.wstart", wst_b);
  // small holds, in the pinned host buffer's layout: status words + ticket, diagnostic records, the
  // scorer reductions (PathSums, CorrSums), then DTW arguments, ticket starts, band-major map and
  // score jobs (one upload), correlations, paths -- so the batch's results come back in ONE copy of
  // the head (each runtime copy is a blit kernel that needs a CU beside the band blocks).  The
  // scorers' O(path) loops run on the device (pair_score_kernel); SONAR_PAIR_HOST_SCORES=1 (A/B,
  // tests) copies correlations and paths back instead and runs them on the host, as a
  // SONAR_PAIR_DUMP does.
  const size_t head_b = stat_b + diag_b + ps_b + cs_b, up_b = args_b + start_b + map_b + sj_b;
  const size_t small_b = head_b + up_b + corr_b + path_b;
  char* small = (char*)dbuf(w, "pb.small", small_b);
  char* corr = small ? small + (head_b + up_b) : nullptr;
  char* path = small ? corr + corr_b : nullptr;
  // SONAR_DTW_TRACE=<file> (diagnostics): every band's sweep timestamps (dtw_band_kernel's trace
  // words) appended to <file> as {pair, band, 8 trace words} records
  const char* trace_path = std::getenv("SONAR_DTW_TRACE");
  char* trb = trace_path ? (char*)dbuf(w, "pb.trace", (size_t)total_bands * 64) : nullptr;
  double* eq = (double*)dbuf(w, "pb.eq", (size_t)maxE * 8);
  double* er = (double*)dbuf(w, "pb.er", (size_t)maxE * 8);
  double* xa = (double*)dbuf(w, "ncc.xa", (size_t)maxE * 8);
  double* xb = (double*)dbuf(w, "ncc.xb", (size_t)maxE * 8);
  double* st = (double*)dbuf(w, "ncc.stats", 64);
  double* up_q = device_ptrs ? nullptr : (double*)dbuf(w, "pairs.q", (size_t)maxn * 8);
  double* up_r = device_ptrs ? nullptr : (double*)dbuf(w, "pairs.r", (size_t)maxn * 8);
  char* h = (char*)sonar::detail::hbuf(w, "pb.host", small_b);
  if (!chroma || !CK || !runs || !Dn || !E || !codes || !wst || !path || !corr || !small || !eq || !er || !xa || !xb ||
      !st || (!device_ptrs && (!up_q || !up_r)) || !h)
    return fail(w, SONAR_ERR_NOMEM, "allocation failed (pair batch)");
  if (dry) {   // reserve only (sonar_align_pairs' sizing pass): the batched-feature buffers too
    if (device_ptrs && !feat_batch(w, pg, sr, sw, hop, fw, q_pcm, r_pcm, chroma, corr, s, true) &&
        w->err.rfind("batch features:", 0) == 0)
      return SONAR_ERR_NOMEM;
    return SONAR_OK;
  }
  int32_t* dstat = (int32_t*)small;                 // per pair: [0..1] plen, [2..3] C[nq][nr], [4..7] sync
  int32_t* ticket = (int32_t*)(small + (size_t)n * 32);
  uint64_t* ddiag = (uint64_t*)(small + stat_b);
  auto* dps = (sonar::host::PathSums*)(small + stat_b + diag_b);
  auto* dcs = (sonar::host::CorrSums*)(small + stat_b + diag_b + ps_b);
  const size_t ab = head_b;                          // where the arguments start
  sonar::DtwArgs* dargs = (sonar::DtwArgs*)(small + ab);
  int64_t* dstart = (int64_t*)(small + ab + args_b);
  char* hstat = h;
  const uint64_t* hdiag = (const uint64_t*)(h + stat_b);
  const auto* hps = (const sonar::host::PathSums*)(h + stat_b + diag_b);
  const auto* hcs = (const sonar::host::CorrSums*)(h + stat_b + diag_b + ps_b);
  sonar::DtwArgs* hargs = (sonar::DtwArgs*)(h + ab);
  int64_t* hstart = (int64_t*)(h + ab + args_b);
  int2* hmap = (int2*)(h + ab + args_b + start_b);
  int2* dmap = (int2*)(small + ab + args_b + start_b);
  auto* hsj = (sonar::ScoreJob*)(h + ab + args_b + start_b + map_b);
  auto* dsj = (const sonar::ScoreJob*)(small + ab + args_b + start_b + map_b);
  char* hcorr = h + head_b + up_b;
  char* hpath = hcorr + corr_b;
  const char* dump_dir = std::getenv("SONAR_PAIR_DUMP");
  const char* hs_env = std::getenv("SONAR_PAIR_HOST_SCORES");
  const bool host_scores = dump_dir || (hs_env && std::atoi(hs_env) != 0);
  HIP_TRY(w, hipMemsetAsync(small, 0, stat_b + diag_b, s));
  // every pair's music features and energy NCC: batched launches over the whole batch when the
  // inputs are on the device and every signal fits the batched kernels (feat_batch), else pair by
  // pair on the worker's scratch
  const bool fb = device_ptrs && feat_batch(w, pg, sr, sw, hop, fw, q_pcm, r_pcm, chroma, corr, s);
  if (!fb && !w->err.empty() && w->err.rfind("batch features:", 0) == 0) return SONAR_ERR_NOMEM;
  int64_t acc = 0;
  for (int i = 0; i < n; ++i) {
    const PairGeo& p = pg[i];
    const double *dq = q_pcm[p.k], *dr = r_pcm[p.k];
    double* cq = (double*)(chroma + p.chroma);
    double* cr = cq + p.Fq * 12;
    if (!fb) {
      if (!device_ptrs) {
        HIP_TRY(w, hipMemcpyAsync(up_q, dq, (size_t)p.nq * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(w, hipMemcpyAsync(up_r, dr, (size_t)p.nr * 8, hipMemcpyHostToDevice, s));
        dq = up_q; dr = up_r;
      }
      int rc = sonar_music_alignment_features(w, dq, p.nq, sr, sw, hop, fw, hop, eq, cq, 1);
      if (rc == SONAR_OK) rc = sonar_music_alignment_features(w, dr, p.nr, sr, sw, hop, fw, hop, er, cr, 1);
      if (rc != SONAR_OK) return rc;
      if (p.corr && sonar::launch_ncc(eq, p.Eq, er, p.Er, p.L, xa, xb, st, (double*)(corr + p.corr_off), s) != 0)
        return fail(w, SONAR_ERR_DEVICE, "ncc launch failed");
    }
    int32_t* sync = dstat + 8 * i + 4;
    sonar::DtwArgs& a = hargs[i];
    a = sonar::DtwArgs{};
    a.q = cq; a.r = cr; a.dim = 12; a.band = -1;
    a.nq = p.g.nq; a.nr = p.g.nr; a.nb = p.g.nb; a.S = p.g.S; a.SW = p.g.SW;
    a.Cn = nullptr; a.CK = (double*)(CK + p.ck); a.runs = (int32_t*)(runs + p.runs); a.Dn = (uint32_t*)(Dn + p.dn); a.E = (uint64_t*)(E + p.e); a.sync = sync;
    a.codes = (uint32_t*)(codes + p.codes); a.plen = (int64_t*)(dstat + 8 * i); a.wstart = (int2*)(wst + p.wst);
    a.pc = (double*)(path + p.path); a.pq = (int32_t*)(a.pc + p.cap); a.pr = a.pq + p.cap;
    a.cnm = (double*)(dstat + 8 * i + 2);
    a.diag = ddiag + (size_t)i * sonar::DTW_DIAG_WORDS;
    a.trace = trb ? (uint64_t*)(trb + (size_t)acc * 64) : nullptr;
    a.dbg_stall = sonar::dtw_dbg_stall_band(true);
    sonar::ScoreJob& sj = hsj[i];
    sj = sonar::ScoreJob{a.pq, a.pr, a.pc, a.plen, p.corr ? (const double*)(corr + p.corr_off) : nullptr,
                         2 * p.L + 1, dps + i, dcs + i};
    hstart[i] = acc;
    acc += p.g.nb;
  }
  hstart[n] = acc;
  // band-major tickets across the batch: band b of every DTW before band b+1 of any, so a block
  // waits about one hand-off for its predecessor band rather than b of them while holding its slot
  {
    int64_t t = 0;
    for (int64_t b = 0; b < maxnb; ++b)
      for (int i = 0; i < n; ++i)
        if (b < pg[i].g.nb) hmap[t++] = make_int2(i, (int)b);
  }
  HIP_TRY(w, hipMemcpyAsync(dargs, hargs, up_b, hipMemcpyHostToDevice, s));
  // the non-finite probe of every pair's chroma in one launch (flags in each pair's sync[2]); the
  // same launch fills every pair's band-edge rows E with the band kernel's sentinel
  int64_t max_el = 0;
  for (const auto& p : pg)
    max_el = std::max({max_el, (p.Fq + p.Fr) * 12, (int64_t)(sonar::dtw_edge_bytes(p.g) / 8)});
  if (sonar::launch_nonfinite_batch(dargs, n, max_el, s) != 0) return fail(w, SONAR_ERR_DEVICE, "dtw launch failed");
  if (sonar::launch_dtw_batch(hargs, dargs, dstart, n, total_bands, max_cap, ticket, s, dmap) != 0)
    return fail(w, SONAR_ERR_DEVICE, "dtw batch launch failed");
  if (!host_scores && sonar::launch_pair_scores(dsj, n, s) != 0) return fail(w, SONAR_ERR_DEVICE, "score launch failed");
  HIP_TRY(w, hipMemcpyAsync(hstat, small, host_scores ? small_b : head_b, hipMemcpyDeviceToHost, s));
  std::vector<uint64_t> htr(trb ? (size_t)total_bands * 8 : 0);
  if (trb) HIP_TRY(w, hipMemcpyAsync(htr.data(), trb, htr.size() * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(w, hipStreamSynchronize(s));
  if (trb) {
    static std::mutex trace_mu;
    std::lock_guard<std::mutex> lk(trace_mu);
    if (FILE* f = std::fopen(trace_path, "ab")) {
      for (int i = 0; i < n; ++i)
        for (int64_t b = 0; b < pg[i].g.nb; ++b) {
          const uint64_t hdr[2] = {(uint64_t)pg[i].k, (uint64_t)b};
          std::fwrite(hdr, 8, 2, f);
          std::fwrite(htr.data() + (size_t)(hstart[i] + b) * 8, 8, 8, f);
        }
      std::fclose(f);
    }
  }
  for (int i = 0; i < n; ++i) {
    const PairGeo& p = pg[i];
    const char* ps = hstat + (size_t)i * 32;
    int64_t P;
    double cnm;
    int32_t sync[4];
    std::memcpy(&P, ps, 8);
    std::memcpy(&cnm, ps + 8, 8);
    std::memcpy(sync, ps + 16, 16);
    sonar_pair_record* rec = &out[p.k];
    if (sync[2]) { redo->emplace_back(p.k, SONAR_PAIR_REDONE_NONFINITE); continue; }
    alignas(8) char sblk[sonar::DTW_SYNC_BYTES];
    std::memcpy(sblk, sync, 16);
    std::memcpy(sblk + 16, hdiag + (size_t)i * sonar::DTW_DIAG_WORDS, 8 * sonar::DTW_DIAG_WORDS);
    const std::string why = sonar::detail::dtw_status(w, sblk);
    if (!why.empty()) {
      if (retry_timeouts) {
        // the band pipeline of this pair timed out: redone once on the single-pair path (exact,
        // separately synchronised); the record carries SONAR_PAIR_REDONE_TIMEOUT and the timeout
        // stays counted in sonar_dtw_counters
        redo->emplace_back(p.k, SONAR_PAIR_REDONE_TIMEOUT);
        continue;
      }
      std::memset(rec, 0, sizeof(*rec));
      rec->status = fail(w, SONAR_ERR_DEVICE, why);
      errs->emplace_back(p.k, why);
      continue;
    }
    if (dump_dir) {
      // tests only: the batched DTW's raw outputs of pair k (path length, C[nq][nr], path costs,
      // query and reference indices) into <dump>/pair_<k>.bin, to be checked against the oracle
      const double* pc = (const double*)(hpath + p.path);
      const std::string fn = std::string(dump_dir) + "/pair_" + std::to_string(p.k) + ".bin";
      if (FILE* f = std::fopen(fn.c_str(), "wb")) {
        std::fwrite(&P, 8, 1, f);
        std::fwrite(&cnm, 8, 1, f);
        std::fwrite(pc, 8, (size_t)P, f);
        std::fwrite(pc + p.cap, 4, (size_t)P, f);
        std::fwrite((const int32_t*)(pc + p.cap) + p.cap, 4, (size_t)P, f);
        std::fclose(f);
      }
    }
    sonar::detail::AlignIn ai;
    ai.q_pcm_len = p.nq; ai.r_pcm_len = p.nr; ai.sample_rate = sr; ai.hop = hop;
    if (p.corr) {
      if (host_scores) ai.corr = (const double*)(hcorr + p.corr_off);
      else ai.corr_sums = hcs + i;
      ai.L = p.L; ai.nqe = p.Eq; ai.nre = p.Er; ai.mlf = p.mlf;
    }
    ai.has_dtw = true;
    if (host_scores) {
      const double* pc = (const double*)(hpath + p.path);
      ai.pc = pc; ai.pq = (const int32_t*)(pc + p.cap); ai.pr = ai.pq + p.cap;
    } else {
      ai.path_sums = hps + i;
    }
    ai.P = P; ai.nqc = p.Fq; ai.nrc = p.Fr; ai.dist = cnm / (double)P;   // dtw.go:88-91
    sonar::detail::align_finish(ai, nullptr, rec);
    rec->status = SONAR_OK;
    rec->flags = 0;
  }
  return SONAR_OK;
}

}  // namespace

extern "C" {

int sonar_align_pairs(sonar_ctx* c, int64_t npairs, const double* const* q_pcm, const int64_t* nq,
                      const double* const* r_pcm, const int64_t* nr, int32_t sample_rate, int32_t stft_window,
                      int32_t hop, int32_t feature_window, double max_lag_seconds, int32_t workers,
                      int32_t device_ptrs, sonar_pair_record* out) {
  if (!c) return SONAR_ERR_INVALID;
  if (npairs < 0 || (npairs > 0 && (!q_pcm || !nq || !r_pcm || !nr || !out)))
    return fail(c, SONAR_ERR_INVALID, "null pair arrays");
  if (npairs == 0) return SONAR_OK;
  const int64_t inflight = workers > 0 ? workers : 128;   // pairs in flight (measured: C5 rises to ~128)
  std::atomic<int> first_err{SONAR_OK};
  auto note = [&](int r, int64_t k, sonar_ctx* w) {
    if (r == SONAR_OK) return;
    int expect = SONAR_OK;
    if (first_err.compare_exchange_strong(expect, r)) c->err = std::string("pair ") + std::to_string(k) + ": " + w->err;
  };
  // SONAR_PAIR_BATCH=0: one pair at a time per worker stream (the unbatched path, for A/B)
  const char* bev = std::getenv("SONAR_PAIR_BATCH");
  const bool batched = !(bev && std::atoi(bev) == 0);
  const char* sev = std::getenv("SONAR_PAIR_STREAMS");
  const int nstreams = batched ? (int)std::max<int64_t>(1, std::min<int64_t>(sev ? std::atoi(sev) : 16, npairs))
                               : (int)std::min<int64_t>(std::min<int64_t>(inflight, 16), npairs);
  int rc = SONAR_OK;
  std::vector<sonar_ctx*>& ws = workers_of(c, nstreams, &rc);
  if (rc != SONAR_OK) return fail(c, rc, "worker context creation failed");
  std::vector<std::thread> th;
  if (!batched) {
    std::atomic<int64_t> next{0};
    for (int t = 0; t < nstreams; ++t) {
      th.emplace_back([&, t] {
        sonar_ctx* w = ws[t];
        for (int64_t k = next.fetch_add(1); k < npairs; k = next.fetch_add(1))
          note(align_one(w, q_pcm[k], nq[k], r_pcm[k], nr[k], sample_rate, stft_window, hop, feature_window,
                         max_lag_seconds, device_ptrs, &out[k]), k, w);
      });
    }
    for (auto& x : th) x.join();
    return first_err.load();
  }
  // batched: pairs validated and sized here; each stream takes batches of up to `per` pairs (the
  // in-flight count split over the streams), cut further by a device-memory budget
  const int64_t per = std::max<int64_t>(1, (inflight + nstreams - 1) / nstreams);
  const char* mev = std::getenv("SONAR_PAIR_BATCH_GB");
  size_t budget = (size_t)((mev ? std::atof(mev) : 24.0) * (1ull << 30));
  {   // every stream holds one batch: keep them within ~70 % of the device memory free now
    size_t fr = 0, tot = 0;
    if (hipSetDevice(c->device) == hipSuccess && hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 0)
      budget = std::min(budget, (size_t)(0.7 * (double)fr / (double)nstreams));
  }
  const int64_t max_lag_samples = (int64_t)(max_lag_seconds * (double)sample_rate);   // alignment.go:104
  std::vector<PairGeo> geo;
  for (int64_t k = 0; k < npairs; ++k) {
    sonar_pair_record* rec = &out[k];
    std::memset(rec, 0, sizeof(*rec));
    int st = SONAR_OK;
    PairGeo p;
    p.k = k; p.nq = nq[k]; p.nr = nr[k];
    if (!q_pcm[k] || !r_pcm[k] || p.nq <= 0 || p.nr <= 0) st = fail(c, SONAR_ERR_EMPTY, "empty signal");
    else if (stft_window <= 0 || hop <= 0) st = fail(c, SONAR_ERR_INVALID, "window and hop size must be positive");
    if (st == SONAR_OK) {
      p.Fq = sonar_stft_frames(p.nq, stft_window, hop);
      p.Fr = sonar_stft_frames(p.nr, stft_window, hop);
      if (p.Fq <= 0 || p.Fr <= 0) st = fail(c, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
      else if (p.Fq + p.Fr > (int64_t)INT32_MAX) st = fail(c, SONAR_ERR_UNSUPPORTED, "sequence too long");
    }
    if (st != SONAR_OK) { rec->status = st; note(st, k, c); continue; }
    p.Eq = sonar_energy_frames(p.nq, feature_window, hop);
    p.Er = sonar_energy_frames(p.nr, feature_window, hop);
    p.corr = p.Eq > 0 && p.Er > 0;
    if (p.corr) {
      p.mlf = std::min(max_lag_samples / hop, std::min(p.Eq, p.Er) - 1);
      p.L = std::max<int64_t>(0, std::min({p.mlf, p.Eq - 1, p.Er - 1}));
    }
    p.g = sonar::dtw_geom(p.Fq, p.Fr);
    p.cap = p.Fq + p.Fr + 1;
    geo.push_back(p);
  }
  std::vector<std::vector<PairGeo>> batches;
  for (size_t i = 0; i < geo.size();) {
    std::vector<PairGeo> b;
    size_t bytes = 0;
    while (i < geo.size() && (int64_t)b.size() < per && (b.empty() || bytes + pair_bytes(geo[i]) <= budget)) {
      bytes += pair_bytes(geo[i]);
      b.push_back(geo[i++]);
    }
    batches.push_back(std::move(b));
  }
  std::atomic<size_t> next{0};
  // SONAR_PAIR_RETRY=0: a pair whose band pipeline timed out is an error (the bench's setting);
  // default: it is redone once on the single-pair path and flagged SONAR_PAIR_REDONE_TIMEOUT
  const char* rtv = std::getenv("SONAR_PAIR_RETRY");
  const bool retry_timeouts = !(rtv && rtv[0] == '0');
  std::mutex rmu;
  std::condition_variable rcv;
  int rdone = 0;
  std::vector<std::vector<std::pair<int64_t, int32_t>>> redo(nstreams);
  std::vector<std::vector<std::pair<int64_t, std::string>>> errs(nstreams);
  for (int t = 0; t < nstreams; ++t) {
    th.emplace_back([&, t] {
      sonar_ctx* w = ws[t];
      // sizing pass: every worker reserves its buffers for the largest of all batches before any
      // worker launches, so no device or pinned allocation (which synchronises the device) happens
      // while other workers' band pipelines run
      for (const auto& b : batches)
        if (align_batch(w, b, q_pcm, r_pcm, sample_rate, stft_window, hop, feature_window, device_ptrs,
                        retry_timeouts, out, &redo[t], &errs[t], true) != SONAR_OK)
          break;                                   // NOMEM: the batch loop's retry path handles it
      // one small fill on the worker's stream: HIP gives a stream its hardware queue at its first
      // command, so every worker's queue exists before any worker's DTW pipeline runs
      if (hipSetDevice(w->device) == hipSuccess) {
        if (void* z = dbuf(w, "pb.touch", 256)) (void)hipMemsetAsync(z, 0, 256, w->stream);
        (void)hipStreamSynchronize(w->stream);
      }
      {
        std::unique_lock<std::mutex> lk(rmu);
        if (++rdone == nstreams) rcv.notify_all();
        else rcv.wait(lk, [&] { return rdone == nstreams; });
      }
      for (size_t bi = next.fetch_add(1); bi < batches.size(); bi = next.fetch_add(1)) {
        int r = align_batch(w, batches[bi], q_pcm, r_pcm, sample_rate, stft_window, hop, feature_window,
                            device_ptrs, retry_timeouts, out, &redo[t], &errs[t]);
        if (r == SONAR_ERR_NOMEM) {
          // the worker's cached buffers are sized by earlier batches, name by name: release them
          // and retry the batch once; then pair by pair on the unbatched path
          sonar::detail::trim_buffers(w);
          r = align_batch(w, batches[bi], q_pcm, r_pcm, sample_rate, stft_window, hop, feature_window, device_ptrs,
                          retry_timeouts, out, &redo[t], &errs[t]);
          if (r == SONAR_ERR_NOMEM) {
            sonar::detail::trim_buffers(w);
            r = SONAR_OK;
            for (const auto& p : batches[bi])
              note(align_one(w, q_pcm[p.k], nq[p.k], r_pcm[p.k], nr[p.k], sample_rate, stft_window, hop,
                             feature_window, max_lag_seconds, device_ptrs, &out[p.k]), p.k, w);
          }
        }
        if (r != SONAR_OK)
          for (const auto& p : batches[bi]) { out[p.k].status = r; note(r, p.k, w); }
      }
      for (const auto& [k, why] : redo[t]) {       // exact single-pair path, flagged in the record
        note(align_one(w, q_pcm[k], nq[k], r_pcm[k], nr[k], sample_rate, stft_window, hop, feature_window,
                       max_lag_seconds, device_ptrs, &out[k]), k, w);
        out[k].flags |= why;
      }
    });
  }
  for (auto& x : th) x.join();
  for (sonar_ctx* w : ws)                            // band-kernel liveness counters to the caller's ctx
    for (int k = 0; k < 4; ++k) { c->dtw_ctr[k] += w->dtw_ctr[k]; w->dtw_ctr[k] = 0; }
  // per-pair device failures (the band pipeline's diagnostic text), lowest pair first
  std::vector<std::pair<int64_t, std::string>> all;
  for (auto& e : errs) all.insert(all.end(), e.begin(), e.end());
  if (!all.empty() && first_err.load() == SONAR_OK) {
    std::sort(all.begin(), all.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    first_err = out[all[0].first].status;
    c->err = "pair " + std::to_string(all[0].first) + ": " + all[0].second;
    if (all.size() > 1) c->err += " (" + std::to_string(all.size() - 1) + " more pairs failed)";
  }
  return first_err.load();
}

int sonar_multi_shard(int64_t n, int32_t W, int32_t H, int32_t G, int32_t g, int64_t* f0, int64_t* f1, int64_t* s0,
                      int64_t* s1) {
  if (W <= 0 || H <= 0 || G <= 0 || g < 0 || g >= G || !f0 || !f1 || !s0 || !s1) return SONAR_ERR_INVALID;
  const int64_t F = sonar_stft_frames(n, W, H);
  if (F <= 0) return SONAR_ERR_TOO_SHORT;
  // every inner boundary even: a shard's frame pairs (mfcc_pair_kernel transforms frames 2p, 2p+1
  // as one complex FFT) are the unsharded call's pairs, so shards reassemble bit-identically
  auto edge = [&](int64_t k) { return k >= G ? F : ((F * k / G) & ~(int64_t)1); };
  *f0 = edge(g);
  *f1 = edge(g + 1);
  if (*f1 <= *f0) { *s0 = *s1 = (*f0) * H; return SONAR_OK; }
  *s0 = (*f0) * H;
  *s1 = std::min<int64_t>((*f1 - 1) * H + W, n);   // a lone frame of a signal shorter than W reads n samples
  return SONAR_OK;
}

int sonar_multi_create(const int32_t* devices, int32_t n, sonar_multi** out) {
  if (!out) return SONAR_ERR_INVALID;
  *out = nullptr;
  if (!devices || n <= 0) return SONAR_ERR_INVALID;
  auto* m = new sonar_multi();
  m->dev.assign(devices, devices + n);
  for (int g = 0; g < n; ++g) {
    sonar_ctx* c = nullptr;
    const int rc = sonar_create(devices[g], &c);
    if (rc != SONAR_OK) { sonar_multi_destroy(m); return rc; }
    m->ctx.push_back(c);
  }
  m->comm.resize(n);
  const ncclResult_t nr = ncclCommInitAll(m->comm.data(), n, m->dev.data());
  if (nr != ncclSuccess) {
    m->comm.clear();
    sonar_multi_destroy(m);
    return SONAR_ERR_DEVICE;
  }
  *out = m;
  return SONAR_OK;
}

void sonar_multi_destroy(sonar_multi* m) {
  if (!m) return;
  for (auto& cm : m->comm) if (cm) ncclCommDestroy(cm);
  for (auto* c : m->ctx) sonar_destroy(c);
  delete m;
}

const char* sonar_multi_last_error(const sonar_multi* m) { return m ? m->err.c_str() : "null multi"; }
int32_t sonar_multi_size(const sonar_multi* m) { return m ? (int32_t)m->ctx.size() : 0; }
sonar_ctx* sonar_multi_ctx(sonar_multi* m, int32_t rank) {
  return (m && rank >= 0 && rank < (int32_t)m->ctx.size()) ? m->ctx[rank] : nullptr;
}

int sonar_fingerprint_multi(sonar_multi* m, const void* pcm, int64_t n, const sonar_fp_cfg* cfg, sonar_fp_out* out) {
  if (!m || !cfg || !out) return mfail(m, SONAR_ERR_INVALID, "null argument");
  if (cfg->device_ptrs) return mfail(m, SONAR_ERR_INVALID, "sonar_fingerprint_multi takes host buffers");
  if (cfg->flags & (SONAR_FP_ZCR | SONAR_FP_ENERGY))
    return mfail(m, SONAR_ERR_UNSUPPORTED, "ZCR / energy read the pre-emphasised sample before a shard");
  if ((cfg->flags & SONAR_FP_SPECTRAL) && out->flux)
    return mfail(m, SONAR_ERR_UNSUPPORTED, "spectral flux of a shard's first frame needs the previous frame");
  if (!pcm || n <= 0) return mfail(m, SONAR_ERR_EMPTY, "empty signal");
  const int W = cfg->window_size, H = cfg->hop_size;
  if (W <= 0) return mfail(m, SONAR_ERR_INVALID, "window size must be positive");
  if (H <= 0) return mfail(m, SONAR_ERR_INVALID, "hop size must be positive");
  if (sonar_stft_frames(n, W, H) <= 0)
    return mfail(m, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
  const int G = (int)m->ctx.size();
  const size_t oe = elt_size(cfg->out_dtype), pe = elt_size(cfg->pcm_dtype);
  const size_t nm = cfg->n_mfcc > 0 ? cfg->n_mfcc : 13, K = (size_t)W / 2 + 1;
  std::vector<int> rcs(G, SONAR_OK);
  std::vector<std::thread> th;
  for (int g = 0; g < G; ++g) {
    th.emplace_back([&, g] {
      int64_t f0, f1, s0, s1;
      sonar_multi_shard(n, W, H, G, g, &f0, &f1, &s0, &s1);
      if (f1 <= f0) return;
      auto at = [&](void* base, size_t cols) -> void* {
        return base ? (void*)((char*)base + (size_t)f0 * cols * oe) : nullptr;
      };
      sonar_fp_out o{};
      o.mfcc = at(out->mfcc, nm);
      o.magnitude = at(out->magnitude, K);
      o.complex = at(out->complex, 2 * K);
      o.phase = at(out->phase, K);
      o.centroid = at(out->centroid, 1);
      o.rolloff = at(out->rolloff, 1);
      o.bandwidth = at(out->bandwidth, 1);
      o.flatness = at(out->flatness, 1);
      o.crest = at(out->crest, 1);
      o.slope = at(out->slope, 1);
      o.low_ratio = at(out->low_ratio, 1);
      o.high_ratio = at(out->high_ratio, 1);
      rcs[g] = sonar_fingerprint(m->ctx[g], (const char*)pcm + (size_t)s0 * pe, s1 - s0, cfg, &o);
    });
  }
  for (auto& x : th) x.join();
  for (int g = 0; g < G; ++g)
    if (rcs[g] != SONAR_OK) return mfail(m, rcs[g], "device " + std::to_string(m->dev[g]) + ": " + m->ctx[g]->err);
  return SONAR_OK;
}

int sonar_fingerprint_multi_gather(sonar_multi* m, const void* const* pcm_dev, int64_t n, const sonar_fp_cfg* cfg,
                                   void* const* mfcc_dev) {
  if (!m || !cfg || !pcm_dev || !mfcc_dev) return mfail(m, SONAR_ERR_INVALID, "null argument");
  if (m->comm.size() != m->ctx.size()) return mfail(m, SONAR_ERR_DEVICE, "no RCCL communicator");
  const int W = cfg->window_size, H = cfg->hop_size, G = (int)m->ctx.size();
  if (W <= 0 || H <= 0) return mfail(m, SONAR_ERR_INVALID, "window and hop size must be positive");
  const int64_t F = sonar_stft_frames(n, W, H);
  if (F <= 0) return mfail(m, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
  std::vector<int64_t> f0(G), f1(G), s0(G), s1(G);
  int64_t maxF = 0;
  for (int g = 0; g < G; ++g) {
    sonar_multi_shard(n, W, H, G, g, &f0[g], &f1[g], &s0[g], &s1[g]);
    maxF = std::max(maxF, f1[g] - f0[g]);
  }
  const size_t oe = elt_size(cfg->out_dtype), nm = cfg->n_mfcc > 0 ? cfg->n_mfcc : 13;
  const size_t shard_bytes = (size_t)maxF * nm * oe;
  sonar_fp_cfg c1 = *cfg;
  c1.flags = SONAR_FP_MFCC;
  c1.device_ptrs = 1;
  std::vector<void*> send(G), recv(G);
  for (int g = 0; g < G; ++g) {             // each device's shard into a padded send buffer
    sonar_ctx* c = m->ctx[g];
    send[g] = dbuf(c, "mg.send", std::max<size_t>(shard_bytes, 16));
    recv[g] = dbuf(c, "mg.recv", std::max<size_t>(shard_bytes * G, 16));
    if (!send[g] || !recv[g]) return mfail(m, SONAR_ERR_NOMEM, "device allocation failed");
    if (f1[g] > f0[g]) {
      sonar_fp_out o{};
      o.mfcc = send[g];
      const int rc = sonar_fingerprint(c, pcm_dev[g], s1[g] - s0[g], &c1, &o);
      if (rc != SONAR_OK) return mfail(m, rc, "device " + std::to_string(m->dev[g]) + ": " + c->err);
    }
  }
  // one all-gather over xGMI (one thread drives every communicator: grouped)
  const ncclDataType_t t = cfg->out_dtype == SONAR_F32 ? ncclFloat32 : ncclFloat64;
  if (ncclGroupStart() != ncclSuccess) return mfail(m, SONAR_ERR_DEVICE, "ncclGroupStart failed");
  for (int g = 0; g < G; ++g) {
    hipSetDevice(m->dev[g]);
    if (ncclAllGather(send[g], recv[g], (size_t)maxF * nm, t, m->comm[g], m->ctx[g]->stream) != ncclSuccess) {
      ncclGroupEnd();
      return mfail(m, SONAR_ERR_DEVICE, "ncclAllGather failed");
    }
  }
  if (ncclGroupEnd() != ncclSuccess) return mfail(m, SONAR_ERR_DEVICE, "ncclGroupEnd failed");
  for (int g = 0; g < G; ++g) {             // drop the padding: shard h's rows at frame f0[h]
    hipSetDevice(m->dev[g]);
    for (int h = 0; h < G; ++h) {
      const size_t bytes = (size_t)(f1[h] - f0[h]) * nm * oe;
      if (bytes && hipMemcpyAsync((char*)mfcc_dev[g] + (size_t)f0[h] * nm * oe, (char*)recv[g] + h * shard_bytes,
                                  bytes, hipMemcpyDeviceToDevice, m->ctx[g]->stream) != hipSuccess)
        return mfail(m, SONAR_ERR_DEVICE, "timeline copy failed");
    }
  }
  for (int g = 0; g < G; ++g) {
    hipSetDevice(m->dev[g]);
    if (hipStreamSynchronize(m->ctx[g]->stream) != hipSuccess) return mfail(m, SONAR_ERR_DEVICE, "synchronize failed");
  }
  return SONAR_OK;
}

int sonar_align_pairs_multi(sonar_multi* m, int64_t npairs, const double* const* q_pcm, const int64_t* nq,
                            const double* const* r_pcm, const int64_t* nr, int32_t sample_rate, int32_t stft_window,
                            int32_t hop, int32_t feature_window, double max_lag_seconds, int32_t workers,
                            sonar_pair_record* out) {
  if (!m) return SONAR_ERR_INVALID;
  if (npairs < 0 || (npairs > 0 && (!q_pcm || !nq || !r_pcm || !nr || !out)))
    return mfail(m, SONAR_ERR_INVALID, "null pair arrays");
  if (npairs == 0) return SONAR_OK;
  if (m->comm.size() != m->ctx.size()) return mfail(m, SONAR_ERR_DEVICE, "no RCCL communicator");
  const int G = (int)m->ctx.size();
  std::vector<int64_t> a(G), b(G);
  int64_t maxc = 0;
  for (int g = 0; g < G; ++g) {
    a[g] = npairs * g / G;
    b[g] = npairs * (g + 1) / G;
    maxc = std::max(maxc, b[g] - a[g]);
  }
  std::vector<sonar_pair_record> local((size_t)npairs);
  std::vector<int> rcs(G, SONAR_OK);
  std::vector<std::thread> th;
  for (int g = 0; g < G; ++g) {
    th.emplace_back([&, g] {
      if (b[g] > a[g])
        rcs[g] = sonar_align_pairs(m->ctx[g], b[g] - a[g], q_pcm + a[g], nq + a[g], r_pcm + a[g], nr + a[g],
                                   sample_rate, stft_window, hop, feature_window, max_lag_seconds, workers, 0,
                                   local.data() + a[g]);
    });
  }
  for (auto& x : th) x.join();
  int first = SONAR_OK;
  for (int g = 0; g < G; ++g)
    if (rcs[g] != SONAR_OK && first == SONAR_OK) { first = rcs[g]; m->err = m->ctx[g]->err; }
  // the records travel through one RCCL all-gather (padded to the largest range)
  const size_t rb = sizeof(sonar_pair_record), shard = (size_t)maxc * rb;
  std::vector<void*> send(G), recv(G);
  for (int g = 0; g < G; ++g) {
    sonar_ctx* c = m->ctx[g];
    hipSetDevice(m->dev[g]);
    send[g] = dbuf(c, "mp.send", std::max<size_t>(shard, 16));
    recv[g] = dbuf(c, "mp.recv", std::max<size_t>(shard * G, 16));
    if (!send[g] || !recv[g]) return mfail(m, SONAR_ERR_NOMEM, "device allocation failed");
    if (b[g] > a[g] && hipMemcpyAsync(send[g], local.data() + a[g], (size_t)(b[g] - a[g]) * rb,
                                      hipMemcpyHostToDevice, c->stream) != hipSuccess)
      return mfail(m, SONAR_ERR_DEVICE, "record upload failed");
  }
  if (ncclGroupStart() != ncclSuccess) return mfail(m, SONAR_ERR_DEVICE, "ncclGroupStart failed");
  for (int g = 0; g < G; ++g) {
    hipSetDevice(m->dev[g]);
    if (ncclAllGather(send[g], recv[g], shard, ncclUint8, m->comm[g], m->ctx[g]->stream) != ncclSuccess) {
      ncclGroupEnd();
      return mfail(m, SONAR_ERR_DEVICE, "ncclAllGather failed");
    }
  }
  if (ncclGroupEnd() != ncclSuccess) return mfail(m, SONAR_ERR_DEVICE, "ncclGroupEnd failed");
  hipSetDevice(m->dev[0]);
  std::vector<char> host(shard * G);
  if (hipMemcpyAsync(host.data(), recv[0], host.size(), hipMemcpyDeviceToHost, m->ctx[0]->stream) != hipSuccess ||
      hipStreamSynchronize(m->ctx[0]->stream) != hipSuccess)
    return mfail(m, SONAR_ERR_DEVICE, "record download failed");
  for (int g = 0; g < G; ++g) {
    hipSetDevice(m->dev[g]);
    hipStreamSynchronize(m->ctx[g]->stream);
    if (b[g] > a[g]) std::memcpy(out + a[g], host.data() + g * shard, (size_t)(b[g] - a[g]) * rb);
  }
  return first;
}

// FindBestMatches over rank-local galleries (comparison.go:197-263, 1107-1152):
// device g ranks the candidates of its own gallery (sonar_find_best_matches on its context), its
// top max_candidates per query travel to every device through one RCCL all-gather, and the lists
// are merged in the single call's order (sonar_merge_matches).  Candidates are numbered globally:
// device g's candidate c is sum_{h<g} nc[h] + c.
int sonar_find_best_matches_multi(sonar_multi* m, sonar_gallery* const* galleries, const int64_t* const* queries,
                                  int64_t nq, const int64_t* const* candidates, const int64_t* nc,
                                  const sonar_compare_cfg* cfg, sonar_match* out, int64_t* n_matches) {
  if (!m) return SONAR_ERR_INVALID;
  if (!galleries || !queries || !nc || !cfg) return mfail(m, SONAR_ERR_INVALID, "null argument");
  if (cfg->max_candidates < 0) return mfail(m, SONAR_ERR_INVALID, "max candidates must not be negative");
  if (m->comm.size() != m->ctx.size()) return mfail(m, SONAR_ERR_DEVICE, "no RCCL communicator");
  const int G = (int)m->ctx.size();
  const int64_t K = cfg->max_candidates;
  if (nq <= 0) return SONAR_OK;
  if (!n_matches || (K > 0 && !out)) return mfail(m, SONAR_ERR_INVALID, "null output");
  for (int g = 0; g < G; ++g)
    if (!galleries[g] || sonar::detail::gallery_ctx(galleries[g]) != m->ctx[g])
      return mfail(m, SONAR_ERR_INVALID, "gallery " + std::to_string(g) + " does not live on rank " + std::to_string(g));
  // per rank: [nq * K matches][nq counts]
  const size_t lb = (size_t)(nq * K) * sizeof(sonar_match), shard = lb + (size_t)nq * 8;
  std::vector<std::vector<char>> local(G, std::vector<char>(shard, 0));
  std::vector<int> rcs(G, SONAR_OK);
  std::vector<std::thread> th;
  for (int g = 0; g < G; ++g) {
    th.emplace_back([&, g] {
      hipSetDevice(m->dev[g]);
      sonar_match* lm = reinterpret_cast<sonar_match*>(local[g].data());
      int64_t* lc = reinterpret_cast<int64_t*>(local[g].data() + lb);
      rcs[g] = sonar_find_best_matches(galleries[g], queries[g], nq, candidates ? candidates[g] : nullptr, nc[g], cfg,
                                       K > 0 ? lm : nullptr, lc);
    });
  }
  for (auto& x : th) x.join();
  for (int g = 0; g < G; ++g)
    if (rcs[g] != SONAR_OK) return mfail(m, rcs[g], "rank " + std::to_string(g) + ": " + m->ctx[g]->err);
  std::vector<void*> send(G), recv(G);
  for (int g = 0; g < G; ++g) {
    sonar_ctx* c = m->ctx[g];
    hipSetDevice(m->dev[g]);
    send[g] = dbuf(c, "mm.send", std::max<size_t>(shard, 16));
    recv[g] = dbuf(c, "mm.recv", std::max<size_t>(shard * G, 16));
    if (!send[g] || !recv[g]) return mfail(m, SONAR_ERR_NOMEM, "device allocation failed");
    if (hipMemcpyAsync(send[g], local[g].data(), shard, hipMemcpyHostToDevice, c->stream) != hipSuccess)
      return mfail(m, SONAR_ERR_DEVICE, "match upload failed");
  }
  if (ncclGroupStart() != ncclSuccess) return mfail(m, SONAR_ERR_DEVICE, "ncclGroupStart failed");
  for (int g = 0; g < G; ++g) {
    hipSetDevice(m->dev[g]);
    if (ncclAllGather(send[g], recv[g], shard, ncclUint8, m->comm[g], m->ctx[g]->stream) != ncclSuccess) {
      ncclGroupEnd();
      return mfail(m, SONAR_ERR_DEVICE, "ncclAllGather failed");
    }
  }
  if (ncclGroupEnd() != ncclSuccess) return mfail(m, SONAR_ERR_DEVICE, "ncclGroupEnd failed");
  hipSetDevice(m->dev[0]);
  std::vector<char> host(shard * G);
  if (hipMemcpyAsync(host.data(), recv[0], host.size(), hipMemcpyDeviceToHost, m->ctx[0]->stream) != hipSuccess ||
      hipStreamSynchronize(m->ctx[0]->stream) != hipSuccess)
    return mfail(m, SONAR_ERR_DEVICE, "match download failed");
  for (int g = 1; g < G; ++g) { hipSetDevice(m->dev[g]); hipStreamSynchronize(m->ctx[g]->stream); }
  std::vector<const sonar_match*> lists(G);
  std::vector<int64_t> counts((size_t)G * nq), base(G, 0);
  for (int g = 0; g < G; ++g) {
    lists[g] = reinterpret_cast<const sonar_match*>(host.data() + g * shard);
    std::memcpy(counts.data() + (size_t)g * nq, host.data() + g * shard + lb, (size_t)nq * 8);
    if (g > 0) base[g] = base[g - 1] + (candidates ? nc[g - 1] : sonar_gallery_size(galleries[g - 1]));
  }
  const int rc = sonar_merge_matches(lists.data(), counts.data(), base.data(), G, nq, (int32_t)K, out, n_matches);
  return rc == SONAR_OK ? SONAR_OK : mfail(m, rc, "merge failed");
}

}  // extern "C"
