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
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ctx.h"

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
  const int nw = (int)std::min<int64_t>(workers > 0 ? workers : 16, npairs);
  int rc = SONAR_OK;
  std::vector<sonar_ctx*>& ws = workers_of(c, nw, &rc);
  if (rc != SONAR_OK) return fail(c, rc, "worker context creation failed");
  std::atomic<int64_t> next{0};
  std::atomic<int> first_err{SONAR_OK};
  std::vector<std::thread> th;
  for (int t = 0; t < nw; ++t) {
    th.emplace_back([&, t] {
      sonar_ctx* w = ws[t];
      for (int64_t k = next.fetch_add(1); k < npairs; k = next.fetch_add(1)) {
        const int r = align_one(w, q_pcm[k], nq[k], r_pcm[k], nr[k], sample_rate, stft_window, hop, feature_window,
                                max_lag_seconds, device_ptrs, &out[k]);
        if (r != SONAR_OK) {
          int expect = SONAR_OK;
          if (first_err.compare_exchange_strong(expect, r)) c->err = std::string("pair ") + std::to_string(k) + ": " + w->err;
        }
      }
    });
  }
  for (auto& x : th) x.join();
  return first_err.load();
}

int sonar_multi_shard(int64_t n, int32_t W, int32_t H, int32_t G, int32_t g, int64_t* f0, int64_t* f1, int64_t* s0,
                      int64_t* s1) {
  if (W <= 0 || H <= 0 || G <= 0 || g < 0 || g >= G || !f0 || !f1 || !s0 || !s1) return SONAR_ERR_INVALID;
  const int64_t F = sonar_stft_frames(n, W, H);
  if (F <= 0) return SONAR_ERR_TOO_SHORT;
  *f0 = F * g / G;
  *f1 = F * (g + 1) / G;
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
  const size_t nm = std::max(cfg->n_mfcc, 1), K = (size_t)W / 2 + 1;
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
  const size_t oe = elt_size(cfg->out_dtype), nm = std::max(cfg->n_mfcc, 1);
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

}  // extern "C"
