// sonar_api.cpp -- the C ABI of include/sonar_gpu.h.
//
// Low-level entries (sonar_fingerprint, sonar_pitch_yin, sonar_chroma_stft,
// sonar_ncc, sonar_dtw) validate exactly like the Go functions they replace,
// stage host buffers when device_ptrs == 0, and launch the HIP kernels.
// High-level entries (sonar_generate_fingerprint, sonar_align_features) are
// the C++ restatement of the Go orchestration above those seams
// (fingerprint/fingerprint.go:137-236, fingerprint/extractors/speech.go:135-550,
// fingerprint/extractors/alignment.go:139-476).  There is no CPU fallback:
// every numeric array comes from a GPU kernel; the host only builds tables
// and runs the O(frames) sequential epilogues the Go code runs.
#include "../../include/sonar_gpu.h"

#include <hip/hip_runtime.h>

#include <mutex>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "ctx.h"
#include "host_dsp.h"
#include "kernels.h"

namespace sonar {
namespace detail {

int fail(sonar_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

void* dbuf(sonar_ctx* c, const std::string& name, size_t bytes) {
  if (bytes == 0) bytes = 16;
  DevBuf& b = c->bufs[name];
  if (b.cap < bytes) {
    if (b.ptr) { hipStreamSynchronize(c->stream); hipFree(b.ptr); b.ptr = nullptr; b.cap = 0; }
    if (hipMalloc(&b.ptr, bytes) != hipSuccess) { b.ptr = nullptr; return nullptr; }
    b.cap = bytes;
  }
  return b.ptr;
}

void* hbuf(sonar_ctx* c, const std::string& name, size_t bytes) {
  if (bytes == 0) bytes = 16;
  DevBuf& b = c->hbufs[name];
  if (b.cap < bytes) {
    if (b.ptr) { hipStreamSynchronize(c->stream); hipHostFree(b.ptr); b.ptr = nullptr; b.cap = 0; }
    if (hipHostMalloc(&b.ptr, bytes, hipHostMallocDefault) != hipSuccess) { b.ptr = nullptr; return nullptr; }
    b.cap = bytes;
  }
  return b.ptr;
}

// brackets the dominant kernel of a call with a HIP event pair on its stream
hipEvent_t timed_begin(sonar_ctx* c, hipStream_t s) {
  if (!c->timing) return nullptr;
  if (c->ev_used == c->ev_pool.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return nullptr;
    c->ev_pool.emplace_back(a, b);
  }
  auto& e = c->ev_pool[c->ev_used];
  hipEventRecord(e.first, s);
  return e.second;
}
void timed_end(sonar_ctx* c, hipStream_t s, hipEvent_t end) {
  if (!end) return;
  hipEventRecord(end, s);
  c->ev_used++;
}

// the cached buffers of one context (not its workers')
namespace {
// idle pinned blocks by capacity; at most kPinnedCache bytes stay cached
struct PinnedPool {
  std::mutex m;
  std::multimap<size_t, void*> idle;
  size_t cached = 0;
};
PinnedPool& pinned_pool() {
  static PinnedPool* p = new PinnedPool();   // never destroyed: blocks may outlive static teardown
  return *p;
}
constexpr size_t kPinnedCache = size_t(8) << 30;
void pinned_release(void* ptr, size_t cap) {
  PinnedPool& pp = pinned_pool();
  std::lock_guard<std::mutex> g(pp.m);
  if (pp.cached + cap > kPinnedCache) { hipHostFree(ptr); return; }
  pp.idle.emplace(cap, ptr);
  pp.cached += cap;
}
}  // namespace

std::shared_ptr<void> pinned_block(size_t bytes) {
  if (bytes == 0) bytes = 64;
  PinnedPool& pp = pinned_pool();
  void* ptr = nullptr;
  size_t cap = 0;
  {
    std::lock_guard<std::mutex> g(pp.m);
    auto it = pp.idle.lower_bound(bytes);
    if (it != pp.idle.end() && it->first <= 2 * bytes + (size_t(64) << 20)) {
      ptr = it->second; cap = it->first;
      pp.cached -= cap;
      pp.idle.erase(it);
    }
  }
  if (!ptr) {
    cap = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
    if (hipHostMalloc(&ptr, cap, hipHostMallocPortable) != hipSuccess) return nullptr;
  }
  return std::shared_ptr<void>(ptr, [cap](void* q) { pinned_release(q, cap); });
}

void pinned_pool_trim() {
  PinnedPool& pp = pinned_pool();
  std::lock_guard<std::mutex> g(pp.m);
  for (auto& kv : pp.idle) hipHostFree(kv.second);
  pp.idle.clear();
  pp.cached = 0;
}

void trim_buffers(sonar_ctx* c) {
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  for (auto& kv : c->bufs) if (kv.second.ptr) hipFree(kv.second.ptr);
  for (auto& kv : c->hbufs) if (kv.second.ptr) hipHostFree(kv.second.ptr);
  c->bufs.clear();
  c->hbufs.clear();
}
}  // namespace detail
}  // namespace sonar

// The WindowConfig literals of ComputeSTFTWithWindow / ComputeSTFTStreaming (spectral.go:290-295,
// :415-420) and extractChromaFeatures (music.go:335-340) set only Type, Size, Normalize and Symmetric:
// Beta and Alpha keep Go's zero value, not DefaultWindowConfig's 8.6 / 0.5 (windowing.go:66-73).  So a
// Kaiser STFT window is I0(0)/I0(0) = 1 everywhere and a Tukey one has no taper (int(0 * N / 2) = 0):
// both are rectangular.
constexpr double kStftBeta = 0.0, kStftAlpha = 0.0;

namespace {
using namespace sonar::detail;

template <typename T>
void* upload(const std::vector<T>& v) {
  void* p = nullptr;
  size_t bytes = std::max<size_t>(16, v.size() * sizeof(T));
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  if (!v.empty()) hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  return p;
}
void* upload_real(const std::vector<double>& v, bool f64) {
  if (f64) return upload(v);
  std::vector<float> f(v.begin(), v.end());
  return upload(f);
}

int64_t go_frames(int64_t n, int W, int H) { return (n - W) / H + 1; }

// Tables of the headline kernel (mfcc_pair.hip).  The filterbank is cut into
// per-lane chunks: a run of consecutive bins whose nonzero filters are the same
// pair (a, b) (a triangle bank has exactly the rising edge of filter j and the
// falling edge of filter j-1 over [p_j, p_{j+1}), mel_scale.go:65-83), split
// into pieces of at most J bins; every filter then sums the partials of its
// chunks in ascending-bin order.  Returns false when the bank does not fit
// (more than 2 filters on one bin, > 64 chunks at J = 16, > 8 chunks per filter).
bool build_pair_tables(const sonar_fp_cfg* cfg, PairTables& t) {
  const int W = 1024, K = W / 2 + 1;
  std::vector<double> win;
  if (!sonar::host::make_window(cfg->window_type, W, true, true, kStftBeta, kStftAlpha, win)) return false;
  sonar::host::MfccTables mt;
  if (!sonar::host::make_mfcc_tables(cfg->sample_rate, cfg->n_mfcc, cfg->n_filters, cfg->filterbank, cfg->low_freq,
                                     cfg->high_freq, cfg->use_lifter != 0, cfg->lifter, W, mt))
    return false;
  if (mt.n_mfcc > 16 || mt.n_mels > 64) return false;
  auto weight = [&](int m, int k) -> double {
    return (k >= mt.lo[m] && k < mt.hi[m]) ? mt.w[mt.woff[m] + (k - mt.lo[m])] : 0.0;
  };
  // runs of bins whose nonzero filters fit in one pair {a, b}: a run may grow from one filter
  // to two (the zero-weight rising start k = l of a triangle opens the run of [l, c)), never
  // shrink (a one-filter tail after a two-filter run starts a run of its own)
  struct Seg { int k0, k1, a, b; };
  std::vector<Seg> segs;
  for (int k = 0; k < K; k++) {
    int act[3], na = 0;
    for (int m = 0; m < mt.n_mels; m++)
      if (k >= mt.lo[m] && k < mt.hi[m]) { if (na == 2) return false; act[na++] = m; }
    if (na == 0) continue;
    if (!segs.empty() && segs.back().k1 == k) {
      Seg& g = segs.back();
      int u[2] = {g.a, g.b}, nu = g.b >= 0 ? 2 : 1;
      bool fits = true;
      if (na < nu) fits = false;
      for (int i = 0; i < na && fits; i++) {
        bool in = false;
        for (int j = 0; j < nu; j++) in |= (u[j] == act[i]);
        if (!in) { if (nu == 2) { fits = false; break; } u[nu++] = act[i]; }
      }
      if (fits) {
        g.k1 = k + 1;
        if (nu == 2) { g.a = std::min(u[0], u[1]); g.b = std::max(u[0], u[1]); }
        continue;
      }
    }
    segs.push_back({k, k + 1, act[0], na > 1 ? act[1] : -1});
  }
  int J = 1;
  for (;; J++) {
    if (J > 16) return false;
    size_t n = 0;
    for (auto& g : segs) n += (g.k1 - g.k0 + J - 1) / J;
    if (n <= 64) break;
  }
  const double scale = cfg->mfcc_input_power ? 1.0 / 16.0 : 0.25;   // |2X|^2 or |2X|^4 from the pair split
  const int JS = J | 1;
  struct Chunk { int k0, seg; };
  std::vector<Chunk> chunks;
  for (size_t gi = 0; gi < segs.size(); gi++)
    for (int k0 = segs[gi].k0; k0 < segs[gi].k1; k0 += J) chunks.push_back({k0, (int)gi});
  chunks.resize(64, Chunk{0, -1});                 // idle lanes read bin 0 with zero weights
  // Lane order of the chunks, per instance.  The filterbank's power-row reads ld2(prow(ks + i)) are
  // ds_read_b64 in the float32 kernel (two 32-lane groups) and ds_read_b128 in the float64 kernel
  // (four 16-lane groups), bank (byte / 4) mod 64: chunks whose rows fall on the same banks in one
  // group serialise (tools/pair_lds_model.py: 59 extra LDS cycles per pair in ascending order at the
  // headline bank in float32, the bulk of its SQ_LDS_BANK_CONFLICT).  A swap search between groups
  // lowers that; the filters still sum their chunks in ascending-bin order (the source lists below
  // follow the chunk order, not the lanes), so the order changes no result bit.
  static const int kB128Group[64] = {0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1, 0, 0,
                                     0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3,
                                     2, 2, 2, 2, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3};
  for (int e = 0; e < 2; e++) {
    const int pad = sonar::mfcc_pair_pad_rows(e), ew = e ? 4 : 2;   // dwords per lane access
    auto group_of = [&](int l) { return e ? kB128Group[l] : l >> 5; };
    auto fb_conflicts = [&](const std::vector<int>& o) {
      int extra = 0;
      for (int i = 0; i < J; i++) {
        int used[4][64][32], nu[4][64] = {};
        for (int l = 0; l < 64; l++) {
          const int k = chunks[o[l]].k0, g = group_of(l);
          const int dw = ew * (k + pad * (k >> 4)) + ew * i + ((i >= 16 - (k & 15)) ? ew * pad : 0);
          for (int d = 0; d < ew; d++) {
            const int b = (dw + d) & 63;
            bool seen = false;
            for (int u = 0; u < nu[g][b]; u++) seen |= used[g][b][u] == dw + d;
            if (!seen && nu[g][b] < 32) used[g][b][nu[g][b]++] = dw + d;
          }
        }
        for (int g = 0; g < (e ? 4 : 2); g++) {
          int mx = 1;
          for (int b = 0; b < 64; b++) mx = std::max(mx, nu[g][b]);
          extra += mx - 1;
        }
      }
      return extra;
    };
    std::vector<int> order(64);
    for (int l = 0; l < 64; l++) order[l] = l;
    for (int best = fb_conflicts(order), improved = 1; improved;) {
      improved = 0;
      for (int a = 0; a < 64; a++)
        for (int b = a + 1; b < 64; b++) {
          if (group_of(a) == group_of(b)) continue;
          std::swap(order[a], order[b]);
          const int c = fb_conflicts(order);
          if (c < best) { best = c; improved = 1; }
          else std::swap(order[a], order[b]);
        }
    }
    std::vector<int> lane_of(64);
    for (int l = 0; l < 64; l++) lane_of[order[l]] = l;
    std::vector<int> ks(64, 0);
    std::vector<double> cw(64 * 2 * JS, 0.0);
    std::vector<std::vector<int>> src(64);
    for (size_t ci = 0; ci < chunks.size(); ci++) {   // chunk order = ascending bins
      const Chunk& ch = chunks[ci];
      if (ch.seg < 0) continue;
      const Seg& g = segs[ch.seg];
      const int lane = lane_of[ci], k0 = ch.k0;
      ks[lane] = k0;
      for (int i = 0; i < J && k0 + i < g.k1; i++) {
        cw[(lane * JS + i) * 2] = weight(g.a, k0 + i) * scale;
        cw[(lane * JS + i) * 2 + 1] = g.b >= 0 ? weight(g.b, k0 + i) * scale : 0.0;
      }
      src[g.a].push_back(2 * lane);
      if (g.b >= 0) src[g.b].push_back(2 * lane + 1);
    }
    std::vector<uint16_t> msrc(64 * 16, 0x8000);
    int max_src = 1;
    for (int m = 0; m < mt.n_mels; m++) {
      if (src[m].size() > 16) return false;
      max_src = std::max(max_src, (int)src[m].size());
      for (size_t i = 0; i < src[m].size(); i++) msrc[i * 64 + m] = (uint16_t)src[m][i];
    }
    t.max_src = max_src;
    t.chunk_w[e] = e ? upload(cw) : upload(std::vector<float>(cw.begin(), cw.end()));
    t.chunk_ks[e] = (int*)upload(ks); t.mel_src[e] = (uint16_t*)upload(msrc);
  }
  const int NMP = (mt.n_mels + 7) / 8 * 8;
  auto dct_rows = [&](int e) {             // [16][NMP + pad]
    const int st = NMP + sonar::mfcc_pair_dct_pad(e);
    std::vector<double> dct(16 * st, 0.0);
    for (int q = 0; q < mt.n_mfcc; q++)
      for (int m = 0; m < mt.n_mels; m++) dct[q * st + m] = mt.dct[(size_t)q * mt.n_mels + m] * mt.lift[q];
    return dct;
  };
  std::vector<double> tw1(64 * 16 * 2), tw2(64 * 2);
  for (int b = 0; b < 64; b++)
    for (int k = 0; k < 16; k++) {
      const double a = -2.0 * M_PI * (double)((b * k) % 1024) / 1024.0;
      tw1[(b * 16 + k) * 2] = std::cos(a); tw1[(b * 16 + k) * 2 + 1] = std::sin(a);
    }
  for (int b = 0; b < 8; b++)
    for (int c = 0; c < 8; c++) {
      const double a = -2.0 * M_PI * (double)(b * c) / 64.0;
      tw2[(b * 8 + c) * 2] = std::cos(a); tw2[(b * 8 + c) * 2 + 1] = std::sin(a);
    }
  // float32 tables = the float64 values rounded once; float64 tables as computed
  auto f32 = [](const std::vector<double>& v) { return std::vector<float>(v.begin(), v.end()); };
  t.window[0] = upload(f32(win)); t.tw1[0] = upload(f32(tw1)); t.tw2[0] = upload(f32(tw2));
  t.dct[0] = upload(f32(dct_rows(0)));
  t.window[1] = upload(win); t.tw1[1] = upload(tw1); t.tw2[1] = upload(tw2);
  t.dct[1] = upload(dct_rows(1));
  t.zeros = upload(std::vector<double>(1024, 0.0));
  t.J = J; t.JS = JS; t.NMP = NMP; t.n_mels = mt.n_mels; t.n_mfcc = mt.n_mfcc;
  t.ok = t.zeros != nullptr;
  for (int i = 0; i < 2; i++)
    t.ok = t.ok && t.window[i] && t.tw1[i] && t.tw2[i] && t.chunk_w[i] && t.dct[i] && t.chunk_ks[i] && t.mel_src[i];
  return t.ok;
}


}  // namespace

// ============================================================ context ====
extern "C" {

int sonar_abi_version(void) { return SONAR_ABI_VERSION; }

int sonar_create(int device, sonar_ctx** out) {
  if (!out) return SONAR_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SONAR_ERR_DEVICE;
  if (device < 0 || device >= n) return SONAR_ERR_INVALID;
  auto* c = new sonar_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SONAR_ERR_DEVICE;
  }
  c->stream = c->own;
  hipEventCreate(&c->ev0);
  hipEventCreate(&c->ev1);
  *out = c;
  return SONAR_OK;
}

void sonar_destroy(sonar_ctx* c) {
  if (!c) return;
  for (sonar_ctx* w : c->workers) sonar_destroy(w);
  c->workers.clear();
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  sonar::detail::ingest_release(c);
  for (auto& kv : c->bufs) if (kv.second.ptr) hipFree(kv.second.ptr);
  for (auto& kv : c->hbufs) if (kv.second.ptr) hipHostFree(kv.second.ptr);
  for (auto& kv : c->fp_tables) {
    FpTables& t = kv.second;
    for (void* p : {(void*)t.window, (void*)t.mel_lo, (void*)t.mel_hi, (void*)t.mel_woff, (void*)t.grp_off,
                    (void*)t.grp_mels, t.mel_w, t.dct, t.lift, t.trig})
      if (p) hipFree(p);
  }
  for (auto& kv : c->pair_tables) {
    PairTables& t = kv.second;
    for (int i = 0; i < 2; i++)
      for (void* p : {t.window[i], t.tw1[i], t.tw2[i], t.chunk_w[i], t.dct[i], (void*)t.chunk_ks[i], (void*)t.mel_src[i]})
        if (p) hipFree(p);
    if (t.zeros) hipFree(t.zeros);
  }
  for (auto& kv : c->chroma_tables) {
    hipFree(kv.second.win); hipFree(kv.second.trig); hipFree(kv.second.map); hipFree(kv.second.cls);
  }
  for (auto& e : c->ev_pool) { hipEventDestroy(e.first); hipEventDestroy(e.second); }
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->fpb_ev) hipEventDestroy(c->fpb_ev);
  if (c->ev1) hipEventDestroy(c->ev1);
  for (auto& e : c->dtw_ev)
    if (e) hipEventDestroy(e);
  for (auto& e : c->side_ev)
    if (e) hipEventDestroy(e);
  if (c->side) hipStreamDestroy(c->side);
  for (auto e : c->chunk_ev)
    if (e) hipEventDestroy(e);
  if (c->copy) hipStreamDestroy(c->copy);
  for (auto e : c->back_ev)
    if (e) hipEventDestroy(e);
  if (c->own) hipStreamDestroy(c->own);
  delete c;
}

const char* sonar_last_error(const sonar_ctx* c) { return c ? c->err.c_str() : "null context"; }

int sonar_set_stream(sonar_ctx* c, void* s) {
  if (!c) return SONAR_ERR_INVALID;
  c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own;
  return SONAR_OK;
}

int sonar_synchronize(sonar_ctx* c) {
  if (!c) return SONAR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return SONAR_OK;
}

int sonar_enable_kernel_timing(sonar_ctx* c, int on) {
  if (!c) return SONAR_ERR_INVALID;
  c->timing = on != 0;
  return SONAR_OK;
}

const char* sonar_last_fp_kernel(sonar_ctx* c) { return c ? c->last_fp_kernel : ""; }


int sonar_trim(sonar_ctx* c) {
  if (!c) return SONAR_ERR_INVALID;
  for (sonar_ctx* w : c->workers) sonar::detail::trim_buffers(w);
  sonar::detail::trim_buffers(c);
  sonar::detail::pinned_pool_trim();
  return SONAR_OK;
}

int sonar_dtw_counters(sonar_ctx* c, int64_t* out4, int32_t reset) {
  if (!c || !out4) return SONAR_ERR_INVALID;
  for (int k = 0; k < 4; ++k) {
    long long v = c->dtw_ctr[k];
    for (sonar_ctx* w : c->workers) v += w->dtw_ctr[k];
    out4[k] = v;
  }
  if (reset) {
    for (int k = 0; k < 4; ++k) c->dtw_ctr[k] = 0;
    for (sonar_ctx* w : c->workers)
      for (int k = 0; k < 4; ++k) w->dtw_ctr[k] = 0;
  }
  return SONAR_OK;
}

int sonar_dtw_last_timing(sonar_ctx* c, double* ms3) {
  if (!c || !ms3) return SONAR_ERR_INVALID;
  for (int k = 0; k < 3; ++k) ms3[k] = c->dtw_ms[k];
  return SONAR_OK;
}

int sonar_last_kernel_ms(sonar_ctx* c, double* ms) {
  if (!c || !ms) return SONAR_ERR_INVALID;
  if (c->ev_used > 0) {   // average over every timed launch since the last query
    HIP_TRY(c, hipEventSynchronize(c->ev_pool[c->ev_used - 1].second));
    double sum = 0.0;
    for (size_t i = 0; i < c->ev_used; ++i) {
      float f = 0.f;
      HIP_TRY(c, hipEventElapsedTime(&f, c->ev_pool[i].first, c->ev_pool[i].second));
      sum += f;
    }
    c->last_ms = sum / (double)c->ev_used;
    c->ev_used = 0;
  }
  *ms = c->last_ms;
  return SONAR_OK;
}

int64_t sonar_stft_frames(int64_t n, int32_t W, int32_t H) {
  if (n <= 0) return SONAR_ERR_EMPTY;
  if (W <= 0 || H <= 0) return SONAR_ERR_INVALID;
  const int64_t F = go_frames(n, W, H);
  return F <= 0 ? SONAR_ERR_TOO_SHORT : F;
}

int64_t sonar_energy_frames(int64_t n, int32_t W, int32_t H) {
  if (n < W || H <= 0 || W <= 0) return 0;
  return (n - W) / H + 1;
}

int64_t sonar_pitch_frames(int64_t n) {
  const int64_t F = (n - 1024) / 512 + 1;
  return F < 0 ? 0 : F;
}

void sonar_fp_cfg_default(sonar_fp_cfg* c) {
  std::memset(c, 0, sizeof(*c));
  c->window_size = 1024;
  c->hop_size = 256;
  c->window_type = SONAR_WIN_HANN;
  c->sample_rate = 44100;
  c->n_mfcc = 13;
  c->n_filters = 26;
  c->filterbank = SONAR_FB_MEL;
  c->use_lifter = 1;
  c->lifter = 22.0;
  c->preemph_alpha = 0.97;
  c->flags = SONAR_FP_MFCC;
  c->precision = SONAR_F32;
  c->pcm_dtype = SONAR_F64;
  c->out_dtype = SONAR_F64;
}

// ======================================================= sonar_fingerprint ==
}  // extern "C"

namespace {
// the headline kernel's tables for a configuration, built once per context
const PairTables& pair_tables_for(sonar_ctx* c, const sonar_fp_cfg* cfg) {
  char key[512];
  std::snprintf(key, sizeof(key), "%d|%d|%d|%d|%.17g|%.17g|%d|%.17g|%d|%d", cfg->window_type, cfg->sample_rate,
                cfg->n_mfcc, cfg->n_filters, cfg->low_freq, cfg->high_freq, cfg->use_lifter, cfg->lifter,
                cfg->filterbank, cfg->mfcc_input_power);
  auto it = c->pair_tables.find(key);
  if (it == c->pair_tables.end()) {
    PairTables t;
    build_pair_tables(cfg, t);
    it = c->pair_tables.emplace(key, t).first;
  }
  return it->second;
}

// tables, LDS carve and work split of one mfcc_pair_kernel launch over NP frame pairs
void fill_pair_params(sonar_ctx* c, const PairTables& t, const sonar_fp_cfg* cfg, int64_t NP,
                      sonar::MfccPairParams& q, bool f64 = false) {
  const int e = f64 ? 1 : 0, es = f64 ? 8 : 4;
  q.f64 = e;
  q.window = t.window[e]; q.tw1 = t.tw1[e]; q.tw2 = t.tw2[e]; q.chunk_w = t.chunk_w[e]; q.dct = t.dct[e];
  q.chunk_ks = t.chunk_ks[e]; q.mel_src = t.mel_src[e]; q.zeros = t.zeros;
  q.J = t.J; q.JS = t.JS; q.max_src = t.max_src; q.NMP = t.NMP; q.n_mels = t.n_mels; q.n_mfcc = t.n_mfcc;
  q.pow2 = cfg->mfcc_input_power != 0;
  auto al = [](int x) { return (x + 15) & ~15; };
  q.lds_src = al(64 * t.JS * 2 * es);
  q.lds_dct = q.lds_src + 64 * 16 * 2;
  q.lds_ctr = q.lds_dct + al(16 * (t.NMP + sonar::mfcc_pair_dct_pad(e)) * es);
  q.lds_tw2 = q.lds_ctr + 16;
  q.lds_wave0 = q.lds_tw2 + (f64 ? 8 * sonar::kPairTw2Row * 16 : 0);   // float64: the stage-2 twiddle table
  // mfcc_pair_kernel: one block per CU (12 waves float32, 8 float64) over a contiguous range of pairs
  // One block per CU.  The float64 waves' 17.4 KB regions beside the largest tables (J = 16,
  // NMP = 64: 29 KB) exceed the 160 KiB of LDS at 8 waves; such a bank runs 7 (or fewer) waves
  q.waves_per_block = sonar::mfcc_pair_waves_per_block(e);
  while (q.waves_per_block > 1 && q.lds_wave0 + q.waves_per_block * sonar::mfcc_pair_wave_bytes(e) > 160 * 1024)
    --q.waves_per_block;
  q.lds_bytes = q.lds_wave0 + q.waves_per_block * sonar::mfcc_pair_wave_bytes(e);
  int dev_cus = 256;
  hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, c->device);
  const int64_t blocks = (int64_t)dev_cus * std::max(1, sonar::mfcc_pair_waves_per_cu(e) / q.waves_per_block);
  q.pairs_per_block = std::max<int64_t>(1, (NP + blocks - 1) / blocks);
}

// The transform kernel of a validated sonar_fingerprint call over F frames (sonar_fp_kernel_plan):
// mfcc_pair_kernel for the float32 MFCC-only configuration at W = 1024 while its 32-bit frame
// indices hold (t = 2 pair + 1 <= F), the general fused kernel for the other fused window sizes,
// the float64 DFT path for any other W.
int fp_plan(const sonar_fp_cfg* cfg, int64_t F) {
  const uint32_t flags = cfg->flags;
  if (!(flags & (SONAR_FP_MFCC | SONAR_FP_MAGNITUDE | SONAR_FP_SPECTRAL | SONAR_FP_COMPLEX | SONAR_FP_PHASE)))
    return SONAR_PLAN_NONE;
  if (!sonar::fingerprint_supported(cfg->window_size)) return SONAR_PLAN_DFT;
  // the pair kernel computes in float32 with float32 PCM and output, or in float64 with float64
  // output (PCM of either type)
  const bool types = cfg->precision == SONAR_F64 ? cfg->out_dtype == SONAR_F64
                                                  : cfg->pcm_dtype != SONAR_F64 && cfg->out_dtype != SONAR_F64;
  const bool pair = types && cfg->window_size == 1024 && (flags & SONAR_FP_MFCC) &&
                    !(flags & (SONAR_FP_MAGNITUDE | SONAR_FP_SPECTRAL | SONAR_FP_COMPLEX | SONAR_FP_PHASE |
                               SONAR_FP_GENERIC | 0x80000000u)) &&
                    F <= SONAR_PAIR_MAX_FRAMES;
  return pair ? SONAR_PLAN_PAIR : SONAR_PLAN_WAVE;
}

// spec_rows_kernel over F float64 |X| rows of K bins into the descriptor outputs (nullable each)
int launch_spec(const double* mag, int64_t F, int K, int sample_rate, bool o64, void* const* d_spec, hipStream_t s,
                int64_t f_lo, int64_t f_hi) {
  sonar::SpecParams sp{};
  sp.mag = mag; sp.F = F; sp.K = K; sp.sample_rate = sample_rate; sp.out_f64 = o64 ? 1 : 0;
  sp.f_first = f_lo; sp.f_last = f_hi;
  for (int d = 0; d < 9; d++) sp.out_spec[d] = d_spec[d];
  // ~24 resident waves per CU over 256 CUs, a contiguous frame run each
  const int64_t target = 256 * 24;
  sp.frames_per_wave = std::max<int64_t>(1, (f_hi - f_lo + target - 1) / target);
  return sonar::launch_spec_rows(sp, s);
}

// ComputeSTFTWithWindow's argument checks (spectral.go:386-412) and the GPU path's own limits, in the
// order sonar_fingerprint applies them: SONAR_OK and the frame count, or the error code + message
int fp_validate(const sonar_fp_cfg* cfg, int64_t n, bool have_pcm, int64_t* F, std::string* msg) {
  if (n <= 0 || !have_pcm) { *msg = "empty signal"; return SONAR_ERR_EMPTY; }
  const int W = cfg->window_size, H = cfg->hop_size;
  if (W <= 0) { *msg = "window size must be positive"; return SONAR_ERR_INVALID; }
  if (H <= 0) { *msg = "hop size must be positive"; return SONAR_ERR_INVALID; }
  *F = go_frames(n, W, H);
  if (*F <= 0) { *msg = "signal too short for given window size and hop size"; return SONAR_ERR_TOO_SHORT; }
  if (fp_plan(cfg, *F) == SONAR_PLAN_DFT) {
    // other window lengths (go-dsp takes any W, spectral.go:131) run the generic DFT path (its
    // |X| scratch feeds spec_rows_kernel for the spectral descriptors)
    if (W > 8192) {
      *msg = "window size " + std::to_string(W) + " above 8192 (generic STFT path)";
      return SONAR_ERR_UNSUPPORTED;
    }
  }
  return SONAR_OK;
}
}  // namespace

extern "C" int32_t sonar_fp_kernel_plan(const sonar_fp_cfg* cfg, int64_t n) {
  if (!cfg) return SONAR_ERR_INVALID;
  int64_t F = 0;
  std::string msg;
  const int rc = fp_validate(cfg, n, true, &F, &msg);
  return rc != SONAR_OK ? rc : fp_plan(cfg, F);
}

namespace sonar {
namespace detail {
// pcm_dev: pcm is already device memory even though the outputs are host buffers
// (cfg->device_ptrs == 0) -- the sonar_fingerprint_f64le path (ingest_api.cpp)
int fingerprint_impl(sonar_ctx* c, const void* pcm, int64_t n, const sonar_fp_cfg* cfg, sonar_fp_out* out,
                     bool pcm_dev, int64_t f_lo, int64_t f_hi) {
  if (!c || !cfg || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  // ComputeSTFTWithWindow validation order (spectral.go:386-412), then the GPU path's limits
  int64_t F = 0;
  {
    std::string msg;
    const int rc = fp_validate(cfg, n, pcm != nullptr, &F, &msg);
    if (rc != SONAR_OK) return fail(c, rc, msg);
  }
  // a frame range [f_lo, f_hi) of the whole signal's STFT (the chunked host-PCM pipeline of the
  // speech extractor): device outputs, the per-frame fused kernel, no energy frames
  if (f_hi < 0 || f_hi > F) f_hi = F;
  if (f_lo < 0) f_lo = 0;
  const bool ranged = f_lo > 0 || f_hi < F;
  if (ranged && (cfg->device_ptrs == 0 || fp_plan(cfg, F) != SONAR_PLAN_WAVE || (cfg->flags & SONAR_FP_ENERGY)))
    return fail(c, SONAR_ERR_UNSUPPORTED, "frame ranges need device outputs and the per-frame fused kernel");
  if (f_hi <= f_lo) return SONAR_OK;
  const int W = cfg->window_size, H = cfg->hop_size;
  const uint32_t flags = cfg->flags;
  // The spectral descriptors always take the float64 transform, whatever `precision` says: the
  // flatness (exp of the mean ln over every bin above 1e-10, spectral_flatness.go:31-73) and the
  // log-log slope (spectral_slope.go:24-63) read leakage bins that sit below an f32 FFT's rounding
  // floor, so an f32 transform cannot hold them to 1e-4.  ~10 % of the kernel.
  const bool f64 = cfg->precision == SONAR_F64 || (flags & SONAR_FP_SPECTRAL) != 0;
  const bool pcm64 = cfg->pcm_dtype == SONAR_F64;
  const bool o64 = cfg->out_dtype == SONAR_F64;
  const int plan = fp_plan(cfg, F);
  const bool need_fft = plan != SONAR_PLAN_NONE;
  const bool generic = plan == SONAR_PLAN_DFT;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const size_t esz_in = pcm64 ? 8 : 4, esz_out = o64 ? 8 : 4;
  const bool dev = cfg->device_ptrs != 0;

  const void* dpcm = pcm;
  if (!dev && !pcm_dev) {
    void* p = dbuf(c, "fp.pcm", (size_t)n * esz_in);
    if (!p) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (pcm)");
    HIP_TRY(c, hipMemcpyAsync(p, pcm, (size_t)n * esz_in, hipMemcpyHostToDevice, s));
    dpcm = p;
  }
  const int K = W / 2 + 1;
  // outputs (device staging when host pointers)
  struct OutMap { void* host; void* devp; size_t bytes; };
  std::vector<OutMap> copies;
  auto out_ptr = [&](void* user, const char* name, size_t count) -> void* {
    if (!user) return nullptr;
    if (dev) return user;
    void* d = dbuf(c, std::string("fp.out.") + name, count * esz_out);
    if (d) copies.push_back({user, d, count * esz_out});
    return d;
  };
  void* d_mfcc = (flags & SONAR_FP_MFCC) ? out_ptr(out->mfcc, "mfcc", (size_t)F * (cfg->n_mfcc > 0 ? cfg->n_mfcc : 13)) : nullptr;
  void* d_mag = (flags & SONAR_FP_MAGNITUDE) ? out_ptr(out->magnitude, "mag", (size_t)F * K) : nullptr;
  if ((flags & SONAR_FP_MFCC) && !d_mfcc) return fail(c, SONAR_ERR_INVALID, "out->mfcc is null or allocation failed");
  if ((flags & SONAR_FP_MAGNITUDE) && !d_mag) return fail(c, SONAR_ERR_INVALID, "out->magnitude is null");
  void* d_cplx = (flags & SONAR_FP_COMPLEX) ? out_ptr(out->complex, "cplx", (size_t)F * K * 2) : nullptr;
  void* d_phase = (flags & SONAR_FP_PHASE) ? out_ptr(out->phase, "phase", (size_t)F * K) : nullptr;
  if ((flags & SONAR_FP_COMPLEX) && !d_cplx) return fail(c, SONAR_ERR_INVALID, "out->complex is null");
  if ((flags & SONAR_FP_PHASE) && !d_phase) return fail(c, SONAR_ERR_INVALID, "out->phase is null");
  void* d_spec[9] = {nullptr};
  if (flags & SONAR_FP_SPECTRAL) {
    void* user[9] = {out->centroid, out->rolloff, out->bandwidth, out->flatness, out->crest, out->slope,
                     out->flux, out->low_ratio, out->high_ratio};
    static const char* nm[9] = {"centroid", "rolloff", "bandwidth", "flatness", "crest", "slope", "flux", "low", "high"};
    for (int d = 0; d < 9; d++) {
      const size_t cnt = (d == 6) ? (size_t)std::max<int64_t>(F - 1, 0) : (size_t)F;
      if (user[d] && cnt > 0) d_spec[d] = out_ptr(user[d], nm[d], cnt);
    }
  }

  c->last_fp_kernel = "";
  if (generic) {
    char key[512];
    std::snprintf(key, sizeof(key), "gen|%d|%d|%d|%d|%d|%d|%.17g|%.17g|%d|%.17g", W, cfg->window_type,
                  cfg->sample_rate, cfg->n_mfcc, cfg->n_filters, cfg->filterbank, cfg->low_freq, cfg->high_freq,
                  cfg->use_lifter, cfg->lifter);
    auto it = c->fp_tables.find(key);
    if (it == c->fp_tables.end()) {
      FpTables t;
      std::vector<double> win;
      if (!sonar::host::make_window(cfg->window_type, W, true, true, kStftBeta, kStftAlpha, win))
        return fail(c, SONAR_ERR_INVALID, "failed to generate window: unsupported window type");
      std::vector<double> trig(2 * (size_t)W);
      for (int m = 0; m < W; ++m) {
        trig[2 * m] = std::cos(2.0 * M_PI * (double)m / (double)W);
        trig[2 * m + 1] = -std::sin(2.0 * M_PI * (double)m / (double)W);
      }
      t.window = upload(win);
      t.trig = upload(trig);
      if (flags & SONAR_FP_MFCC) {
        sonar::host::MfccTables mt;
        if (!sonar::host::make_mfcc_tables(cfg->sample_rate, cfg->n_mfcc, cfg->n_filters, cfg->filterbank,
                                           cfg->low_freq, cfg->high_freq, cfg->use_lifter != 0, cfg->lifter, W, mt))
          return fail(c, SONAR_ERR_INVALID, "failed to initialize MFCC: failed to create mel filter bank");
        t.mel_lo = (int*)upload(mt.lo); t.mel_hi = (int*)upload(mt.hi); t.mel_woff = (int*)upload(mt.woff);
        t.mel_w = upload(mt.w); t.dct = upload(mt.dct); t.lift = upload(mt.lift);
        t.n_mels = mt.n_mels; t.n_mfcc = mt.n_mfcc; t.nnz = (int)mt.w.size();
        if (!t.mel_lo || !t.mel_w || !t.dct || !t.lift) return fail(c, SONAR_ERR_NOMEM, "table upload failed");
      }
      if (!t.window || !t.trig) return fail(c, SONAR_ERR_NOMEM, "table upload failed");
      it = c->fp_tables.emplace(key, t).first;
    }
    FpTables& t = it->second;
    if ((flags & SONAR_FP_MFCC) && !t.mel_lo) {                   // tables built by a non-MFCC call first
      sonar::host::MfccTables mt;
      if (!sonar::host::make_mfcc_tables(cfg->sample_rate, cfg->n_mfcc, cfg->n_filters, cfg->filterbank,
                                         cfg->low_freq, cfg->high_freq, cfg->use_lifter != 0, cfg->lifter, W, mt))
        return fail(c, SONAR_ERR_INVALID, "failed to initialize MFCC: failed to create mel filter bank");
      t.mel_lo = (int*)upload(mt.lo); t.mel_hi = (int*)upload(mt.hi); t.mel_woff = (int*)upload(mt.woff);
      t.mel_w = upload(mt.w); t.dct = upload(mt.dct); t.lift = upload(mt.lift);
      t.n_mels = mt.n_mels; t.n_mfcc = mt.n_mfcc; t.nnz = (int)mt.w.size();
    }
    double* mag = (double*)dbuf(c, "fp.gen.mag", (size_t)F * K * 8);
    if (!mag) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (spectrogram)");
    hipEvent_t tend = timed_begin(c, s);
    if (sonar::launch_stft_dft(dpcm, pcm64, n, F, W, H, (const double*)t.window, (const double*)t.trig, mag, d_mag,
                               d_cplx, d_phase, o64, s) != 0)
      return fail(c, SONAR_ERR_DEVICE, "stft launch failed");
    if ((flags & SONAR_FP_MFCC) &&
        sonar::launch_mfcc_rows(mag, F, K, t.mel_lo, t.mel_hi, t.mel_woff, (const double*)t.mel_w, t.n_mels,
                                (const double*)t.dct, (const double*)t.lift, t.n_mfcc, cfg->mfcc_input_power, d_mfcc,
                                o64, s) != 0)
      return fail(c, SONAR_ERR_DEVICE, "mfcc launch failed");
    if ((flags & SONAR_FP_SPECTRAL) && launch_spec(mag, F, K, cfg->sample_rate, o64, d_spec, s, 0, F) != 0)
      return fail(c, SONAR_ERR_DEVICE, "spectral descriptor launch failed");
    timed_end(c, s, tend);
    c->last_fp_kernel = "stft_dft_kernel";
  }
  // headline path: float32 MFCC only at W = 1024 (mfcc_pair.hip); SONAR_FP_GENERIC forces fp_kernel.hip
  bool pair_done = false;
  if (plan == SONAR_PLAN_PAIR) {
    const PairTables& t = pair_tables_for(c, cfg);
    if (t.ok) {
      sonar::MfccPairParams q{};
      fill_pair_params(c, t, cfg, (F + 1) / 2, q, f64);
      q.pcm = dpcm; q.pcm_f64 = pcm64 ? 1 : 0; q.n = n; q.F = F; q.H = H;
      q.out = d_mfcc;
#ifdef HL_STAMP
      const char* stamp_path = std::getenv("SONAR_HL_STAMP");
      const int64_t nw = ((F + 1) / 2 + q.pairs_per_block - 1) / q.pairs_per_block * q.waves_per_block;
      if (stamp_path) q.stamp = (uint64_t*)dbuf(c, "hl.stamp", (size_t)nw * 24);
#endif
      hipEvent_t tend = timed_begin(c, s);
      const int lrc = sonar::launch_mfcc_pair(q, s);
      if (lrc == -4) return fail(c, SONAR_ERR_UNSUPPORTED, "too many frames for one mfcc_pair_kernel launch");
      if (lrc != 0)
        return fail(c, SONAR_ERR_DEVICE, std::string("mfcc kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
      timed_end(c, s, tend);
#ifdef HL_STAMP
      if (q.stamp) {   // diagnostics: every wave's {start, end} appended to the file
        std::vector<uint64_t> h((size_t)nw * 3);
        HIP_TRY(c, hipMemcpyAsync(h.data(), q.stamp, h.size() * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipStreamSynchronize(s));
        if (FILE* f = std::fopen(stamp_path, "ab")) { std::fwrite(h.data(), 8, h.size(), f); std::fclose(f); }
      }
#endif
      pair_done = true;
      c->last_fp_kernel = "mfcc_pair_kernel";
    }
  }
  if (need_fft && !generic && !pair_done) {
    // Spectral descriptors (round 6): the transform writes float64 |X| rows to HBM (the caller's
    // Magnitude output when it is float64, else a scratch of F x K doubles) and spec_rows_kernel
    // reduces them.  The fused SPEC epilogue (one wave per SIMD) remains only for a float32
    // Magnitude output beside the descriptors, or when the scratch cannot be allocated.
    const bool spec_req = (flags & SONAR_FP_SPECTRAL) != 0;
    double* spec_mag = nullptr;
    if (spec_req && f64 && !(d_mag && !o64))
      spec_mag = d_mag ? (double*)d_mag : (double*)dbuf(c, "fp.specmag", (size_t)F * K * 8);
    const bool spec = spec_req && !spec_mag;            // the fused SPEC epilogue
    const int NB = sonar::fp_batch_frames(W, f64 ? 1 : 0, spec ? 1 : 0);
    const int PRE = sonar::fp_pre_rows(W, spec);
    sonar::FpParams p{};
    p.pcm = dpcm; p.n = n; p.pcm_f64 = pcm64; p.F = F; p.W = W; p.H = H;
    p.f_first = f_lo; p.f_last = f_hi;
    p.flags = spec ? flags : (flags & ~(uint32_t)SONAR_FP_SPECTRAL);
    p.input_power = cfg->mfcc_input_power;
    p.n_groups = 64 / NB;
    p.sample_rate = cfg->sample_rate;
    p.out_f64 = o64;
    p.out_mfcc = d_mfcc;
    p.out_mag = spec_mag ? (void*)spec_mag : d_mag;
    p.mag_f64 = spec_mag ? 1 : (int)o64;
    p.out_cplx = d_cplx;
    p.out_phase = d_phase;
    for (int d = 0; d < 9; d++) p.out_spec[d] = d_spec[d];
    // tables, cached per configuration
    char key[512];
    std::snprintf(key, sizeof(key), "%d|%d|%d|%d|%d|%d|%.17g|%.17g|%d|%.17g|%d|%d", W, cfg->window_type,
                  cfg->sample_rate, cfg->n_mfcc, cfg->n_filters, cfg->filterbank, cfg->low_freq, cfg->high_freq,
                  cfg->use_lifter, cfg->lifter, (int)f64, NB);
    auto it = c->fp_tables.find(key);
    if (it == c->fp_tables.end()) {
      FpTables t;
      std::vector<double> win;
      if (!sonar::host::make_window(cfg->window_type, W, true, true, kStftBeta, kStftAlpha, win))
        return fail(c, SONAR_ERR_INVALID, "failed to generate window: unsupported window type");
      t.window = upload_real(win, f64);
      sonar::host::MfccTables mt;
      if (!sonar::host::make_mfcc_tables(cfg->sample_rate, cfg->n_mfcc, cfg->n_filters, cfg->filterbank, cfg->low_freq,
                                         cfg->high_freq, cfg->use_lifter != 0, cfg->lifter, W, mt))
        return fail(c, SONAR_ERR_INVALID, "failed to initialize MFCC: failed to create mel filter bank");
      std::vector<int> off, mels;
      sonar::host::balance_groups(mt, 64 / NB, off, mels);
      t.mel_lo = (int*)upload(mt.lo); t.mel_hi = (int*)upload(mt.hi); t.mel_woff = (int*)upload(mt.woff);
      t.grp_off = (int*)upload(off); t.grp_mels = (int*)upload(mels);
      t.mel_w = upload_real(mt.w, f64); t.dct = upload_real(mt.dct, f64); t.lift = upload_real(mt.lift, f64);
      t.n_mels = mt.n_mels; t.n_mfcc = mt.n_mfcc; t.nnz = (int)mt.w.size();
      if (!t.window || !t.mel_lo || !t.mel_w || !t.dct || !t.lift) return fail(c, SONAR_ERR_NOMEM, "table upload failed");
      it = c->fp_tables.emplace(key, t).first;
    }
    const FpTables& t = it->second;
    p.window = t.window;
    p.n_mels = t.n_mels; p.n_mfcc = t.n_mfcc; p.nnz = t.nnz;
    p.mel_lo = t.mel_lo; p.mel_hi = t.mel_hi; p.mel_woff = t.mel_woff; p.mel_w = t.mel_w;
    p.grp_off = t.grp_off; p.grp_mels = t.grp_mels; p.dct = t.dct; p.lift = t.lift;
    // LDS carve: twiddle tables (shared), then one region per wave
    const int esz = f64 ? 8 : 4;
    const int R = W / 128, FR = R >= 8 ? 1 : 8 / R, G = R * FR / 8;
    auto al = [](int x) { return (x + 15) & ~15; };
    p.lds_tab_t1 = 0;
    p.lds_tab_t2 = al(R * 64 * 2 * esz);
    p.lds_tab_t3 = p.lds_tab_t2 + al(64 * 2 * esz);
    p.lds_tab_mel = p.lds_tab_t3 + al(G * 8 * 64 * 2 * esz);
    p.lds_tab_w = p.lds_tab_mel + al((4 * t.n_mels + p.n_groups + 1) * 4);
    p.lds_tab_dct = p.lds_tab_w + al(std::max(t.nnz, 1) * esz);
    p.lds_wave0 = p.lds_tab_dct + al((t.n_mfcc * t.n_mels + t.n_mfcc) * esz);
    p.lds_logmel = al((PRE + NB) * K * esz);
    p.lds_stage = p.lds_logmel + al(NB * (t.n_mels + 1) * esz);
    p.lds_wave_stride = p.lds_stage + al(NB * t.n_mfcc * esz);
    p.waves_per_block = 4;
    while (p.waves_per_block > 1 && p.lds_wave0 + p.waves_per_block * p.lds_wave_stride > 160 * 1024) p.waves_per_block--;
    p.lds_bytes = p.lds_wave0 + p.waves_per_block * p.lds_wave_stride;
    if (p.lds_bytes > 160 * 1024) return fail(c, SONAR_ERR_UNSUPPORTED, "LDS budget exceeded");
    // frames per wave: about 12 resident waves per CU, equal shares, multiple of NB
    int dev_cus = 256;
    hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, c->device);
    const int64_t target_waves = (int64_t)dev_cus * 12;
    int64_t fpw = (f_hi - f_lo + target_waves - 1) / target_waves;
    fpw = std::max<int64_t>(NB, (fpw + NB - 1) / NB * NB);
    p.frames_per_wave = fpw;
    hipEvent_t tend = timed_begin(c, s);
    const int rc = sonar::launch_fingerprint(p, f64, s);
    c->last_fp_kernel = "fp_wave_kernel";
    if (rc != 0) return fail(c, SONAR_ERR_DEVICE, std::string("fingerprint kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    if (spec_mag && launch_spec(spec_mag, F, K, cfg->sample_rate, o64, d_spec, s, f_lo, f_hi) != 0)
      return fail(c, SONAR_ERR_DEVICE, "spectral descriptor launch failed");
    timed_end(c, s, tend);
  }
  if (flags & SONAR_FP_ZCR) {
    void* d = out_ptr(out->zcr, "zcr", (size_t)F);
    if (!d) return fail(c, SONAR_ERR_INVALID, "out->zcr is null");
    if (sonar::launch_zcr(dpcm, pcm64, n, F, W, H, cfg->preemph_alpha, cfg->sample_rate, d, o64, s, f_lo, f_hi) != 0)
      return fail(c, SONAR_ERR_DEVICE, "zcr launch failed");
  }
  if (flags & SONAR_FP_ENERGY) {
    const int64_t Fe = sonar_energy_frames(n, cfg->energy_window, cfg->energy_hop);
    if (Fe > 0) {
      void* d = out_ptr(out->energy, "energy", (size_t)Fe);
      if (!d) return fail(c, SONAR_ERR_INVALID, "out->energy is null");
      if (sonar::launch_energy(dpcm, pcm64, n, Fe, cfg->energy_window, cfg->energy_hop, cfg->preemph_alpha, d, o64, s) != 0)
        return fail(c, SONAR_ERR_DEVICE, "energy launch failed");
    }
  }
  if (!dev) {
    for (auto& m : copies) HIP_TRY(c, hipMemcpyAsync(m.host, m.devp, m.bytes, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SONAR_OK;
}
}  // namespace detail
}  // namespace sonar

extern "C" {

int sonar_fingerprint(sonar_ctx* c, const void* pcm, int64_t n, const sonar_fp_cfg* cfg, sonar_fp_out* out) {
  return sonar::detail::fingerprint_impl(c, pcm, n, cfg, out, cfg && cfg->device_ptrs != 0);
}

// SpectralAnalyzer.ComputeSTFTBatch (fingerprint/analyzers/spectral.go:234-285): every signal through
// ComputeSTFTWithWindow with one configuration; the first failing signal (by index) reports
// "error processing signal i: <its error>" (:276-281).  The f32 MFCC configuration at W = 1024 runs
// all signals' frame pairs in ONE mfcc_pair_kernel launch (segment table, mfcc_pair.hip SEG); any
// other configuration runs sonar_fingerprint per signal on the context's stream.
int sonar_fingerprint_batch(sonar_ctx* c, const void* const* pcm, const int64_t* n, int32_t count,
                            const sonar_fp_cfg* cfg, sonar_fp_out* out) {
  if (!c) return SONAR_ERR_INVALID;
  if (count <= 0) return fail(c, SONAR_ERR_EMPTY, "no signals provided");
  if (!pcm || !n || !cfg || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  const int W = cfg->window_size, H = cfg->hop_size;
  auto sig_fail = [&](int i, int code, const std::string& msg) {
    return fail(c, code, "error processing signal " + std::to_string(i) + ": " + msg);
  };
  // ComputeSTFTWithWindow's checks per signal, in its order (spectral.go:386-412)
  for (int i = 0; i < count; i++) {
    if (n[i] <= 0 || !pcm[i]) return sig_fail(i, SONAR_ERR_EMPTY, "empty signal");
    if (W <= 0) return sig_fail(i, SONAR_ERR_INVALID, "window size must be positive");
    if (H <= 0) return sig_fail(i, SONAR_ERR_INVALID, "hop size must be positive");
    if (go_frames(n[i], W, H) <= 0)
      return sig_fail(i, SONAR_ERR_TOO_SHORT, "signal too short for given window size and hop size");
  }
  const bool dev = cfg->device_ptrs != 0;
  int64_t pairs_total = 0;                 // the one launch's 32-bit frame indices run over the whole batch
  for (int i = 0; i < count; i++) pairs_total += (go_frames(n[i], W, H) + 1) / 2;
  const bool one_launch = W == 1024 && cfg->flags == SONAR_FP_MFCC && cfg->precision == SONAR_F32 &&
                          cfg->pcm_dtype == SONAR_F32 && cfg->out_dtype == SONAR_F32 &&
                          2 * pairs_total <= SONAR_PAIR_MAX_FRAMES;
  const PairTables* tp = one_launch ? &pair_tables_for(c, cfg) : nullptr;
  if (!tp || !tp->ok) {
    for (int i = 0; i < count; i++) {
      const int rc = sonar::detail::fingerprint_impl(c, pcm[i], n[i], cfg, &out[i], dev);
      if (rc != SONAR_OK) return sig_fail(i, rc, c->err);
    }
    return SONAR_OK;
  }
  const PairTables& t = *tp;
  for (int i = 0; i < count; i++)
    if (!out[i].mfcc) return fail(c, SONAR_ERR_INVALID, "out[" + std::to_string(i) + "].mfcc is null");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  // segment table {pcm address, n, F, out address, first pair} in pinned staging, and the batch's
  // buffers; the staging is reused once the previous call's table upload has completed
  const size_t seg_n = 5 * (size_t)count + 1;
  if (c->fpb_ev) HIP_TRY(c, hipEventSynchronize(c->fpb_ev));
  else HIP_TRY(c, hipEventCreateWithFlags(&c->fpb_ev, hipEventDisableTiming));
  int64_t* seg = (int64_t*)hbuf(c, "fpb.seg", seg_n * 8);
  if (!seg) return fail(c, SONAR_ERR_NOMEM, "pinned allocation failed (batch table)");
  int64_t NP = 0, ns = 0, nf = 0;
  for (int i = 0; i < count; i++) {
    const int64_t F = go_frames(n[i], W, H);
    // frames whose W samples lie inside the signal (F itself unless n < W: Go's count truncates)
    seg[2 * (size_t)count + i] = F; seg[(size_t)count + i] = n[i] >= W ? std::min<int64_t>(F, (n[i] - W) / H + 1) : 0;
    seg[4 * (size_t)count + i] = NP;
    NP += (F + 1) / 2; ns += n[i]; nf += F;
  }
  seg[5 * (size_t)count] = NP;
  float* dpcm = nullptr;
  float* dout = nullptr;
  if (!dev) {
    dpcm = (float*)dbuf(c, "fpb.pcm", (size_t)ns * 4);
    dout = (float*)dbuf(c, "fpb.mfcc", (size_t)nf * t.n_mfcc * 4);
    if (!dpcm || !dout) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (batch)");
  }
  int64_t po = 0, fo = 0;
  for (int i = 0; i < count; i++) {
    if (dev) {
      seg[i] = (int64_t)(uintptr_t)pcm[i];
      seg[3 * (size_t)count + i] = (int64_t)(uintptr_t)out[i].mfcc;
    } else {
      HIP_TRY(c, hipMemcpyAsync(dpcm + po, pcm[i], (size_t)n[i] * 4, hipMemcpyHostToDevice, s));
      seg[i] = (int64_t)(uintptr_t)(dpcm + po);
      seg[3 * (size_t)count + i] = (int64_t)(uintptr_t)(dout + fo * t.n_mfcc);
    }
    po += n[i]; fo += seg[2 * (size_t)count + i];
  }
  int64_t* dseg = (int64_t*)dbuf(c, "fpb.seg", seg_n * 8);
  if (!dseg) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (batch table)");
  HIP_TRY(c, hipMemcpyAsync(dseg, seg, seg_n * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipEventRecord(c->fpb_ev, s));
  sonar::MfccPairParams q{};
  fill_pair_params(c, t, cfg, NP, q);
  q.F = 2 * NP; q.H = H;
  q.seg = dseg; q.nseg = count;
  hipEvent_t tend = timed_begin(c, s);
  const int lrc = sonar::launch_mfcc_pair(q, s);
  if (lrc == -4) return fail(c, SONAR_ERR_UNSUPPORTED, "too many frames for one mfcc_pair_kernel launch");
  if (lrc != 0)
    return fail(c, SONAR_ERR_DEVICE, std::string("mfcc kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
  timed_end(c, s, tend);
  c->last_fp_kernel = "mfcc_pair_kernel";
  if (!dev) {
    fo = 0;
    for (int i = 0; i < count; i++) {
      const int64_t F = seg[2 * (size_t)count + i];
      HIP_TRY(c, hipMemcpyAsync(out[i].mfcc, dout + fo * t.n_mfcc, (size_t)F * t.n_mfcc * 4, hipMemcpyDeviceToHost, s));
      fo += F;
    }
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SONAR_OK;
}

// ========================================================= YIN, chroma ====
int sonar_pitch_yin(sonar_ctx* c, const double* pcm, int64_t n, int32_t sr, double* pitch, double* conf, int32_t* tau,
                    int32_t device_ptrs) {
  if (!c) return SONAR_ERR_INVALID;
  const int64_t F = sonar_pitch_frames(n);
  if (F == 0) return SONAR_OK;
  if (!pcm || !pitch || !conf) return fail(c, SONAR_ERR_INVALID, "null buffer");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const double* dp = pcm;
  double *dpi = pitch, *dco = conf;
  int32_t* dta = tau;
  if (!device_ptrs) {
    void* b = dbuf(c, "yin.pcm", n * 8);
    dpi = (double*)dbuf(c, "yin.p", F * 8);
    dco = (double*)dbuf(c, "yin.c", F * 8);
    dta = tau ? (int32_t*)dbuf(c, "yin.t", F * 4) : nullptr;
    if (!b || !dpi || !dco) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    HIP_TRY(c, hipMemcpyAsync(b, pcm, n * 8, hipMemcpyHostToDevice, s));
    dp = (const double*)b;
  }
  if (sonar::launch_yin(dp, n, F, 512, sr, dpi, dco, dta, s) != 0) return fail(c, SONAR_ERR_DEVICE, "yin launch failed");
  if (!device_ptrs) {
    HIP_TRY(c, hipMemcpyAsync(pitch, dpi, F * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(conf, dco, F * 8, hipMemcpyDeviceToHost, s));
    if (tau) HIP_TRY(c, hipMemcpyAsync(tau, dta, F * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SONAR_OK;
}

int sonar_chroma_stft(sonar_ctx* c, const double* pcm, int64_t n, int64_t F, int32_t hop, int32_t sr, int32_t preprocess,
                      double* chroma, int32_t device_ptrs) {
  if (!c) return SONAR_ERR_INVALID;
  if (!pcm || n <= 0 || F <= 0) return fail(c, SONAR_ERR_INVALID, "invalid input data");
  if (hop <= 0) return fail(c, SONAR_ERR_INVALID, "hop size must be positive");
  const int fs = (int)(n / F);                                    // music.go:331
  if (fs <= 0) return fail(c, SONAR_ERR_INVALID, "window size must be positive");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const double* dp = pcm;
  double* dout = chroma;
  if (!device_ptrs) {
    void* b = dbuf(c, "chroma.pcm", n * 8);
    dout = (double*)dbuf(c, "chroma.out", F * 12 * 8);
    if (!b || !dout) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    HIP_TRY(c, hipMemcpyAsync(b, pcm, n * 8, hipMemcpyHostToDevice, s));
    dp = (const double*)b;
  }
  const double* y = dp;
  if (preprocess) {
    double* yb = (double*)dbuf(c, "chroma.y", n * 8);
    if (!yb) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    double* dcs = (double*)dbuf(c, "chroma.dcscratch", sonar::dc_preemph_scratch_bytes(n));
    if (!dcs) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    if (sonar::launch_dc_preemph(dp, n, 0.995, 0.95, yb, dcs, s) != 0) return fail(c, SONAR_ERR_DEVICE, "dc launch failed");
    y = yb;
  }
  const sonar_ctx::ChromaT* ct = sonar::detail::chroma_tables_for(c, fs, sr);
  if (!ct) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  const int* cls = (const int*)ct->cls;
  if (sonar::launch_chroma(y, n, F, hop, fs, (const double*)ct->win, (const double*)ct->trig,
                           (const int*)ct->map, cls, dout, s) != 0)
    return fail(c, SONAR_ERR_UNSUPPORTED, "chroma launch failed (frame size too large for LDS?)");
  if (!device_ptrs) {
    HIP_TRY(c, hipMemcpyAsync(chroma, dout, F * 12 * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SONAR_OK;
}

}  // extern "C"

namespace sonar {
namespace detail {
// the chroma tables of frame size fs at sample rate sr (ChromaSTFT, chroma_stft.go:45-138), built
// once per context: Hann window, the bin -> class map, the FFT twiddles, per-class bin lists
const sonar_ctx::ChromaT* chroma_tables_for(sonar_ctx* c, int fs, int sr) {
  const std::string key = std::to_string(fs) + "|" + std::to_string(sr);
  auto it = c->chroma_tables.find(key);
  if (it == c->chroma_tables.end()) {
    std::vector<double> win;
    sonar::host::make_window(SONAR_WIN_HANN, fs, true, true, kStftBeta, kStftAlpha, win);
    std::vector<int> map = sonar::host::chroma_map(fs, sr);
    std::vector<double> trig(2 * (size_t)fs);
    for (int m = 0; m < fs; m++) {
      trig[2 * m] = std::cos(2.0 * M_PI * (double)m / (double)fs);
      trig[2 * m + 1] = -std::sin(2.0 * M_PI * (double)m / (double)fs);
    }
    // per chroma class, its bins in ascending order (the fold order of music.go:366-372)
    std::vector<int> cls(13 + map.size());
    int e = 0;
    for (int b = 0; b < 12; ++b) {
      cls[b] = e;
      for (size_t k = 0; k < map.size(); ++k)
        if (map[k] == b) cls[13 + e++] = (int)k;
    }
    cls[12] = e;
    const sonar_ctx::ChromaT t{upload(win), upload(trig), upload(map), upload(cls)};
    if (!t.win || !t.trig || !t.map || !t.cls) return nullptr;
    it = c->chroma_tables.emplace(key, t).first;
  }
  return &it->second;
}
}  // namespace detail
}  // namespace sonar

extern "C" {

// ================================================================ NCC ====
int sonar_ncc(sonar_ctx* c, const double* a, int64_t na, const double* b, int64_t nb, int32_t max_lag, double* corr,
              double* metrics, int32_t device_ptrs) {
  if (!c) return SONAR_ERR_INVALID;
  if (na <= 0 || nb <= 0 || !a || !b) return fail(c, SONAR_ERR_EMPTY, "empty signals provided");
  int64_t L = max_lag;                                            // calculateActualMaxLag :452-461
  L = std::min<int64_t>(L, na - 1);
  L = std::min<int64_t>(L, nb - 1);
  L = std::max<int64_t>(L, 0);
  const int64_t nl = 2 * L + 1;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const double *da = a, *db = b;
  if (!device_ptrs) {
    double* pa = (double*)dbuf(c, "ncc.a", na * 8);
    double* pb = (double*)dbuf(c, "ncc.b", nb * 8);
    if (!pa || !pb) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    HIP_TRY(c, hipMemcpyAsync(pa, a, na * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(pb, b, nb * 8, hipMemcpyHostToDevice, s));
    da = pa; db = pb;
  }
  double* xa = (double*)dbuf(c, "ncc.xa", na * 8);
  double* xb = (double*)dbuf(c, "ncc.xb", nb * 8);
  double* st = (double*)dbuf(c, "ncc.stats", 64);
  double* dc = (device_ptrs && corr) ? corr : (double*)dbuf(c, "ncc.corr", nl * 8);
  if (!xa || !xb || !st || !dc) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  hipEvent_t tend = timed_begin(c, s);
  if (sonar::launch_ncc(da, na, db, nb, L, xa, xb, st, dc, s) != 0) return fail(c, SONAR_ERR_DEVICE, "ncc launch failed");
  timed_end(c, s, tend);
  std::vector<double> hc(nl);
  HIP_TRY(c, hipMemcpyAsync(hc.data(), dc, nl * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  if (corr && !device_ptrs) std::memcpy(corr, hc.data(), nl * 8);
  if (metrics) {
    const auto m = sonar::host::ncc_metrics(hc.data(), nl, L, na, nb);
    const double v[10] = {m.peak_corr, (double)m.peak_lag, (double)m.peak_index, m.p_value, m.snr, m.sharpness,
                          m.second_peak, m.psl, (double)m.overlap, (double)m.num_lags};
    std::memcpy(metrics, v, sizeof(v));
  }
  return SONAR_OK;
}

// ================================================================ DTW ====
int sonar_dtw(sonar_ctx* c, const double* q, int64_t nq, const double* r, int64_t nr, int32_t dim, int32_t band,
              double* distance, int32_t* path_q, int32_t* path_r, double* path_cost, int64_t* path_len, double* cost,
              int32_t device_ptrs) {
  if (!c) return SONAR_ERR_INVALID;
  if (nq <= 0 || nr <= 0 || !q || !r) return fail(c, SONAR_ERR_EMPTY, "empty sequences provided");
  if (dim <= 0) return fail(c, SONAR_ERR_INVALID, "feature dimension must be positive");
  if (nq + nr > (int64_t)INT32_MAX) return fail(c, SONAR_ERR_UNSUPPORTED, "sequence too long");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const double *dq = q, *dr = r;
  if (!device_ptrs) {
    double* pq = (double*)dbuf(c, "dtw.q", nq * dim * 8);
    double* pr = (double*)dbuf(c, "dtw.r", nr * dim * 8);
    if (!pq || !pr) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    HIP_TRY(c, hipMemcpyAsync(pq, q, nq * dim * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(pr, r, nr * dim * 8, hipMemcpyHostToDevice, s));
    dq = pq; dr = pr;
  }
  const sonar::DtwGeom g = sonar::dtw_geom(nq, nr);
  // the full cost store only when the caller asks for the cost matrix; otherwise every 64th
  // column (CK) and the path costs recomputed per visited tile
  const bool full = cost != nullptr;
  double* Cn = full ? (double*)dbuf(c, "dtw.Cn", sonar::dtw_cn_bytes(g)) : nullptr;
  double* CK = full ? nullptr : (double*)dbuf(c, "dtw.CK", sonar::dtw_ck_bytes(g));
  int32_t* runs = full ? nullptr : (int32_t*)dbuf(c, "dtw.runs", (size_t)sonar::dtw_run_words(g) * 4);
  double* cnm_d = (double*)dbuf(c, "dtw.cnm", 8);
  uint32_t* Dn = (uint32_t*)dbuf(c, "dtw.Dn", sonar::dtw_dn_bytes(g));
  uint64_t* E = (uint64_t*)dbuf(c, "dtw.E", sonar::dtw_edge_bytes(g));
  int32_t* sync = (int32_t*)dbuf(c, "dtw.sync", sonar::DTW_SYNC_BYTES);
  const int64_t cap = nq + nr + 1;
  uint32_t* codes = (uint32_t*)dbuf(c, "dtw.codes", ((cap + 1023) / 1024) * 64 * 4);
  int64_t* pl = (int64_t*)dbuf(c, "dtw.plen", 16);
  if ((full ? !Cn : (!CK || !runs)) || !cnm_d || !Dn || !E || !sync || !codes || !pl)
    return fail(c, SONAR_ERR_NOMEM, "device allocation failed (cost matrix)");
  // math.Min's NaN / -Inf / -0 rules only matter when an input is not finite
  bool fast = true;
  if (!device_ptrs) {
    for (int64_t k = 0; k < nq * dim && fast; ++k) fast = std::isfinite(q[k]);
    for (int64_t k = 0; k < nr * dim && fast; ++k) fast = std::isfinite(r[k]);
  } else {
    HIP_TRY(c, hipMemsetAsync(sync + 2, 0, 4, s));
    if (sonar::launch_nonfinite(dq, nq * dim, sync + 2, s) || sonar::launch_nonfinite(dr, nr * dim, sync + 2, s))
      return fail(c, SONAR_ERR_DEVICE, "dtw launch failed");
    int32_t nf = 0;
    HIP_TRY(c, hipMemcpyAsync(&nf, sync + 2, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    fast = nf == 0;
  }
  // SONAR_DTW_TRACE=<file>: per-band timestamps of the sweep (diagnostics only)
  const char* trace_path = std::getenv("SONAR_DTW_TRACE");
  uint64_t* trace = trace_path ? (uint64_t*)dbuf(c, "dtw.trace", (size_t)g.nb * 64) : nullptr;
  for (auto& e : c->dtw_ev)
    if (!e) HIP_TRY(c, hipEventCreate(&e));
  hipEvent_t tend = timed_begin(c, s);
  HIP_TRY(c, hipEventRecord(c->dtw_ev[0], s));
  if (sonar::launch_dtw(dq, dr, dim, band, fast, g, Cn, Dn, E, sync, codes, pl, trace, s, c->dtw_ev[1], CK) != 0)
    return fail(c, SONAR_ERR_DEVICE, "dtw launch failed");
  HIP_TRY(c, hipEventRecord(c->dtw_ev[2], s));
  timed_end(c, s, tend);
  if (trace) {
    std::vector<uint64_t> t((size_t)g.nb * 8);
    HIP_TRY(c, hipMemcpyAsync(t.data(), trace, t.size() * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (FILE* f = std::fopen(trace_path, "wb")) { std::fwrite(t.data(), 8, t.size(), f); std::fclose(f); }
  }
  int64_t P = 0;
  alignas(8) char sblk[sonar::DTW_SYNC_BYTES];
  HIP_TRY(c, hipMemcpyAsync(&P, pl, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(sblk, sync, sizeof(sblk), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  {
    const std::string why = sonar::detail::dtw_status(c, sblk);
    if (!why.empty()) return fail(c, SONAR_ERR_DEVICE, why);
  }
  int32_t* oq = path_q; int32_t* orr = path_r; double* oc = path_cost;
  if (!device_ptrs) {
    oq = (int32_t*)dbuf(c, "dtw.pq", cap * 4);
    orr = (int32_t*)dbuf(c, "dtw.pr", cap * 4);
    oc = (double*)dbuf(c, "dtw.pc", cap * 8);
    if (!oq || !orr || !oc) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (path)");
  }
  int2* wstart = (int2*)dbuf(c, "dtw.wstart", (size_t)((P + 15) / 16 + 1) * sizeof(int2));
  if (!wstart) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (path)");
  if (sonar::launch_dtw_path_cost(Cn, g, codes, P, wstart, oq, orr, oc, s) != 0 ||
      (!full && sonar::launch_dtw_path_tiles(sonar::detail::tile_args(dq, dr, dim, band, g, E, CK, runs, oq, orr, oc,
                                                                        pl, cnm_d), P, s) != 0))
    return fail(c, SONAR_ERR_DEVICE, "dtw path launch failed");
  HIP_TRY(c, hipEventRecord(c->dtw_ev[3], s));
  double cNM = 0;
  HIP_TRY(c, hipMemcpyAsync(&cNM, full ? Cn + sonar::dtw_cn_index(g, nq, nr) : cnm_d, 8, hipMemcpyDeviceToHost, s));
  double* cost_dev = cost;
  if (cost && !device_ptrs) {
    cost_dev = (double*)dbuf(c, "dtw.cost", (size_t)nq * (nr + 1) * 8);
    if (!cost_dev) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (cost output)");
  }
  if (cost && sonar::launch_dtw_cost_rowmajor(Cn, g, cost_dev, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "dtw cost launch failed");
  if (!device_ptrs) {
    if (path_q) HIP_TRY(c, hipMemcpyAsync(path_q, oq, P * 4, hipMemcpyDeviceToHost, s));
    if (path_r) HIP_TRY(c, hipMemcpyAsync(path_r, orr, P * 4, hipMemcpyDeviceToHost, s));
    if (path_cost) HIP_TRY(c, hipMemcpyAsync(path_cost, oc, P * 8, hipMemcpyDeviceToHost, s));
    if (cost) HIP_TRY(c, hipMemcpyAsync(cost, cost_dev, (size_t)nq * (nr + 1) * 8, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  for (int k = 0; k < 3; ++k) {
    float f = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&f, c->dtw_ev[k], c->dtw_ev[k + 1]));
    c->dtw_ms[k] = f;
  }
  if (path_len) *path_len = P;
  if (distance) *distance = cNM / (double)P;                      // dtw.go:88-91
  return SONAR_OK;
}

}  // extern "C"

// ============================================= deferred-sync pair pieces ====
namespace sonar {
namespace detail {

std::string dtw_status(sonar_ctx* c, const void* sync_block) {
  int32_t sync[4];
  uint64_t d[sonar::DTW_DIAG_WORDS];
  std::memcpy(sync, sync_block, 16);
  std::memcpy(d, static_cast<const char*>(sync_block) + 16, sizeof(d));
  c->dtw_ctr[0] += (long long)d[13];
  c->dtw_ctr[1] += (long long)d[14];
  c->dtw_ctr[3] += (long long)d[15];
  if (!sync[1]) return std::string();
  c->dtw_ctr[2] += 1;
  static const char* roles[] = {"?", "edge", "feeder", "sweep", "code", "distance", "loader"};
  std::string roles_hit;
  for (int k = 0; k < 6; ++k)
    if (sync[1] & (1 << k)) roles_hit += std::string(roles_hit.empty() ? "" : "+") + roles[k + 1];
  char buf[768];
  if (!(d[0] >> 63)) {
    std::snprintf(buf, sizeof(buf), "dtw band pipeline timed out (roles %s; no diagnostic record)", roles_hit.c_str());
    return buf;
  }
  const int role = (int)((d[0] >> 56) & 0x7F);
  const uint64_t ticks = d[11] & 0xFFFFFFFFFFull;
  std::snprintf(buf, sizeof(buf),
                "dtw band pipeline timed out (roles %s): first %s wave, band %u ticket %u, no progress for %.3f s "
                "(%llu k polls); prog %u cprog %u efill %u rdy %d dchunk %u/%u/%u/%u edge target %u of %u; "
                "E[efill+1] sc1 %016llx after-acquire %016llx system %016llx rmw-agent %016llx rmw-system %016llx; "
                "first sentinel column %lld; xcc %u hw_id %08x; waves timed out %llu; refresh fences %llu (%llu hit)",
                roles_hit.c_str(), roles[role >= 1 && role <= 6 ? role : 0], (unsigned)(d[0] & 0xFFFFFFFF),
                (unsigned)((d[0] >> 32) & 0xFFFFFF), ticks * 1e-8, (unsigned long long)(d[11] >> 40),
                (unsigned)(d[1] & 0xFFFFFFFF), (unsigned)(d[1] >> 32), (unsigned)(d[2] & 0xFFFFFFFF),
                (int)(int32_t)(d[2] >> 32), (unsigned)(d[3] & 0xFFFF), (unsigned)((d[3] >> 16) & 0xFFFF),
                (unsigned)((d[3] >> 32) & 0xFFFF), (unsigned)((d[3] >> 48) & 0xFFFF), (unsigned)(d[4] & 0xFFFFFFFF),
                (unsigned)(d[4] >> 32), (unsigned long long)d[5], (unsigned long long)d[6], (unsigned long long)d[7],
                (unsigned long long)d[8], (unsigned long long)d[9], (long long)(int64_t)d[10], (unsigned)(d[12] & 0xFF),
                (unsigned)(d[12] >> 32), (unsigned long long)d[15], (unsigned long long)d[13],
                (unsigned long long)d[14]);
  return buf;
}

sonar::DtwArgs tile_args(const double* q, const double* r, int dim, int band, const sonar::DtwGeom& g, uint64_t* E,
                         double* CK, int32_t* runs, int32_t* pq, int32_t* pr, double* pc, int64_t* plen, double* cnm) {
  sonar::DtwArgs a{};
  a.q = q; a.r = r; a.dim = dim; a.band = band;
  a.nq = g.nq; a.nr = g.nr; a.nb = g.nb; a.S = g.S; a.SW = g.SW;
  a.E = E; a.CK = CK; a.runs = runs; a.pq = pq; a.pr = pr; a.pc = pc; a.plen = plen; a.cnm = cnm;
  return a;
}

void ncc_metrics_host(const double* corr, int64_t L, int64_t na, int64_t nb, double* metrics) {
  const auto m = sonar::host::ncc_metrics(corr, 2 * L + 1, L, na, nb);
  const double v[10] = {m.peak_corr, (double)m.peak_lag, (double)m.peak_index, m.p_value, m.snr, m.sharpness,
                        m.second_peak, m.psl, (double)m.overlap, (double)m.num_lags};
  std::memcpy(metrics, v, sizeof(v));
}

// sonar_ncc's launch half: the correlation lands in pinned host memory once the stream drains
int ncc_enqueue(sonar_ctx* c, const double* da, int64_t na, const double* db, int64_t nb, int32_t max_lag,
                double** hcorr, int64_t* Lout) {
  if (na <= 0 || nb <= 0 || !da || !db) return fail(c, SONAR_ERR_EMPTY, "empty signals provided");
  int64_t L = max_lag;                                            // calculateActualMaxLag :452-461
  L = std::max<int64_t>(std::min({L, na - 1, nb - 1}), 0);
  const int64_t nl = 2 * L + 1;
  hipStream_t s = c->stream;
  double* xa = (double*)dbuf(c, "ncc.xa", na * 8);
  double* xb = (double*)dbuf(c, "ncc.xb", nb * 8);
  double* st = (double*)dbuf(c, "ncc.stats", 64);
  double* dc = (double*)dbuf(c, "ncc.corr", nl * 8);
  double* hc = (double*)hbuf(c, "ncc.corr", nl * 8);
  if (!xa || !xb || !st || !dc || !hc) return fail(c, SONAR_ERR_NOMEM, "allocation failed (ncc)");
  if (sonar::launch_ncc(da, na, db, nb, L, xa, xb, st, dc, s) != 0) return fail(c, SONAR_ERR_DEVICE, "ncc launch failed");
  HIP_TRY(c, hipMemcpyAsync(hc, dc, nl * 8, hipMemcpyDeviceToHost, s));
  *hcorr = hc;
  *Lout = L;
  return SONAR_OK;
}

// sonar_dtw's launch half for device sequences: the non-finite probe runs on the device and the
// FAST (finite-input) pipeline is launched without waiting for it; dtw_finish re-runs the exact
// math.Min pipeline in the rare case the probe fired
int dtw_enqueue(sonar_ctx* c, const double* dq, int64_t nq, const double* dr, int64_t nr, int32_t dim, int32_t band,
                DtwPending* p) {
  if (nq <= 0 || nr <= 0 || !dq || !dr) return fail(c, SONAR_ERR_EMPTY, "empty sequences provided");
  if (dim <= 0) return fail(c, SONAR_ERR_INVALID, "feature dimension must be positive");
  if (nq + nr > (int64_t)INT32_MAX) return fail(c, SONAR_ERR_UNSUPPORTED, "sequence too long");
  hipStream_t s = c->stream;
  const sonar::DtwGeom g = sonar::dtw_geom(nq, nr);
  double* CK = (double*)dbuf(c, "dtw.CK", sonar::dtw_ck_bytes(g));
  uint32_t* Dn = (uint32_t*)dbuf(c, "dtw.Dn", sonar::dtw_dn_bytes(g));
  uint64_t* E = (uint64_t*)dbuf(c, "dtw.E", sonar::dtw_edge_bytes(g));
  int32_t* sync = (int32_t*)dbuf(c, "dtw.sync", sonar::DTW_SYNC_BYTES);
  const int64_t cap = nq + nr + 1;
  uint32_t* codes = (uint32_t*)dbuf(c, "dtw.codes", ((cap + 1023) / 1024) * 64 * 4);
  int64_t* pl = (int64_t*)dbuf(c, "dtw.plen", 16);
  int64_t* st = (int64_t*)hbuf(c, "dtw.status", 8 + sonar::DTW_SYNC_BYTES);
  if (!CK || !Dn || !E || !sync || !codes || !pl || !st) return fail(c, SONAR_ERR_NOMEM, "allocation failed (dtw)");
  HIP_TRY(c, hipMemsetAsync(sync + 2, 0, 4, s));
  if (sonar::launch_nonfinite(dq, nq * dim, sync + 2, s) || sonar::launch_nonfinite(dr, nr * dim, sync + 2, s))
    return fail(c, SONAR_ERR_DEVICE, "dtw launch failed");
  if (sonar::launch_dtw(dq, dr, dim, band, true, g, nullptr, Dn, E, sync, codes, pl, nullptr, s, nullptr, CK) != 0)
    return fail(c, SONAR_ERR_DEVICE, "dtw launch failed");
  HIP_TRY(c, hipMemcpyAsync(st, pl, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(st + 1, sync, sonar::DTW_SYNC_BYTES, hipMemcpyDeviceToHost, s));
  *p = DtwPending{dq, dr, nq, nr, dim, band, st};
  return SONAR_OK;
}

// after the caller's stream sync: decode the path into pinned host arrays (one more sync)
int dtw_finish(sonar_ctx* c, DtwPending* p, const int32_t** hq, const int32_t** hr, const double** hc, int64_t* Pout,
               double* distance) {
  hipStream_t s = c->stream;
  const sonar::DtwGeom g = sonar::dtw_geom(p->nq, p->nr);
  const int64_t cap = p->nq + p->nr + 1;
  double* CK = (double*)dbuf(c, "dtw.CK", sonar::dtw_ck_bytes(g));
  uint32_t* Dn = (uint32_t*)dbuf(c, "dtw.Dn", sonar::dtw_dn_bytes(g));
  uint64_t* E = (uint64_t*)dbuf(c, "dtw.E", sonar::dtw_edge_bytes(g));
  int32_t* sync = (int32_t*)dbuf(c, "dtw.sync", sonar::DTW_SYNC_BYTES);
  uint32_t* codes = (uint32_t*)dbuf(c, "dtw.codes", ((cap + 1023) / 1024) * 64 * 4);
  int64_t* pl = (int64_t*)dbuf(c, "dtw.plen", 16);
  int32_t* runs = (int32_t*)dbuf(c, "dtw.runs", (size_t)sonar::dtw_run_words(g) * 4);
  double* cnm_d = (double*)dbuf(c, "dtw.cnm", 8);
  if (!runs || !cnm_d) return fail(c, SONAR_ERR_NOMEM, "allocation failed (dtw path)");
  int32_t nfw[3];
  std::memcpy(nfw, p->st + 1, 12);
  if (nfw[2] != 0) {                                              // non-finite input: exact math.Min rules
    if (sonar::launch_dtw(p->dq, p->dr, p->dim, p->band, false, g, nullptr, Dn, E, sync, codes, pl, nullptr, s, nullptr,
                          CK))
      return fail(c, SONAR_ERR_DEVICE, "dtw launch failed");
    HIP_TRY(c, hipMemcpyAsync(p->st, pl, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(p->st + 1, sync, sonar::DTW_SYNC_BYTES, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    std::memcpy(nfw, p->st + 1, 8);
  }
  {
    const std::string why = dtw_status(c, p->st + 1);
    if (!why.empty()) return fail(c, SONAR_ERR_DEVICE, why);
  }
  const int64_t P = p->st[0];
  int32_t* oq = (int32_t*)dbuf(c, "dtw.pq", cap * 4);
  int32_t* orr = (int32_t*)dbuf(c, "dtw.pr", cap * 4);
  double* oc = (double*)dbuf(c, "dtw.pc", cap * 8);
  int2* wstart = (int2*)dbuf(c, "dtw.wstart", (size_t)((P + 15) / 16 + 1) * sizeof(int2));
  // one pinned block: cost(N,M), path costs, then the two index arrays
  char* h = (char*)hbuf(c, "dtw.path", 8 + (size_t)cap * 16);
  if (!oq || !orr || !oc || !wstart || !h) return fail(c, SONAR_ERR_NOMEM, "allocation failed (dtw path)");
  if (sonar::launch_dtw_path_cost(nullptr, g, codes, P, wstart, oq, orr, oc, s) != 0 ||
      sonar::launch_dtw_path_tiles(tile_args(p->dq, p->dr, p->dim, p->band, g, E, CK, runs, oq, orr, oc, pl, cnm_d), P,
                                   s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "dtw path launch failed");
  double* hcnm = (double*)h;
  double* hcost = hcnm + 1;
  int32_t* hpq = (int32_t*)(hcost + cap);
  int32_t* hpr = hpq + cap;
  HIP_TRY(c, hipMemcpyAsync(hcnm, cnm_d, 8, hipMemcpyDeviceToHost, s));
  if (P > 0) {
    HIP_TRY(c, hipMemcpyAsync(hcost, oc, P * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(hpq, oq, P * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(hpr, orr, P * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  *hq = hpq; *hr = hpr; *hc = hcost;
  *Pout = P;
  *distance = *hcnm / (double)P;                                  // dtw.go:88-91
  return SONAR_OK;
}

}  // namespace detail
}  // namespace sonar

extern "C" {

// ========================================================= formants ====
namespace {
int formant_geometry(int sr, int* W, int* p) {
  *W = sr >= 16000 ? 2048 : 1024;                    // NewFormantAnalyzer (format.go:48-69)
  *p = 12 + sr / 1000;
  return 0;
}
int run_formants(sonar_ctx* c, const double* pcm, int64_t n, int sr, int64_t frames, int64_t hop, bool ok_len,
                 sonar_formant_frame* out, double* coeffs, double* refl, int device_ptrs) {
  int W, p;
  formant_geometry(sr, &W, &p);
  if (p > 64) return fail(c, SONAR_ERR_UNSUPPORTED, "LPC order above 64 (sample rate > 52 kHz)");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  std::vector<double> ham(W);
  for (int i = 0; i < W; ++i) ham[i] = 0.54 - 0.46 * std::cos(2.0 * M_PI * (double)i / (double)(W - 1));
  double* dham = (double*)dbuf(c, "lpc.ham", W * 8);
  if (!dham) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
  HIP_TRY(c, hipMemcpyAsync(dham, ham.data(), W * 8, hipMemcpyHostToDevice, s));
  const double* dp = pcm;
  sonar_formant_frame* dout = out;
  double *dco = coeffs, *dre = refl;
  if (!device_ptrs) {
    double* b = (double*)dbuf(c, "lpc.pcm", std::max<int64_t>(n, 1) * 8);
    dout = (sonar_formant_frame*)dbuf(c, "lpc.out", std::max<int64_t>(frames, 1) * sizeof(sonar_formant_frame));
    dco = coeffs ? (double*)dbuf(c, "lpc.coeffs", std::max<int64_t>(frames, 1) * (p + 1) * 8) : nullptr;
    dre = refl ? (double*)dbuf(c, "lpc.refl", std::max<int64_t>(frames, 1) * p * 8) : nullptr;
    if (!b || !dout || (coeffs && !dco) || (refl && !dre)) return fail(c, SONAR_ERR_NOMEM, "device allocation failed");
    HIP_TRY(c, hipMemcpyAsync(b, pcm, n * 8, hipMemcpyHostToDevice, s));
    dp = b;
  }
  hipEvent_t tend = timed_begin(c, s);
  if (sonar::launch_formants(dp, frames, hop, W, p, sr, ok_len ? 1 : 0, dham, dout, dco, dre, s) != 0)
    return fail(c, SONAR_ERR_DEVICE, "formant launch failed");
  timed_end(c, s, tend);
  if (!device_ptrs) {
    HIP_TRY(c, hipMemcpyAsync(out, dout, frames * sizeof(sonar_formant_frame), hipMemcpyDeviceToHost, s));
    if (coeffs) HIP_TRY(c, hipMemcpyAsync(coeffs, dco, frames * (p + 1) * 8, hipMemcpyDeviceToHost, s));
    if (refl) HIP_TRY(c, hipMemcpyAsync(refl, dre, frames * p * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return SONAR_OK;
}
}  // namespace

extern "C" {

int64_t sonar_formant_frame_count(int64_t n, int32_t sample_rate, int32_t frame_size, int32_t hop_size) {
  int W, p;
  formant_geometry(sample_rate, &W, &p);
  if (frame_size <= 0) frame_size = W;
  if (hop_size <= 0) hop_size = frame_size / 2;
  if (hop_size <= 0) return 0;
  return n > frame_size ? (n - frame_size - 1) / hop_size + 1 : 0;   // for i := 0; i < n-frameSize; i += hop
}

int sonar_formants(sonar_ctx* c, const double* pcm, int64_t n, int32_t sample_rate, int32_t frame_size,
                   int32_t hop_size, sonar_formant_frame* out, double* lpc_coeffs, double* reflection,
                   int32_t device_ptrs) {
  if (!c) return SONAR_ERR_INVALID;
  if (sample_rate <= 0) return fail(c, SONAR_ERR_INVALID, "sample rate must be positive");
  int W, p;
  formant_geometry(sample_rate, &W, &p);
  if (frame_size <= 0) frame_size = W;
  if (hop_size <= 0) hop_size = frame_size / 2;
  if (hop_size <= 0) return fail(c, SONAR_ERR_INVALID, "hop size must be positive");
  const int64_t frames = sonar_formant_frame_count(n, sample_rate, frame_size, hop_size);
  if (frames == 0) return SONAR_OK;
  if (!pcm || !out) return fail(c, SONAR_ERR_INVALID, "null buffer");
  return run_formants(c, pcm, n, sample_rate, frames, hop_size, frame_size >= W, out, lpc_coeffs, reflection,
                      device_ptrs);
}

}  // extern "C"

int sonar_analyze_formants_host(sonar_ctx* c, const double* pcm, int64_t n, int sample_rate, sonar_formant_frame* out) {
  int W, p;
  formant_geometry(sample_rate, &W, &p);
  return run_formants(c, pcm, n, sample_rate, 1, 0, n >= W, out, nullptr, nullptr, 0);
}

// ====================================================== result object ====
int sonar_result_get(const sonar_result* r, const char* name, const double** data, int64_t* rows, int64_t* cols) {
  if (!r || !name) return SONAR_ERR_INVALID;
  for (const auto& a : r->arrays)
    if (a.name == name) {
      if (data) *data = a.data();
      if (rows) *rows = a.rows;
      if (cols) *cols = a.cols;
      return SONAR_OK;
    }
  return SONAR_ERR_INVALID;
}
int sonar_result_count(const sonar_result* r) { return r ? (int)r->arrays.size() : 0; }
const char* sonar_result_name(const sonar_result* r, int i) {
  return (r && i >= 0 && i < (int)r->arrays.size()) ? r->arrays[i].name.c_str() : nullptr;
}
void sonar_result_free(sonar_result* r) { delete r; }

}  // extern "C"
