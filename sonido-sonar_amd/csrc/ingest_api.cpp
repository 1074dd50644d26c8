// ingest_api.cpp -- the input side of path A:
//
//   sonar_ingest_f64le   Decoder.bytesToFloat64 + processFFmpegOutput's empty check
//                        (transcode/decoder.go:850-871, :782-787), with ffmpeg writing "-f f64le"
//                        (decoder.go:709), ending in device memory instead of a Go []float64.
//
// The Go decoder walks the byte slice once, one binary.LittleEndian.Uint64 per sample.  Here the
// byte stream is cut into chunks that cross PCIe from a ring of pinned host slots: a persistent
// pool of host threads fills slot i+1 (a copy, or the f64 -> f32 rounding in HOST_CONVERT mode)
// while the DMA engine drains slot i on the ctx stream, so the host fill, the PCIe transfer and
// (DEVICE_CONVERT with f32 output) the conversion kernel overlap.  A slot is refilled only after
// the event recorded behind its copy has completed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ctx.h"
#include "kernels.h"

using sonar::detail::dbuf;
using sonar::detail::fail;

namespace {

constexpr int kSlots = 3;
constexpr size_t kSlotBytes = size_t(32) << 20;  // bytes that cross PCIe per chunk

// Persistent fork-join pool: run(fn) calls fn(t, T) on T threads (the caller is thread 0).
class HostPool {
 public:
  explicit HostPool(int T) : T_(T) {
    for (int t = 1; t < T_; t++) th_.emplace_back([this, t] { loop(t); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return T_; }
  void run(const std::function<void(int, int)>& fn) {
    if (T_ == 1) { fn(0, 1); return; }
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      pending_ = T_ - 1;
      gen_++;
    }
    cv_.notify_all();
    fn(0, T_);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int, int)>* fn;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
      }
      (*fn)(t, T_);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  int T_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
  const std::function<void(int, int)>* fn_ = nullptr;
};

int default_threads() {
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int v = std::atoi(e);
    if (v > 0) return std::min(v, 64);
  }
  const int hw = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(16, hw));
}

}  // namespace

struct IngestState {
  void* slot[kSlots] = {nullptr};
  hipEvent_t ev[kSlots] = {nullptr};
  bool live[kSlots] = {false};
  HostPool* pool = nullptr;
};

namespace sonar {
namespace detail {
void ingest_release(sonar_ctx* c) {
  IngestState* st = c->ingest;
  if (!st) return;
  for (int i = 0; i < kSlots; i++) {
    if (st->ev[i]) { hipEventSynchronize(st->ev[i]); hipEventDestroy(st->ev[i]); }
    if (st->slot[i]) hipHostFree(st->slot[i]);
  }
  delete st->pool;
  delete st;
  c->ingest = nullptr;
}
}  // namespace detail
}  // namespace sonar

extern "C" {

int sonar_ingest_f64le(sonar_ctx* c, const void* bytes, int64_t nbytes, int32_t out_dtype, int32_t mode,
                       int32_t host_threads, void* d_out, int64_t* n_samples) {
  if (!c || !n_samples) return fail(c, SONAR_ERR_INVALID, "null argument");
  if (out_dtype != SONAR_F32 && out_dtype != SONAR_F64) return fail(c, SONAR_ERR_INVALID, "out_dtype");
  if (mode != SONAR_INGEST_DEVICE_CONVERT && mode != SONAR_INGEST_HOST_CONVERT)
    return fail(c, SONAR_ERR_INVALID, "mode");
  // bytesToFloat64: trim to a multiple of 8 (decoder.go:852-855); no samples -> error (:785-787)
  const int64_t n = nbytes > 0 ? nbytes / 8 : 0;
  *n_samples = n;
  if (n == 0 || !bytes) return fail(c, SONAR_ERR_EMPTY, "no audio samples decoded");
  if (!d_out) return SONAR_OK;
  if ((uintptr_t)d_out & 15) return fail(c, SONAR_ERR_INVALID, "d_out must be 16-byte aligned");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;

  IngestState* st = c->ingest;
  if (!st) {
    // build the whole state before publishing it: a failure part-way leaves c->ingest null
    IngestState* fresh = new IngestState();
    hipError_t e = hipSuccess;
    for (int i = 0; i < kSlots && e == hipSuccess; i++) {
      e = hipHostMalloc(&fresh->slot[i], kSlotBytes, hipHostMallocDefault);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&fresh->ev[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
      for (int i = 0; i < kSlots; i++) {
        if (fresh->slot[i]) (void)hipHostFree(fresh->slot[i]);
        if (fresh->ev[i]) (void)hipEventDestroy(fresh->ev[i]);
      }
      delete fresh;
      return fail(c, SONAR_ERR_DEVICE, hipGetErrorString(e));
    }
    st = c->ingest = fresh;
  }
  const int T = host_threads > 0 ? std::min(host_threads, 64) : default_threads();
  if (!st->pool || st->pool->size() != T) {
    delete st->pool;
    st->pool = new HostPool(T);
  }

  const bool f32 = out_dtype == SONAR_F32;
  const bool host_cvt = f32 && mode == SONAR_INGEST_HOST_CONVERT;
  const bool dev_cvt = f32 && !host_cvt;
  const size_t pcie_esz = host_cvt ? 4 : 8, out_esz = f32 ? 4 : 8;
  const int64_t chunk = (int64_t)(kSlotBytes / pcie_esz);  // samples per slot (multiple of 4)
  double* stage = nullptr;
  if (dev_cvt) {
    stage = (double*)dbuf(c, "ingest.stage", (size_t)kSlots * kSlotBytes);
    if (!stage) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (ingest staging)");
  }
  const unsigned char* src = (const unsigned char*)bytes;
  char* dst = (char*)d_out;

  for (int64_t off = 0, i = 0; off < n; off += chunk, i++) {
    const int k = (int)(i % kSlots);
    const int64_t m = std::min(chunk, n - off);
    if (st->live[k]) HIP_TRY(c, hipEventSynchronize(st->ev[k]));
    void* slot = st->slot[k];
    const unsigned char* in = src + off * 8;
    // fill: the T threads take contiguous 4 KB-aligned stripes of the chunk
    st->pool->run([&](int t, int TT) {
      const int64_t per = ((m + TT - 1) / TT + 511) & ~int64_t(511);
      const int64_t a = std::min(m, (int64_t)t * per), b = std::min(m, a + per);
      if (a >= b) return;
      if (!host_cvt) {
        std::memcpy((char*)slot + a * 8, in + a * 8, (size_t)(b - a) * 8);
      } else {
        float* o = (float*)slot;
        for (int64_t j = a; j < b; j++) {
          double v;
          std::memcpy(&v, in + j * 8, 8);  // LittleEndian.Uint64 + Float64frombits on x86-64
          o[j] = (float)v;                 // round to nearest even
        }
      }
    });
    if (dev_cvt) {
      double* sk = stage + (size_t)k * (kSlotBytes / 8);
      HIP_TRY(c, hipMemcpyAsync(sk, slot, (size_t)m * 8, hipMemcpyHostToDevice, s));
      HIP_TRY(c, hipEventRecord(st->ev[k], s));
      if (sonar::launch_f64_to_f32(sk, (float*)(dst + off * out_esz), m, s) != 0)
        return fail(c, SONAR_ERR_DEVICE, "f64_to_f32 launch failed");
    } else {
      HIP_TRY(c, hipMemcpyAsync(dst + off * out_esz, slot, (size_t)m * pcie_esz, hipMemcpyHostToDevice, s));
      HIP_TRY(c, hipEventRecord(st->ev[k], s));
    }
    st->live[k] = true;
  }
  return SONAR_OK;
}

int sonar_fingerprint_f64le(sonar_ctx* c, const void* bytes, int64_t nbytes, int32_t mode,
                           const sonar_fp_cfg* cfg, sonar_fp_out* out) {
  if (!c || !cfg || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  if (cfg->device_ptrs) return fail(c, SONAR_ERR_INVALID, "sonar_fingerprint_f64le takes host output buffers");
  // the samples reach the device in the caller's pcm_dtype: F64 keeps Go's []float64 end to end,
  // F32 rounds each sample to nearest even (float32(x)) on the host threads or on the device
  const int32_t pdt = cfg->pcm_dtype == SONAR_F64 ? SONAR_F64 : SONAR_F32;
  if (cfg->pcm_dtype != SONAR_F32 && cfg->pcm_dtype != SONAR_F64) return fail(c, SONAR_ERR_INVALID, "pcm_dtype");
  const size_t esz = pdt == SONAR_F64 ? 8 : 4;
  int64_t n = 0;
  int rc = sonar_ingest_f64le(c, bytes, nbytes, pdt, mode, 0, nullptr, &n);
  if (rc != SONAR_OK) return rc;
  // same validation order as ComputeSTFTWithWindow before any device work (spectral.go:386-412)
  if (cfg->window_size <= 0 || cfg->hop_size <= 0 || (n - cfg->window_size) / cfg->hop_size + 1 <= 0)
    return sonar::detail::fingerprint_impl(c, bytes, n, cfg, out, false);
  void* d = dbuf(c, "ingest.pcm", (size_t)n * esz);
  if (!d) return fail(c, SONAR_ERR_NOMEM, "device allocation failed (ingest pcm)");
  rc = sonar_ingest_f64le(c, bytes, nbytes, pdt, mode, 0, d, &n);
  if (rc != SONAR_OK) return rc;
  sonar_fp_cfg f = *cfg;
  f.pcm_dtype = pdt;
  return sonar::detail::fingerprint_impl(c, d, n, &f, out, true);
}

}  // extern "C"
