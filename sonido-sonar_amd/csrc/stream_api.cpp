// stream_api.cpp -- SpectralAnalyzer.ComputeSTFTStreaming / STFTStreamer.ProcessChunk
// (fingerprint/analyzers/spectral.go:287-374) on the device.
//
// The Go streamer appends each chunk to a buffer and, while the buffer holds a full window, emits
// the windowed FFT of its first W samples and drops min(hop, len) samples (:322-366).  Every frame
// therefore starts a whole number of hops after the buffer's start, and after a push of n samples
// to a buffer of len samples the emitted frames are exactly the STFT frames of the contiguous
// [buffer | chunk] at hop H: F = (len + n - W) / H + 1 (0 below W -- no zero-padded short frame as in
// ComputeSTFTWithWindow), and what stays is [F H, len + n) (nothing once F H >= len + n: the Go
// clear at "hopSize >= len(s.buffer)", which also drops the rest of a skip longer than the buffer
// when H > W).  So the device keeps that tail (< W samples for H <= W) in a ping-pong pair of
// buffers, copies each chunk behind it and runs ONE fused STFT launch over [tail | chunk].
//
// The launch is the per-frame fused kernel (fp_wave_kernel, or stft_dft_kernel for other window
// sizes): each frame's arithmetic is its own, so any chunking gives rows bit-identical to one
// sonar_fingerprint call over the whole stream with the same kernel (SONAR_FP_GENERIC for the f32
// MFCC configuration).  The headline mfcc_pair_kernel is not used here: it transforms frames
// (2p, 2p+1) as one complex FFT, so a frame's bits depend on its partner, and a push that ends on
// an even frame has no partner yet (Go emits it at once).
#include "../../include/sonar_gpu.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>

#include "ctx.h"

using sonar::detail::fail;

struct sonar_stft_stream {
  sonar_ctx* c = nullptr;
  sonar_fp_cfg cfg{};
  void* buf[2] = {nullptr, nullptr};   // [tail | chunk] of the current push, and the next tail
  int cur = 0;
  int64_t cap = 0;                     // samples per buffer
  int64_t len = 0;                     // samples held (len(s.buffer))
  size_t esz = 4;
};

namespace {

constexpr uint32_t kStreamFlags = SONAR_FP_MFCC | SONAR_FP_MAGNITUDE | SONAR_FP_COMPLEX | SONAR_FP_PHASE;

// frames ProcessChunk emits when n samples arrive on top of `len` buffered ones (H > 0)
int64_t stream_frames(int64_t len, int64_t n, int W, int H) {
  if (n <= 0) return 0;                // an empty chunk returns (nil, nil) at once (:323-325)
  const int64_t tot = len + n;
  return tot < W ? 0 : (tot - W) / H + 1;
}

int grow(sonar_stft_stream* st, int64_t need) {
  if (need <= st->cap) return SONAR_OK;
  sonar_ctx* c = st->c;
  int64_t cap = std::max<int64_t>(st->cap * 2, std::max<int64_t>(need, std::max<int64_t>(2 * st->cfg.window_size, 1 << 16)));
  void* nb[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++)
    if (hipMalloc(&nb[k], (size_t)cap * st->esz) != hipSuccess) {
      if (nb[0]) (void)hipFree(nb[0]);
      return fail(c, SONAR_ERR_NOMEM, "device allocation failed (stream buffer)");
    }
  hipError_t e = hipSuccess;
  if (st->len > 0)
    e = hipMemcpyAsync(nb[0], st->buf[st->cur], (size_t)st->len * st->esz, hipMemcpyDeviceToDevice, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {                       // the old buffers stay; the new pair must not leak
    for (int k = 0; k < 2; k++) (void)hipFree(nb[k]);
    return fail(c, SONAR_ERR_DEVICE, std::string("stream buffer copy: ") + hipGetErrorString(e));
  }
  for (int k = 0; k < 2; k++)
    if (st->buf[k]) (void)hipFree(st->buf[k]);
  st->buf[0] = nb[0]; st->buf[1] = nb[1];
  st->cur = 0;
  st->cap = cap;
  return SONAR_OK;
}

}  // namespace

extern "C" {

int sonar_stft_stream_create(sonar_ctx* c, const sonar_fp_cfg* cfg, sonar_stft_stream** out) {
  if (!c || !cfg || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  *out = nullptr;
  const int W = cfg->window_size;
  // WindowGenerator.Generate's checks, wrapped as ComputeSTFTStreaming does (:297-300, windowing.go:180-187)
  if (W <= 0)
    return fail(c, SONAR_ERR_INVALID, "failed to generate window: window size must be positive: " + std::to_string(W));
  if (W > 1048576)
    return fail(c, SONAR_ERR_INVALID, "failed to generate window: window size too large: " + std::to_string(W));
  if (cfg->window_type < SONAR_WIN_HANN || cfg->window_type > SONAR_WIN_WELCH)
    return fail(c, SONAR_ERR_INVALID, "failed to generate window: unsupported window type");
  if (cfg->flags & ~kStreamFlags)
    return fail(c, SONAR_ERR_UNSUPPORTED,
                "the streamer emits magnitude, phase, complex and MFCC rows only (SpectrogramFrame, spectral.go:369-374)");
  if (!(cfg->flags & kStreamFlags)) return fail(c, SONAR_ERR_INVALID, "no output requested");
  if (!sonar::fingerprint_supported(W) && W > 8192)
    return fail(c, SONAR_ERR_UNSUPPORTED, "window size " + std::to_string(W) + " above 8192 (generic STFT path)");
  auto* st = new sonar_stft_stream();
  st->c = c;
  st->cfg = *cfg;
  st->cfg.flags |= SONAR_FP_GENERIC;                  // the per-frame kernel (see the header comment)
  st->esz = cfg->pcm_dtype == SONAR_F64 ? 8 : 4;
  *out = st;
  return SONAR_OK;
}

int64_t sonar_stft_stream_frames(const sonar_stft_stream* st, int64_t n) {
  if (!st) return SONAR_ERR_INVALID;
  if (st->cfg.hop_size <= 0)              // the push would fail (sonar_stft_stream_push) once a frame is due
    return (n > 0 && st->len + n >= st->cfg.window_size) ? SONAR_ERR_INVALID : 0;
  return stream_frames(st->len, n, st->cfg.window_size, st->cfg.hop_size);
}

int64_t sonar_stft_stream_buffered(const sonar_stft_stream* st) { return st ? st->len : SONAR_ERR_INVALID; }

int sonar_stft_stream_push(sonar_stft_stream* st, const void* chunk, int64_t n, sonar_fp_out* out, int64_t* frames) {
  if (!st) return SONAR_ERR_INVALID;
  sonar_ctx* c = st->c;
  if (frames) *frames = 0;
  if (n <= 0) return SONAR_OK;                        // (:323-325)
  if (!chunk || !out) return fail(c, SONAR_ERR_INVALID, "null argument");
  const int W = st->cfg.window_size, H = st->cfg.hop_size;
  const int64_t tot = st->len + n;
  if (tot >= W && H <= 0) {
    // the first emitted frame would advance the buffer by hopSize: a negative one is a slice panic
    // (s.buffer[s.hopSize:], :359), zero never advances and Go's loop does not terminate (:334)
    if (H < 0) {
      char msg[96];
      std::snprintf(msg, sizeof(msg), "runtime error: slice bounds out of range [%d:]", H);
      return fail(c, SONAR_ERR_PANIC, msg);
    }
    return fail(c, SONAR_ERR_INVALID, "hop size must be positive (STFTStreamer.ProcessChunk never advances at 0)");
  }
  HIP_TRY(c, hipSetDevice(c->device));
  int rc = grow(st, tot);
  if (rc != SONAR_OK) return rc;
  const size_t esz = st->esz;
  char* b = static_cast<char*>(st->buf[st->cur]);
  HIP_TRY(c, hipMemcpyAsync(b + (size_t)st->len * esz, chunk, (size_t)n * esz,
                            st->cfg.device_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
  const int64_t F = stream_frames(st->len, n, W, H);
  if (F > 0) {
    rc = sonar::detail::fingerprint_impl(c, b, tot, &st->cfg, out, true);
    if (rc != SONAR_OK) return rc;
    const int64_t keep0 = std::min<int64_t>(F * (int64_t)H, tot);
    const int64_t keep = tot - keep0;
    if (keep > 0)
      HIP_TRY(c, hipMemcpyAsync(st->buf[1 - st->cur], b + (size_t)keep0 * esz, (size_t)keep * esz,
                                hipMemcpyDeviceToDevice, c->stream));
    st->cur = 1 - st->cur;
    st->len = keep;
  } else {
    st->len = tot;
  }
  if (!st->cfg.device_ptrs) HIP_TRY(c, hipStreamSynchronize(c->stream));   // the host chunk may be reused
  if (frames) *frames = F;
  return SONAR_OK;
}

void sonar_stft_stream_destroy(sonar_stft_stream* st) {
  if (!st) return;
  if (st->c) (void)hipStreamSynchronize(st->c->stream);
  for (int k = 0; k < 2; k++)
    if (st->buf[k]) (void)hipFree(st->buf[k]);
  delete st;
}

}  // extern "C"
