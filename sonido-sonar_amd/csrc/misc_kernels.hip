// misc_kernels.hip -- per-frame side features of the hot path (gfx950).
//
//  zcr_kernel      ZeroCrossingRate.Compute on pre-emphasised frames
//                  (algorithms/spectral/zero_crossing_rate.go:37-52, called at
//                  fingerprint/extractors/speech.go:351-358)
//  energy_wave_kernel  Energy.ComputeShortTimeEnergy (algorithms/temporal/energy.go:25-50)
//  yin_kernel      PitchDetector.detectPitchYin core (algorithms/tonal/pitch_detection.go:282-420)
//  chroma_kernel   ChromaSTFT.ComputeChroma on one music-extractor frame
//                  (algorithms/chroma/chroma_stft.go:45-138, fingerprint/extractors/music.go:327-376)
//  dc_block/carry_kernel  DCRemoval.Process + PreEmphasis.Process (music.go:245-259)
//
// Decision-bearing arithmetic (sign tests, sums feeding thresholds) is float64
// with explicit _rn intrinsics: no FMA contraction, Go's evaluation order.
#include <algorithm>
#include <atomic>

#include "kernels.h"

#pragma clang fp contract(off)

namespace sonar {

namespace {
// y[i] = x[i] - alpha * x[i-1], x[-1] = 0 (pre_emphasis.go:150-153), rounded like Go
__device__ __forceinline__ double pre_x(const void* pcm, int f64, int64_t i) {
  return f64 ? ((const double*)pcm)[i] : (double)((const float*)pcm)[i];
}
__device__ __forceinline__ double preemph(const void* pcm, int f64, int64_t i, double alpha) {
  const double x = pre_x(pcm, f64, i);
  const double prev = i > 0 ? pre_x(pcm, f64, i - 1) : 0.0;
  return __dsub_rn(x, __dmul_rn(alpha, prev));
}
__device__ __forceinline__ void store_out(void* out, int f64, int64_t i, double v) {
  if (f64) ((double*)out)[i] = v; else ((float*)out)[i] = (float)v;
}
}  // namespace

// one wave per frame; crossing count is an exact integer reduction
__global__ __launch_bounds__(256) void zcr_kernel(const void* pcm, int pcm_f64, int64_t n, int64_t f0, int64_t F,
                                                  int W, int H, double alpha, int sr, void* out, int out_f64) {
  const int lane = threadIdx.x & 63;
  const int64_t t = f0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // frames [f0, F)
  if (t >= F) return;
  const int64_t s = t * H;
  int64_t e = s + W; if (e > n) e = n;
  const int64_t len = e - s;
  int cnt = 0;
  for (int64_t i = s + 1 + lane; i < e; i += 64) {
    const double a = preemph(pcm, pcm_f64, i - 1, alpha), b = preemph(pcm, pcm_f64, i, alpha);
    cnt += ((a >= 0 && b < 0) || (a < 0 && b >= 0)) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (lane == 0) {
    double r = 0.0;
    if (len >= 2) r = __ddiv_rn((double)cnt, __ddiv_rn((double)len, (double)sr));
    store_out(out, out_f64, t, r);
  }
}

// a batched launch's job (blockIdx.y, or blockIdx.x for one-wave kernels) into SGPRs
template <class J>
__device__ __forceinline__ J load_job(const J* p) {
  static_assert(sizeof(J) % 4 == 0, "read as dwords");
  J r;
  const int* src = reinterpret_cast<const int*>(p);
  int* dst = reinterpret_cast<int*>(&r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(J) / 4); ++k) dst[k] = __builtin_amdgcn_readfirstlane(src[k]);
  return r;
}

// Phase boundary of a wave-private LDS exchange (see mfcc_pair.hip): DS ops stay on their side,
// and every DS op of the phase has retired before another lane's words are read or overwritten.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Energy.ComputeShortTimeEnergy (energy.go:25-50) of pre-emphasised frames, every lane one frame:
// Go's order needs each frame's sum as ONE sequential chain, so the lane count is the frame count.
// A wave owns 64 consecutive frames and walks them in rounds of kEnP = 8 samples: each round it
// loads the 64 frames' next 8 samples (8 rows x 8 columns per load instruction), transposes them
// through a wave-private LDS tile [frame][10 doubles] (row stride 80 B: the lanes' b128 reads hit
// distinct banks), and every lane adds its frame's 8 terms.  Same operations in the same order as
// Go: y = x - alpha x_prev, ss += y * y, sqrt(ss / W).  No span limit (any W, H).
// Footprint sized for C5, where these blocks run beside the DTW band kernel's two blocks per CU
// (104 KB of LDS, 4 waves x 104 VGPRs per SIMD): 20 KB of LDS per 4-wave block and 54 VGPRs (no
// register prefetch of the next round), so one fits next to them.  (The first round-4 form --
// 16-sample rounds, 37 KB, 148 VGPRs with the prefetch -- fitted beside none.)
constexpr int kEnP = 8;                  // samples per round
constexpr int kEnRow = kEnP + 2;         // LDS row stride in doubles

template <bool BJ>
__global__ __launch_bounds__(256) void energy_wave_kernel(const void* pcm, int pcm_f64, int64_t n, int64_t fbase,
                                                          int64_t Fe, int W, int H, double alpha, void* out,
                                                          int out_f64, const MfJob* jobs) {
  SONAR_FEAT_PRIO();
  __shared__ __attribute__((aligned(16))) double tile[4][64 * kEnRow];
  if constexpr (BJ) {
    const MfJob j = load_job(jobs + blockIdx.y);
    pcm = j.y; n = j.n; Fe = j.Fe; out = j.energy;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t f0 = fbase + ((int64_t)blockIdx.x * 4 + w) * 64;   // this wave's first frame; frames [fbase, Fe)
  if (f0 >= Fe) return;
  double* tl = tile[w];
  // loader role: round sample (row r = 8 i + lane / 8, column c = lane % 8)
  const int lr = lane >> 3, lc = lane & 7;
  auto load_round = [&](int k0, double (&v)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t g = (f0 + 8 * i + lr) * (int64_t)H + k0 + lc;
      v[i] = g < n ? pre_x(pcm, pcm_f64, g) : 0.0;
    }
  };
  const int64_t s = (f0 + lane) * (int64_t)H;                    // this lane's frame start
  double prev = (s > 0 && s - 1 < n) ? pre_x(pcm, pcm_f64, s - 1) : 0.0;
  double ss = 0.0;
  // alpha 0 (the raw-PCM RMS of ShortTimeEnergy callers): no pre-emphasis at all, so a non-finite
  // previous sample cannot turn 0 * x[n-1] into NaN
  const bool pre = alpha != 0.0;
  for (int k0 = 0; k0 < W; k0 += kEnP) {
    {
      double nx[8];
      load_round(k0, nx);
#pragma unroll
      for (int i = 0; i < 8; ++i) tl[(8 * i + lr) * kEnRow + lc] = nx[i];
    }
    wave_lds_sync();
    double cur[kEnP];
#pragma unroll
    for (int j = 0; j < kEnP; j += 2) {
      const double2 v2 = *reinterpret_cast<const double2*>(tl + lane * kEnRow + j);
      cur[j] = v2.x; cur[j + 1] = v2.y;
    }
    wave_lds_sync();
    if (k0 + kEnP <= W) {
#pragma unroll
      for (int j = 0; j < kEnP; ++j) {
        const double y = pre ? __dsub_rn(cur[j], __dmul_rn(alpha, prev)) : cur[j];
        prev = cur[j];
        ss = __dadd_rn(ss, __dmul_rn(y, y));
      }
    } else {
      for (int j = 0; j < W - k0; ++j) {
        const double y = pre ? __dsub_rn(cur[j], __dmul_rn(alpha, prev)) : cur[j];
        prev = cur[j];
        ss = __dadd_rn(ss, __dmul_rn(y, y));
      }
    }
  }
  if (f0 + lane < Fe) store_out(out, out_f64, f0 + lane, sqrt(__ddiv_rn(ss, (double)W)));
}

// YIN per 1024-sample frame (hop 512 for extractHarmonicFeatures, 256 for the voice-quality
// period scan), PitchDetector.detectPitchYin (pitch_detection.go:349-420) after preprocessFrame
// (:282-314).  One wave per frame (round 6; rounds 1-5: a 256-thread block per frame, two tau per
// thread reading both operands of every term from LDS, and one thread running the CMNDF with 1,022
// dependent divisions: 23 ms per hour of 44.1 kHz audio).
//  * difference function d(tau) = sum_j (x_j - x_{j+tau})^2, j < 512: lane l owns tau = 8 l + r,
//    r < 8, eight independent chains in Go's j order (unfused: bit-exact).  The operands x_{j+tau}
//    of a lane's eight chains slide by one per j, so they stay in a 16-register window refilled
//    with 8 LDS reads per 8 j; x_j is an LDS broadcast.  8 x 8 terms = 192 f64 VALU per 16 LDS
//    reads: the kernel is FP64-VALU-bound (3 ops per term, 2.4e11 per hour at hop 512).
//  * CMNDF running sum (:368-372) is Go's sequential chain over tau = 1..511: a wave-uniform add
//    chain fed by v_readlane, each lane keeping the partial sums of its own tau; then the two
//    divisions per tau in parallel across lanes.
//  * the first tau below the threshold that is a local minimum (:375-384) by a ballot, parabolic
//    interpolation and the frequency gate (:391-417, 743-764) on uniform values.
__constant__ double c_yin_win[1024];

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__global__ __launch_bounds__(256) void yin_kernel(const double* pcm, int64_t n, int64_t f0, int64_t frames, int64_t hop,
                                                  int sr, double* pitch, double* conf, int32_t* tau_out) {
  __shared__ double xs[4][1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t fi = f0 + (int64_t)blockIdx.x * 4 + w;       // frames [f0, frames)
  if (fi >= frames) return;
  const int64_t s = fi * hop;
  if (s + 1024 > n) {   // DetectPitch rejects frames != WindowSize (pitch_detection.go:226)
    if (lane == 0) { pitch[fi] = 0; conf[fi] = 0; if (tau_out) tau_out[fi] = -2; }
    return;
  }
  double* xw = xs[w];
  for (int i = lane; i < 1024; i += 64) {  // applyPreEmphasis :300-314 (fresh per frame), window :292-294
    const double x = pcm[s + i];
    const double y = (i == 0) ? x : __dsub_rn(x, __dmul_rn(0.97, pcm[s + i - 1]));
    xw[i] = __dmul_rn(y, c_yin_win[i]);
  }
  wave_lds_sync();
  const int t0 = 8 * lane;
  double acc[8], win[16];
#pragma unroll
  for (int r = 0; r < 8; ++r) { acc[r] = 0.0; win[r] = xw[t0 + r]; }
  for (int jb = 0; jb < 512; jb += 8) {                  // difference function :353-362
#pragma unroll
    for (int r = 0; r < 8; ++r) win[8 + r] = xw[jb + t0 + 8 + r];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const double xj = xw[jb + jj];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const double d = __dsub_rn(xj, win[jj + r]);
        acc[r] = __dadd_rn(acc[r], __dmul_rn(d, d));
      }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) win[r] = win[8 + r];
  }
  // CMNDF :364-372: runningSum over tau = 1..511 in order (wave-uniform chain)
  double run = 0.0, myrun[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) myrun[r] = 0.0;
  for (int L = 0; L < 64; ++L) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (L == 0 && r == 0) continue;                    // tau = 0 is not summed
      run = __dadd_rn(run, readlane_f64(acc[r], L));
      myrun[r] = (lane == L) ? run : myrun[r];
    }
  }
  double cm[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int tau = t0 + r;
    cm[r] = tau == 0 ? 1.0 : __ddiv_rn(acc[r], __ddiv_rn(myrun[r], (double)tau));
  }
  // first tau in 1..510 with cm < 0.15 and cm[tau] < cm[tau + 1] (:375-384)
  const double nxt0 = __shfl_down(cm[0], 1, 64);         // lane + 1's tau 8 (l + 1)
  int fr = 8;
#pragma unroll
  for (int r = 7; r >= 0; --r) {
    const int tau = t0 + r;
    const double nx = r < 7 ? cm[r + 1] : nxt0;
    if (tau >= 1 && cm[r] < 0.15 && tau + 1 < 512 && cm[r] < nx) fr = r;
  }
  const unsigned long long bal = __ballot(fr < 8);
  int mt = -1;
  if (bal) {
    const int L = __ffsll((long long)bal) - 1;
    mt = 8 * L + __builtin_amdgcn_readlane(fr, L);
  }
  double p = 0.0, c = 0.0;
  if (mt > 0) {                                          // wave-uniform from here
    auto cm_at = [&](int tau) {                         // cm of a uniform tau, without a dynamic index
      const int r = tau & 7, L = tau >> 3;
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) { const double t = readlane_f64(cm[q], L); v = (r == q) ? t : v; }
      return v;
    };
    const double y2 = cm_at(mt);
    double period = (double)mt;                          // parabolicInterpolation :743-764
    if (mt < 511) {
      const double y1 = cm_at(mt - 1), y3 = cm_at(mt + 1);
      const double a = __ddiv_rn(__dadd_rn(__dsub_rn(y1, __dmul_rn(2.0, y2)), y3), 2.0);
      const double b = __ddiv_rn(__dsub_rn(y3, y1), 2.0);
      if (a != 0.0) period = __dadd_rn((double)mt, __ddiv_rn(-b, __dmul_rn(2.0, a)));
    }
    const double f = __ddiv_rn((double)sr, period);
    const double cf = __dsub_rn(1.0, y2);
    if (f >= 80.0 && f <= 1000.0) { p = f; c = cf; }
  }
  if (lane == 0) {
    pitch[fi] = p; conf[fi] = c;
    if (tau_out) tau_out[fi] = mt;
  }
}

// chroma of one frame per block: direct DFT of length fs (any fs), |X|^2 folded to 12 bins.
// trig table (cos, sin of -2 pi m/fs): copied into LDS when it fits (trig_lds), else read from
// global memory (L1/L2 resident).
__global__ __launch_bounds__(256) void chroma_kernel(const double* y, int64_t n, int64_t frames, int hop, int fs,
                                                     const double* win, const double* trig_g, const int* cmap,
                                                     double* out, int trig_lds, int fft) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* seg = (double*)smem;                 // fs
  double* pw = seg + fs;                        // K + 12
  const int K = fs / 2 + 1;
  const int64_t t = blockIdx.x;
  if (t >= frames) return;
  const int64_t s = t * hop;
  const double* trig = trig_g;
  if (trig_lds) {
    double* tl = pw + K + 12 + ((K + 12) & 1);    // 16-B aligned, 2 fs
    for (int i = threadIdx.x; i < fs; i += blockDim.x)
      reinterpret_cast<double2*>(tl)[i] = reinterpret_cast<const double2*>(trig_g)[i];
    trig = tl;
  }
  if (fft) {
    // power-of-two frame (fs = 256 at every BASELINE config, F6): radix-2 DIT FFT in LDS, like the
    // go-dsp radix-2 path the reference runs (O(fs log fs) instead of the O(fs^2) direct DFT)
    double* fre = pw + K + 12 + ((K + 12) & 1) + (trig_lds ? 2 * fs : 0);
    double* fim = fre + fs;
    int lg = 0;
    while ((1 << lg) < fs) ++lg;
    for (int i = threadIdx.x; i < fs; i += blockDim.x) {
      const double v = (s + i < n) ? y[s + i] : 0.0;   // zero pad (music.go:351-357)
      const int r = (int)(__brev((unsigned)i) >> (32 - lg));
      fre[r] = v * win[i];
      fim[r] = 0.0;
    }
    __syncthreads();
    for (int h = 1; h < fs; h <<= 1) {
      const int tstep = fs / (2 * h);
      for (int bf = threadIdx.x; bf < fs / 2; bf += blockDim.x) {
        const int k = bf & (h - 1), i0 = ((bf - k) << 1) + k, i1 = i0 + h;
        const double wr = trig[2 * (k * tstep)], wi = trig[2 * (k * tstep) + 1];
        const double xr = fre[i1], xi = fim[i1];
        const double tr = xr * wr - xi * wi, ti = xr * wi + xi * wr;
        const double ar = fre[i0], ai = fim[i0];
        fre[i0] = ar + tr; fim[i0] = ai + ti;
        fre[i1] = ar - tr; fim[i1] = ai - ti;
      }
      __syncthreads();
    }
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
      const double mag = hypot(fre[k], fim[k]);
      pw[k] = mag * mag;
    }
    __syncthreads();
  } else {
  for (int i = threadIdx.x; i < fs; i += blockDim.x) {
    const double v = (s + i < n) ? y[s + i] : 0.0;   // zero pad (music.go:351-357)
    seg[i] = v * win[i];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    double re = 0.0, im = 0.0;
    int idx = 0;
    for (int m = 0; m < fs; ++m) {
      re += seg[m] * trig[2 * idx];
      im += seg[m] * trig[2 * idx + 1];
      idx += k; if (idx >= fs) idx -= fs;
    }
    const double mag = hypot(re, im);
    pw[k] = mag * mag;
  }
  __syncthreads();
  }
  if (threadIdx.x < 12) {
    double acc = 0.0;
    for (int k = 0; k < K; ++k) if (cmap[k] == (int)threadIdx.x) acc += pw[k];  // ascending-k order
    pw[K + threadIdx.x] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int b = 0; b < 12; ++b) tot += pw[K + b];
    for (int b = 0; b < 12; ++b) out[t * 12 + b] = (tot > 1e-10) ? pw[K + b] / tot : pw[K + b];
  }
}

// chroma_kernel's FFT path for power-of-two frames of 256..2048 samples, one wave per frame and
// 4 frames per block: the same radix-2 DIT butterflies (same pairs, twiddles and operation order,
// so the same bits), but a lane holds the 4 points of a two-stage group in registers, so a frame
// makes one LDS round trip per two stages with no block barrier after the twiddle table; |X|^2
// folds into the 12 classes through per-class bin lists (ascending bins: chroma_kernel's order).
// cls = [13 offsets][bins]: class b owns cls[13 + cls[b] .. 13 + cls[b+1]).
template <int PPL, bool BJ = false>
__global__ __launch_bounds__(256) void chroma_wave_kernel(const double* y, int64_t n, int64_t frames, int hop,
                                                          const double* win, const double* trig_g, const int* cls,
                                                          double* out, const MfJob* jobs) {
  SONAR_FEAT_PRIO();
  if constexpr (BJ) {
    const MfJob j = load_job(jobs + blockIdx.y);
    y = j.y; n = j.n; frames = j.F; out = j.chroma;
    if ((int64_t)blockIdx.x * 4 >= frames) return;
  }
  constexpr int FS = 64 * PPL, K = FS / 2 + 1;
  constexpr int LG = PPL == 4 ? 8 : (PPL == 8 ? 9 : (PPL == 16 ? 10 : 11));
  static_assert((1 << LG) == FS, "power-of-two frame");
  __shared__ __attribute__((aligned(16))) double2 tw[FS / 2];
  __shared__ __attribute__((aligned(16))) double2 xs[4][FS];
  __shared__ double pw[4][K + 12];
  for (int m = threadIdx.x; m < FS / 2; m += 256) tw[m] = reinterpret_cast<const double2*>(trig_g)[m];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 4 + w;
  if (t >= frames) return;
  const int64_t s = t * hop;
  double2* x = xs[w];
  double* p = pw[w];
#pragma unroll
  for (int u = 0; u < PPL; ++u) {
    const int i = lane + 64 * u;
    const double v = (s + i < n) ? y[s + i] : 0.0;      // zero pad (music.go:351-357)
    x[__brev((unsigned)i) >> (32 - LG)] = make_double2(v * win[i], 0.0);
  }
  // a ← a + t, b ← a - t with t = b * w (chroma_kernel's operation order)
  auto bfly = [](double2& a, double2& b, double2 wv) {
    const double tr = b.x * wv.x - b.y * wv.y, ti = b.x * wv.y + b.y * wv.x;
    const double ar = a.x, ai = a.y;
    a = make_double2(ar + tr, ai + ti);
    b = make_double2(ar - tr, ai - ti);
  };
  int h = 1;
  for (; 4 * h <= FS; h *= 4) {                          // stages h and 2h
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int ts1 = FS / (2 * h), ts2 = FS / (4 * h);
#pragma unroll
    for (int u = 0; u < PPL / 4; ++u) {
      const int g = lane + 64 * u, k = g & (h - 1), p0 = ((g - k) << 2) + k;
      double2 a0 = x[p0], a1 = x[p0 + h], a2 = x[p0 + 2 * h], a3 = x[p0 + 3 * h];
      const double2 w1 = tw[k * ts1];
      bfly(a0, a1, w1);
      bfly(a2, a3, w1);
      bfly(a0, a2, tw[k * ts2]);
      bfly(a1, a3, tw[(k + h) * ts2]);
      x[p0] = a0; x[p0 + h] = a1; x[p0 + 2 * h] = a2; x[p0 + 3 * h] = a3;
    }
  }
  if (h < FS) {                                          // odd stage count: the last stage alone
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int u = 0; u < PPL / 2; ++u) {
      const int k = lane + 64 * u;                       // h = FS / 2: twiddle step 1
      double2 a0 = x[k], a1 = x[k + h];
      bfly(a0, a1, tw[k]);
      x[k] = a0; x[k + h] = a1;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (int k = lane; k < K; k += 64) {
    const double2 c = x[k];
    const double mag = hypot(c.x, c.y);
    p[k] = mag * mag;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (lane < 12) {
    double acc = 0.0;
    for (int e = cls[lane]; e < cls[lane + 1]; ++e) acc += p[cls[13 + e]];
    p[K + lane] = acc;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (lane < 12) {
    double tot = 0.0;
#pragma unroll
    for (int b = 0; b < 12; ++b) tot += p[K + b];
    const double v = p[K + lane];
    out[t * 12 + lane] = (tot > 1e-10) ? v / tot : v;
  }
}

// SpectralAnalyzer.ComputeSTFTWithWindow for a window length the fused kernels do not take
// (any W up to 8192: go-dsp's FFTReal runs Bluestein for non-powers of two, analyzers/spectral.go:131):
// one block per frame, the windowed frame (and the (cos, -sin) table when it fits) in LDS, one
// thread per bin running the DFT sum in float64 in index order.  Writes |X| (float64 scratch for
// the MFCC pass) and the requested Magnitude / Complex / Phase rows; frames Go skips
// (spectral.go:524-534) stay zero.
template <typename P>
__global__ __launch_bounds__(256) void stft_dft_kernel(const P* pcm, int64_t n, int64_t F, int W, int H,
                                                       const double* win, const double2* trig_g, int trig_lds,
                                                       double* mag, void* out_mag, void* out_cplx, void* out_phase,
                                                       int out_f64) {
  extern __shared__ __attribute__((aligned(16))) double dsm[];
  const int64_t t = blockIdx.x;
  if (t >= F) return;
  const int K = W / 2 + 1;
  double2* tl = reinterpret_cast<double2*>(dsm);
  double* xs = dsm + (trig_lds ? 2 * W : 0);
  const int64_t s0 = t * H;
  const bool valid = s0 + W <= n;
  if (trig_lds)
    for (int i = threadIdx.x; i < W; i += 256) tl[i] = trig_g[i];
  for (int i = threadIdx.x; i < W; i += 256) xs[i] = valid ? (double)pcm[s0 + i] * win[i] : 0.0;
  __syncthreads();
  const double2* tr = trig_lds ? tl : trig_g;
  for (int k = threadIdx.x; k < K; k += 256) {
    double re = 0.0, im = 0.0;
    int idx = 0;
    for (int m = 0; m < W; ++m) {
      const double2 c = tr[idx];
      re += xs[m] * c.x;
      im += xs[m] * c.y;
      idx += k;
      if (idx >= W) idx -= W;
    }
    const double a = hypot(re, im);                  // cmplx.Abs (spectral.go:492)
    const int64_t o = t * K + k;
    mag[o] = a;
    auto put = [&](void* dst, int64_t i, double v) {
      if (out_f64) reinterpret_cast<double*>(dst)[i] = v; else reinterpret_cast<float*>(dst)[i] = (float)v;
    };
    if (out_mag) put(out_mag, o, a);
    if (out_cplx) { put(out_cplx, 2 * o, re); put(out_cplx, 2 * o + 1, im); }
    if (out_phase) put(out_phase, o, atan2(im, re));
  }
}

// MFCC.ComputeFrames on |X| rows (mfcc.go:126-143, 215-227): one wave per frame, the mel sums in
// ascending-bin order, ln with the 1e-10 floor, DCT-II in ascending order, lifter -- the
// operations and order of the fused kernels' epilogue, in float64
__global__ __launch_bounds__(64) void mfcc_rows_kernel(const double* mag, int64_t F, int K, const int* lo,
                                                       const int* hi, const int* woff, const double* w, int n_mels,
                                                       const double* dct, const double* lift, int n_mfcc,
                                                       int input_power, void* out, int out_f64) {
  __shared__ double lm[512];
  const int64_t t = blockIdx.x;
  if (t >= F) return;
  const int lane = threadIdx.x;
  const double* row = mag + t * K;
  for (int m = lane; m < n_mels; m += 64) {
    double sm = 0.0;
    const double* wm = w + woff[m] - lo[m];
    for (int k = lo[m]; k < hi[m]; ++k) {
      double v = row[k] * row[k];                     // |X|^2
      if (input_power) v = v * v;                     // F5
      sm += v * wm[k];
    }
    lm[m] = sm > 0.0 ? log(sm) : log(1e-10);
  }
  __syncthreads();
  for (int kk = lane; kk < n_mfcc; kk += 64) {
    double sm = 0.0;
    for (int q = 0; q < n_mels; ++q) sm += lm[q] * dct[kk * n_mels + q];
    const double v = sm * lift[kk];
    if (out_f64) reinterpret_cast<double*>(out)[t * n_mfcc + kk] = v;
    else reinterpret_cast<float*>(out)[t * n_mfcc + kk] = (float)v;
  }
}

int launch_stft_dft(const void* pcm, int pcm_f64, int64_t n, int64_t F, int W, int H, const double* win,
                    const double* trig, double* mag, void* out_mag, void* out_cplx, void* out_phase, int out_f64,
                    hipStream_t s) {
  if (F <= 0) return 0;
  if (W > 8192) return -4;
  const int trig_lds = (size_t)W * 24 <= 64 * 1024;
  const size_t lds = (size_t)W * 8 * (trig_lds ? 3 : 1);
  if (pcm_f64)
    hipLaunchKernelGGL(stft_dft_kernel<double>, dim3((unsigned)F), dim3(256), lds, s, (const double*)pcm, n, F, W, H,
                       win, (const double2*)trig, trig_lds, mag, out_mag, out_cplx, out_phase, out_f64);
  else
    hipLaunchKernelGGL(stft_dft_kernel<float>, dim3((unsigned)F), dim3(256), lds, s, (const float*)pcm, n, F, W, H,
                       win, (const double2*)trig, trig_lds, mag, out_mag, out_cplx, out_phase, out_f64);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_mfcc_rows(const double* mag, int64_t F, int K, const int* lo, const int* hi, const int* woff,
                     const double* w, int n_mels, const double* dct, const double* lift, int n_mfcc, int input_power,
                     void* out, int out_f64, hipStream_t s) {
  if (F <= 0) return 0;
  if (n_mels > 512) return -4;
  hipLaunchKernelGGL(mfcc_rows_kernel, dim3((unsigned)F), dim3(64), 0, s, mag, F, K, lo, hi, woff, w, n_mels, dct, lift,
                     n_mfcc, input_power, out, out_f64);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_zcr(const void* pcm, int pcm_f64, int64_t n, int64_t F, int W, int H, double alpha, int sr, void* out,
               int out_f64, hipStream_t s, int64_t f0, int64_t f1) {
  if (f1 < 0 || f1 > F) f1 = F;
  if (f1 <= f0) return 0;
  hipLaunchKernelGGL(zcr_kernel, dim3((unsigned)((f1 - f0 + 3) / 4)), dim3(256), 0, s, pcm, pcm_f64, n, f0, f1, W, H,
                     alpha, sr, out, out_f64);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_energy(const void* pcm, int pcm_f64, int64_t n, int64_t Fe, int W, int H, double alpha, void* out,
                  int out_f64, hipStream_t s, int64_t f0, int64_t f1) {
  if (f1 < 0 || f1 > Fe) f1 = Fe;
  if (f1 <= f0) return 0;
  if (W <= 0 || H <= 0) return -4;
  hipLaunchKernelGGL(energy_wave_kernel<false>, dim3((unsigned)((f1 - f0 + 255) / 256)), dim3(256), 0, s, pcm, pcm_f64,
                     n, f0, f1, W, H, alpha, out, out_f64, (const MfJob*)nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// EnergyEntropy of extractEnergyFeatures (extractors/speech.go:429-433): -e ln(e + 1e-10) where e > 0
__global__ __launch_bounds__(256) void energy_entropy_kernel(const double* e, int64_t n, double* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = e[i];
    out[i] = v > 0.0 ? -v * log(v + 1e-10) : 0.0;
  }
}

int launch_energy_entropy(const double* e, int64_t n, double* out, hipStream_t s) {
  if (n <= 0) return 0;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(energy_entropy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, e, n, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_yin(const double* pcm, int64_t n, int64_t frames, int64_t hop, int sr, double* pitch, double* conf,
               int32_t* tau, hipStream_t s, int64_t f0, int64_t f1) {
  // the window table is a per-device symbol: uploaded once per device of the process
  static std::atomic<uint64_t> init_mask{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -5;
  if (!(init_mask.load() & (1ull << dev))) {   // symmetric Hann without normalisation, pitch_detection.go:316-345
    double w[1024];
    for (int i = 0; i < 1024; i++) w[i] = 0.5 * (1.0 - cos(2.0 * M_PI * (double)i / 1023.0));
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_yin_win), w, sizeof(w)) != hipSuccess) return -5;
    init_mask.fetch_or(1ull << dev);
  }
  if (f1 < 0 || f1 > frames) f1 = frames;
  if (f1 <= f0) return 0;
  hipLaunchKernelGGL(yin_kernel, dim3((unsigned)((f1 - f0 + 3) / 4)), dim3(256), 0, s, pcm, n, f0, f1, hop, sr, pitch,
                     conf, tau);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// VoiceQualityAnalyzer period amplitudes (algorithms/speech/voice_quality.go:200-207, 330-338):
// RMS of each extracted pitch period, one thread per period, summed in Go's sample order
__global__ __launch_bounds__(256) void period_rms_kernel(const double* y, const int64_t* start, const int64_t* len,
                                                         int64_t np, double* amp) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= np) return;
  const double* p = y + start[k];
  const int64_t L = len[k];
  double r = 0.0;
  for (int64_t j = 0; j < L; ++j) r = __dadd_rn(r, __dmul_rn(p[j], p[j]));
  amp[k] = sqrt(__ddiv_rn(r, (double)L));
}

// calculateHNR autocorrelation (voice_quality.go:255-267) of one 2048-sample frame:
// ac[lag] = sum_{i < 2048-lag} x[i] x[i+lag] / (2048-lag), one thread per lag, Go's order
__global__ __launch_bounds__(256) void hnr_autocorr_kernel(const double* fr, double* ac) {
  __shared__ double x[2048];
  for (int i = threadIdx.x; i < 2048; i += 256) x[i] = fr[i];
  __syncthreads();
  const int lag = blockIdx.x * 256 + threadIdx.x;
  double sm = 0.0;
  for (int i = 0; i < 2048 - lag; ++i) sm = __dadd_rn(sm, __dmul_rn(x[i], x[i + lag]));
  ac[lag] = __ddiv_rn(sm, (double)(2048 - lag));
}

int launch_period_rms(const double* y, const int64_t* start, const int64_t* len, int64_t np, double* amp,
                      hipStream_t s) {
  if (np <= 0) return 0;
  hipLaunchKernelGGL(period_rms_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, y, start, len, np, amp);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_hnr_autocorr(const double* frame2048, double* ac, hipStream_t s) {
  hipLaunchKernelGGL(hnr_autocorr_kernel, dim3(8), dim3(256), 0, s, frame2048, ac);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_chroma(const double* y, int64_t n, int64_t frames, int hop, int fs, const double* window,
                  const double* trig, const int* cmap, const int* cls, double* out, hipStream_t s) {
  if (frames <= 0) return 0;
  if (cls && (fs == 256 || fs == 512)) {
    const dim3 grid((unsigned)((frames + 3) / 4));
    const MfJob* none = nullptr;
    if (fs == 256) hipLaunchKernelGGL((chroma_wave_kernel<4>), grid, dim3(256), 0, s, y, n, frames, hop, window, trig, cls, out, none);
    else hipLaunchKernelGGL((chroma_wave_kernel<8>), grid, dim3(256), 0, s, y, n, frames, hop, window, trig, cls, out, none);
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
  const int K = fs / 2 + 1;
  size_t lds = sizeof(double) * ((size_t)fs + K + 12);
  if (lds > 160 * 1024) return -4;
  // the trig table joins the frame in LDS while the block stays small (fs = 256 at every
  // BASELINE config, F6): 6 KB per block instead of a global read per MAC
  const size_t lds_t = sizeof(double) * ((size_t)fs + K + 12 + ((K + 12) & 1) + 2 * (size_t)fs);
  const int trig_lds = lds_t <= 32 * 1024;
  if (trig_lds) lds = lds_t;
  // radix-2 FFT for power-of-two frames whose (re, im) work arrays still fit next to the rest
  const int fft = (fs & (fs - 1)) == 0 && fs >= 2 && lds + 16 * (size_t)fs <= 48 * 1024;
  if (fft) lds += 16 * (size_t)fs + 8;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)chroma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(chroma_kernel, dim3((unsigned)frames), dim3(256), lds, s, y, n, frames, hop, fs, window, trig,
                     cmap, out, trig_lds, fft);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// DC removal y[n] = x[n] - x[n-1] + R y[n-1] (dc_removal.go:101-124) followed by pre-emphasis
// z[n] = y[n] - alpha y[n-1] (pre_emphasis.go:135-155), both from zero state, lane-dense:
//  * a 256-thread block owns kDcBlk = 2,048 samples, lane c the 8-sample chunk c.  The block stages
//    its samples (and the one before) in LDS with coalesced loads; every lane runs Go's recurrence
//    over its chunk from a zero state, which gives the chunk's affine map Y -> e_c + R^8 Y.
//  * an inclusive Kogge-Stone scan of the 256 maps (6 shuffle levels per wave, then the waves'
//    totals through LDS) gives every chunk's map from the block start.
//  * pass (1) stores the block's map (its end value from a zero start); pass (2), one wave per
//    signal, chains the blocks' maps (dc_carry_kernel: Y_b = ends[b] + R^2048 Y_{b-1}); pass (3)
//    redoes (1)'s scan, takes chunk c's start state from the block's true start, re-runs Go's
//    recurrence over the chunk and writes z back through LDS with coalesced stores.
// Every sample goes through Go's sequential recurrence from a start state equal to Go's up to the
// scan's rounding (a few ulp of |Y|, reassociated affine maps), outputs within ~1e-15 of Go's
// relative to the signal scale (tests: chroma 1e-9, energies 1e-12, the NCC peak exact).
// The round-3 form ran 256-sample chunks with 16 of a block's 256 lanes busy.  Block size: 18 KB
// of LDS and <= 96 VGPRs, so one fits on a CU beside the DTW band kernel's two blocks under C5
// (the first round-4 form, 4,096-sample blocks, needed 35 KB).
constexpr int kDcL = 8;                               // samples per lane
constexpr int kDcBlk = 256 * kDcL;                    // samples per block
static_assert(kDcL == 8, "dc_slot pads one slot per kDcL samples");
__device__ __forceinline__ int dc_slot(int i) { return i + (i >> 3); }   // lane stride 9 doubles
constexpr int kDcSlots = kDcBlk + 1 + (kDcBlk + 1) / kDcL + 1;      // > dc_slot(kDcBlk)

template <bool WRITE, bool BJ = false>
__global__ __launch_bounds__(256) void dc_block_kernel(const double* x, int64_t n, double R, double RL, double alpha,
                                                       const double* ystart, double* ends, double* z,
                                                       const MfJob* jobs) {
  SONAR_FEAT_PRIO();
  __shared__ double xs[kDcSlots];
  __shared__ double wtot[2][4];                       // the waves' inclusive totals (B, A)
  if constexpr (BJ) {
    const MfJob j = load_job(jobs + blockIdx.y);
    x = j.x; n = j.n; ystart = j.ystart; ends = j.ends; z = j.y;
  }
  const int64_t base = (int64_t)blockIdx.x * kDcBlk;  // first sample of the block
  if (base >= n) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int span = (int)min((int64_t)kDcBlk, n - base);
  for (int i = tid; i <= span; i += 256) {            // xs[slot(i)] = x[base - 1 + i]
    const int64_t g = base - 1 + i;
    xs[dc_slot(i)] = g >= 0 ? x[g] : 0.0;
  }
  __syncthreads();
  const int c0 = kDcL * tid;                           // chunk start (block-relative)
  const int m = min(kDcL, max(0, span - c0));         // valid samples of this chunk
  double v[kDcL + 1];                                  // v[0] = x[s - 1], v[1..16] = the chunk
#pragma unroll
  for (int j = 0; j <= kDcL; ++j) v[j] = xs[dc_slot(c0 + j)];
  // the chunk's response from a zero state
  double e = 0.0;
#pragma unroll
  for (int j = 0; j < kDcL; ++j)
    if (j < m) e = __dadd_rn(__dsub_rn(v[j + 1], v[j]), __dmul_rn(R, e));
  // inclusive scan of the maps (B, A): (B2, A2) o (B1, A1) = (B2 + A2 B1, A2 A1)
  double B = e, A = RL;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double Bp = __shfl_up(B, d, 64), Ap = __shfl_up(A, d, 64);
    if (lane >= d) { B = __dadd_rn(B, __dmul_rn(A, Bp)); A = __dmul_rn(A, Ap); }
  }
  if (lane == 63) { wtot[0][w] = B; wtot[1][w] = A; }
  __syncthreads();
  double Bw = 0.0, Aw = 1.0;                           // the earlier waves' composite
  for (int u = 0; u < w; ++u) {
    const double Bu = wtot[0][u], Au = wtot[1][u];
    Bw = __dadd_rn(Bu, __dmul_rn(Au, Bw));
    Aw = __dmul_rn(Au, Aw);
  }
  if (!WRITE) {
    if (tid == 255) ends[blockIdx.x] = __dadd_rn(B, __dmul_rn(A, Bw));   // the block's end from zero
    return;
  }
  // chunk c's start: the exclusive composite applied to the block's true start Yb
  const double Yb = ystart[blockIdx.x];
  double Be = __shfl_up(B, 1, 64), Ae = __shfl_up(A, 1, 64);
  if (lane == 0) { Be = 0.0; Ae = 1.0; }
  Be = __dadd_rn(Be, __dmul_rn(Ae, Bw));
  Ae = __dmul_rn(Ae, Aw);
  double y1 = (tid == 0) ? Yb : __dadd_rn(Be, __dmul_rn(Ae, Yb));
  // every lane read its inputs before the scan's barrier above: z goes straight back into xs
  // (slot c0 + j = sample base + c0 + j), with no register copy of the chunk's outputs
#pragma unroll
  for (int j = 0; j < kDcL; ++j) {
    const double yv = __dadd_rn(__dsub_rn(v[j + 1], v[j]), __dmul_rn(R, y1));
    xs[dc_slot(c0 + j)] = __dsub_rn(yv, __dmul_rn(alpha, y1));
    y1 = yv;
  }
  __syncthreads();
  for (int i = tid; i < span; i += 256) z[base + i] = xs[dc_slot(i)];
}

// one wave: ystart[c] = Y_{c-1}, Y_c = ends[c] + RC Y_{c-1}, Y_{-1} = 0 over the blocks' maps.
// Each 64-block group is a 6-step Kogge-Stone scan of the affine maps Y -> B + A Y (lane c ends
// with the map of blocks [i, c]), then one carry from the previous group.
template <bool BJ = false>
__global__ __launch_bounds__(64) void dc_carry_kernel(const double* ends, int64_t T, double RC, double* ystart,
                                                      const MfJob* jobs) {
  SONAR_FEAT_PRIO();
  if constexpr (BJ) {   // one wave per job
    const MfJob j = load_job(jobs + blockIdx.x);
    ends = j.ends; T = j.T; ystart = j.ystart;
  }
  const int lane = threadIdx.x;
  double Yin = 0.0;
  for (int64_t i = 0; i < T; i += 64) {
    double B = i + lane < T ? ends[i + lane] : 0.0;
    double A = RC;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const double Bp = __shfl_up(B, d, 64), Ap = __shfl_up(A, d, 64);
      if (lane >= d) { B = __dadd_rn(B, __dmul_rn(A, Bp)); A = __dmul_rn(A, Ap); }
    }
    const double Y = __dadd_rn(B, __dmul_rn(A, Yin));    // Y_{i+lane}
    const double prev = __shfl_up(Y, 1, 64);
    if (i + lane < T) ystart[i + lane] = lane == 0 ? Yin : prev;
    Yin = __shfl(Y, 63, 64);
  }
}

namespace {
double dc_pow(double R, int k) {                       // R^k by repeated products (host)
  double r = 1.0;
  for (int i = 0; i < k; ++i) r *= R;
  return r;
}
}  // namespace

int64_t dc_chunks(int64_t n) { return (n + kDcBlk - 1) / kDcBlk; }
size_t dc_preemph_scratch_bytes(int64_t n) { return (size_t)(2 * dc_chunks(n) + 2) * 8; }

int launch_dc_preemph(const double* x, int64_t n, double R, double alpha, double* y, double* scratch, hipStream_t s) {
  if (n <= 0) return 0;
  const int64_t T = dc_chunks(n);
  double* ends = scratch;
  double* ystart = scratch + T;
  const double RL = dc_pow(R, kDcL), RC = dc_pow(R, kDcBlk);
  const MfJob* none = nullptr;
  hipLaunchKernelGGL((dc_block_kernel<false>), dim3((unsigned)T), dim3(256), 0, s, x, n, R, RL, 0.0, nullptr, ends,
                     nullptr, none);
  hipLaunchKernelGGL((dc_carry_kernel<false>), dim3(1), dim3(64), 0, s, ends, T, RC, ystart, none);
  hipLaunchKernelGGL((dc_block_kernel<true>), dim3((unsigned)T), dim3(256), 0, s, x, n, R, RL, alpha, ystart, nullptr,
                     y, none);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// MusicFeatureExtractor energy + chroma of many signals in five launches (jobs on the device in
// djobs, the same on the host in hjobs for the grid sizes): DC removal + pre-emphasis (the same
// three passes as launch_dc_preemph), ShortTimeEnergy of the pre-emphasised signal (alpha 0, as
// music_features_impl), chroma (chroma_wave_kernel, fs 256 or 512; tables shared by every job).
// Returns -1 without launching when a job does not fit those kernels (the caller then runs the
// per-signal path).
int launch_music_features_batch(const MfJob* hjobs, const MfJob* djobs, int nj, int W, int H, int fs,
                                const double* window, const double* trig, const int* cls, hipStream_t s) {
  if (nj <= 0) return 0;
  if (nj > 65535 || !cls || (fs != 256 && fs != 512) || W <= 0 || H <= 0) return -1;
  int64_t maxT = 1, maxFe = 1, maxF = 1;
  for (int k = 0; k < nj; ++k) {
    if (hjobs[k].n <= 0 || hjobs[k].F <= 0) return -1;
    maxT = std::max(maxT, hjobs[k].T);
    maxFe = std::max(maxFe, hjobs[k].Fe);
    maxF = std::max(maxF, hjobs[k].F);
  }
  const double R = 0.995, alpha = 0.95;        // music.go:245-259 (dc_removal / pre_emphasis defaults)
  const double RL = dc_pow(R, kDcL), RC = dc_pow(R, kDcBlk);
  const dim3 gdc((unsigned)maxT, (unsigned)nj);
  hipLaunchKernelGGL((dc_block_kernel<false, true>), gdc, dim3(256), 0, s, nullptr, 0, R, RL, 0.0, nullptr, nullptr,
                     nullptr, djobs);
  hipLaunchKernelGGL((dc_carry_kernel<true>), dim3((unsigned)nj), dim3(64), 0, s, nullptr, 0, RC, nullptr, djobs);
  hipLaunchKernelGGL((dc_block_kernel<true, true>), gdc, dim3(256), 0, s, nullptr, 0, R, RL, alpha, nullptr, nullptr,
                     nullptr, djobs);
  hipLaunchKernelGGL((energy_wave_kernel<true>), dim3((unsigned)((maxFe + 255) / 256), (unsigned)nj), dim3(256), 0, s,
                     nullptr, 1, 0, 0, 0, W, H, 0.0, nullptr, 1, djobs);
  const dim3 gch((unsigned)((maxF + 3) / 4), (unsigned)nj);
  if (fs == 256)
    hipLaunchKernelGGL((chroma_wave_kernel<4, true>), gch, dim3(256), 0, s, nullptr, 0, 0, H, window, trig, cls, nullptr, djobs);
  else
    hipLaunchKernelGGL((chroma_wave_kernel<8, true>), gch, dim3(256), 0, s, nullptr, 0, 0, H, window, trig, cls, nullptr, djobs);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---- speech-extractor helpers -------------------------------------------
// y = PreEmphasis.ProcessBuffer(x) (pre_emphasis.go:184-190), float64 output
__global__ void preemph_kernel(const void* pcm, int pcm_f64, int64_t i0, int64_t i1, double alpha, double* y) {
  for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = preemph(pcm, pcm_f64, i, alpha);
}

// per-block partials over y: {max|y|, sum|y|, sum y^2, sign changes}, reduced on the host
// in block order (speech.go:383-393 peak/average amplitude; speech_analysis.go:135-162 ZCR/RMS)
__global__ __launch_bounds__(256) void stats_kernel(const double* y, int64_t n, double* part) {
  __shared__ double sm[4][256];
  double mx = 0, sa = 0, s2 = 0, cr = 0;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
  for (int64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
    const double v = y[i], a = fabs(v);
    mx = a > mx ? a : mx; sa += a; s2 += v * v;
    if (i > 0) { const double u = y[i - 1]; cr += ((u >= 0 && v < 0) || (u < 0 && v >= 0)) ? 1.0 : 0.0; }
  }
  sm[0][threadIdx.x] = mx; sm[1][threadIdx.x] = sa; sm[2][threadIdx.x] = s2; sm[3][threadIdx.x] = cr;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sm[0][threadIdx.x] = sm[0][threadIdx.x] > sm[0][threadIdx.x + o] ? sm[0][threadIdx.x] : sm[0][threadIdx.x + o];
      for (int q = 1; q < 4; q++) sm[q][threadIdx.x] += sm[q][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) for (int q = 0; q < 4; q++) part[4 * blockIdx.x + q] = sm[q][0];
}

// SpeechFeatureExtractor.extractSpectralTilt (speech.go:552-585): frames of 1024 at hop 512
__global__ void tilt_kernel(const double* y, int64_t n, int64_t frames, double* tilt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= frames) return;
  const int64_t s = i * 512;
  int64_t e = s + 1024; if (e > n) e = n;
  double hi = 0.0, lo = 0.0;
  for (int64_t j = s + 1; j < e; ++j) {
    const double d = __dsub_rn(y[j], y[j - 1]);
    hi = __dadd_rn(hi, __dmul_rn(d, d));
    lo = __dadd_rn(lo, __dmul_rn(y[j], y[j]));
  }
  tilt[i] = lo > 0 ? -10.0 * log10(hi / lo) : 0.0;
}

int launch_preemph(const void* pcm, int pcm_f64, int64_t n, double alpha, double* y, hipStream_t s, int64_t i0,
                   int64_t i1) {
  if (i1 < 0 || i1 > n) i1 = n;
  if (i1 <= i0) return 0;
  int64_t blocks = (i1 - i0 + 255) / 256; if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(preemph_kernel, dim3((unsigned)blocks), dim3(256), 0, s, pcm, pcm_f64, i0, i1, alpha, y);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
int launch_stats(const double* y, int64_t n, double* part, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(stats_kernel, dim3(blocks), dim3(256), 0, s, y, n, part);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
int launch_tilt(const double* y, int64_t n, int64_t frames, double* tilt, hipStream_t s) {
  if (frames <= 0) return 0;
  hipLaunchKernelGGL(tilt_kernel, dim3((unsigned)((frames + 255) / 256)), dim3(256), 0, s, y, n, frames, tilt);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---- PCM ingest (sonar_ingest_f64le, ingest_api.cpp) ----------------------
// f64 -> f32, round-to-nearest-even like Go's float32(x) and numpy astype; 4 samples per lane
// (two 16-B loads, one 16-B store), HBM-bound at 12 B per sample.
__global__ __launch_bounds__(256) void f64_to_f32_kernel(const double* __restrict__ in, float* __restrict__ out,
                                                         int64_t n) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const double2 a = reinterpret_cast<const double2*>(in)[2 * i];
    const double2 b = reinterpret_cast<const double2*>(in)[2 * i + 1];
    reinterpret_cast<float4*>(out)[i] = make_float4((float)a.x, (float)a.y, (float)b.x, (float)b.y);
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (float)in[i];
}

int launch_f64_to_f32(const double* in, float* out, int64_t n, hipStream_t s) {
  if (n <= 0) return 0;
  if (((uintptr_t)in & 15) || ((uintptr_t)out & 15)) return -2;
  int64_t blocks = ((n >> 2) + 255) / 256; if (blocks > 8192) blocks = 8192; if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(f64_to_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace sonar
