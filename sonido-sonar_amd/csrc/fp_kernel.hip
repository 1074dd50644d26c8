// fp_kernel.hip -- fused per-frame DSP for gfx950 (CDNA4, wave64).
//
// Replaces, for one batch of frames:
//   SpectralAnalyzer.ComputeSTFTWithWindow   fingerprint/analyzers/spectral.go:385-545
//     (frame t = x[tH : tH+W] * normalised symmetric window, go-dsp FFTReal, |X_k|, k <= W/2)
//   MFCC.Compute / ComputeFrames             algorithms/spectral/mfcc.go:113-191
//     (|X|^2 -> dense filterbank -> ln (floor 1e-10) -> DCT-II -> lifter)
//   per-frame spectral descriptors            fingerprint/extractors/speech.go:320-367, :438-458
//
// Layout / schedule (see DESIGN.md "Kernel 1"):
//  * one block = 256 threads = 4 waves = one tile of `tile_f` frames; blocks are
//    persistent over a contiguous run of tiles (halo re-reads hit L2).
//  * a wave computes FR frames at a time (FR = 8/R for R < 8): the W-point real
//    FFT is a M = W/2 = 64*R point complex FFT of z[n] = x[2n] + i x[2n+1]:
//      step 1: lane b holds z[64a+b] (a < R) -> R-point DFT in registers, twiddle w_M^{bc}
//      step 2: 64-point DFT across lanes for every column c, done as 8 x 8:
//              LDS exchange A, DFT8, twiddle w_64^{fg}, LDS exchange B, DFT8
//      step 3: real split X_k = E_k + w_W^k O_k (partner bin M-k through LDS)
//    Exchanges use XOR-swizzled addresses chosen so every ds_write_b32 / ds_read_b32
//    is bank-conflict-free (searched offline, tools/ in DESIGN.md).  The scratch
//    is the frame's own LDS spectrum row, so a tile needs only tile_f * (M+1) words.
//  * epilogue with lane = frame: thread (frame f, group g); group g owns a set of
//    filterbank rows balanced by nonzero count (sparse triangle sums in Go's
//    ascending-bin order), then the DCT rows g, g+G, ...; results are staged in
//    LDS and written with coalesced stores.
#include "kernels.h"
#include "twiddles.h"

namespace sonar {

namespace {

constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n >> 1); }
constexpr int bitrev(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; i++) r = (r << 1) | ((x >> i) & 1);
  return r;
}

// In-register forward DFT of size N (N | 64), radix-2 DIT, compile-time twiddles.
template <typename T, int N>
__device__ __forceinline__ void dft_reg(T (&re)[N], T (&im)[N]) {
  constexpr int LB = ilog2(N);
#pragma unroll
  for (int i = 0; i < N; i++) {
    const int j = bitrev(i, LB);
    if (i < j) {
      T t = re[i]; re[i] = re[j]; re[j] = t;
      t = im[i]; im[i] = im[j]; im[j] = t;
    }
  }
#pragma unroll
  for (int len = 2; len <= N; len <<= 1) {
    const int half = len >> 1;
#pragma unroll
    for (int k = 0; k < half; k++) {
      const int ti = k * (64 / len);
#pragma unroll
      for (int i = k; i < N; i += len) {
        const int j = i + half;
        T xr, xi;
        if (ti == 0) {
          xr = re[j]; xi = im[j];
        } else if (ti == 16) {  // * (-i)
          xr = im[j]; xi = -re[j];
        } else {
          const T wr = (T)TW64R[ti], wi = (T)TW64I[ti];
          xr = re[j] * wr - im[j] * wi;
          xi = re[j] * wi + im[j] * wr;
        }
        re[j] = re[i] - xr; im[j] = im[i] - xi;
        re[i] = re[i] + xr; im[i] = im[i] + xi;
      }
    }
  }
}

// orders LDS traffic of one wave (cross-lane exchange through LDS)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <typename T>
__device__ __forceinline__ T load_pcm(const void* pcm, int pcm_f64, int64_t i) {
  if (pcm_f64) return (T)((const double*)pcm)[i];
  return (T)((const float*)pcm)[i];
}

template <typename T>
__device__ __forceinline__ void store_out(void* out, int out_f64, int64_t i, T v) {
  if (out_f64) ((double*)out)[i] = (double)v;
  else ((float*)out)[i] = (float)v;
}

__device__ __forceinline__ float dev_log(float x) { return logf(x); }
__device__ __forceinline__ double dev_log(double x) { return log(x); }

template <typename T>
__device__ __forceinline__ void sincos_turns(double turns, T& c, T& s) {
  // e^{2 pi i turns}; evaluated in double then rounded to T
  double sd, cd;
  sincospi(2.0 * turns, &sd, &cd);
  c = (T)cd; s = (T)sd;
}

}  // namespace

template <typename T, int R>
__global__ __launch_bounds__(256, 2) void fp_tile_kernel(FpParams p) {
  constexpr int FR = (R >= 8) ? 1 : 8 / R;   // frames per wave pass
  constexpr int V = R * FR;                   // values per lane
  constexpr int G = V / 8;                    // 8-column groups
  constexpr int M = 64 * R;                   // complex FFT size
  constexpr int K = M + 1;                    // bins per frame (LDS row stride)

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* Prow = reinterpret_cast<T*>(smem + p.lds_P);
  T* logmel = reinterpret_cast<T*>(smem + p.lds_logmel);
  T* stage = reinterpret_cast<T*>(smem + p.lds_stage);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const T* win = reinterpret_cast<const T*>(p.window);

  // ---- per-lane constants, identical for every frame ----------------------
  T we[R], wo[R];                        // window at the lane's even/odd samples
#pragma unroll
  for (int a = 0; a < R; a++) {
    const int n0 = 2 * (64 * a + lane);
    we[a] = win[n0];
    wo[a] = win[n0 + 1];
  }
  T t1r[R], t1i[R];                      // w_M^{lane * c}
#pragma unroll
  for (int c = 0; c < R; c++) sincos_turns<T>(-(double)((lane * c) % M) / (double)M, t1r[c], t1i[c]);
  const int f2 = lane & 7;               // step-2 role: column cl2 = lane >> 3, f = lane & 7
  const int cl2 = lane >> 3;
  T t2r[8], t2i[8];                      // w_64^{f * g}
#pragma unroll
  for (int g = 0; g < 8; g++) sincos_turns<T>(-(double)((f2 * g) % 64) / 64.0, t2r[g], t2i[g]);
  const int g3 = lane >> 3;              // step-3 role: lane = 8 g + cl
  const int cl3 = lane & 7;
  T t3r[G][8], t3i[G][8];                // w_W^k for the lane's output bins
#pragma unroll
  for (int gm = 0; gm < G; gm++) {
    const int col = 8 * gm + cl3;
    const int c = col % R;
#pragma unroll
    for (int h = 0; h < 8; h++) {
      const int k = c + R * g3 + 8 * R * h;
      sincos_turns<T>(-(double)k / (double)(2 * M), t3r[gm][h], t3i[gm][h]);
    }
  }

  const int64_t chunk = (p.ntiles + gridDim.x - 1) / gridDim.x;
  const int64_t tile_begin = (int64_t)blockIdx.x * chunk;
  const int64_t tile_end = min(p.ntiles, tile_begin + chunk);
  const int units = p.tile_f / FR;

  for (int64_t tile = tile_begin; tile < tile_end; ++tile) {
    const int64_t tb = tile * p.stride - p.r0;   // frame of LDS row 0

    // ======================= FFT phase: wave-private =======================
    for (int u = wave; u < units; u += 4) {
      const int rb = u * FR;
      T* S = Prow + (int64_t)rb * K;             // scratch = the unit's own rows
      bool any = false;
      T xr[FR][R], xi[FR][R];
#pragma unroll
      for (int fr = 0; fr < FR; fr++) {
        const int64_t t = tb + rb + fr;
        const bool exists = (t >= 0) && (t < p.F);
        // Go skips frames whose end passes the signal (spectral.go:524-534): row stays all-zero
        const bool valid = exists && (t * p.H + p.W <= p.n);
        any |= exists;
        const int64_t s0 = t * p.H;
#pragma unroll
        for (int a = 0; a < R; a++) {
          const int64_t n0 = s0 + 2 * (64 * a + lane);
          T e = 0, o = 0;
          if (valid) {
            e = load_pcm<T>(p.pcm, p.pcm_f64, n0);
            o = load_pcm<T>(p.pcm, p.pcm_f64, n0 + 1);
          }
          xr[fr][a] = e * we[a];
          xi[fr][a] = o * wo[a];
        }
      }
      if (!any) continue;   // wave-uniform

      // step 1: R-point DFT over a, twiddle w_M^{lane c}
#pragma unroll
      for (int fr = 0; fr < FR; fr++) {
        dft_reg<T, R>(xr[fr], xi[fr]);
#pragma unroll
        for (int c = 1; c < R; c++) {
          const T a_ = xr[fr][c], b_ = xi[fr][c];
          xr[fr][c] = a_ * t1r[c] - b_ * t1i[c];
          xi[fr][c] = a_ * t1i[c] + b_ * t1r[c];
        }
      }
      // value for column col = fr*R + c  ->  flat index col
      T yr[G][8], yi[G][8];
      // exchange A: write S[gm*512 + 64*cl + (lane ^ 8cl)], read S[gm*512 + 64*cl2 + ((8e+f2) ^ 8cl2)]
#pragma unroll
      for (int plane = 0; plane < 2; plane++) {
#pragma unroll
        for (int col = 0; col < V; col++) {
          const int gm = col >> 3, cl = col & 7;
          const T v = plane ? xi[col / R][col % R] : xr[col / R][col % R];
          S[gm * 512 + 64 * cl + (lane ^ (8 * cl))] = v;
        }
        wave_lds_sync();
#pragma unroll
        for (int gm = 0; gm < G; gm++)
#pragma unroll
          for (int e = 0; e < 8; e++) {
            const T v = S[gm * 512 + 64 * cl2 + ((8 * e + f2) ^ (8 * cl2))];
            if (plane) yi[gm][e] = v; else yr[gm][e] = v;
          }
        wave_lds_sync();
      }
      // step 2: DFT8 over e, twiddle w_64^{f g}
#pragma unroll
      for (int gm = 0; gm < G; gm++) {
        dft_reg<T, 8>(yr[gm], yi[gm]);
#pragma unroll
        for (int g = 1; g < 8; g++) {
          const T a_ = yr[gm][g], b_ = yi[gm][g];
          yr[gm][g] = a_ * t2r[g] - b_ * t2i[g];
          yi[gm][g] = a_ * t2i[g] + b_ * t2r[g];
        }
      }
      // exchange B: write S[gm*512 + 64*cl2 + ((8g+f2) ^ (9cl2 & 63))], read with lane = 8g3 + cl3
      T zr[G][8], zi[G][8];
#pragma unroll
      for (int plane = 0; plane < 2; plane++) {
#pragma unroll
        for (int gm = 0; gm < G; gm++)
#pragma unroll
          for (int g = 0; g < 8; g++)
            S[gm * 512 + 64 * cl2 + ((8 * g + f2) ^ ((9 * cl2) & 63))] = plane ? yi[gm][g] : yr[gm][g];
        wave_lds_sync();
#pragma unroll
        for (int gm = 0; gm < G; gm++)
#pragma unroll
          for (int f = 0; f < 8; f++) {
            const T v = S[gm * 512 + 64 * cl3 + ((8 * g3 + f) ^ ((9 * cl3) & 63))];
            if (plane) zi[gm][f] = v; else zr[gm][f] = v;
          }
        wave_lds_sync();
      }
      // step 3: DFT8 over f -> h;  lane holds Z_fr[c + R*g3 + 8R*h] for its columns
#pragma unroll
      for (int gm = 0; gm < G; gm++) dft_reg<T, 8>(zr[gm], zi[gm]);

      // real split: partner Z_fr[(M-k) mod M] through LDS (one plane at a time)
      T pr_[G][8], pi_[G][8];
#pragma unroll
      for (int plane = 0; plane < 2; plane++) {
#pragma unroll
        for (int gm = 0; gm < G; gm++) {
          const int col = 8 * gm + cl3, fr = col / R, c = col % R;
#pragma unroll
          for (int h = 0; h < 8; h++) {
            const int k = c + R * g3 + 8 * R * h;
            S[fr * M + k] = plane ? zi[gm][h] : zr[gm][h];
          }
        }
        wave_lds_sync();
#pragma unroll
        for (int gm = 0; gm < G; gm++) {
          const int col = 8 * gm + cl3, fr = col / R, c = col % R;
#pragma unroll
          for (int h = 0; h < 8; h++) {
            const int k = c + R * g3 + 8 * R * h;
            const T v = S[fr * M + ((M - k) & (M - 1))];
            if (plane) pi_[gm][h] = v; else pr_[gm][h] = v;
          }
        }
        wave_lds_sync();
      }
      // X_k = E + w O,  E = (A + B)/2, O = -i (A - B)/2, A = Z[k], B = conj(Z[M-k])
#pragma unroll
      for (int gm = 0; gm < G; gm++) {
        const int col = 8 * gm + cl3, fr = col / R, c = col % R;
        T* row = Prow + (int64_t)(rb + fr) * K;
#pragma unroll
        for (int h = 0; h < 8; h++) {
          const int k = c + R * g3 + 8 * R * h;
          const T ar = zr[gm][h], ai = zi[gm][h];
          const T br = pr_[gm][h], bi = -pi_[gm][h];
          const T er = (T)0.5 * (ar + br), ei = (T)0.5 * (ai + bi);
          const T or_ = (T)0.5 * (ai - bi), oi = (T)-0.5 * (ar - br);
          const T xr_ = er + (t3r[gm][h] * or_ - t3i[gm][h] * oi);
          const T xi_ = ei + (t3r[gm][h] * oi + t3i[gm][h] * or_);
          T pw = xr_ * xr_ + xi_ * xi_;
          row[k] = p.store_mag ? sqrt(pw) : pw;
          if (k == 0) {                 // Nyquist bin M = E_0 - O_0 (both real)
            const T xn = er - or_;
            row[M] = p.store_mag ? fabs(xn) : xn * xn;
          }
        }
      }
    }
    __syncthreads();

    // ======================= epilogue: lane = frame ========================
    const int nvalid_hi = (int)min((int64_t)p.tile_f, p.F - tb);   // rows < nvalid_hi exist
    const int rlo = (tb + p.r0 < 0) ? (int)(-tb) : p.r0;           // first output row

    if (p.out_mag) {   // SpectrogramResult.Magnitude rows, coalesced flat copy
      const int64_t first = tb + rlo;
      const int64_t cnt = (int64_t)(nvalid_hi - rlo) * K;
      for (int64_t i = threadIdx.x; i < cnt; i += 256) {
        T v = Prow[(int64_t)rlo * K + i];
        store_out<T>(p.out_mag, p.out_f64, first * K + i, p.store_mag ? v : sqrt(v));
      }
    }

    if (p.out_mfcc) {
      const int f = threadIdx.x % p.tile_f;
      const int grp = threadIdx.x / p.tile_f;
      const T* wts = reinterpret_cast<const T*>(p.mel_w);
      const bool act = (f >= rlo) && (f < nvalid_hi);
      if (act) {
        const T* row = Prow + (int64_t)f * K;
        for (int q = p.grp_off[grp]; q < p.grp_off[grp + 1]; ++q) {
          const int m = p.grp_mels[q];
          const int lo = p.mel_lo[m], hi = p.mel_hi[m];
          const T* w = wts + p.mel_woff[m] - lo;
          T s = 0;
          for (int k = lo; k < hi; ++k) {
            T pv = row[k];
            if (p.store_mag) pv = pv * pv;        // |X|^2
            if (p.input_power) pv = pv * pv;      // F5: Compute() squares |X|^2 again
            s += pv * w[k];
          }
          logmel[f * (p.n_mels + 1) + m] = (s > (T)0) ? dev_log(s) : dev_log((T)1e-10);
        }
      }
      __syncthreads();
      if (act) {
        const T* dct = reinterpret_cast<const T*>(p.dct);
        const T* lift = reinterpret_cast<const T*>(p.lift);
        const T* lm = logmel + f * (p.n_mels + 1);
        for (int kk = grp; kk < p.n_mfcc; kk += p.n_groups) {
          const T* d = dct + kk * p.n_mels;
          T s = 0;
          for (int n = 0; n < p.n_mels; ++n) s += lm[n] * d[n];
          stage[f * p.n_mfcc + kk] = s * lift[kk];
        }
      }
      __syncthreads();
      const int64_t first = tb + rlo;
      const int64_t cnt = (int64_t)(nvalid_hi - rlo) * p.n_mfcc;
      for (int64_t i = threadIdx.x; i < cnt; i += 256)
        store_out<T>(p.out_mfcc, p.out_f64, first * p.n_mfcc + i, stage[rlo * p.n_mfcc + i]);
    }
    __syncthreads();   // LDS rows are rewritten by the next tile
  }
}

bool fingerprint_supported(int W) {
  return W == 128 || W == 256 || W == 512 || W == 1024 || W == 2048;
}

template <typename T, int R>
static int launch_t(const FpParams& p, hipStream_t s) {
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int64_t grid = (int64_t)ncu * 2;
  if (grid > p.ntiles) grid = p.ntiles;
  if (grid < 1) grid = 1;
  auto kern = fp_tile_kernel<T, R>;
  if (p.lds_bytes > 64 * 1024)
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), p.lds_bytes, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_fingerprint(const FpParams& p, int f64, hipStream_t s) {
  const int R = p.W / 128;
  if (f64) {
    switch (R) {
      case 1: return launch_t<double, 1>(p, s);
      case 2: return launch_t<double, 2>(p, s);
      case 4: return launch_t<double, 4>(p, s);
      case 8: return launch_t<double, 8>(p, s);
      case 16: return launch_t<double, 16>(p, s);
    }
  } else {
    switch (R) {
      case 1: return launch_t<float, 1>(p, s);
      case 2: return launch_t<float, 2>(p, s);
      case 4: return launch_t<float, 4>(p, s);
      case 8: return launch_t<float, 8>(p, s);
      case 16: return launch_t<float, 16>(p, s);
    }
  }
  return -4;
}

}  // namespace sonar
