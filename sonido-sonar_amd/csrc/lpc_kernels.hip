// lpc_kernels.hip -- row a13 of the hot path on gfx950: LPC formant analysis,
// FormantAnalyzer.AnalyzeFormants (algorithms/speech/format.go:85-124) per frame
// of FormantAnalyzer.AnalyzeMultipleFrames (format.go:427-449).
//
// One 256-thread block per frame:
//   preprocessSignal (:127-146)   pre-emphasis 0.97 then symmetric Hamming, into LDS
//   LPCAnalyzer.Analyze (lpc.go:44-82) with R = Correlations[:p+1] of
//     AutoCorrelation(1024) (stats/correlation.go:669-684): the reference reaches
//     these through a z-scored FFT cross-correlation; on the device they are the
//     same sums evaluated directly, r(k) = sum_i z[i] z[i+k] for the p+1 lags
//     k = L .. L-p (F11: the array starts at lag -L), one partial per thread
//   levinsonDurbin (lpc.go:85-135)  lane 0, in place as written
//   GetSpectralEnvelope (lpc.go:233-265)  513 points across the block, the angles by
//     rotation recurrence
//   findSpectralPeaks / bandwidth / confidence (format.go:148-300)  the first wave, by ballots
//     with the serial scans' exact outcome; validate / spacing / VTL / quality (:300-411) lane 0
#include "../../include/sonar_gpu.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace sonar {

constexpr int LPC_MAXP = 64;

namespace {
// a rejected frame still gets a complete record (the output buffer is reused across calls)
__device__ void clear_record(sonar_formant_frame* o, int status, int p) {
  o->status = status;
  o->n_formants = 0;
  for (int i = 0; i < 4; ++i) o->frequency[i] = o->bandwidth[i] = o->amplitude[i] = o->confidence[i] = 0.0;
  o->vocal_tract_length = 0.0;
  o->quality = 0.0;
  o->stable = 0;
  o->lpc_order = p;
}
__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }   // finite operands only
__device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : b; }

template <int NT>
__device__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}
}  // namespace

#ifndef FMT_MIN_BLOCKS
#define FMT_MIN_BLOCKS 5   // 0.614-0.618 against 0.635-0.641 ms at 1 (profiles/r06bg_formant_minblocks_ab.log)
#endif
__global__ __launch_bounds__(256, FMT_MIN_BLOCKS) void formant_kernel(const double* pcm, int64_t hop, int W, int p, int sr,
                                                      int frame_ok_len, const double* ham, sonar_formant_frame* out,
                                                      double* coeffs, double* refl) {
  __shared__ double x[2048];
  __shared__ double red[4];
  __shared__ double Rp[1][LPC_MAXP + 1];
  __shared__ double a[LPC_MAXP + 1], kr[LPC_MAXP];
  __shared__ double env[513];
  const int tid = threadIdx.x;
  const int64_t f = blockIdx.x;
  const double* sig = pcm + f * hop;
  sonar_formant_frame* o = out + f;

  if (!frame_ok_len) {                              // len(frame) < windowSize (format.go:86-88)
    if (tid == 0) { clear_record(o, 1, p); o->gain = 0.0; o->residual_energy = 0.0; }
    return;
  }
  #pragma unroll 8
  for (int i = tid; i < W; i += 256) {
    const double v = i == 0 ? sig[0] : sig[i] - 0.97 * sig[i - 1];
    x[i] = v * ham[i];
  }
  __syncthreads();
  // normalize (correlation.go:464-501): mean, population variance, z-score
  double s = 0.0;
  #pragma unroll 8
  for (int i = tid; i < W; i += 256) s += x[i];
  const double mean = block_sum<256>(s, red) / (double)W;
  s = 0.0;
  #pragma unroll 8
  for (int i = tid; i < W; i += 256) { const double d = x[i] - mean; s += d * d; }
  const double sd = sqrt(block_sum<256>(s, red) / (double)W);
  __syncthreads();
  #pragma unroll 8
  for (int i = tid; i < W; i += 256) x[i] = sd < 1e-10 ? x[i] - mean : (x[i] - mean) / sd;
  __syncthreads();
  // R[m] = r(L - m), L = min(1024, W-1)
  const int L = W - 1 < 1024 ? W - 1 : 1024;
  const int lane = tid & 63, wv = tid >> 6;
  for (int m = wv; m <= p; m += 4) {                  // wave wv: lags L-m for m = wv, wv+4, ...
    const int k = L - m;
    double v = 0.0;
    #pragma unroll 4
    for (int i = lane; i + k < W; i += 64) v += x[i] * x[i + k];
    for (int sh = 32; sh > 0; sh >>= 1) v += __shfl_xor(v, sh, 64);
    if (lane == 0) Rp[0][m] = v;
  }
  __syncthreads();

  if (tid == 0) {
    const double* R = Rp[0];
    int status = 0;
    double E = R[0];
    for (int i = 0; i <= p; ++i) { a[i] = 0.0; if (i < p) kr[i] = 0.0; }
    if (R[0] == 0) status = 3;
    else {
      a[0] = 1.0;
      for (int i = 1; i <= p; ++i) {
        double num = R[i];
        for (int j = 1; j < i; ++j) num -= a[j] * R[i - j];
        if (E == 0) { status = 4; break; }
        kr[i - 1] = num / E;
        a[i] = kr[i - 1];
        for (int j = 1; j < i; ++j) a[j] = a[j] - kr[i - 1] * a[i - j];   // in place, as written
        E *= (1 - kr[i - 1] * kr[i - 1]);
        if (E <= 0) break;
      }
    }
    o->status = status;
    o->lpc_order = p;
    o->residual_energy = E;
    o->gain = sqrt(E);
    red[0] = status;
    red[1] = E;
  }
  __syncthreads();
  const int status = (int)red[0];
  const double E = red[1];
  if (status != 0) {
    if (tid == 0) clear_record(o, status, p);
    return;
  }
  if (coeffs) for (int i = tid; i <= p; i += 256) coeffs[f * (p + 1) + i] = a[i];
  if (refl) for (int i = tid; i < p; i += 256) refl[f * p + i] = kr[i];
  // spectral envelope, nfft = 1024 (findFormantsFromLPC format.go:150)
  // (cos, sin) of the angles -i w by the rotation recurrence from (cos w, -sin w): within
  // ~i ulp of cos(-i w) (the libm calls cost ~150 VALU each and were ~80 % of the kernel;
  // tools/formant_microbench.py, DESIGN.md Kernel 3c); Go's sums in Go's order
  for (int kk = tid; kk <= 512; kk += 256) {
    const double w = 2.0 * M_PI * (double)kk / 1024.0;
    const double c1 = cos(w), s1 = -sin(w);
    double cr = c1, si = s1;
    double rp = 1.0, ip = 0.0;
#pragma unroll 4
    for (int i = 1; i <= p; ++i) {
      rp += a[i] * cr;
      ip += a[i] * si;
      const double nc = cr * c1 - si * s1, ns = si * c1 + cr * s1;
      cr = nc;
      si = ns;
    }
    const double mg = sqrt(rp * rp + ip * ip);
    env[kk] = mg > 0 ? 1.0 / mg : 0.0;
  }
  __syncthreads();
  // findSpectralPeaks + bandwidths + confidences (format.go:148-300) by the first wave: every
  // search is wave-parallel with the serial loop's exact outcome (the same comparisons; a ballot's
  // lowest set lane is the loop's first hit), so no LDS read sits in a one-lane dependent chain
  if (tid >= 64) return;
  int stable = 1;
  {
    bool bad = false;
    for (int i = lane + 1; i <= p; i += 64) bad = bad || fabs(a[i]) >= 1.0;
    if (__ballot(bad)) stable = 0;
  }
  const double res = (double)sr / 1024.0;
  double maxv = 0.0;                                  // Go's strict '>' scan from 0: NaN never taken
  for (int i = lane; i < 513; i += 64) { const double e = env[i]; if (e > maxv) maxv = e; }
  for (int sh = 32; sh > 0; sh >>= 1) { const double o = __shfl_xor(maxv, sh, 64); if (o > maxv) maxv = o; }
  double fq[4], bw[4], am[4], cf[4];
  int nf = 0;
  if (maxv != 0) {
    for (int base = 1; base < 512 && nf < 4; base += 64) {   // peaks are ascending: the first 4 survive the cut
      const int i = base + lane;
      bool ok = false;
      if (i < 512) {
        const double e = env[i];
        ok = e > env[i - 1] && e > env[i + 1] && e / maxv > 0.1;
        const double fr = (double)i * res;
        ok = ok && !(fr < 50.0 || fr > (double)sr / 2.0);
      }
      uint64_t bal = __ballot(ok);
      while (bal && nf < 4) {
        const int pk = base + __ffsll((long long)bal) - 1;
        bal &= bal - 1;
        const double ei = env[pk], fr = (double)pk * res, hh = ei / 2.0;
        int li = pk, ri = pk;
        for (int t0 = pk - 1; t0 >= 0; t0 -= 64) {      // the nearest t < pk with env[t] <= hh
          const int t = t0 - lane;
          const uint64_t q = __ballot(t >= 0 && env[t] <= hh);
          if (q) { li = t0 - (__ffsll((long long)q) - 1); break; }
        }
        for (int t0 = pk + 1; t0 < 513; t0 += 64) {     // the nearest t > pk with env[t] <= hh
          const int t = t0 + lane;
          const uint64_t q = __ballot(t < 513 && env[t] <= hh);
          if (q) { ri = t0 + (__ffsll((long long)q) - 1); break; }
        }
        double b = (double)(ri - li) * res;
        if (b < 50.0) b = 50.0; else if (b > 500.0) b = 500.0;
        double c = 1.0;
        if (fr >= 300 && fr <= 3500) c *= 1.0;
        else if (fr >= 100 && fr <= 5000) c *= 0.7;
        else c *= 0.3;
        c *= dmin(ei, 1.0);
        if (b >= 50 && b <= 300) c *= 1.0;
        else if (b >= 30 && b <= 500) c *= 0.8;
        else c *= 0.5;
        c = dmax(0.0, dmin(1.0, c));
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (u == nf) { fq[u] = fr; bw[u] = b; am[u] = ei; cf[u] = c; }
        ++nf;
      }
    }
  }
  if (lane != 0) return;
  double vf[4], vb[4], va[4], vc[4];
  int nv = 0;
  for (int i = 0; i < nf; ++i) {
    if (fq[i] < 50.0 || fq[i] > (double)sr / 2.0) continue;
    if (cf[i] < 0.2) continue;
    if (bw[i] <= 0 || bw[i] > 1000) continue;
    vf[nv] = fq[i]; vb[nv] = bw[i]; va[nv] = am[i]; vc[nv] = cf[i]; ++nv;
  }
  if (nv > 1) {
    int ns = 1;
    for (int i = 1; i < nv; ++i) {
      if (vf[i] - vf[ns - 1] >= 200.0) { vf[ns] = vf[i]; vb[ns] = vb[i]; va[ns] = va[i]; vc[ns] = vc[i]; ++ns; }
      else if (vc[i] > vc[ns - 1]) { vf[ns - 1] = vf[i]; vb[ns - 1] = vb[i]; va[ns - 1] = va[i]; vc[ns - 1] = vc[i]; }
    }
    nv = ns;
  }
  double vtl = 17.5;
  if (nv > 0) {
    double tot = 0.0;
    int cnt = 0;
    for (int i = 0; i < nv; ++i)
      if (vf[i] > 0 && vc[i] > 0.3) {
        const double v = (2.0 * (i + 1) - 1.0) * 35000.0 / (4.0 * vf[i]);
        if (v >= 10.0 && v <= 25.0) { tot += v; ++cnt; }
      }
    if (cnt > 0) vtl = tot / (double)cnt;
  }
  double quality = 0.0;
  if (nv > 0) {
    double ac = 0.0;
    for (int i = 0; i < nv; ++i) ac += vc[i];
    ac /= (double)nv;
    const double lq = E > 0 ? dmax(0.0, 1.0 - dmin(1.0, E)) : 1.0;
    quality = (dmin((double)nv / 3.0, 1.0) + ac + lq + (stable ? 1.0 : 0.0)) / 4.0;
  }
  o->n_formants = nv;
  for (int i = 0; i < 4; ++i) {
    const bool v = i < nv;
    o->frequency[i] = v ? vf[i] : 0.0;
    o->bandwidth[i] = v ? vb[i] : 0.0;
    o->amplitude[i] = v ? va[i] : 0.0;
    o->confidence[i] = v ? vc[i] : 0.0;
  }
  o->vocal_tract_length = vtl;
  o->quality = quality;
  o->stable = stable;
}

int launch_formants(const double* pcm, int64_t frames, int64_t hop, int W, int p, int sr, int frame_ok_len,
                    const double* ham, sonar_formant_frame* out, double* coeffs, double* refl, hipStream_t s) {
  if (frames <= 0) return 0;
  if (p > LPC_MAXP || W > 2048) return -4;
  hipLaunchKernelGGL(formant_kernel, dim3((unsigned)frames), dim3(256), 0, s, pcm, hop, W, p, sr, frame_ok_len, ham,
                     out, coeffs, refl);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace sonar
