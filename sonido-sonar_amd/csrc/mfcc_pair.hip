// mfcc_pair.hip -- fused STFT(1024) -> mel -> ln -> DCT-II (MFCC) for gfx950, float32 / float64.
//
// Replaces, for the headline configuration (MFCC output only, W = 1024):
//   SpectralAnalyzer.ComputeSTFTWithWindow   fingerprint/analyzers/spectral.go:385-545
//     (frame t = x[tH : tH+W] * normalised window, forward DFT, k <= W/2)
//   MFCC.ComputeFrames / Compute             algorithms/spectral/mfcc.go:113-191
//     (|X|^2 [or |X|^4, F5] -> filterbank -> ln (floor 1e-10) -> DCT-II -> lifter)
// The general kernel (fp_kernel.hip) keeps every other mode (magnitude, spectral descriptors,
// other window sizes, float64 arithmetic with float32 output).
//
// Templated on the arithmetic type T (round 6): float for the headline, double for the same
// configuration at the reference's precision (float64 PCM or float32 PCM widened, float64 MFCC out);
// the data movement is the same with 64-bit values (two 32-bit permlane / DPP moves per value, LDS
// rows twice as wide, 8 waves per CU instead of 12).
//
// One wave = one PAIR of frames at a time (DESIGN.md "Kernel 1"):
//  * z[n] = w[n] (x_t[n] + i x_{t+1}[n]) is one 1024-point complex FFT; the two
//    real spectra separate as X_t = (Z_k + conj Z_{-k}) / 2, X_{t+1} = (Z_k - conj Z_{-k}) / 2i,
//    so only |.|^2 of those sums is needed -- no real-split twiddles.
//  * n = 64 a + b (lane b, register a): pass 1 = DFT16 over a in registers, then
//    w_1024^{b k1}.  k = k1 + 16 k2, k2 = c0 + 8 c1; b = b0 + 8 b1.
//  * T1: register bits 0-2 <-> lane bits 3-5 by v_permlane32_swap (bit 5),
//    v_permlane16_swap (bit 4) and a DPP row_ror:8 exchange (bit 3) -- no LDS.
//    Lane b0 + 8 (k1 & 7) then holds b1 (and k1 >> 3) in registers: pass 2 =
//    two DFT8 over b1, twiddle w_64^{b0 c0}.
//  * T2: one LDS transpose (b64, lane stride 136 B: conflict-free reads) to the
//    "combo" layout: lane L holds the combos (k1, c0) with residues r and 128 - r
//    (r = k1 + 16 c0), 8 values b0 each; pass 3 = two DFT8 over b0 gives
//    Z[r + 128 c1] and Z[128 - r + 128 c1], so Z_k and Z_{1024-k} meet in one lane.
//    Lane 63 holds the two self-paired residues 0 and 64 (operand selects).
//  * power spectra of both frames -> LDS [bin][2] (aliasing the dead T2 buffer),
//    filterbank as per-lane bin chunks of one filter pair each (rise/fall
//    partials, weights from an LDS table), partial sums -> ln -> DCT (+lifter)
//    on 52 lanes, coalesced stores.
#include <type_traits>

#include "kernels.h"

namespace sonar {

namespace {

template <typename T> struct cx { T x, y; };
template <typename T> __device__ __forceinline__ cx<T> cadd(cx<T> a, cx<T> b) { return {a.x + b.x, a.y + b.y}; }
template <typename T> __device__ __forceinline__ cx<T> csub(cx<T> a, cx<T> b) { return {a.x - b.x, a.y - b.y}; }
template <typename T> __device__ __forceinline__ cx<T> cmul(cx<T> a, cx<T> w) {
  return {a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x};
}
template <typename T> __device__ __forceinline__ cx<T> negi(cx<T> a) { return {a.y, -a.x}; }   // -i a
template <typename T> struct K_ {
  static constexpr T C = (T)0.70710678118654752440;                       // sqrt(2)/2
  static constexpr T c1 = (T)0.92387953251128675613, s1 = (T)0.38268343236508977173;
};
template <typename T> __device__ __forceinline__ cx<T> w8_1(cx<T> a) {   // a (1 - i)/sqrt2
  return {K_<T>::C * (a.x + a.y), K_<T>::C * (a.y - a.x)};
}
template <typename T> __device__ __forceinline__ cx<T> w8_3(cx<T> a) {   // a (-1 - i)/sqrt2
  return {K_<T>::C * (a.y - a.x), -K_<T>::C * (a.x + a.y)};
}

// forward DFT4 in place
template <typename T>
__device__ __forceinline__ void dft4(cx<T>& a0, cx<T>& a1, cx<T>& a2, cx<T>& a3) {
  const cx<T> t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = negi(csub(a1, a3));
  a0 = cadd(t0, t2); a2 = csub(t0, t2); a1 = cadd(t1, t3); a3 = csub(t1, t3);
}

// forward DFT8 of v[o + s*j], j = 0..7, natural-order output in place
template <int O, int S, typename T, int N>
__device__ __forceinline__ void dft8(cx<T> (&v)[N]) {
  cx<T> e0 = v[O], e1 = v[O + 2 * S], e2 = v[O + 4 * S], e3 = v[O + 6 * S];
  cx<T> o0 = v[O + S], o1 = v[O + 3 * S], o2 = v[O + 5 * S], o3 = v[O + 7 * S];
  dft4(e0, e1, e2, e3);
  dft4(o0, o1, o2, o3);
  o1 = w8_1(o1); o2 = negi(o2); o3 = w8_3(o3);
  v[O + S] = cadd(e1, o1); v[O + 5 * S] = csub(e1, o1);
  v[O + 3 * S] = cadd(e3, o3); v[O + 7 * S] = csub(e3, o3);
  v[O] = cadd(e0, o0); v[O + 4 * S] = csub(e0, o0);
  v[O + 2 * S] = cadd(e2, o2); v[O + 6 * S] = csub(e2, o2);
}

// w16^j, j in 1..9
template <int J, typename T> __device__ __forceinline__ cx<T> w16(cx<T> a) {
  if constexpr (J == 4) return negi(a);
  else if constexpr (J == 2) return w8_1(a);
  else if constexpr (J == 6) return w8_3(a);
  else {
    constexpr T cr = (J == 1) ? K_<T>::c1 : (J == 3) ? K_<T>::s1 : -K_<T>::c1;   // J = 9: cos(9 pi/8) = -cos(pi/8)
    constexpr T ci = (J == 1) ? -K_<T>::s1 : (J == 3) ? -K_<T>::c1 : K_<T>::s1;  //        -sin(9 pi/8) = sin(pi/8)
    return cmul(a, cx<T>{cr, ci});
  }
}

// forward DFT16 of v[0..15] in place (natural-order output), 4 x 4; INNER = false: the inner DFT4s
// were done by the caller (dft16_windowed)
template <bool INNER = true, typename T>
__device__ __forceinline__ void dft16(cx<T> (&v)[16]) {
  // inner DFT4 over n1 of v[4 n1 + n2] -> Y[n2][k1] stored at v[4 k1 + n2]
  if (INNER) {
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) dft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
  }
  v[4 + 1] = w16<1>(v[4 + 1]); v[4 + 2] = w16<2>(v[4 + 2]); v[4 + 3] = w16<3>(v[4 + 3]);
  v[8 + 1] = w16<2>(v[8 + 1]); v[8 + 2] = w16<4>(v[8 + 2]); v[8 + 3] = w16<6>(v[8 + 3]);
  v[12 + 1] = w16<3>(v[12 + 1]); v[12 + 2] = w16<6>(v[12 + 2]); v[12 + 3] = w16<9>(v[12 + 3]);
  // outer DFT4 over n2 for each k1: X[k1 + 4 k2] = sum_n2 Y'[n2][k1] w4^{n2 k2}
  cx<T> o[16];
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++) {
    cx<T> a0 = v[4 * k1], a1 = v[4 * k1 + 1], a2 = v[4 * k1 + 2], a3 = v[4 * k1 + 3];
    dft4(a0, a1, a2, a3);
    o[k1] = a0; o[k1 + 4] = a1; o[k1 + 8] = a2; o[k1 + 12] = a3;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = o[i];
}

__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

// DFT16 of the windowed pair z[a] = w[a] (xr[a] + i xi[a]): the window multiply is fused into the
// inner DFT4s' first butterflies (w0 x0 +- w8 x8 as one product and two FMAs, 48 VALU instead of 64).
// PCM of type P (float or double) is widened to T here.
template <typename T, typename P>
__device__ __forceinline__ void dft16_windowed(const P (&xr)[16], const P (&xi)[16], const T (&w)[16],
                                               cx<T> (&v)[16]) {
#pragma unroll
  for (int n2 = 0; n2 < 4; n2++) {
    const int a0 = n2, a1 = 4 + n2, a2 = 8 + n2, a3 = 12 + n2;
    const T p0r = (T)xr[a0] * w[a0], p0i = (T)xi[a0] * w[a0], p1r = (T)xr[a1] * w[a1], p1i = (T)xi[a1] * w[a1];
    const cx<T> t0 = {fma_((T)xr[a2], w[a2], p0r), fma_((T)xi[a2], w[a2], p0i)};
    const cx<T> t1 = {fma_(-(T)xr[a2], w[a2], p0r), fma_(-(T)xi[a2], w[a2], p0i)};
    const cx<T> t2 = {fma_((T)xr[a3], w[a3], p1r), fma_((T)xi[a3], w[a3], p1i)};
    const cx<T> t3 = negi(cx<T>{fma_(-(T)xr[a3], w[a3], p1r), fma_(-(T)xi[a3], w[a3], p1i)});
    v[a0] = cadd(t0, t2); v[a2] = csub(t0, t2); v[a1] = cadd(t1, t3); v[a3] = csub(t1, t3);
  }
  dft16<false>(v);
}

__device__ __forceinline__ float f_of(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t u_of(float f) { return __float_as_uint(f); }

// register bit <-> lane bit 5 for the pair (a, b): a' = [a_lo, b_lo], b' = [a_hi, b_hi]
__device__ __forceinline__ void swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(u_of(a), u_of(b), false, false);
  a = f_of(r[0]); b = f_of(r[1]);
}
__device__ __forceinline__ void swap32(double& a, double& b) {   // both 32-bit halves
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)__double2loint(a), (uint32_t)__double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)__double2hiint(a), (uint32_t)__double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]); b = __hiloint2double((int)hi[1], (int)lo[1]);
}
// register bit <-> lane bit 4: a' = rows {a0, b0, a2, b2}, b' = {a1, b1, a3, b3}
__device__ __forceinline__ void swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(u_of(a), u_of(b), false, false);
  a = f_of(r[0]); b = f_of(r[1]);
}
__device__ __forceinline__ void swap16(double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)__double2loint(a), (uint32_t)__double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)__double2hiint(a), (uint32_t)__double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]); b = __hiloint2double((int)hi[1], (int)lo[1]);
}
// register bit <-> lane bit 3 (lane ^ 8 = row_ror:8 inside each 16-lane row) for 4 pairs:
// a' = bit3 ? ror8(b) : a,  b' = bit3 ? b : ror8(a), as v_cndmask_b32 with a DPP source
// (VOP2 reads its mask from VCC, set here; s_nop 1 covers the VALU-write -> DPP-read hazard).
// The leading s_nop 4 keeps any in-flight VALU write of VCC from before the block off the mask.
__device__ __forceinline__ void swap8x4(float (&a)[4], float (&b)[4], uint64_t m_lo, uint64_t m_hi) {
#ifdef SONAR_SWAP8_BUILTIN   // compiler-managed form (4 VALU per pair and plane instead of 2)
  const bool hi = (__lane_id() & 8) != 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const float ra = f_of((uint32_t)__builtin_amdgcn_update_dpp(0, (int)u_of(a[i]), 0x128, 0xf, 0xf, false));
    const float rb = f_of((uint32_t)__builtin_amdgcn_update_dpp(0, (int)u_of(b[i]), 0x128, 0xf, 0xf, false));
    const float na = hi ? rb : a[i], nb = hi ? b[i] : ra;
    a[i] = na; b[i] = nb;
  }
  return;
#endif
  float na[4], nb[4];
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b64 vcc, %[mlo]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_dpp %[na0], %[b0], %[a0], vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[na1], %[b1], %[a1], vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[na2], %[b2], %[a2], vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[na3], %[b3], %[a3], vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_mov_b64 vcc, %[mhi]\n\t"
      "v_cndmask_b32_dpp %[nb0], %[a0], %[b0], vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[nb1], %[a1], %[b1], vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[nb2], %[a2], %[b2], vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[nb3], %[a3], %[b3], vcc row_ror:8 row_mask:0xf bank_mask:0xf"
      : [na0] "=&v"(na[0]), [na1] "=&v"(na[1]), [na2] "=&v"(na[2]), [na3] "=&v"(na[3]),
        [nb0] "=&v"(nb[0]), [nb1] "=&v"(nb[1]), [nb2] "=&v"(nb[2]), [nb3] "=&v"(nb[3])
      : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]),
        [b0] "v"(b[0]), [b1] "v"(b[1]), [b2] "v"(b[2]), [b3] "v"(b[3]), [mlo] "s"(m_lo), [mhi] "s"(m_hi)
      : "vcc");
#pragma unroll
  for (int i = 0; i < 4; i++) { a[i] = na[i]; b[i] = nb[i]; }
}
// the same for four doubles: the exchange moves each 32-bit half
__device__ __forceinline__ void swap8x4(double (&a)[4], double (&b)[4], uint64_t m_lo, uint64_t m_hi) {
  float al[4], ah[4], bl[4], bh[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    al[i] = __int_as_float(__double2loint(a[i])); ah[i] = __int_as_float(__double2hiint(a[i]));
    bl[i] = __int_as_float(__double2loint(b[i])); bh[i] = __int_as_float(__double2hiint(b[i]));
  }
  swap8x4(al, bl, m_lo, m_hi);
  swap8x4(ah, bh, m_lo, m_hi);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    a[i] = __hiloint2double(__float_as_int(ah[i]), __float_as_int(al[i]));
    b[i] = __hiloint2double(__float_as_int(bh[i]), __float_as_int(bl[i]));
  }
}

// Phase boundary of the wave-private LDS exchanges: the fence and wave barrier keep the
// compiler from moving DS ops across it; the explicit lgkmcnt(0) retires every DS op of the
// phase before the next phase reads other lanes' words (defensive; costs < 2 % here).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#ifndef SONAR_NO_LGKM_SYNC
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
  __builtin_amdgcn_wave_barrier();
}

// T2 destination byte offsets (float32 layout: complex units x 8) for lanes with k1 & 7 == 0:
// [h][c0] -> L3 * 136 + slot * 64 (see comboLane in DESIGN.md / the header comment); scaled by the
// complex size for float64
constexpr int kT2Irreg[2][8] = {
    {63 * 136, 60 * 136, 61 * 136, 62 * 136, 63 * 136 + 64, 62 * 136 + 64, 61 * 136 + 64, 60 * 136 + 64},
    {56 * 136, 57 * 136, 58 * 136, 59 * 136, 59 * 136 + 64, 58 * 136 + 64, 57 * 136 + 64, 56 * 136 + 64}};

// power rows [bin][2 frames]: bin k at row k + PAD (k >> 4) -- pad rows after every 16 bins make the
// split's stores (bins k1 + 16 c0 across a lane group) conflict-free: two for the float32 kernel's
// 8-B rows, one for the float64 kernel's 16-B rows (mfcc_pair_pad_rows); rows cover the chunk
// over-read up to bin 527; with two pad rows they take the dummy bin-512 stores of lanes != 63
template <int PAD = 2> __host__ __device__ constexpr int prow(int k) { return k + PAD * (k >> 4); }
constexpr int kPRows = 600;

// one wave's LDS region for arithmetic type T (bytes)
template <typename T> struct Lay {
  static constexpr int ES = (int)sizeof(T), CB = 2 * ES;       // element, complex
  static constexpr int T2Stride = 17 * CB;                     // bytes per lane row of the T2 buffer (17 complex)
  static constexpr int WaveBytes = 64 * T2Stride + 16;         // + a complex that stays zero (unused filter sources)
  static constexpr int PB = 2 * ES;                            // power row: [2 frames]
  static constexpr int PadR = mfcc_pair_pad_rows(ES == 8);     // pad rows per 16 power rows
  // partial sums: float32 [64 lanes][a0 a1 b0 b1]; float64 two planes [2][64 lanes][2] (16-B lane
  // stride: a 32-B stride puts an 8-lane ds_write_b128 group on every bank twice)
  static constexpr int PartOff = kPRows * PB;
  static constexpr int LogOff = PartOff + 64 * 4 * ES;         // logmel [2][NMP]
  static_assert(LogOff + 2 * 64 * ES <= WaveBytes, "wave region");
};

template <typename T> struct V2;
template <> struct V2<float> { using type = float2; };
template <> struct V2<double> { using type = double2; };
template <typename T> __device__ __forceinline__ void st2(unsigned char* a, T x, T y) {
  *reinterpret_cast<typename V2<T>::type*>(a) = typename V2<T>::type{x, y};
}
template <typename T> __device__ __forceinline__ cx<T> ld2(const unsigned char* a) {
  const auto u = *reinterpret_cast<const typename V2<T>::type*>(a);
  return {u.x, u.y};
}
__device__ __forceinline__ float lnf_(float x) { return __logf(x); }
__device__ __forceinline__ double lnf_(double x) { return log(x); }
__device__ __forceinline__ float lane32_other(float s) {           // lane ^ 32's value (lanes < 32)
  const auto r = __builtin_amdgcn_permlane32_swap(u_of(s), u_of(s), false, false);
  return f_of(r[1]);
}
__device__ __forceinline__ double lane32_other(double s) {
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)__double2loint(s), (uint32_t)__double2loint(s), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)__double2hiint(s), (uint32_t)__double2hiint(s), false, false);
  return __hiloint2double((int)hi[1], (int)lo[1]);
}

template <typename T> struct template_ty { using type = T; };

}  // namespace


// JT / MS / NH: compile-time chunk length, sources per filter and DCT half-length for the
// headline bank (40 mels at 44.1 kHz: 12 / 8 / 20); 0 = read from p (runtime loops).
// SEG: a batch of signals (sonar_fingerprint_batch) -- p.seg is the segment table, the pair index
// runs over all signals' frame pairs, and each wave follows its range across signal boundaries.
// HC: compile-time hop (256: frame t+1 is frame t shifted by four 64-sample rows, so a pair loads 20
// rows instead of 32 and holds 20 PCM registers) or 0 (runtime p.H, both frames loaded).
// T: arithmetic / output type (float: the headline; double: 8 waves per block); P: PCM type.
template <typename T, typename P, bool POW2, int JT, int MS, int NH, bool SEG, int HC>
__global__ __launch_bounds__(sizeof(T) == 8 ? 512 : 768, 1) void mfcc_pair_kernel(MfccPairParams p) {
  using L = Lay<T>;
  using C = cx<T>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // ---- shared tables -> LDS ---------------------------------------------------
  C* s_cw = reinterpret_cast<C*>(smem);                                            // [64][J] (wa, wb)
  uint16_t* s_src = reinterpret_cast<uint16_t*>(smem + p.lds_src);                 // [16][64] source byte offsets
  T* s_dct = reinterpret_cast<T*>(smem + p.lds_dct);                               // [16][NMP + DP], lifter folded
  constexpr int DP = mfcc_pair_dct_pad(sizeof(T) == 8);
  const C* g_cw = reinterpret_cast<const C*>(p.chunk_w);
  for (int i = threadIdx.x; i < 64 * p.JS; i += blockDim.x) s_cw[i] = g_cw[i];
  // as byte offsets into the wave's region: a partial sum's pair (PartOff + 2 ES idx), or for an
  // unused source (bit 15) the complex that stays zero past the T2 rows
  for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
    const uint32_t idx = p.mel_src[i];
    s_src[i] = (uint16_t)((idx & 0x8000u) ? 64 * L::T2Stride
                          : L::PartOff + (sizeof(T) == 8 ? 16 * (int)(idx >> 1) + 1024 * (int)(idx & 1)
                                                         : 2 * L::ES * (int)idx));
  }
  const T* g_dct = reinterpret_cast<const T*>(p.dct);
  for (int i = threadIdx.x; i < 16 * (p.NMP + DP); i += blockDim.x) s_dct[i] = g_dct[i];
  if (sizeof(T) == 8) {   // the float64 instance's stage-2 twiddle table, rows of kPairTw2Row complex
    C* t = reinterpret_cast<C*>(smem + p.lds_tw2);
    for (int i = threadIdx.x; i < 64; i += blockDim.x) t[(i >> 3) * kPairTw2Row + (i & 7)] = reinterpret_cast<const C*>(p.tw2)[i];
  }
  int* s_next = reinterpret_cast<int*>(smem + p.lds_ctr);                          // the block's pair counter
  if (threadIdx.x == 0) *s_next = 0;
  unsigned char* wb = smem + p.lds_wave0 + wave * L::WaveBytes;
  // Zero the wave's region once: the filterbank chunks read up to 11 rows past bin 512 with
  // zero weight, and some of those bytes (the unused 17th complex of T2 lane rows 33/34) are
  // never written by this kernel -- stale LDS from an earlier launch can hold NaN/Inf, and
  // 0 * NaN would turn the last filter into ln(1e-10) (seen in tools/pair_stress2.py).
  for (int i = lane; i < L::WaveBytes / 16; i += 64)
    *reinterpret_cast<float4*>(wb + 16 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();

  // ---- per-lane constants ---------------------------------------------------------
  // float64 register budget (8 waves per CU = 256 VGPRs each): the per-lane constants that the
  // float32 kernel keeps in registers are re-read or derived per pair instead -- the window from
  // global memory (L1/L2-resident 8 KB) at each pair's pass 1 (WIN_G), w_1024^{lane k1} from four
  // held powers (k1 = 1, 2, 4, 8) by 11 complex products (TW1_R), w_64^{b0 c0} from an LDS table
  // (TW2_L: 8 distinct rows per wave, broadcast reads).  The same moves in the float32 kernel (16
  // waves per CU at 128 VGPRs) measured slower (DESIGN.md Kernel 1a, profiles/r06y_*).
  constexpr bool D = sizeof(T) == 8;
  constexpr bool WIN_G = D, TW1_R = D, TW2_L = D;
  const T* g_win = reinterpret_cast<const T*>(p.window);
  T win[16];
  if constexpr (!WIN_G) {
#pragma unroll
    for (int a = 0; a < 16; a++) win[a] = g_win[64 * a + lane];
  }
  const C* g_tw1 = reinterpret_cast<const C*>(p.tw1);
  const C* g_tw2 = reinterpret_cast<const C*>(p.tw2);
  C tw1[16];                                    // w_1024^{lane k1}
#pragma unroll
  for (int k = 1; k < 16; k++)
    if (!TW1_R || k == 1 || k == 2 || k == 4 || k == 8) tw1[k] = g_tw1[lane * 16 + k];
  const int b0 = lane & 7, kl = lane >> 3;
  C tw2[8];                                     // w_64^{b0 c0}
  // (rows of 9 complex: the 8 rows a wave reads at once land on distinct banks -- rows of 8 put
  // them all on one bank of the ds_read2_b64's mod-32 banking, 8-way)
  const C* s_tw2 = reinterpret_cast<const C*>(smem + p.lds_tw2) + b0 * kPairTw2Row;
  if constexpr (!TW2_L) {
#pragma unroll
    for (int c = 1; c < 8; c++) tw2[c] = g_tw2[b0 * 8 + c];
  }
  // lane masks for the bit-3 exchange: m_hi3 = lanes with bit 3 set, m_lo3 = the rest
  const uint64_t m_hi3 = 0xff00ff00ff00ff00ull, m_lo3 = ~m_hi3;
  // T2 write bases (regular lanes, kl != 0): h = 0 -> + stride c0, h = 1 -> + stride (7 - c0)
  const int t2b0 = (kl - 1) * 8 * L::T2Stride + L::CB * b0;
  const int t2b1 = (7 - kl) * 8 * L::T2Stride + 8 * L::CB + L::CB * b0;
  // combo residues of this lane (as T2 reader / split)
  int rA;
  if (lane < 56) rA = (lane >> 3) + 1 + 16 * (lane & 7);
  else if (lane < 60) rA = 8 + 16 * (lane - 56);
  else if (lane < 63) rA = 16 * (lane - 59);
  else rA = 0;
  const int rB = (lane == 63) ? 64 : 128 - rA;
  const bool self = (lane == 63);
  constexpr int PR = L::PadR;
  const int pA = prow<PR>(rA) * L::PB, pB = prow<PR>(rB) * L::PB;   // power row byte offsets (+(128 + 8 PR) rows per 128 bins)
  const int p8 = L::PB * (self ? prow<PR>(512) : 18 * (lane & 31) + 16 + (lane >> 5));   // bin 512, or a pad row (PR = 2)
  const int ks = p.chunk_ks[lane];                           // mel chunk start bin
  const int nmp = p.NMP;
  // the ln phase's source byte offsets, loop-invariant per lane: in registers when the hop-256 PCM
  // reuse leaves room (HC = 256, MS known), so that phase is one LDS round trip instead of two
#ifndef HL_SRC_REGS
#define HL_SRC_REGS 1
#endif
  constexpr bool SRC_REGS = HL_SRC_REGS && HC == 256 && MS > 0;
  uint32_t srco[SRC_REGS ? MS : 1];
  if constexpr (SRC_REGS) {
#pragma unroll
    for (int i = 0; i < MS; i++) srco[i] = s_src[64 * i + lane];
  }

  // ---- this block's pairs, handed to its waves one at a time --------------------------
  // The block (one per CU) owns the contiguous pairs [pb, pe); each wave takes the next
  // unclaimed pair from an LDS counter.  A static split per wave left the kernel waiting for its
  // slowest waves: the youngest of a SIMD's three waves loses every issue tie to the older two
  // (arbitration is by priority, then age) and finished its equal share ~15 % later
  // (tools/hl_stamp.py, profiles/r05j_stamp.log).  Pair indices are 32-bit (the host checks the
  // count), so the wave-uniform compares stay scalar.
  const int NP = (int)((p.F + 1) >> 1);
  const int64_t pb64 = (int64_t)blockIdx.x * p.pairs_per_block;
  const int pb = (int)min((int64_t)NP, pb64);
  const int pe = (int)min((int64_t)NP, pb64 + p.pairs_per_block);
  const int H = HC ? HC : p.H;
  auto claim = [&]() -> int {
    int v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(s_next, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return pb + __builtin_amdgcn_readfirstlane(v);
  };

  // The signal a pair belongs to (wave-uniform).  One signal: pairs [0, NP) of p.pcm / p.out.  SEG:
  // seg = {pcm address[nseg], frames inside the signal[nseg], F[nseg], out address[nseg], first
  // pair[nseg + 1]}; the loads (one pair ahead) and the processing each keep their own cursor,
  // advanced monotonically.  Fin: frames t with t H + W <= n (= F unless the signal is shorter than
  // W: Go's frame count truncates toward zero), the rest read zeros.
  struct Sig { const P* pcm; T* out; int Fin, F, p0, p1, s; };
  // The table is read with vector loads (the kernel's stores keep it off the scalar cache); the
  // values are wave-uniform, so readfirstlane parks them in SGPRs.
  auto ld = [&](int i) {
    const int64_t v = p.seg[i];
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
  };
  auto sig_at = [&](int s) {
    const int ns = p.nseg;
    Sig g;
    g.pcm = reinterpret_cast<const P*>(ld(s)); g.Fin = (int)ld(ns + s); g.F = (int)ld(2 * ns + s);
    g.out = reinterpret_cast<T*>(ld(3 * ns + s)); g.p0 = (int)ld(4 * ns + s); g.p1 = (int)ld(4 * ns + s + 1);
    g.s = s;
    return g;
  };
  Sig gl, gp;
  if (SEG) {
    int lo = 0, hi = p.nseg - 1;                        // last signal whose first pair <= pb
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (ld(4 * p.nseg + mid) <= pb) lo = mid; else hi = mid - 1;
    }
    gl = sig_at(lo);
  } else {
    const int Fin = p.n >= 1024 ? (int)min(p.F, (p.n - 1024) / H + 1) : 0;
    gl = Sig{reinterpret_cast<const P*>(p.pcm), reinterpret_cast<T*>(p.out), Fin, (int)p.F, 0, NP, 0};
  }
  gp = gl;
  auto advance = [&](Sig& g, int pi) {
    if (SEG) while (pi >= g.p1) g = sig_at(g.s + 1);
  };

  auto frame_ok = [&](const Sig& g, int t) { return t < g.Fin; };
  const P* zeros = reinterpret_cast<const P*>(p.zeros);
  // The pair's PCM: xr = frame t's 16 rows (sample 64 a + lane), xe = frame t+1's rows that frame t
  // lacks (HC = 256: its last four, frame t+1 = frame t from row 4 on; else all 16).  Unconditional loads: a frame past the signal (the last
  // pair's second frame of an odd F, or a frame of a signal shorter than W) reads p.zeros instead
  // -- a wave-uniform pointer select, so the loaded registers have one definition and stay in place
  // across the loop's back edge.
  constexpr int NE = HC == 256 ? 4 : 16;
  auto load_pair = [&](int pi, P (&xr)[16], P (&xe)[NE]) {
    advance(gl, pi);
    const int t = 2 * (pi - gl.p0);
    const bool ok1 = frame_ok(gl, t + 1);
    const P* f0 = frame_ok(gl, t) ? gl.pcm + t * (int64_t)H : zeros;
    const P* f1 = !ok1 ? zeros : (HC == 256 ? f0 + 1024 : gl.pcm + (t + 1) * (int64_t)H);
#pragma unroll
    for (int a = 0; a < 16; a++) xr[a] = f0[lane + 64 * a];
#pragma unroll
    for (int a = 0; a < NE; a++) xe[a] = f1[lane + 64 * a];
  };

  // Phase-dependent issue priority: a wave in the LDS-bound epilogue (pass 3, power rows,
  // filterbank, ln, DCT: five LDS phases, few VALU) runs at s_setprio 1 and issues ahead of the
  // waves in the VALU-bound FFT passes (0), so its short VALU bursts between LDS round trips are not
  // queued behind 3-6 wave-instructions of FFT arithmetic, and its LDS traffic overlaps their VALU
  // work.  Same-box A/B (profiles/r04n_ab.log, r04x4_ab.log): 0.475-0.481 ms against 0.505-0.509 ms
  // at one priority; the reverse order 0.483-0.492 ms; the epilogue at 3, or priority from the T2
  // transpose on, no better.
  // one pair; the next pair's PCM (nxt, claimed one pair ahead) is loaded during it, and the pair
  // after that is claimed in its DCT phase, whose LDS drain returns the counter with the data
  auto process = [&](int pi, int nxt, P (&xr)[16], P (&xe)[NE]) -> int {
    advance(gp, pi);
#ifndef HL_PHASE_PRIO
#define HL_PHASE_PRIO 1
#endif
    if (HL_PHASE_PRIO) __builtin_amdgcn_s_setprio(0);
    C v[16];
    // ---- pass 1: DFT16 over a (the window fused into its first butterflies), twiddle w_1024^{b k1}
    if constexpr (HC == 256) {
      // frame t+1 = rows 4..15 of frame t + its own last four.  Past the signal (the last pair of an
      // odd F) xe is zero and the partner is frame t's tail: its row is never stored, and frame t's
      // bits depend only on frame t's samples, identically in single and batched calls
      P xi[16];
#pragma unroll
      for (int a = 0; a < 16; a++) xi[a] = a < 12 ? xr[a + 4] : xe[a - 12];
      if constexpr (WIN_G) {
        T wl[16];
#pragma unroll
        for (int a = 0; a < 16; a++) wl[a] = g_win[64 * a + lane];
        dft16_windowed(xr, xi, wl, v);
      } else {
        dft16_windowed(xr, xi, win, v);
      }
    } else {
      if constexpr (WIN_G) {
        T wl[16];
#pragma unroll
        for (int a = 0; a < 16; a++) wl[a] = g_win[64 * a + lane];
        dft16_windowed(xr, xe, wl, v);
      } else {
        dft16_windowed(xr, xe, win, v);
      }
    }
    // the next pair's PCM into the same registers, now that this pair's samples are windowed: in
    // flight during the whole pair, and no register copies across the loop's back edge
    // (unconditional, so the registers carry one definition round the loop: the last pair of the
    // wave's range loads itself again)
    load_pair(nxt < pe ? nxt : pi, xr, xe);
    if constexpr (TW1_R) {
      C w[16];
      w[1] = tw1[1]; w[2] = tw1[2]; w[4] = tw1[4]; w[8] = tw1[8];
      w[3] = cmul(w[1], w[2]); w[5] = cmul(w[4], w[1]); w[6] = cmul(w[4], w[2]); w[7] = cmul(w[4], w[3]);
#pragma unroll
      for (int k = 9; k < 16; k++) w[k] = cmul(w[8], w[k - 8]);
#pragma unroll
      for (int k = 1; k < 16; k++) v[k] = cmul(v[k], w[k]);
    } else {
#pragma unroll
      for (int k = 1; k < 16; k++) v[k] = cmul(v[k], tw1[k]);
    }
    // ---- T1: register bits 0-2 <-> lane bits 3-5 --------------------------------
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((j & 4) == 0) { swap32(v[j].x, v[j + 4].x); swap32(v[j].y, v[j + 4].y); }
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((j & 2) == 0) { swap16(v[j].x, v[j + 2].x); swap16(v[j].y, v[j + 2].y); }
    {
      T ea[4], eb[4];
#pragma unroll
      for (int pl = 0; pl < 4; pl++) {        // (plane, half): 4 pairs each
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int j = 2 * i + 8 * (pl >> 1);
          ea[i] = (pl & 1) ? v[j].y : v[j].x;
          eb[i] = (pl & 1) ? v[j + 1].y : v[j + 1].x;
        }
        swap8x4(ea, eb, m_lo3, m_hi3);
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int j = 2 * i + 8 * (pl >> 1);
          if (pl & 1) { v[j].y = ea[i]; v[j + 1].y = eb[i]; } else { v[j].x = ea[i]; v[j + 1].x = eb[i]; }
        }
      }
    }
    // ---- pass 2: DFT8 over b1 (registers 8h + b1), twiddle w_64^{b0 c0} -----------
    dft8<0, 1>(v);
    dft8<8, 1>(v);
#pragma unroll
    for (int c = 1; c < 8; c++) {
      const C w = TW2_L ? s_tw2[c] : tw2[c];
      v[c] = cmul(v[c], w); v[8 + c] = cmul(v[8 + c], w);
    }
    // ---- T2: LDS transpose into the combo layout ---------------------------------
    if (kl != 0) {
#pragma unroll
      for (int c = 0; c < 8; c++) {
        st2<T>(wb + t2b0 + L::T2Stride * c, v[c].x, v[c].y);
        st2<T>(wb + t2b1 + L::T2Stride * (7 - c), v[8 + c].x, v[8 + c].y);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 8; c++) {
        st2<T>(wb + L::CB * b0 + kT2Irreg[0][c] * (L::CB / 8), v[c].x, v[c].y);
        st2<T>(wb + L::CB * b0 + kT2Irreg[1][c] * (L::CB / 8), v[8 + c].x, v[8 + c].y);
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = ld2<T>(wb + lane * L::T2Stride + L::CB * j);
    wave_lds_sync();
    if (HL_PHASE_PRIO) __builtin_amdgcn_s_setprio(1);
    // ---- pass 3: DFT8 over b0 for both combos --------------------------------------
    dft8<0, 1>(v);    // A[c1] = Z[rA + 128 c1]
    dft8<8, 1>(v);    // B[c1] = Z[rB + 128 c1]
    // ---- power spectra of both frames: P_t = |Za + conj Zb|^2, P_t+1 = |Za - conj Zb|^2
    //      (the 1/4 is folded into the filterbank weights)
    auto pw = [&](C a, C b, int off) {
      const T sr = a.x + b.x, si = a.y - b.y, dr = a.x - b.x, di = a.y + b.y;
      T p0 = sr * sr + si * si, p1 = dr * dr + di * di;
      if (POW2) { p0 *= p0; p1 *= p1; }
      st2<T>(wb + off, p0, p1);
    };
    constexpr int R128 = (128 + 8 * PR) * L::PB;                // power rows of 128 bins (pad rows included)
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const C sec = self ? v[(8 - c) & 7] : v[15 - c];         // B[7 - c], or A[(8 - c) & 7] on lane 63
      pw(v[c], sec, pA + R128 * c);
    }
    pw(self ? v[12] : v[4], v[11], pB + 3 * R128);             // (A4, B3) / lane 63: (B4, B3)
#pragma unroll
    for (int c = 5; c < 8; c++) {
      const C fst = self ? v[8 + c] : v[c];                    // lane 63: (B5, B2), (B6, B1), (B7, B0)
      pw(fst, v[15 - c], pB + R128 * (7 - c));
    }
    {                                                           // bin 512 (lane 63: (A4, A4))
      const T p0 = v[4].x * v[4].x * (T)4, p1 = v[4].y * v[4].y * (T)4;   // |2 a|^2 -> 4 a^2
      if (PR == 2 || self) {                                    // one pad row: lane 63 alone
        if (POW2) st2<T>(wb + p8, p0 * p0, p1 * p1); else st2<T>(wb + p8, p0, p1);
      }
    }
    wave_lds_sync();
    // ---- filterbank: lane chunk [ks, ks + J) of one filter pair ----------------------
    {
      T a0 = 0, a1 = 0, c0 = 0, c1 = 0;
      const unsigned char* pr = wb + prow<PR>(ks) * L::PB;
      const int ib = 16 - (ks & 15);                          // first i past a pad pair
      const C* cw = s_cw + lane * p.JS;
      const int J = JT ? JT : p.J;
#pragma unroll
      for (int i = 0; i < J; i++) {
        const C pp = ld2<T>(pr + L::PB * i + (i >= ib ? PR * L::PB : 0));
        const C w = cw[i];
        a0 += w.x * pp.x; a1 += w.x * pp.y;
        c0 += w.y * pp.x; c1 += w.y * pp.y;
      }
      if constexpr (sizeof(T) == 8) {
        st2<T>(wb + L::PartOff + 16 * lane, a0, a1);
        st2<T>(wb + L::PartOff + 1024 + 16 * lane, c0, c1);
      } else {
        st2<T>(wb + L::PartOff + 4 * L::ES * lane, a0, a1);
        st2<T>(wb + L::PartOff + 4 * L::ES * lane + 2 * L::ES, c0, c1);
      }
    }
    wave_lds_sync();
    // ---- ln of the filter sums (lane = filter) ----------------------------------------
    if (lane < nmp) {
      const int ms = MS ? MS : p.max_src;
      const C q0 = ld2<T>(wb + (SRC_REGS ? srco[0] : s_src[lane]));   // every filter has a source
      T m0 = q0.x, m1 = q0.y;
#pragma unroll
      for (int i = 1; i < ms; i++) {
        const C q = ld2<T>(wb + (SRC_REGS ? srco[SRC_REGS ? i : 0] : s_src[64 * i + lane]));
        m0 += q.x;
        m1 += q.y;
      }
      const T lf = (T)-23.025850929940457;                      // ln(1e-10)
      T l0 = m0 > (T)0 ? lnf_(m0) : lf, l1 = m1 > (T)0 ? lnf_(m1) : lf;
      if (lane >= p.n_mels) { l0 = 0; l1 = 0; }
      T* lm = reinterpret_cast<T*>(wb + L::LogOff);
      lm[lane] = l0; lm[nmp + lane] = l1;
    }
    wave_lds_sync();
    {
      // ---- DCT-II (+ lifter): lane = q + 16 f + 32 h, half h of the filters ----------------
      const int q = lane & 15, f = (lane >> 4) & 1, hh = lane >> 5;
      const int half = NH ? NH : (nmp >> 1);
      const T* lm = reinterpret_cast<const T*>(wb + L::LogOff) + f * nmp + hh * half;
      const T* d = s_dct + q * (nmp + DP) + hh * half;        // row stride NMP + DP
      auto dot4 = [&](int m) -> T {                             // 4 terms, in the float32 kernel's order
        if constexpr (sizeof(T) == 4) {
          const float4 x = *reinterpret_cast<const float4*>(lm + m);
          const float4 y = *reinterpret_cast<const float4*>(d + m);
          return x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
        } else {
          const double2 x0 = *reinterpret_cast<const double2*>(lm + m), x1 = *reinterpret_cast<const double2*>(lm + m + 2);
          const double2 y0 = *reinterpret_cast<const double2*>(d + m), y1 = *reinterpret_cast<const double2*>(d + m + 2);
          return x0.x * y0.x + x0.y * y0.y + x1.x * y1.x + x1.y * y1.y;
        }
      };
      T s = dot4(0);                                            // half >= 4 (NMP is a multiple of 8)
      if constexpr (NH > 0) {
#pragma unroll
        for (int m = 4; m < NH; m += 4) s += dot4(m);
      } else {
        for (int m = 4; m < half; m += 4) s += dot4(m);
      }
      s += lane32_other(s);                                     // lanes < 32: + lane + 32
      const int64_t t = 2 * (pi - gp.p0) + f;
      if (hh == 0 && q < p.n_mfcc && t < gp.F) gp.out[t * p.n_mfcc + q] = s;
      int v = 0;
      if (lane == 0) v = __hip_atomic_fetch_add(s_next, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      wave_lds_sync();
      return pb + __builtin_amdgcn_readfirstlane(v);
    }
  };

#ifdef HL_STAMP
  const uint64_t t_begin = __builtin_amdgcn_s_memrealtime();
  int done = 0;
#endif
  int cur = claim();
  if (cur < pe) {
    int nxt = claim();
    P ar[16], ae[NE];
    load_pair(cur, ar, ae);
    for (;;) {
      const int nn = process(cur, nxt, ar, ae);
#ifdef HL_STAMP
      ++done;
#endif
      if (nxt >= pe) break;
      cur = nxt;
      nxt = nn;
    }
  }
#ifdef HL_STAMP
  if (p.stamp && lane == 0) {
    const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    p.stamp[3 * gw] = t_begin;
    p.stamp[3 * gw + 1] = __builtin_amdgcn_s_memrealtime();
    p.stamp[3 * gw + 2] = (uint64_t)done;
  }
#endif
}


int launch_mfcc_pair(const MfccPairParams& p, hipStream_t s) {
  const int64_t NP = (p.F + 1) >> 1;
  // 32-bit pair AND frame indices in the kernel (t = 2 (pi - p0) + 1 <= 2 NP): the host routes larger
  // calls to fp_wave_kernel (sonar_fp_kernel_plan), so this is a guard, reported as unsupported
  if (2 * NP > SONAR_PAIR_MAX_FRAMES) return -4;
  const int64_t grid = (NP + p.pairs_per_block - 1) / p.pairs_per_block;
  const bool head = p.J == 12 && p.max_src <= 8 && p.NMP == 40;
#ifndef HL_HOP256
#define HL_HOP256 1
#endif
  const bool h256 = HL_HOP256 && p.H == 256 && head;   // the headline configuration's hop
  auto pick = [&](auto tp, auto pp, auto seg) {
    using T = typename decltype(tp)::type;
    using P = typename decltype(pp)::type;
    constexpr bool S = decltype(seg)::value;
    if (h256) return p.pow2 ? mfcc_pair_kernel<T, P, true, 12, 8, 20, S, 256> : mfcc_pair_kernel<T, P, false, 12, 8, 20, S, 256>;
    return p.pow2 ? (head ? mfcc_pair_kernel<T, P, true, 12, 8, 20, S, 0> : mfcc_pair_kernel<T, P, true, 0, 0, 0, S, 0>)
                  : (head ? mfcc_pair_kernel<T, P, false, 12, 8, 20, S, 0> : mfcc_pair_kernel<T, P, false, 0, 0, 0, S, 0>);
  };
  if (p.nseg > 0 && p.f64) return -5;   // the batch table is float32 only
  template_ty<float> f32t; template_ty<double> f64t;
  decltype(pick(f32t, f32t, std::false_type{})) kern;
  if (!p.f64) kern = p.nseg > 0 ? pick(f32t, f32t, std::true_type{}) : pick(f32t, f32t, std::false_type{});
  else if (p.pcm_f64) kern = pick(f64t, f64t, std::false_type{});
  else kern = pick(f64t, f32t, std::false_type{});
  if (p.lds_bytes > 64 * 1024)
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes);
  if (p.waves_per_block < 1 || p.waves_per_block > mfcc_pair_waves_per_block(p.f64) || p.lds_bytes > 160 * 1024) return -5;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * p.waves_per_block), p.lds_bytes, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int mfcc_pair_wave_bytes(int f64) { return f64 ? Lay<double>::WaveBytes : Lay<float>::WaveBytes; }
int mfcc_pair_waves_per_block(int f64) { return f64 ? 8 : 12; }
int mfcc_pair_waves_per_cu(int f64) { return f64 ? 8 : 12; }
int mfcc_pair_rows() { return kPRows; }

}  // namespace sonar
