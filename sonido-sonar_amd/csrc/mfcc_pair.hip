// mfcc_pair.hip -- fused STFT(1024) -> mel -> ln -> DCT-II (MFCC) for gfx950, float32.
//
// Replaces, for the headline configuration (float32, MFCC output only, W = 1024):
//   SpectralAnalyzer.ComputeSTFTWithWindow   fingerprint/analyzers/spectral.go:385-545
//     (frame t = x[tH : tH+W] * normalised window, forward DFT, k <= W/2)
//   MFCC.ComputeFrames / Compute             algorithms/spectral/mfcc.go:113-191
//     (|X|^2 [or |X|^4, F5] -> filterbank -> ln (floor 1e-10) -> DCT-II -> lifter)
// The general kernel (fp_kernel.hip) keeps every other mode (f64, magnitude,
// spectral descriptors, other window sizes).
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

struct cf { float x, y; };
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf w) { return {a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x}; }
__device__ __forceinline__ cf negi(cf a) { return {a.y, -a.x}; }          // -i a
constexpr float kC = 0.70710678118654752440f;                              // sqrt(2)/2
__device__ __forceinline__ cf w8_1(cf a) { return {kC * (a.x + a.y), kC * (a.y - a.x)}; }   // a (1 - i)/sqrt2
__device__ __forceinline__ cf w8_3(cf a) { return {kC * (a.y - a.x), -kC * (a.x + a.y)}; }  // a (-1 - i)/sqrt2

// forward DFT4 in place
__device__ __forceinline__ void dft4(cf& a0, cf& a1, cf& a2, cf& a3) {
  const cf t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = negi(csub(a1, a3));
  a0 = cadd(t0, t2); a2 = csub(t0, t2); a1 = cadd(t1, t3); a3 = csub(t1, t3);
}

// forward DFT8 of v[o + s*j], j = 0..7, natural-order output in place
template <int O, int S, int N>
__device__ __forceinline__ void dft8(cf (&v)[N]) {
  cf e0 = v[O], e1 = v[O + 2 * S], e2 = v[O + 4 * S], e3 = v[O + 6 * S];
  cf o0 = v[O + S], o1 = v[O + 3 * S], o2 = v[O + 5 * S], o3 = v[O + 7 * S];
  dft4(e0, e1, e2, e3);
  dft4(o0, o1, o2, o3);
  o1 = w8_1(o1); o2 = negi(o2); o3 = w8_3(o3);
  v[O + S] = cadd(e1, o1); v[O + 5 * S] = csub(e1, o1);
  v[O + 3 * S] = cadd(e3, o3); v[O + 7 * S] = csub(e3, o3);
  v[O] = cadd(e0, o0); v[O + 4 * S] = csub(e0, o0);
  v[O + 2 * S] = cadd(e2, o2); v[O + 6 * S] = csub(e2, o2);
}

// w16^j, j in 1..9
template <int J> __device__ __forceinline__ cf w16(cf a) {
  if constexpr (J == 4) return negi(a);
  else if constexpr (J == 2) return w8_1(a);
  else if constexpr (J == 6) return w8_3(a);
  else {
    constexpr float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
    constexpr float cr = (J == 1) ? c1 : (J == 3) ? s1 : -c1;      // J = 9: cos(9 pi/8) = -cos(pi/8)
    constexpr float ci = (J == 1) ? -s1 : (J == 3) ? -c1 : s1;     //        -sin(9 pi/8) = sin(pi/8)
    return cmul(a, cf{cr, ci});
  }
}

// forward DFT16 of v[0..15] in place (natural-order output), 4 x 4; INNER = false: the inner DFT4s
// were done by the caller (dft16_windowed)
template <bool INNER = true>
__device__ __forceinline__ void dft16(cf (&v)[16]) {
  // inner DFT4 over n1 of v[4 n1 + n2] -> Y[n2][k1] stored at v[4 k1 + n2]
  if (INNER) {
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) dft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
  }
  v[4 + 1] = w16<1>(v[4 + 1]); v[4 + 2] = w16<2>(v[4 + 2]); v[4 + 3] = w16<3>(v[4 + 3]);
  v[8 + 1] = w16<2>(v[8 + 1]); v[8 + 2] = w16<4>(v[8 + 2]); v[8 + 3] = w16<6>(v[8 + 3]);
  v[12 + 1] = w16<3>(v[12 + 1]); v[12 + 2] = w16<6>(v[12 + 2]); v[12 + 3] = w16<9>(v[12 + 3]);
  // outer DFT4 over n2 for each k1: X[k1 + 4 k2] = sum_n2 Y'[n2][k1] w4^{n2 k2}
  cf o[16];
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++) {
    cf a0 = v[4 * k1], a1 = v[4 * k1 + 1], a2 = v[4 * k1 + 2], a3 = v[4 * k1 + 3];
    dft4(a0, a1, a2, a3);
    o[k1] = a0; o[k1 + 4] = a1; o[k1 + 8] = a2; o[k1 + 12] = a3;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = o[i];
}

// DFT16 of the windowed pair z[a] = w[a] (xr[a] + i xi[a]): the window multiply is fused into the
// inner DFT4s' first butterflies (w0 x0 +- w8 x8 as one product and two FMAs, 48 VALU instead of 64)
__device__ __forceinline__ void dft16_windowed(const float (&xr)[16], const float (&xi)[16], const float (&w)[16],
                                               cf (&v)[16]) {
#pragma unroll
  for (int n2 = 0; n2 < 4; n2++) {
    const int a0 = n2, a1 = 4 + n2, a2 = 8 + n2, a3 = 12 + n2;
    const float p0r = xr[a0] * w[a0], p0i = xi[a0] * w[a0], p1r = xr[a1] * w[a1], p1i = xi[a1] * w[a1];
    const cf t0 = {__builtin_fmaf(xr[a2], w[a2], p0r), __builtin_fmaf(xi[a2], w[a2], p0i)};
    const cf t1 = {__builtin_fmaf(-xr[a2], w[a2], p0r), __builtin_fmaf(-xi[a2], w[a2], p0i)};
    const cf t2 = {__builtin_fmaf(xr[a3], w[a3], p1r), __builtin_fmaf(xi[a3], w[a3], p1i)};
    const cf t3 = negi(cf{__builtin_fmaf(-xr[a3], w[a3], p1r), __builtin_fmaf(-xi[a3], w[a3], p1i)});
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
// register bit <-> lane bit 4: a' = rows {a0, b0, a2, b2}, b' = {a1, b1, a3, b3}
__device__ __forceinline__ void swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(u_of(a), u_of(b), false, false);
  a = f_of(r[0]); b = f_of(r[1]);
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

// T2 destination byte offsets (float2 units x 8) for lanes with k1 & 7 == 0:
// [h][c0] -> L3 * 136 + slot * 64 (see comboLane in DESIGN.md / the header comment)
constexpr int kT2Irreg[2][8] = {
    {63 * 136, 60 * 136, 61 * 136, 62 * 136, 63 * 136 + 64, 62 * 136 + 64, 61 * 136 + 64, 60 * 136 + 64},
    {56 * 136, 57 * 136, 58 * 136, 59 * 136, 59 * 136 + 64, 58 * 136 + 64, 57 * 136 + 64, 56 * 136 + 64}};

constexpr int kT2Stride = 136;          // bytes per lane row of the T2 buffer (17 float2)
constexpr int kWaveBytes = 64 * kT2Stride + 16;   // + a float2 that stays zero (unused filter sources)
// power rows [bin][2 frames]: bin k at row k + 2 (k >> 4) -- two pad rows per 16 bins make the
// split's stores (bins k1 + 16 c0 across a lane group) conflict-free; rows cover the chunk
// over-read up to bin 527; the pad rows take the dummy bin-512 stores of lanes != 63
__host__ __device__ constexpr int prow(int k) { return k + 2 * (k >> 4); }
constexpr int kPRows = 600;
constexpr int kPartOff = kPRows * 8;    // partial sums [64 lanes][a0 a1 b0 b1]
constexpr int kLogOff = kPartOff + 64 * 16;   // logmel [2][NMP]

}  // namespace

// JT / MS / NH: compile-time chunk length, sources per filter and DCT half-length for the
// headline bank (40 mels at 44.1 kHz: 12 / 8 / 20); 0 = read from p (runtime loops).
// SEG: a batch of signals (sonar_fingerprint_batch) -- p.seg is the segment table, the pair index
// runs over all signals' frame pairs, and each wave follows its range across signal boundaries.
// HC: compile-time hop (256: frame t+1 is frame t shifted by four 64-sample rows, so a pair loads 20
// rows instead of 32 and holds 20 PCM registers) or 0 (runtime p.H, both frames loaded).
template <bool POW2, int JT, int MS, int NH, bool SEG, int HC>
__global__ __launch_bounds__(768, 1) void mfcc_pair_kernel(MfccPairParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // ---- shared tables -> LDS ---------------------------------------------------
  float2* s_cw = reinterpret_cast<float2*>(smem);                                  // [64][J] (wa, wb)
  uint16_t* s_src = reinterpret_cast<uint16_t*>(smem + p.lds_src);                 // [16][64] source byte offsets
  float* s_dct = reinterpret_cast<float*>(smem + p.lds_dct);                       // [16][NMP + 4], lifter folded
  for (int i = threadIdx.x; i < 64 * p.JS; i += blockDim.x) s_cw[i] = p.chunk_w[i];
  // as byte offsets into the wave's region: a partial sum's float2 (kPartOff + 8 idx), or for an
  // unused source (bit 15) the float2 that stays zero past the T2 rows
  for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
    const uint32_t idx = p.mel_src[i];
    s_src[i] = (uint16_t)((idx & 0x8000u) ? 64 * kT2Stride : kPartOff + 8 * (int)idx);
  }
  for (int i = threadIdx.x; i < 16 * (p.NMP + 4); i += blockDim.x) s_dct[i] = p.dct[i];
  int* s_next = reinterpret_cast<int*>(smem + p.lds_ctr);                          // the block's pair counter
  if (threadIdx.x == 0) *s_next = 0;
  unsigned char* wb = smem + p.lds_wave0 + wave * kWaveBytes;
  // Zero the wave's region once: the filterbank chunks read up to 11 rows past bin 512 with
  // zero weight, and some of those bytes (the unused 17th float2 of T2 lane rows 33/34) are
  // never written by this kernel -- stale LDS from an earlier launch can hold NaN/Inf, and
  // 0 * NaN would turn the last filter into ln(1e-10) (seen in tools/pair_stress2.py).
  for (int i = lane; i < kWaveBytes / 16; i += 64)
    *reinterpret_cast<float4*>(wb + 16 * i) = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();

  // ---- per-lane constants ---------------------------------------------------------
  float win[16];
#pragma unroll
  for (int a = 0; a < 16; a++) win[a] = p.window[64 * a + lane];
  cf tw1[16];                                   // w_1024^{lane k1}
#pragma unroll
  for (int k = 1; k < 16; k++) { const float2 v = p.tw1[lane * 16 + k]; tw1[k] = {v.x, v.y}; }
  const int b0 = lane & 7, kl = lane >> 3;
  cf tw2[8];                                    // w_64^{b0 c0}
#pragma unroll
  for (int c = 1; c < 8; c++) { const float2 v = p.tw2[b0 * 8 + c]; tw2[c] = {v.x, v.y}; }
  // lane masks for the bit-3 exchange: m_hi3 = lanes with bit 3 set, m_lo3 = the rest
  const uint64_t m_hi3 = 0xff00ff00ff00ff00ull, m_lo3 = ~m_hi3;
  // T2 write bases (regular lanes, kl != 0): h = 0 -> + 136 c0, h = 1 -> + 136 (7 - c0)
  const int t2b0 = (kl - 1) * 8 * kT2Stride + 8 * b0;
  const int t2b1 = (7 - kl) * 8 * kT2Stride + 64 + 8 * b0;
  // combo residues of this lane (as T2 reader / split)
  int rA;
  if (lane < 56) rA = (lane >> 3) + 1 + 16 * (lane & 7);
  else if (lane < 60) rA = 8 + 16 * (lane - 56);
  else if (lane < 63) rA = 16 * (lane - 59);
  else rA = 0;
  const int rB = (lane == 63) ? 64 : 128 - rA;
  const bool self = (lane == 63);
  const int pA = prow(rA) * 8, pB = prow(rB) * 8;             // power row byte offsets (+1152 per 128 bins)
  const int p8 = 8 * (self ? prow(512) : 18 * (lane & 31) + 16 + (lane >> 5));   // bin 512, or a pad row
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
  // The block (one per CU, 12 waves) owns the contiguous pairs [pb, pe); each wave takes the next
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
  struct Sig { const float* pcm; float* out; int Fin, F, p0, p1, s; };
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
    g.pcm = reinterpret_cast<const float*>(ld(s)); g.Fin = (int)ld(ns + s); g.F = (int)ld(2 * ns + s);
    g.out = reinterpret_cast<float*>(ld(3 * ns + s)); g.p0 = (int)ld(4 * ns + s); g.p1 = (int)ld(4 * ns + s + 1);
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
    gl = Sig{p.pcm, p.out, Fin, (int)p.F, 0, NP, 0};
  }
  gp = gl;
  auto advance = [&](Sig& g, int pi) {
    if (SEG) while (pi >= g.p1) g = sig_at(g.s + 1);
  };

  auto frame_ok = [&](const Sig& g, int t) { return t < g.Fin; };
  // The pair's PCM: xr = frame t's 16 rows (sample 64 a + lane), xe = frame t+1's rows that frame t
  // lacks (HC = 256: its last four, frame t+1 = frame t from row 4 on; else all 16).  Unconditional loads: a frame past the signal (the last
  // pair's second frame of an odd F, or a frame of a signal shorter than W) reads p.zeros instead
  // -- a wave-uniform pointer select, so the loaded registers have one definition and stay in place
  // across the loop's back edge.
  constexpr int NE = HC == 256 ? 4 : 16;
  auto load_pair = [&](int pi, float (&xr)[16], float (&xe)[NE]) {
    advance(gl, pi);
    const int t = 2 * (pi - gl.p0);
    const bool ok1 = frame_ok(gl, t + 1);
    const float* f0 = frame_ok(gl, t) ? gl.pcm + t * (int64_t)H : p.zeros;
    const float* f1 = !ok1 ? p.zeros : (HC == 256 ? f0 + 1024 : gl.pcm + (t + 1) * (int64_t)H);
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
  auto process = [&](int pi, int nxt, float (&xr)[16], float (&xe)[NE]) -> int {
    advance(gp, pi);
#ifndef HL_PHASE_PRIO
#define HL_PHASE_PRIO 1
#endif
    if (HL_PHASE_PRIO) __builtin_amdgcn_s_setprio(0);
    cf v[16];
    // ---- pass 1: DFT16 over a (the window fused into its first butterflies), twiddle w_1024^{b k1}
    if constexpr (HC == 256) {
      // frame t+1 = rows 4..15 of frame t + its own last four.  Past the signal (the last pair of an
      // odd F) xe is zero and the partner is frame t's tail: its row is never stored, and frame t's
      // bits depend only on frame t's samples, identically in single and batched calls
      float xi[16];
#pragma unroll
      for (int a = 0; a < 16; a++) xi[a] = a < 12 ? xr[a + 4] : xe[a - 12];
      dft16_windowed(xr, xi, win, v);
    } else {
      dft16_windowed(xr, xe, win, v);
    }
    // the next pair's PCM into the same registers, now that this pair's samples are windowed: in
    // flight during the whole pair, and no register copies across the loop's back edge
    // (unconditional, so the registers carry one definition round the loop: the last pair of the
    // wave's range loads itself again)
    load_pair(nxt < pe ? nxt : pi, xr, xe);
#pragma unroll
    for (int k = 1; k < 16; k++) v[k] = cmul(v[k], tw1[k]);
    // ---- T1: register bits 0-2 <-> lane bits 3-5 --------------------------------
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((j & 4) == 0) { swap32(v[j].x, v[j + 4].x); swap32(v[j].y, v[j + 4].y); }
#pragma unroll
    for (int j = 0; j < 16; j++)
      if ((j & 2) == 0) { swap16(v[j].x, v[j + 2].x); swap16(v[j].y, v[j + 2].y); }
    {
      float ea[4], eb[4];
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
    for (int c = 1; c < 8; c++) { v[c] = cmul(v[c], tw2[c]); v[8 + c] = cmul(v[8 + c], tw2[c]); }
    // ---- T2: LDS transpose into the combo layout ---------------------------------
    if (kl != 0) {
#pragma unroll
      for (int c = 0; c < 8; c++) {
        *reinterpret_cast<float2*>(wb + t2b0 + kT2Stride * c) = make_float2(v[c].x, v[c].y);
        *reinterpret_cast<float2*>(wb + t2b1 + kT2Stride * (7 - c)) = make_float2(v[8 + c].x, v[8 + c].y);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 8; c++) {
        *reinterpret_cast<float2*>(wb + 8 * b0 + kT2Irreg[0][c]) = make_float2(v[c].x, v[c].y);
        *reinterpret_cast<float2*>(wb + 8 * b0 + kT2Irreg[1][c]) = make_float2(v[8 + c].x, v[8 + c].y);
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const float2 u = *reinterpret_cast<const float2*>(wb + lane * kT2Stride + 8 * j);
      v[j] = {u.x, u.y};
    }
    wave_lds_sync();
    if (HL_PHASE_PRIO) __builtin_amdgcn_s_setprio(1);
    // ---- pass 3: DFT8 over b0 for both combos --------------------------------------
    dft8<0, 1>(v);    // A[c1] = Z[rA + 128 c1]
    dft8<8, 1>(v);    // B[c1] = Z[rB + 128 c1]
    // ---- power spectra of both frames: P_t = |Za + conj Zb|^2, P_t+1 = |Za - conj Zb|^2
    //      (the 1/4 is folded into the filterbank weights)
    auto pw = [&](cf a, cf b, int off) {
      const float sr = a.x + b.x, si = a.y - b.y, dr = a.x - b.x, di = a.y + b.y;
      float p0 = sr * sr + si * si, p1 = dr * dr + di * di;
      if (POW2) { p0 *= p0; p1 *= p1; }
      *reinterpret_cast<float2*>(wb + off) = make_float2(p0, p1);
    };
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const cf sec = self ? v[(8 - c) & 7] : v[15 - c];        // B[7 - c], or A[(8 - c) & 7] on lane 63
      pw(v[c], sec, pA + 1152 * c);
    }
    pw(self ? v[12] : v[4], v[11], pB + 3456);                 // (A4, B3) / lane 63: (B4, B3)
#pragma unroll
    for (int c = 5; c < 8; c++) {
      const cf fst = self ? v[8 + c] : v[c];                   // lane 63: (B5, B2), (B6, B1), (B7, B0)
      pw(fst, v[15 - c], pB + 1152 * (7 - c));
    }
    {                                                           // bin 512 (lane 63: (A4, A4))
      const float p0 = v[4].x * v[4].x * 4.f, p1 = v[4].y * v[4].y * 4.f;   // |2 a|^2 -> 4 a^2
      *reinterpret_cast<float2*>(wb + p8) = POW2 ? make_float2(p0 * p0, p1 * p1) : make_float2(p0, p1);
    }
    wave_lds_sync();
    // ---- filterbank: lane chunk [ks, ks + J) of one filter pair ----------------------
    {
      float a0 = 0.f, a1 = 0.f, c0 = 0.f, c1 = 0.f;
      const unsigned char* pr = wb + prow(ks) * 8;
      const int ib = 16 - (ks & 15);                          // first i past a pad pair
      const float2* cw = s_cw + lane * p.JS;
      const int J = JT ? JT : p.J;
#pragma unroll
      for (int i = 0; i < J; i++) {
        const float2 pp = *reinterpret_cast<const float2*>(pr + 8 * i + (i >= ib ? 16 : 0));
        const float2 w = cw[i];
        a0 += w.x * pp.x; a1 += w.x * pp.y;
        c0 += w.y * pp.x; c1 += w.y * pp.y;
      }
      *reinterpret_cast<float4*>(wb + kPartOff + 16 * lane) = make_float4(a0, a1, c0, c1);
    }
    wave_lds_sync();
    // ---- ln of the filter sums (lane = filter) ----------------------------------------
    if (lane < nmp) {
      const int ms = MS ? MS : p.max_src;
      const float2 q0 = *reinterpret_cast<const float2*>(wb + (SRC_REGS ? srco[0] : s_src[lane]));   // every filter has a source
      float m0 = q0.x, m1 = q0.y;
#pragma unroll
      for (int i = 1; i < ms; i++) {
        const float2 q = *reinterpret_cast<const float2*>(wb + (SRC_REGS ? srco[SRC_REGS ? i : 0] : s_src[64 * i + lane]));
        m0 += q.x;
        m1 += q.y;
      }
      const float lf = -23.025850929940457f;                    // ln(1e-10)
      float l0 = m0 > 0.f ? __logf(m0) : lf, l1 = m1 > 0.f ? __logf(m1) : lf;
      if (lane >= p.n_mels) { l0 = 0.f; l1 = 0.f; }
      float* lm = reinterpret_cast<float*>(wb + kLogOff);
      lm[lane] = l0; lm[nmp + lane] = l1;
    }
    wave_lds_sync();
    {
      // ---- DCT-II (+ lifter): lane = q + 16 f + 32 h, half h of the filters ----------------
      const int q = lane & 15, f = (lane >> 4) & 1, hh = lane >> 5;
      const int half = NH ? NH : (nmp >> 1);
      const float* lm = reinterpret_cast<const float*>(wb + kLogOff) + f * nmp + hh * half;
      const float* d = s_dct + q * (nmp + 4) + hh * half;     // row stride NMP + 4: 11 x 16 B slots
      float s;                                                  // half >= 4 (NMP is a multiple of 8)
      {
        const float4 x = *reinterpret_cast<const float4*>(lm);
        const float4 y = *reinterpret_cast<const float4*>(d);
        s = x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
      }
#pragma unroll
      for (int m = 4; m < half; m += 4) {
        const float4 x = *reinterpret_cast<const float4*>(lm + m);
        const float4 y = *reinterpret_cast<const float4*>(d + m);
        s += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
      }
      const auto r = __builtin_amdgcn_permlane32_swap(u_of(s), u_of(s), false, false);
      s += f_of(r[1]);                                          // lanes < 32: + lane + 32
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
    float ar[16], ae[NE];
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
  auto pick = [&](auto seg) {
    constexpr bool S = decltype(seg)::value;
    if (h256) return p.pow2 ? mfcc_pair_kernel<true, 12, 8, 20, S, 256> : mfcc_pair_kernel<false, 12, 8, 20, S, 256>;
    return p.pow2 ? (head ? mfcc_pair_kernel<true, 12, 8, 20, S, 0> : mfcc_pair_kernel<true, 0, 0, 0, S, 0>)
                  : (head ? mfcc_pair_kernel<false, 12, 8, 20, S, 0> : mfcc_pair_kernel<false, 0, 0, 0, S, 0>);
  };
  auto kern = p.nseg > 0 ? pick(std::true_type{}) : pick(std::false_type{});
  if (p.lds_bytes > 64 * 1024)
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, p.lds_bytes);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * mfcc_pair_waves_per_block()), p.lds_bytes, s, p);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int mfcc_pair_wave_bytes() { return kWaveBytes; }
int mfcc_pair_waves_per_block() { return 12; }
int mfcc_pair_waves_per_cu() { return 12; }
int mfcc_pair_rows() { return kPRows; }

}  // namespace sonar
