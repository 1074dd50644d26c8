// pk_complex.h -- packed-f32 complex arithmetic for gfx950 (CDNA4), used by mfcc_pair.hip.
//
// A complex value lives in one even-aligned VGPR pair (re, im).  Every helper is ONE VOP3P
// instruction on both halves (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32), so one wave64 issue
// retires 128 f32 results: the f32 VALU peak (MI355X_MICROARCH.md: 64 FLOP/clk/SIMD) is only
// reachable through the packed forms -- plain v_add/v_fma_f32 run at half of it.  Operand
// swizzles (-i b, swapped halves, one half broadcast) are VOP3P source selects, not extra
// instructions:
//   op_sel[i]    = which half of source i feeds the LOW result,
//   op_sel_hi[i] = which half of source i feeds the HIGH result (default 1 = high),
//   neg_lo[i] / neg_hi[i] negate source i's input to the low / high result.
// tools/pk_selftest.hip checks every helper against scalar arithmetic on the GPU.
#pragma once
#include <hip/hip_runtime.h>

namespace sonar {
namespace pk {

typedef float cf __attribute__((ext_vector_type(2)));
constexpr float kC = 0.70710678118654752440f;   // sqrt(2)/2

#define SONAR_PK2(name, ins)                             \
  __device__ __forceinline__ cf name(cf a, cf b) {       \
    cf d;                                                \
    asm(ins : "=v"(d) : "v"(a), "v"(b));                 \
    return d;                                            \
  }
#define SONAR_PK3(name, ins)                             \
  __device__ __forceinline__ cf name(cf a, cf b, cf c) { \
    cf d;                                                \
    asm(ins : "=v"(d) : "v"(a), "v"(b), "v"(c));         \
    return d;                                            \
  }

SONAR_PK2(cadd, "v_pk_add_f32 %0, %1, %2")                                                // a + b
SONAR_PK2(csub, "v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]")                      // a - b
SONAR_PK2(cadd_mi, "v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]")   // a + (-i) b
SONAR_PK2(csub_mi, "v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]")   // a - (-i) b
SONAR_PK2(pmul, "v_pk_mul_f32 %0, %1, %2")                                                // elementwise
SONAR_PK3(pfma, "v_pk_fma_f32 %0, %1, %2, %3")                                            // a * b + c
// (a.x + b.x, a.x - b.x) and (a.y - b.y, a.y + b.y): Z_k +- conj Z_-k of the two real frames
SONAR_PK2(split_re, "v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,0] neg_hi:[0,1]")
SONAR_PK2(split_im, "v_pk_add_f32 %0, %1, %2 op_sel:[1,1] neg_lo:[0,1]")
// c + a.x * b  /  c + a.y * b  (one weight broadcast to both frames)
SONAR_PK3(fma_bx, "v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]")
SONAR_PK3(fma_by, "v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0]")
// x * w.x  /  x * w.y  (one window sample broadcast to the pair of frames)
SONAR_PK2(mul_bx, "v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]")
SONAR_PK2(mul_by, "v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]")

// complex product a * w: t = (a.x w.x, a.x w.y); d = t + (-a.y w.y, a.y w.x)
__device__ __forceinline__ cf cmul(cf a, cf w) {
  cf t, d;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(d) : "v"(a), "v"(w), "v"(t));
  return d;
}
// (a.x + a.y, a.y - a.x) = sqrt(2) a w8^1
__device__ __forceinline__ cf swapadd(cf a) {
  cf d;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(a));
  return d;
}
__device__ __forceinline__ cf kk() { return cf{kC, kC}; }
// e + kC s,  e - kC s
__device__ __forceinline__ cf fma_k(cf s, cf e) { return pfma(s, kk(), e); }
__device__ __forceinline__ cf fnma_k(cf s, cf e) {
  cf d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(d) : "v"(s), "v"(kk()), "v"(e));
  return d;
}
// e + (-i) kC s = (e.x + kC s.y, e.y - kC s.x),  e - (-i) kC s
__device__ __forceinline__ cf fma_k_mi(cf s, cf e) {
  cf d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=v"(d) : "v"(s), "v"(kk()), "v"(e));
  return d;
}
__device__ __forceinline__ cf fnma_k_mi(cf s, cf e) {
  cf d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=v"(d) : "v"(s), "v"(kk()), "v"(e));
  return d;
}
// kC s,  (-i) kC s = (kC s.y, -kC s.x)
__device__ __forceinline__ cf mul_k(cf s) { return pmul(s, kk()); }
__device__ __forceinline__ cf mul_k_mi(cf s) {
  cf d;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1] neg_hi:[1,0]" : "=v"(d) : "v"(s), "v"(kk()));
  return d;
}
// -i a = (a.y, -a.x)
__device__ __forceinline__ cf negi(cf a) { return cf{a.y, -a.x}; }
// (|a + conj b|^2, |a - conj b|^2): the power of both real frames at one bin
__device__ __forceinline__ cf pw2(cf a, cf b) {
  const cf sr = split_re(a, b), si = split_im(a, b);
  return pfma(si, si, pmul(sr, sr));
}

#undef SONAR_PK2
#undef SONAR_PK3

}  // namespace pk
}  // namespace sonar
