// lzq_su2.h -- two-level (SU(2)) helpers shared by the LZ propagators (lzq_propagator.hip,
// lzq_profile.hip).  Not ABI.
#pragma once
#include <hip/hip_runtime.h>

namespace lzq {

struct Cplx {
  double re, im;
};

// <u|psi> for u = (u0, u1)
__host__ __device__ __forceinline__ Cplx inner(Cplx u0, Cplx u1, Cplx p0, Cplx p1) {
  return {u0.re * p0.re + u0.im * p0.im + u1.re * p1.re + u1.im * p1.im,
          u0.re * p0.im - u0.im * p0.re + u1.re * p1.im - u1.im * p1.re};
}

// cos(x) and sin(x)/x as even Taylor polynomials in x2 = x^2 for x2 <= 1 (truncation < 1e-17;
// a Magnus step's rotation angle |n| ~ E dt <= 1 at >= 3 steps per radian), else through
// sincos.  Replaces sqrt + sincos + a division per step; the numpy restatements use libm.
static __constant__ double kSincC[9] = {0x1.0000000000000p+0,  -0x1.5555555555555p-3, 0x1.1111111111111p-7,
                                        -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26,
                                        0x1.6124613a86d09p-33,  -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49};
static __constant__ double kCosC[10] = {0x1.0000000000000p+0,  -0x1.0000000000000p-1, 0x1.5555555555555p-5,
                                        -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22,
                                        0x1.1eed8eff8d898p-29,  -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45,
                                        -0x1.6827863b97d97p-53};
// Three-address FP64 fma.  The Horner steps below add a loop-invariant coefficient; written as
// __builtin_fma the compiler picks the two-address v_fmac_f64 and copies the coefficient into the
// accumulator first (one v_mov_b64 per term, ~19 per Magnus step); v_fma_f64 needs no copy.
#ifndef LZQ_SU2_FMA3
#define LZQ_SU2_FMA3 1  // 0: __builtin_fma (tools/ablate_prop.py)
#endif
__device__ __forceinline__ double fma3(double a, double b, double c) {
  if (!LZQ_SU2_FMA3) return __builtin_fma(a, b, c);
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// The same with a wave-uniform addend (a Horner coefficient) pinned to an SGPR pair: v_fma_f64 reads
// one scalar operand for free, so the constants need neither VGPRs nor the per-step v_mov copies the
// register allocator otherwise inserts to rebuild them (round 4: ~17 VALU per profile Magnus step).
__device__ __forceinline__ double fma3s(double a, double b, double c) {
  if (!LZQ_SU2_FMA3) return __builtin_fma(a, b, c);
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

__device__ __forceinline__ void cos_sinc(double x2, double& cs, double& sc) {
  if (x2 <= 1.0) {
    double ps = kSincC[8], pc = kCosC[9];
#pragma unroll
    for (int k = 7; k >= 0; --k) ps = fma3s(ps, x2, kSincC[k]);
#pragma unroll
    for (int k = 8; k >= 0; --k) pc = fma3s(pc, x2, kCosC[k]);
    sc = ps;
    cs = pc;
  } else {
    const double x = sqrt(x2);
    double sn;
    sincos(x, &sn, &cs);
    sc = sn / x;
  }
}

// The same for |n|^2 <= 1/4 with the Taylor series cut at 7 (sinc) and 8 (cos) terms (< 1e-16
// there), and at 7 + 7 for |n|^2 <= 1/8 (< 6e-18); both propagators step at >= 3 steps per
// radian, where |n|^2 <~ 0.12.  Beyond 1/4 the full series (and sincos beyond 1).
#ifndef LZQ_SU2_SHORTSC
#define LZQ_SU2_SHORTSC 1
#endif
#ifndef LZQ_SU2_SHORT8
#define LZQ_SU2_SHORT8 1  // |n|^2 <= 1/8 (the usual step): 7 + 7 terms (< 6e-18)
#endif
__device__ __forceinline__ void cos_sinc_short(double x2, double& cs, double& sc) {
  if (LZQ_SU2_SHORT8 && x2 <= 0.125) {
    double ps = kSincC[6], pc = kCosC[6];
#pragma unroll
    for (int k = 5; k >= 0; --k) ps = fma3s(ps, x2, kSincC[k]);
#pragma unroll
    for (int k = 5; k >= 0; --k) pc = fma3s(pc, x2, kCosC[k]);
    sc = ps;
    cs = pc;
  } else if (LZQ_SU2_SHORTSC && x2 <= 0.25) {
    double ps = kSincC[6], pc = kCosC[7];
#pragma unroll
    for (int k = 5; k >= 0; --k) ps = fma3s(ps, x2, kSincC[k]);
#pragma unroll
    for (int k = 6; k >= 0; --k) pc = fma3s(pc, x2, kCosC[k]);
    sc = ps;
    cs = pc;
  } else {
    cos_sinc(x2, cs, sc);
  }
}

// cos|n| and sin|n|/|n| of a step (cos_sinc_short's values): the usual |n|^2 <= 1/8 inline, the
// rest out of line, so the longer series' coefficients hold no registers in the step loops
// (lzq_profile.hip's Magnus step, lzq_propagator.hip's core steps)
#ifndef LZQ_SU2_COLD_SC
#define LZQ_SU2_COLD_SC 1  // 0: cos_sinc_short inline (tools/ablate_profile.py, tools/ablate_prop.py)
#endif
struct CosSinc {
  double cs, sc;
};
static __device__ __noinline__ CosSinc cos_sinc_cold(double x2) {
  CosSinc r;
  cos_sinc_short(x2, r.cs, r.sc);
  return r;
}
__device__ __forceinline__ void cos_sinc_step(double x2, double& cs, double& sc) {
  if (!LZQ_SU2_COLD_SC || !LZQ_SU2_SHORT8) {
    cos_sinc_short(x2, cs, sc);
  } else if (x2 <= 0.125) {
    double ps = kSincC[6], pc = kCosC[6];
#pragma unroll
    for (int k = 5; k >= 0; --k) ps = fma3s(ps, x2, kSincC[k]);
#pragma unroll
    for (int k = 5; k >= 0; --k) pc = fma3s(pc, x2, kCosC[k]);
    sc = ps;
    cs = pc;
  } else {
    const CosSinc r = cos_sinc_cold(x2);
    cs = r.cs;
    sc = r.sc;
  }
}

// psi <- exp(-i n.sigma) psi, with cs = cos|n| and (sx, sy, sz) = sin|n|/|n| * n:
// U11 = cs - i sz ; U12 = -sy - i sx ; U21 = sy - i sx ; U22 = cs + i sz
__device__ __forceinline__ void su2_apply(double cs, double sx, double sy, double sz, Cplx& p0, Cplx& p1) {
#define FMA __builtin_fma
  Cplx q0, q1;
  q0.re = FMA(cs, p0.re, FMA(sz, p0.im, FMA(-sy, p1.re, sx * p1.im)));
  q0.im = FMA(cs, p0.im, FMA(-sz, p0.re, FMA(-sy, p1.im, -(sx * p1.re))));
  q1.re = FMA(sy, p0.re, FMA(sx, p0.im, FMA(cs, p1.re, -(sz * p1.im))));
  q1.im = FMA(sy, p0.im, FMA(-sx, p0.re, FMA(cs, p1.im, sz * p1.re)));
#undef FMA
  p0 = q0;
  p1 = q1;
}

}  // namespace lzq
