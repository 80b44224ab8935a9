// lzq_exp2.h -- the FP64 exponential of the KJMA inner loop (fpy:163), CDNA4 form.
//
// The reference evaluates, per (y, z_k) node, exp(c * g4_k) with c = -(I_p/6) e^y <= 0
// (fpy:163).  The kernel evaluates the same quantity as 2^(c2 * g4_k) with c2 = c*log2(e)
// rounded once per y-node (not per z-node), in 17 FP64 VALU issue slots per node instead
// of the ~23 of the generic ROCm exp(double):
//
//   u  = c2*g            v_mul_f64
//   kd = rint(u)         v_rndne_f64
//   r  = fma(c2,g,-kd)   v_fma_f64     r in [-1/2, 1/2], one rounding
//   k  = (int)kd         v_cvt_i32_f64 saturating: |u| >= 2^31 gives INT_MIN -> result 0
//   p  = 1 + r*q(r)      11 x v_fma_f64, degree-11 minimax (tools/exp2_poly.py): 0.63 ulp
//   2^u = ldexp(p, k)    v_ldexp_f64   exact scaling, gradual underflow to 0 like libm
//
// No overflow / NaN / positive-argument handling is needed: g4_k >= 0 (checked when the
// table is built) and c2 < 0, so u <= 0.  For |u| >= 2^52 the reduction is meaningless
// but p stays finite (|r| < 2^30) and ldexp(p, INT_MIN) is 0, the exact answer.
// Accuracy vs the libm exp of the oracle: the rounding of c2 costs |u|*2^-53 relative,
// i.e. < 1e-13 even where u ~ -1000 (and those nodes are ~1e-300 of the sum).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LZQ_HD __host__ __device__ __forceinline__
#else
#define LZQ_HD static inline
#endif

namespace lzq {

// 2^r = 1 + r*(A1 + r*(A2 + ... + r*A11)) on [-1/2, 1/2]; tools/exp2_poly.py 11
constexpr double kExp2A1 = 0x1.62e42fefa39efp-1;
constexpr double kExp2A2 = 0x1.ebfbdff82c5a4p-3;
constexpr double kExp2A3 = 0x1.c6b08d7049fe8p-5;
constexpr double kExp2A4 = 0x1.3b2ab6fba0119p-7;
constexpr double kExp2A5 = 0x1.5d87fe78cd6d4p-10;
constexpr double kExp2A6 = 0x1.4309130ed8da0p-13;
constexpr double kExp2A7 = 0x1.ffcbfba97fab8p-17;
constexpr double kExp2A8 = 0x1.62bfc79d2fa58p-20;
constexpr double kExp2A9 = 0x1.b5267ce2583c7p-24;
constexpr double kExp2A10 = 0x1.e61b4fc4ab239p-28;
constexpr double kExp2A11 = 0x1.e79bb37875897p-32;
constexpr double kLog2E = 0x1.71547652b82fep0;  // log2(e) rounded to nearest

LZQ_HD double exp2_poly(double r) {
  double q = __builtin_fma(r, kExp2A11, kExp2A10);
  q = __builtin_fma(r, q, kExp2A9);
  q = __builtin_fma(r, q, kExp2A8);
  q = __builtin_fma(r, q, kExp2A7);
  q = __builtin_fma(r, q, kExp2A6);
  q = __builtin_fma(r, q, kExp2A5);
  q = __builtin_fma(r, q, kExp2A4);
  q = __builtin_fma(r, q, kExp2A3);
  q = __builtin_fma(r, q, kExp2A2);
  q = __builtin_fma(r, q, kExp2A1);
  return __builtin_fma(r, q, 1.0);
}

// Saturating double -> int32 (v_cvt_i32_f64 semantics: out-of-range clamps, NaN -> 0).
LZQ_HD int32_t cvt_i32_sat(double kd) {
#if defined(__HIP_DEVICE_COMPILE__)
  int32_t k;
  asm("v_cvt_i32_f64 %0, %1" : "=v"(k) : "v"(kd));
  return k;
#else
  if (kd != kd) return 0;
  if (kd <= -2147483648.0) return INT32_MIN;
  if (kd >= 2147483647.0) return INT32_MAX;
  return (int32_t)kd;
#endif
}

// 2^(c2*g) for c2*g <= 0 (see header comment).
LZQ_HD double exp2_nonpos(double c2, double g) {
  double u = c2 * g;
  double kd = __builtin_rint(u);
  double r = __builtin_fma(c2, g, -kd);
  int32_t k = cvt_i32_sat(kd);
  return __builtin_ldexp(exp2_poly(r), k);
}

// ---------------------------------------------------------------------------------------
// Table-driven variant (default): 2^u = 2^e * T[j] * 2^(r/256),  u*256 = 256 e + j + r,
// T[j] = 2^(j/256) (2 KB, staged in LDS once per block), |r| <= 1/2 so r/256 <= 2^-9 and a
// degree-4 Taylor polynomial is accurate to 3.8e-17 (0.17 ulp).  Per node: 11 FP64 VALU
// (mul, rndne, fma, cvt, 3 fma + mul, fma, ldexp, + the caller's accumulate) + 3 integer
// VALU (and, shift for the LDS address, arithmetic shift for e) + one ds_read_b64.  The LDS
// table has 256 distinct 8-byte entries, so a wave64 read is at most 8-way bank-conflicted
// and is usually far less (lanes of one wave hold neighbouring y-nodes).
constexpr int kTabBits = 8;
constexpr int kTabN = 1 << kTabBits;
constexpr double kTabB1 = 0x1.62e42fefa39efp-9;   // (ln2/256)^1 / 1!
constexpr double kTabB2 = 0x1.ebfbdff82c58fp-19;  // (ln2/256)^2 / 2!
constexpr double kTabB3 = 0x1.c6b08d704a0c0p-29;  // (ln2/256)^3 / 3!
constexpr double kTabB4 = 0x1.3b2ab6fba4e77p-39;  // (ln2/256)^4 / 4!

// 2^(c2N*g / 256) for c2N*g <= 0 with c2N = 256*c2; tab[j] = 2^(j/256).
LZQ_HD double exp2_nonpos_tab(double c2N, double g, const double* tab) {
  double u = c2N * g;
  double kd = __builtin_rint(u);
  double r = __builtin_fma(c2N, g, -kd);
  int32_t k = cvt_i32_sat(kd);
  int32_t j = k & (kTabN - 1);
  int32_t e = k >> kTabBits;  // arithmetic shift: floor(k / 256); INT_MIN -> -2^23 -> 0 result
  double T = tab[j];
  double q = r * __builtin_fma(r, __builtin_fma(r, __builtin_fma(r, kTabB4, kTabB3), kTabB2), kTabB1);
  return __builtin_ldexp(__builtin_fma(T, q, T), e);
}

}  // namespace lzq
