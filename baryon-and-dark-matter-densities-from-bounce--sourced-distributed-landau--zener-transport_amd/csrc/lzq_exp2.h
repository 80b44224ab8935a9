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
#include <math.h>
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

// fma(a, b, c) with the addend c in an SGPR pair: one VOP3 v_fma_f64 on the device.  Left to
// itself the compiler keeps Horner coefficients in VGPRs (hoisted out of loops: 2 VGPRs each)
// and emits v_mov_b64 + v_fmac_f64 (addend = destination) per step, 2 VALU instead of 1.
#ifndef LZQ_EXP2_VVS
#define LZQ_EXP2_VVS 0  // 1: exp2_poly Horner steps through fma_vvs (ODE A/B: -3.5% narrow, +1% stiff; off)
#endif
LZQ_HD double fma_vvs(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
#else
  return __builtin_fma(a, b, c);
#endif
}

LZQ_HD double exp2_poly(double r) {
#if !LZQ_EXP2_VVS
#define fma_vvs __builtin_fma
#endif
  double q = fma_vvs(r, kExp2A11, kExp2A10);
  q = fma_vvs(r, q, kExp2A9);
  q = fma_vvs(r, q, kExp2A8);
  q = fma_vvs(r, q, kExp2A7);
  q = fma_vvs(r, q, kExp2A6);
  q = fma_vvs(r, q, kExp2A5);
  q = fma_vvs(r, q, kExp2A4);
  q = fma_vvs(r, q, kExp2A3);
  q = fma_vvs(r, q, kExp2A2);
  q = fma_vvs(r, q, kExp2A1);
#if !LZQ_EXP2_VVS
#undef fma_vvs
#endif
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

// 2^(c2*g + bias) for c2*g <= 0 (see header comment); bias = kOmegaBias when the caller's
// weights are the scaled omega' = omega * 2^-512 of the z table.
LZQ_HD double exp2_nonpos(double c2, double g, int32_t bias = 0) {
  double u = c2 * g;
  double kd = __builtin_rint(u);
  double r = __builtin_fma(c2, g, -kd);
  int32_t k = cvt_i32_sat(kd);  // INT_MIN + bias stays hugely negative -> 0
  return __builtin_ldexp(exp2_poly(r), k + bias);
}

// ---------------------------------------------------------------------------------------
// Table-driven variant (default).  2^(u/N) for u = c2N*g <= 0 (u in 1/N-octave units):
//   u = N e + j + r,  k = N e + j = round(u),  |r| <= 1/2,
//   2^(u/N) = 2^e * T[j] * (1 + q(r)),  T[j] = 2^(j/N),  q(r) = r*(B1 + r*(B2 + ...)),
// q a minimax polynomial of degree LZQ_POLYDEG in r (tools/exp2_tab_poly.py; absolute error
// |dq| of q is the relative error of T*(1+q)).  The kernel (lzq_kernels.hip, zsum) never
// forms 2^e with ldexp: the LDS table stores T'[j] with its high word pre-biased so that ONE
// integer add of (k << S), S = 20 - BITS, gives T[j] * 2^(e + 512) (tab_scale), and the z
// table's weights carry the compensating 2^-512 (kOmegaBias).  k is clamped to
// KMIN = -1534 N so that e + 512 >= -1022 keeps that product a normal double.
//
//   BITS DEG  LDS/block  |dq| (minimax)     VALU/node  C2 points/s (1 GPU)
//     8   4     2 KB     1.9e-17 (0.1 ulp)   12.5       3.17e5  (round-1 kernel: ldexp path)
//    12   2    32 KB     2.5e-14 (114 ulp)   11.4       3.54e5  (ldexp path, 2-op address)
//    13   2    64 KB     3.2e-15 (14 ulp)    10         4.64e5  (LZQ_SQFORM=0)
//    13   2sq  64 KB     1.73e-14 (78 ulp)   9          5.25e5  (default: completed square, below)
// The 13-bit address is ONE v_lshlrev_b16 ((k << 3) mod 2^16 = 8*(k mod 8192)).  The default's
// 1.73e-14 bound moves Y_B by at most that much (relative), 6e5 x inside the north_star 1e-8
// gate; tests/test_exp2_host.py pins every row against mpmath.
#ifndef LZQ_TABBITS
#define LZQ_TABBITS 13
#endif
#ifndef LZQ_POLYDEG
#define LZQ_POLYDEG 2
#endif

template <int BITS, int DEG>
struct TabPoly;  // coefficients B1..B_DEG of 2^(r/2^BITS) - 1 ~= r*(B1 + r*(B2 + ...))
template <>
struct TabPoly<8, 4> {  // Taylor: (ln2/256)^i / i!
  static constexpr double B[4] = {0x1.62e42fefa39efp-9, 0x1.ebfbdff82c58fp-19, 0x1.c6b08d704a0c0p-29,
                                  0x1.3b2ab6fba4e77p-39};
};
template <>
struct TabPoly<10, 3> {
  static constexpr double B[3] = {0x1.62e42fefa39efp-11, 0x1.ebfbe03972542p-23, 0x1.c6b08dae13771p-35};
};
template <>
struct TabPoly<12, 2> {
  static constexpr double B[2] = {0x1.62e42ff4f7b0ap-13, 0x1.ebfbdffcafed4p-27};
};
template <>
struct TabPoly<12, 3> {
  static constexpr double B[3] = {0x1.62e42fefa39efp-13, 0x1.ebfbdffc40b8ap-27, 0x1.c6b08d7426a2bp-41};
};
template <>
struct TabPoly<13, 2> {
  static constexpr double B[2] = {0x1.62e42ff0f8a36p-14, 0x1.ebfbdff94d3e0p-29};
};
template <>
struct TabPoly<14, 2> {
  static constexpr double B[2] = {0x1.62e42feff8e01p-15, 0x1.ebfbdff874923p-31};
};
template <>
struct TabPoly<14, 3> {
  static constexpr double B[3] = {0x1.62e42fefa39efp-15, 0x1.ebfbdff86d9eep-31, 0x1.c6b08d7087d56p-47};
};

// Completed-square form of the degree-2 step (LZQ_SQFORM, default on for 13 bits / degree 2):
//   2^(r/N) ~= C * ((r + A)^2 + beta),  A an INTEGER,
// so that s = r + A comes out of the reduction at no extra cost (w = (M + A) - t is exact
// because M + A is, then s = fma(c2N, g, w) rounds once), the polynomial is ONE fma
// q = fma(s, s, beta), and C is folded into the table, T''[j] = C * 2^(j/N).  The node is then
//   t, w, s, address, exponent insert, q, v = T'' * q, F += omega' * v  = 8 VALU (was 9).
// A = N/ln2 would be Taylor's centre (11818.47); the nearest integers cost accuracy: the
// minimax (C, beta) at A = 11819 leaves |2^(r/N) - p(r)| <= 1.73e-14 relative on [-1/2, 1/2]
// (A = 11818: 2.16e-14) -- 6e5 x inside the north_star 1e-8 gate (tests/test_exp2_host.py
// pins it against mpmath).  C ~ 2^-27.06 lowers the table's exponents by 28, so KMIN is
// -1506 N (e + 512 - 28 >= -1022 keeps T''*2^(e+512) normal); those clamped nodes still
// contribute omega*2^u with u < -1506 octaves, which rounds away exactly.
#ifndef LZQ_SQFORM
#define LZQ_SQFORM 1
#endif

constexpr int kTabBits = LZQ_TABBITS;
constexpr int kTabN = 1 << kTabBits;
constexpr int kPolyDeg = LZQ_POLYDEG;
constexpr bool kSqForm = LZQ_SQFORM && kTabBits == 13 && kPolyDeg == 2;
constexpr double kSqA = 11819.0;
constexpr double kSqBeta = 139678307.60123383601;  // tools/exp2_tab_poly.py --sq 11819
constexpr long double kSqC = 3.5795199663544010274e-9L;
constexpr int kTabShift = 20 - kTabBits;          // (k << S) = (e << 20) + (j << S)
constexpr int32_t kOmegaBias = 512;               // T' carries 2^512, omega' carries 2^-512
constexpr int32_t kTabKMin = (kSqForm ? -1506 : -1534) * kTabN;  // T'*2^(e+512) stays normal
static_assert(kTabBits >= 8 && kTabBits <= 16, "table bits");
static_assert((int64_t)kTabKMin * (1 << kTabShift) >= INT32_MIN, "k << S must not overflow");

// q(r) = r*(B1 + r*(B2 + ...)): DEG-1 fma + 1 mul, coefficients passed in (so that a caller
// can hold B1 in a VGPR across its loop: a VOP3 op reads at most one SGPR on gfx950, and the
// compiler otherwise re-materialises the copy every iteration)
template <int DEG>
LZQ_HD double tab_q_with(double r, const double (&B)[DEG]) {
  double acc = B[DEG - 1];
#pragma unroll
  for (int i = DEG - 2; i >= 0; --i) acc = __builtin_fma(r, acc, B[i]);
  return r * acc;
}

// Exact value of table entry j before its one rounding (host side): 2^(j/N), times C in the
// completed-square form.
static inline long double tab_exact(int32_t j) {
  const long double T = exp2l((long double)j / (long double)kTabN);
  return kSqForm ? T * kSqC : T;
}

// Table entry j as stored (host side): tab_exact(j) rounded once, high word pre-biased by
// (512 << 20) - (j << S) (mod 2^32).
static inline uint64_t tab_entry_bits(long double T_exact, int32_t j) {
  const uint64_t b = __builtin_bit_cast(uint64_t, (double)T_exact);
  const uint32_t hi = (uint32_t)(b >> 32) + ((uint32_t)kOmegaBias << 20) - ((uint32_t)j << kTabShift);
  return ((uint64_t)hi << 32) | (b & 0xffffffffu);
}

// LDS byte address of entry (k mod N) from the low word k of the clamped magic sum.
LZQ_HD uint32_t tab_byte_addr(uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (kTabBits == 13) {
    uint32_t a;  // 16-bit shift, upper half zeroed: (k << 3) & 0xffff = 8 * (k & 8191)
    asm("v_lshlrev_b16_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
        : "=v"(a) : "v"(k));
    return a;
  }
#endif
  return (k & (uint32_t)(kTabN - 1)) << 3;
}

// T'[j] with its high word advanced by k << S:  T[j] * 2^(e + 512).
// (written on a 2 x u32 vector so that the compiler emits one v_lshl_add_u32 on the high
// VGPR of the pair, not a 64-bit add)
typedef uint32_t lzq_u32x2 __attribute__((vector_size(8)));
LZQ_HD double tab_scale(double Tp, uint32_t k) {
  lzq_u32x2 w = __builtin_bit_cast(lzq_u32x2, Tp);
  w[1] = w[1] + (k << kTabShift);
  return __builtin_bit_cast(double, w);
}

// Host/device reference of one table-variant node: returns 2^(u/N) * 2^512 exactly as the
// kernel forms it (the kernel multiplies by omega' = omega * 2^-512 inside its accumulate).
// tabp = table as stored (tab_entry_bits).  c2N*g <= 0, |c2N*g| < 2^51.
LZQ_HD double exp2_tab_scaled(double c2N, double g, const double* tabp) {
  constexpr double kMagic = 0x1.8p52;
  const double t = __builtin_fma(c2N, g, kMagic);
  const double tc = __builtin_fmax(t, kMagic + (double)kTabKMin);
  const uint32_t k = (uint32_t)__builtin_bit_cast(uint64_t, tc);
  const double Ts = tab_scale(tabp[tab_byte_addr(k) >> 3], k);
  if constexpr (kSqForm) {
    const double s = __builtin_fma(c2N, g, (kMagic + kSqA) - t);  // r + A, one rounding
    return Ts * __builtin_fma(s, s, kSqBeta);
  }
  const double kd = t - kMagic;
  const double r = __builtin_fma(c2N, g, -kd);
  const double q = tab_q_with<kPolyDeg>(r, TabPoly<kTabBits, kPolyDeg>::B);
  return __builtin_fma(Ts, q, Ts);
}

}  // namespace lzq
