// lzq_kernels.hip -- CDNA4 (gfx950) kernels + C ABI of the bounce-sourced LZ yield engine.
//
// Hot path (fpy = /root/reference/first_principles_yields.py):
//   Y_B = trapz_y[ P J(y) A/V(y) W(y) / (s H T) |dT/dy| ]          fpy:231-267
//   A/V(y) = pref(y) * trapz_z[ z^2 e^-z exp(c(y) g4(z)) ]          fpy:158-165
// with 8000 y-nodes x 1200 z-nodes per parameter point.
//
// Mapping:
//   * one 64-lane wavefront owns one parameter point; lane l takes y-nodes l, l+64, ...;
//     no barriers (besides staging the exp table) and no atomics; 16 independent wavefronts
//     per 1024-thread block, two blocks per CU (8 waves per SIMD);
//   * the point-invariant z tables {g4_k, omega'_k} (omega = z^2 e^-z x trapezoid weight,
//     scaled by 2^-512) are read with wave-uniform addresses -> scalar loads into SGPRs, so
//     every FP64 VALU op of the inner loop takes its table operand from an SGPR;
//   * the inner exp is the pre-biased 8192-entry LDS table of lzq_exp2.h: 9-10 VALU per
//     (y, z) node including the accumulate (zsum below);
//   * per-lane partial sums over its y-nodes are combined by a fixed xor-butterfly, so the
//     result is a pure function of the point: independent of launch geometry, batch
//     composition and GPU count (SURVEY §8e bit-identity across W = 1,2,4,8).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/lzq.h"
#include "lzq_exp2.h"
#include "lzq_internal.h"
#include "lzq_physics.h"

namespace lzq {

constexpr int kNZ = LZQ_NZ;
constexpr int kWaveSize = 64;
// The block is sized so that the LDS copies of the exp table that fit in a CU's 160 KB carry
// the waves: 64-KB table (default) -> two 1024-thread blocks per CU = 8 waves per SIMD, with
// LZQ_MIN_WAVES = 8 capping the kernel at 64 VGPRs (its few spills sit outside the z-loop;
// +2.2% over 4 waves/SIMD, tools/ablate_builds.py).
#ifndef LZQ_BLOCK
#define LZQ_BLOCK ((8 << LZQ_TABBITS) > 81920 ? 1024 : (8 << LZQ_TABBITS) > 40960 ? 1024 : 256)
#endif
constexpr int kBlock = LZQ_BLOCK;
constexpr int kWavesPerBlock = kBlock / kWaveSize;
#ifndef LZQ_KUNROLL
#define LZQ_KUNROLL 8
#endif
#ifndef LZQ_YB
#define LZQ_YB 1
#endif
// __launch_bounds__ second argument = minimum waves per SIMD (8: <= 64 VGPRs; see LZQ_BLOCK)
#ifndef LZQ_MIN_WAVES
#define LZQ_MIN_WAVES 8
#endif
// z-table source: 0 = wave-uniform scalar loads (SGPR operands), 1 = staged in LDS and read
// with broadcast ds_read_b128 (keeps every LGKM operation of the loop in order, so the
// compiler can use counted lgkmcnt waits instead of draining behind SMEM)
#ifndef LZQ_ZLDS
#define LZQ_ZLDS 0
#endif
#ifndef LZQ_YFACT_EARLY
#define LZQ_YFACT_EARLY 0
#endif
// re-form y / e^y / weight after the z-loop instead of keeping them live across it
#ifndef LZQ_Y_RECOMPUTE
#define LZQ_Y_RECOMPUTE 1
#endif
// keep yb_wave's per-lane running sum in the wave's LDS slot instead of a VGPR pair
#ifndef LZQ_ACC_LDS
#define LZQ_ACC_LDS 1
#endif
constexpr int kKUnroll = LZQ_KUNROLL;  // z-nodes per scalar-load batch (must divide 1200)
constexpr int kYB = LZQ_YB;            // y-nodes per lane per pass (independent chains)
static_assert(kNZ % kKUnroll == 0, "z unroll must divide nz");

struct ZNode {
  double g4;     // fpy:156 gamma4(z_k), verbatim cancelling form
  double omega;  // z_k^2 e^{-z_k} * trapezoid weight of node k
};

// ---------------------------------------------------------------------------------------
// per-point quadrature setup (wave-uniform values)
// ---------------------------------------------------------------------------------------
struct QuadSetup {
  double y_lo, y_hi, step, delta;  // ys = linspace(y_lo, y_hi, n)    fpy:247
  int64_t n;
  bool empty;                      // y_hi <= y_lo -> Y_B = 0         fpy:242-243
  double pref0;                    // (I_p/2)(beta/v_w)               fpy:162
  double cneg;                     // -(I_p/6)                        fpy:163
  double Bc, Tp, dT0, sig, m, m3, flux, P, g_star, g_star_s;
  double H0;      // 1.66 sqrt(g*) / M_Pl             fpy:85
  double s0;      // (2 pi^2/45) g*s                   fpy:88
  double c_rel;   // g * 3 zeta3/(4 pi^2) | g zeta3/pi^2   fpy:96-99
  double c_nr;    // g (m/2pi)^1.5                     fpy:104
  double v0;      // pi * max(m, 1e-20)                fpy:117
  double isig;    // 1/sig: y_factors multiplies instead of dividing
};

// Move a wave-uniform double into SGPRs (two v_readfirstlane_b32): the per-point constants
// then occupy scalar registers instead of ~44 VGPRs across the z-loop.
__device__ __forceinline__ double uniform(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// x**1.5 as x*sqrt(x) (<= 2 ulp from pow; the device pow is ~100 VALU and ~40 VGPRs)
__device__ __forceinline__ double pow15(double x) { return x * sqrt(x); }

__device__ __forceinline__ QuadSetup quad_setup(const lzq_point& pt, double P, double T_lo, double T_hi,
                                                int32_t n_y) {
  QuadSetup s;
  const double B = pt.beta_over_H, Tp = pt.T_p_GeV;
  // fpy:234-243
  double y_lo = pymax(y_of_T(T_hi, Tp, B), -80.0);
  double y_hi = pymin(y_of_T(T_lo, Tp, B), +50.0);
  s.empty = !(y_hi > y_lo);
  s.y_lo = y_lo;
  s.y_hi = y_hi;
  s.n = n_y > LZQ_NY_MIN ? n_y : LZQ_NY_MIN;  // fpy:246
  s.delta = y_hi - y_lo;
  s.step = s.delta / (double)(s.n - 1);
  // AoverVKernel constants fpy:146-151
  double v_w = pymax(pt.v_w, 1e-12);
  double H_p = H_std(Tp, pt.g_star);
  double beta = B * H_p;
  s.pref0 = (pt.I_p / 2.0) * (beta / v_w);
  s.cneg = -(pt.I_p / 6.0);
  // fpy:250-262
  s.Bc = pymax(B, 1e-30);
  s.Tp = Tp;
  s.dT0 = -(Tp / s.Bc);
  s.sig = pymax(pt.source_shape_sigma_y, 1e-6);
  s.m = pt.m_chi_GeV;
  s.m3 = pt.m_chi_GeV / 3.0;
  s.flux = pt.incident_flux_scale;
  s.P = P;
  s.g_star = pt.g_star;
  s.g_star_s = pt.g_star_s;
  s.H0 = 1.66 * sqrt(pt.g_star);
  s.s0 = (2.0 * (kPi * kPi) / 45.0) * pt.g_star_s;
  s.c_rel = (pt.stats == 0) ? pt.g_chi * (3.0 * kZeta3 / (4.0 * (kPi * kPi))) : pt.g_chi * (kZeta3 / (kPi * kPi));
  s.c_nr = pt.g_chi * pow15(pt.m_chi_GeV / (2.0 * kPi));
  s.v0 = kPi * pymax(pt.m_chi_GeV, 1e-20);
  s.isig = 1.0 / s.sig;
  double* f[] = {&s.y_lo, &s.y_hi, &s.step, &s.delta, &s.pref0, &s.cneg, &s.Bc, &s.Tp, &s.dT0, &s.sig, &s.m,
                 &s.m3, &s.flux, &s.P, &s.g_star, &s.g_star_s, &s.H0, &s.s0, &s.c_rel, &s.c_nr, &s.v0,
                 &s.isig};
#pragma unroll
  for (double* v : f) *v = uniform(*v);
  return s;
}

// A loop-invariant double materialised once in a VGPR (opaque to re-materialisation).
__device__ __forceinline__ double vgpr_const(double x) {
  double v;
  asm volatile("v_mov_b64 %0, %1" : "=v"(v) : "s"(x));
  return v;
}

// e^x for the per-y factors (<= 1 ulp, like the device libm exp).  Cody-Waite reduction
// x = k ln2 + r, |r| <= ln2/2, Taylor series to r^13 (truncation < 5e-18), ldexp.  The 15
// constants are read from constant memory through an offset made opaque per call, so they
// come in by scalar loads where needed: the libm exp's coefficients were hoisted out of the
// y-loop into VGPRs and spilled to scratch across the z-loop (which needs ~60 of 64 VGPRs).
#ifndef LZQ_YFAST
#define LZQ_YFAST 7  // bit mask (A/B builds): 1 SGPR Horner steps, 2 rsqrt, 4 1/sigma product
#endif

__constant__ double kExpC[15] = {
    0x1.6124613a86d09p-33, 0x1.1eed8eff8d898p-29, 0x1.ae64567f544e4p-26, 0x1.27e4fb7789f5cp-22,
    0x1.71de3a556c734p-19, 0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-13, 0x1.6c16c16c16c17p-10,
    0x1.1111111111111p-7,  0x1.5555555555555p-5,  0x1.5555555555555p-3,  0x1.0p-1,  // 1/13! .. 1/2!
    0x1.71547652b82fep+0,                                                           // 1/ln2
    0x1.62e42fefa39efp-1,  0x1.abc9e3b39803fp-56};                                  // ln2 hi, lo
__device__ __forceinline__ double exp_sc(double x) {
  int o = 0;
  asm volatile("" : "+s"(o));
  const double* c = kExpC + o;
  x = x < -1100.0 ? -1100.0 : x;  // NaN passes through both
  x = x > 710.0 ? 710.0 : x;
  const double k = __builtin_rint(x * c[12]);
  double r = __builtin_fma(-k, c[13], x);
  r = __builtin_fma(-k, c[14], r);
  double p = c[0];
#pragma unroll
  for (int i = 1; i < 12; ++i) p = (LZQ_YFAST & 1) ? fma_vvs(p, r, c[i]) : __builtin_fma(p, r, c[i]);
  p = __builtin_fma(p, r, 1.0);  // (e^r - 1) / r
  p = __builtin_fma(p, r, 1.0);  // e^r
  return __builtin_ldexp(p, (int)k);
}

// numpy.linspace element (handles numpy's step == 0 branch as well)
__device__ __forceinline__ double y_node(const QuadSetup& s, int j) {  // n_y is int32
  const int n = (int)s.n;
  if (j == n - 1) return s.y_hi;
  if (s.step == 0.0) return ((double)j / (double)(n - 1)) * s.delta + s.y_lo;
  return (double)j * s.step + s.y_lo;
}

// Per-y factors of the integrand of fpy:264-265 that do not depend on F, computed BEFORE the
// z-loop so that only these 7 doubles (not the whole QuadSetup) stay live across it.  The
// post-loop combination keeps the reference's rounding order:
//   SB = ((P*J)*Av)*W,  integrand = SB/((s*H)*T)*|dT/dy|,  Av = (pref0*expy)*F.
struct YFactors {
  double PJ;     // P * J(T)                        fpy:260,264
  double W;      // window                          fpy:262
  double sHT;    // (s*H)*T                         fpy:258-259,265
  double adTdy;  // |dT/dy|                         fpy:255,265
  double pexp;   // pref0 * expy  (A/V prefactor)   fpy:162
  double w;      // trapezoid weight of the node    fpy:267
  double live;   // 1 if y <= 50 (fpy:159), else 0
};

// 1/sqrt(d) for a positive normal d: v_rsq_f64, then the Goldschmidt iteration that the
// compiler's correctly rounded sqrt uses (g -> sqrt(d), h -> 1/(2 sqrt(d))); <= 2 ulp.
__device__ __forceinline__ double rsqrt_pos(double d) {
  const double r = __builtin_amdgcn_rsq(d);
  double g = d * r, h = 0.5 * r;
  double e = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  e = __builtin_fma(-g, h, 0.5);
  h = __builtin_fma(h, e, h);
  return 2.0 * h;
}

// The fixed-exponent powers of numpy's `**` (SVML pow, <= 1 ulp) are evaluated with products
// (<= 3 ulp): denom**-0.5 and denom**-1.5 from one reciprocal square root, T**3 = (T*T)*T,
// T**1.5 = T sqrt T; the quotients by per-point constants (y/sigma, H's 1/M_Pl) are products
// with their reciprocals.  This keeps the per-y work small (the device pow(double) is
// ~100 VALU and ~40 VGPRs; a division or a sqrt ~10-16) and moves results by ~1e-16 relative
// (tests: worst golden error unchanged at 1e-13).
__device__ __forceinline__ YFactors y_factors(const QuadSetup& s, double y, double expy, double wt) {
  YFactors f;
  double T, dTdy, H;
  if (LZQ_YFAST & 2) {
    // 2y/B stays a correctly rounded division: near y = -B/2 (T_max/T_p large) 1 + 2y/B cancels,
    // and the product with a rounded 2/B moved Y_B by 6.7e-13 on a golden point (diag_golden.py)
    const double denom = pymax(1.0 + 2.0 * y / s.Bc, 1e-12);  // fpy:252-253
    const double rs = rsqrt_pos(denom);
    T = s.Tp * rs;                                           // fpy:254
    dTdy = s.dT0 * ((rs * rs) * rs);                         // fpy:255  denom**(-1.5)
    H = s.H0 * T * T * (1.0 / kMplGeV);                      // fpy:258 via fpy:85
  } else {
    const double denom = pymax(1.0 + 2.0 * y / s.Bc, 1e-12);
    const double sd = sqrt(denom);
    T = s.Tp / sd;
    dTdy = s.dT0 * (1.0 / (denom * sd));
    H = s.H0 * T * T / kMplGeV;
  }
  double T3 = (T * T) * T;
  double sE = s.s0 * T3;                                  // fpy:259 via fpy:88
  double n_eq, vbar;                                      // fpy:90-120, strict T > m/3 branch
  if (T > s.m3) {
    n_eq = s.c_rel * T3;
    vbar = 1.0;
  } else {
    n_eq = s.c_nr * (T * sqrt(T)) * exp_sc(-s.m / pymax(T, 1e-30));
    vbar = sqrt(pymax(8.0 * T / s.v0, 0.0));
  }
  double J = s.flux * 0.25 * n_eq * vbar;                 // fpy:260
  double q = (LZQ_YFAST & 4) ? y * s.isig : y / s.sig;
  f.W = exp_sc(-0.5 * (q * q));                              // fpy:262
  f.PJ = s.P * J;
  f.sHT = sE * H * T;
  f.adTdy = fabs(dTdy);
  f.pexp = s.pref0 * expy;
  f.w = wt;
  f.live = (y > 50.0) ? 0.0 : 1.0;
  return f;
}

__device__ __forceinline__ double integrand_from(const YFactors& f, double F) {
  double Av = f.live != 0.0 ? f.pexp * F : 0.0;           // fpy:159-165
  double SB = f.PJ * Av * f.W;                            // fpy:264
  return SB / f.sHT * f.adTdy;                            // fpy:265
}

// trapezoid weight of y-node j: (d_{j-1} + d_j)/2 with d = diff(ys)      fpy:267
__device__ __forceinline__ double y_weight(const QuadSetup& s, int j, double y) {
  double dl = (j > 0) ? y - y_node(s, j - 1) : 0.0;
  double dr = (j + 1 < (int)s.n) ? y_node(s, j + 1) - y : 0.0;
  return 0.5 * (dl + dr);
}

// exp variants of the inner loop (lzq_tune(LZQ_TUNE_EXP, ...))
enum ExpVariant { kExpPoly11 = 0, kExpTable = 1 };

// Scale of c2 expected by the variant (2^(c2*g) for poly11, 2^(c2N*g/256) for the table).
template <int EXPV>
__device__ __forceinline__ double c2_scale() { return EXPV == kExpTable ? (double)kTabN : 1.0; }

// F(c2) = sum_k omega_k 2^(c2 g4_k) for YB independent y-nodes per lane.
//
// The loop is VALU-issue bound: an FP64 instruction costs 4.4 cycles per wave64 on gfx950 and an
// integer / FP32 one ~2.5 (tools/ubench_valu.hip, pure streams); in this kernel a node's 8.48
// VALU instructions take 30.9 SIMD-cycles, 79% of them in the 6.1 FP64 FMA/MUL/ADD
// (profiles/round2/pmc_summary.json).  So the loop is built to minimise the instruction count,
// FP64 first.  Table variant, per (y, z) node:
//
//   t  = fma(c2, g, M)          M = 1.5*2^52: t = M + round(u), u = c2*g in 1/N-octave units
//   kd = t - M                  exact
//   r  = fma(c2, g, -kd)        u - round(u) in [-1/2, 1/2], one rounding
//   tc = max(t, M + KMIN)       clamp to e >= -1534 octaves (also keeps lo32 in int range)
//   a  = (lo32(tc) & (N-1))*8   LDS byte address: ONE v_lshlrev_b16 for N = 8192
//   T' = lds[a]                 T'.hi = hi(2^(j/N)) - (j << S) + (512 << 20), S = 20 - BITS
//   T'.hi += lo32(tc) << S      ONE v_lshl_add_u32: T' = 2^(j/N) * 2^(e+512), e = floor(k/N)
//   q  = r*(B1 + r*B2)          2 FP64
//   v  = fma(T', q, T')         = 2^(u/N) * 2^512, always a normal double (e+512 >= -1022)
//   F  = fma(omega', v, F)      omega' = omega * 2^-512 (z table), so omega'*v = omega*2^u
//
// = 10 VALU per node (round-1 kernel: 12.5).  The default completed-square form (kSqForm,
// lzq_exp2.h) replaces kd, r, q and the T*(1+q) fma by
//   w  = (M + A) - t            exact (M + A an integer below 2^53)
//   s  = fma(c2, g, w)          r + A, one rounding
//   v  = T'' * fma(s, s, beta)  T'' = C * 2^(j/N) * 2^(e+512) from the same lookup + insert
// = 9 VALU per node, 8 on clamp-free passes.  The last fma rounds the exact product omega*2^u
// once, so gradual underflow is exact; clamped nodes (u < -1534 octaves) contribute
// omega*2^-1534*(...) which rounds away exactly like the underflowed 0 it stands for.
// For |u| < 2^51 (every non-dead lane, checked on the host) t is exact; dead lanes (whose
// every node k >= 1 underflows) run with c2 = 0 and are zeroed, so no input reaches the
// loop with |u| >= 2^51.
//
// CLAMP = false drops the max (9 VALU/node) on passes whose lanes all satisfy |c2N|*g_max <=
// N*1534 (no node can leave the clamp range); zsum_dispatch picks it per pass.
template <int YB, int EXPV, bool CLAMP = true>
__device__ __forceinline__ void zsum(const ZNode* __restrict__ zt, const double* tab, const double (&c2)[YB],
                                     double (&F)[YB], int kend) {
#pragma unroll
  for (int b = 0; b < YB; ++b) F[b] = 0.0;
  if constexpr (EXPV == kExpTable) {
    constexpr double kMagic = 0x1.8p52;
    constexpr double kTClamp = kMagic + (double)kTabKMin;  // exact
    const double Mv = vgpr_const(kMagic);
    const double MAv = kMagic + kSqA;  // exact (an integer below 2^53)
    // plain form: polynomial coefficients, B1 pinned in a VGPR for the whole loop (see tab_q_with)
    double Bv[kPolyDeg];
#pragma unroll
    for (int i = 0; i < kPolyDeg; ++i) Bv[i] = TabPoly<kTabBits, kPolyDeg>::B[i];
    if constexpr (!kSqForm) Bv[0] = vgpr_const(Bv[0]);
    const char* tabb = reinterpret_cast<const char*>(tab);
    for (int k = 0; k < kend; k += kKUnroll) {
      double g4[kKUnroll], om[kKUnroll];
#pragma unroll
      for (int kk = 0; kk < kKUnroll; ++kk) {
        g4[kk] = zt[k + kk].g4;
        om[kk] = zt[k + kk].omega;
      }
      // phases: reduction + addresses for the whole batch, then the lookups (in flight
      // together), then polynomial + accumulate
      double r[YB][kKUnroll], T[YB][kKUnroll];
      uint32_t kc[YB][kKUnroll], a[YB][kKUnroll];
#pragma unroll
      for (int kk = 0; kk < kKUnroll; ++kk)
#pragma unroll
        for (int b = 0; b < YB; ++b) {
          const double t = __builtin_fma(c2[b], g4[kk], Mv);
          if constexpr (kSqForm) {
            r[b][kk] = __builtin_fma(c2[b], g4[kk], MAv - t);  // s = r + A (lzq_exp2.h)
          } else {
            const double kd = t - Mv;
            r[b][kk] = __builtin_fma(c2[b], g4[kk], -kd);
          }
          const double tc = CLAMP ? __builtin_fmax(t, kTClamp) : t;
          kc[b][kk] = (uint32_t)__builtin_bit_cast(uint64_t, tc);
          a[b][kk] = tab_byte_addr(kc[b][kk]);
        }
#pragma unroll
      for (int kk = 0; kk < kKUnroll; ++kk)
#pragma unroll
        for (int b = 0; b < YB; ++b) T[b][kk] = *reinterpret_cast<const double*>(tabb + a[b][kk]);
#pragma unroll
      for (int kk = 0; kk < kKUnroll; ++kk)
#pragma unroll
        for (int b = 0; b < YB; ++b) {
          const double Ts = tab_scale(T[b][kk], kc[b][kk]);
          if constexpr (kSqForm) {
            F[b] = __builtin_fma(om[kk], Ts * __builtin_fma(r[b][kk], r[b][kk], kSqBeta), F[b]);
          } else {
            const double q = tab_q_with<kPolyDeg>(r[b][kk], Bv);
            F[b] = __builtin_fma(om[kk], __builtin_fma(Ts, q, Ts), F[b]);
          }
        }
    }
  } else {
    for (int k = 0; k < kend; k += kKUnroll) {
#pragma unroll
      for (int kk = 0; kk < kKUnroll; ++kk) {
        const double g = zt[k + kk].g4, om = zt[k + kk].omega;
#pragma unroll
        for (int b = 0; b < YB; ++b) F[b] = __builtin_fma(om, exp2_nonpos(c2[b], g, kOmegaBias), F[b]);
      }
    }
  }
}

// Pass-level wrapper: "dead" lanes, c2 * g4_1 <= -N*1077 (every node k >= 1 underflows to
// exactly 0: g4 is increasing and omega_0 = 0), run the loop with c2 = 0 and are zeroed
// afterwards -- the same instruction stream, the exact zero.
//
// The z grid: NZ > 0 is the compile-time node count of the reference's default grid
// (fpy:142, LZQ_NZ = 1200: the headline kernels); NZ = 0 reads the padded node count nzp of a
// runtime (nz, z_max) grid (AoverVKernel(..., z_max, nz), fpy:141-156).  Padding nodes repeat the
// last g4 with omega = 0: each adds an exact +0, so F is the sum over the nz real nodes.  On a
// fine grid (small g4_1) a live lane can reach |u| >= 2^51 at later nodes, where the magic-
// constant reduction is inexact; every such node has u < KMIN, takes the clamped path (the
// clamp-free test below sees it), and its term omega' * T''(KMIN) * ((A + O(|u| 2^-52))^2 + beta)
// stays below 2^-1074 for |u| < 2^200, so it rounds away exactly like the underflow it stands
// for (tests/test_exp2_host.py); build_ztable bounds |u| by that on the host.
//
// truncate != 0 (lzq_tune LZQ_TUNE_TRUNCATE; NOT used by the headline bench, which is dense
// per SURVEY §8d): the pass stops at kend, the first z-node (rounded up to the unroll) beyond
// which every live lane has c2*g4_k < -1080 octaves.  Those nodes add omega*2^u < 2^-1080 to
// F, which the accumulate's rounding discards exactly, so F is bit-identical to the dense sum.
// (Needs g4 non-decreasing over the grid: the host passes truncate = 0 for a grid whose
// rounded g4 is not.)
template <int YB, int EXPV, int NZ = 0>
__device__ __forceinline__ void zsum_dispatch(const ZNode* __restrict__ zt, int nzp, const double* tab,
                                              const double (&c2)[YB], double (&F)[YB], int truncate = 0) {
  const int nz = NZ > 0 ? NZ : nzp;
  const double g_1 = zt[1].g4, g_max = zt[nz - 1].g4;
  bool dead[YB], small = true;
  double c2e[YB];
#pragma unroll
  for (int b = 0; b < YB; ++b) {
    dead[b] = c2[b] * g_1 <= -c2_scale<EXPV>() * 1077.0;
    c2e[b] = dead[b] ? 0.0 : c2[b];
    small = small && c2e[b] * g_max >= (double)kTabKMin;  // every node stays >= KMIN
  }
  int kend = nz;
  if (truncate) {
    // largest per-lane threshold g_thr = -1080 N / c2 (live lanes; dead lanes impose none,
    // c2 = 0 lanes never underflow)
    double thr = 0.0;
#pragma unroll
    for (int b = 0; b < YB; ++b) {
      const double tb = dead[b] ? 0.0 : (c2e[b] < 0.0 ? (-1080.0 * c2_scale<EXPV>()) / c2e[b] : __builtin_inf());
      thr = pymax(thr, tb);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) thr = pymax(thr, __shfl_xor(thr, off, kWaveSize));
    thr = uniform(thr);
    // first k with g4_k > thr (g4 increasing): scalar binary search over the z table
    int lo = 0, hi = nz;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (zt[mid].g4 > thr) hi = mid;
      else lo = mid + 1;
    }
    kend = (lo + kKUnroll - 1) / kKUnroll * kKUnroll;
  }
  if (EXPV == kExpTable && __all(small))
    zsum<YB, EXPV, false>(zt, tab, c2e, F, kend);
  else
    zsum<YB, EXPV, true>(zt, tab, c2e, F, kend);
#pragma unroll
  for (int b = 0; b < YB; ++b) F[b] = dead[b] ? 0.0 : F[b];
}

// Stage the exp table (N doubles, see lzq_exp2.h) in LDS (every thread of the block must call this).
template <int EXPV>
__device__ __forceinline__ const double* stage_table(const double* __restrict__ gtab, double* lds) {
  if (EXPV != kExpTable) return nullptr;
  for (int i = threadIdx.x; i < kTabN; i += blockDim.x) lds[i] = gtab[i];
  __syncthreads();
  return lds;
}

// LDS image of the per-block tables: z nodes (19.2 KB) followed by the exp table.
struct LdsTables {
  ZNode z[kNZ];
  double t[kTabN];
};

// Stage both tables (global layout: ZNode[kNZ] then double[kTabN], see ensure_device).
template <int EXPV>
__device__ __forceinline__ void stage_tables(const ZNode* __restrict__ gz, LdsTables* lds) {
  const double* src = reinterpret_cast<const double*>(gz);
  double* dst = reinterpret_cast<double*>(lds);
  constexpr int n = 2 * kNZ + (EXPV == kExpTable ? kTabN : 0);
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

// Fixed-order xor butterfly over the 64 lanes (every lane ends with the same sum).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWaveSize);
  return v;
}

// Lane index 0..63, re-derived where it is used (v_mbcnt; volatile, so it is not kept live).
__device__ __forceinline__ int lane_id() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Y_B of one point by one wavefront.  fpy:231-267
//
// Nothing but the z-loop's own state is held in registers across the z-loop (which needs ~60
// of the 64 VGPRs at 8 waves/SIMD):
//   * the point's QuadSetup lives in the wave's LDS slot (~44 SGPRs otherwise); each pass
//     re-reads the fields it needs with broadcast ds_reads, through a slot index made opaque
//     per pass so that the reads are not hoisted back out of the y-loop;
//   * y, e^y and the weight are re-formed after the z-loop (same operations, same bits);
//   * the lane's running sum over its y-nodes sits in the slot (LZQ_ACC_LDS).
// Without this the kernel spilled ~200 B/lane to scratch around every z-loop.
// MODE (see lzq_sweep_grid_reuse): kYbDense computes every F(y_j) = sum_k omega_k 2^(c2_j g_k)
// itself (the headline); kYbTable computes them the same way and stores them to Fout instead of
// integrating; kYbReuse reads them from Fin (a table written by kYbTable for a point with the
// same y-grid and A/V kernel) and integrates.  The F values and the integration are the same
// operations in the same lane order in every mode, so Y_B is bit-identical.
enum YbMode { kYbDense = 0, kYbReuse = 1, kYbTable = 2 };

template <int YB, int EXPV, int MODE = kYbDense, int NZ = 0, typename Slot>
__device__ double yb_wave(Slot* slots, int w, const ZNode* __restrict__ zt, int nzp, const double* tab, int truncate,
                          const double* __restrict__ Fin = nullptr, double* __restrict__ Fout = nullptr) {
  static_assert(MODE == kYbDense || !LZQ_YFACT_EARLY, "table modes re-form the y-factors after the z-loop");
  if (slots[w].s.empty) return 0.0;
  // y-node counts are int32 (n_y of the C ABI): 32-bit loop bounds save the SGPRs that
  // would otherwise spill around the z-loop
  const int n = (int)__builtin_bit_cast(int64_t, uniform(__builtin_bit_cast(double, slots[w].s.n)));  // SGPR
  const int per_pass = kWaveSize * YB;
#if LZQ_ACC_LDS
  slots[w].acc[lane_id()] = 0.0;
#else
  double acc = 0.0;
#endif
  for (int base = 0; base < n; base += per_pass) {
    // only y, e^y and the weight stay live across the z-loop (LZQ_YFACT_EARLY=1: the 7
    // y-factors instead); the y-factors are formed after it
    double yv[YB], ey[YB], wt[YB];
#if LZQ_YFACT_EARLY
    YFactors fy[YB];
#endif
    double F[YB];
    if constexpr (MODE == kYbReuse) {
      const int lane = lane_id();
#pragma unroll
      for (int b = 0; b < YB; ++b) {
        const int j = base + b * kWaveSize + lane;
        F[b] = Fin[j < n ? j : n - 1];
      }
    } else {
      const int lane = lane_id();
      int wo = w;
      asm volatile("" : "+s"(wo));
      const QuadSetup& s = slots[wo].s;
      double c2[YB];
#pragma unroll
      for (int b = 0; b < YB; ++b) {
        const int j = base + b * kWaveSize + lane;
        const int jj = j < n ? j : n - 1;  // tail lanes recompute the last node with weight 0
        yv[b] = y_node(s, jj);
        ey[b] = exp_sc(pymax(pymin(yv[b], 50.0), -50.0));                          // fpy:161
        c2[b] = ((s.cneg * ey[b]) * kLog2E) * c2_scale<EXPV>();                 // fpy:163 c, log2 units
        wt[b] = j < n ? y_weight(s, jj, yv[b]) : 0.0;
#if LZQ_YFACT_EARLY
        fy[b] = y_factors(s, yv[b], ey[b], wt[b]);
#endif
      }
      zsum_dispatch<YB, EXPV, NZ>(zt, nzp, tab, c2, F, truncate);
      if constexpr (MODE == kYbTable) {
#pragma unroll
        for (int b = 0; b < YB; ++b) {
          const int j = base + b * kWaveSize + lane;
          if (j < n) Fout[j] = F[b];
        }
        continue;
      }
    }
    int wr = w;
    asm volatile("" : "+s"(wr));
    const int lane2 = lane_id();
    if (MODE == kYbReuse || (LZQ_Y_RECOMPUTE && !LZQ_YFACT_EARLY)) {
      const QuadSetup& sr = slots[wr].s;
#pragma unroll
      for (int b = 0; b < YB; ++b) {
        const int j = base + b * kWaveSize + lane2;
        const int jj = j < n ? j : n - 1;
        yv[b] = y_node(sr, jj);
        ey[b] = exp_sc(pymax(pymin(yv[b], 50.0), -50.0));
        wt[b] = j < n ? y_weight(sr, jj, yv[b]) : 0.0;
      }
    }
#if LZQ_ACC_LDS
    double acc = slots[wr].acc[lane2];
#endif
#pragma unroll
    for (int b = 0; b < YB; ++b) {
#if !LZQ_YFACT_EARLY
      const YFactors f = y_factors(slots[wr].s, yv[b], ey[b], wt[b]);
#else
      const YFactors& f = fy[b];
#endif
      acc = __builtin_fma(f.w, integrand_from(f, F[b]), acc);
    }
#if LZQ_ACC_LDS
    slots[wr].acc[lane2] = acc;
#endif
  }
#if LZQ_ACC_LDS
  return wave_sum(slots[w].acc[lane_id()]);
#else
  return wave_sum(acc);
#endif
}

// fpy:372-384 (fast path) + fpy:413-417, split around the quadrature: epilogue_pre forms every
// field that does not depend on Y_B before the z-loops (so the point record need not stay live
// across them), epilogue_finish adds Y_B with the same operations and rounding order.
struct EpiPre {
  lzq_yield o;  // Y_chi, rho_DM_kg_m3, P_used set
  int valid;    // regime is thermal / nonthermal
};

__device__ __forceinline__ EpiPre epilogue_pre(const lzq_point& pt, double P) {
  const double T_p = pt.T_p_GeV;
  const double T_hi = pt.T_max_over_Tp * T_p;
  double Ychi;
  if (pt.regime == LZQ_THERMAL) {
    Ychi = n_chi_eq(T_hi, pt.m_chi_GeV, pt.g_chi, pt.stats) / s_entropy(T_hi, pt.g_star_s);
  } else if (pt.regime == LZQ_NONTHERMAL) {
    if (pt.has_Y_chi_init) Ychi = pt.Y_chi_init;
    else if (pt.has_n_chi_at_Tp) Ychi = pt.n_chi_at_Tp_GeV3 / pymax(s_entropy(T_p, pt.g_star_s), 1e-300);
    else Ychi = 1.0e-12;
  } else {
    Ychi = __builtin_nan("");  // reference: UnboundLocalError
  }
  EpiPre e;
  const double nDM0 = Ychi * kS0M3;
  e.o.Y_B = 0.0;
  e.o.rho_B_kg_m3 = 0.0;
  e.o.DM_over_B = 0.0;
  e.o.Y_chi = Ychi;
  e.o.rho_DM_kg_m3 = nDM0 * (pt.m_chi_GeV * kGeVToKg);
  e.o.P_used = P;
  e.valid = pt.regime == LZQ_THERMAL || pt.regime == LZQ_NONTHERMAL;
  return e;
}

__device__ __forceinline__ lzq_yield epilogue_finish(const EpiPre& e, double YB) {
  lzq_yield o = e.o;
  const double nB0 = YB * kS0M3;
  o.Y_B = YB;
  o.rho_B_kg_m3 = nB0 * kMProtonKg;
  o.DM_over_B = o.rho_DM_kg_m3 / pymax(o.rho_B_kg_m3, 1e-300);
  if (!e.valid) o.Y_B = o.rho_B_kg_m3 = o.rho_DM_kg_m3 = o.DM_over_B = __builtin_nan("");
  return o;
}

// Per-wave LDS slot of the quadrature kernels (one point per wavefront).
struct WaveSlot {
  QuadSetup s;
  EpiPre e;
#if LZQ_ACC_LDS
  double acc[kWaveSize];  // per-lane running sums of yb_wave
#endif
};

// Park the (wave-uniform) setup and epilogue inputs in the wave's slot.  Lane 0 writes; LDS
// operations of one wavefront complete in order, the fence makes that formal for the compiler.
__device__ __forceinline__ void park(WaveSlot& slot, const QuadSetup& s, const EpiPre& e, int lane) {
  if (lane == 0) {
    slot.s = s;
    slot.e = e;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Quadrature of the parked point, then lane 0 stores its yields.
template <int YB, int EXPV, int NZ>
__device__ __forceinline__ void point_yields(WaveSlot* slots, int w, const ZNode* __restrict__ zt, int nzp,
                                             const double* tab, int lane, int truncate, lzq_yield* out) {
  const double Y_B = yb_wave<YB, EXPV, kYbDense, NZ>(slots, w, zt, nzp, tab, truncate);
  if (lane == 0) *out = epilogue_finish(slots[w].e, Y_B);
}

// ---------------------------------------------------------------------------------------
// point sources
// ---------------------------------------------------------------------------------------
struct GridSpec {
  int32_t n_axes;
  int32_t field[LZQ_MAX_AXES];
  int64_t n[LZQ_MAX_AXES];
  int64_t stride[LZQ_MAX_AXES];
  const double* values[LZQ_MAX_AXES];
  int64_t tstride[LZQ_MAX_AXES];  // lzq_sweep_grid_reuse: stride in the z-sum table index (0: axis not in it)
};

__device__ __forceinline__ void set_field(lzq_point& p, int32_t f, double v, double& delta, double& m_mix,
                                          double& dprime) {
  switch (f) {  // explicit switch: a runtime-indexed store would push the struct to scratch
    case LZQ_F_M_CHI: p.m_chi_GeV = v; break;
    case LZQ_F_G_CHI: p.g_chi = v; break;
    case LZQ_F_T_P: p.T_p_GeV = v; break;
    case LZQ_F_BETA_OVER_H: p.beta_over_H = v; break;
    case LZQ_F_V_W: p.v_w = v; break;
    case LZQ_F_I_P: p.I_p = v; break;
    case LZQ_F_G_STAR: p.g_star = v; break;
    case LZQ_F_G_STAR_S: p.g_star_s = v; break;
    case LZQ_F_P: p.P_chi_to_B = v; break;
    case LZQ_F_SIGMA_Y: p.source_shape_sigma_y = v; break;
    case LZQ_F_FLUX: p.incident_flux_scale = v; break;
    case LZQ_F_T_MAX_OVER_TP: p.T_max_over_Tp = v; break;
    case LZQ_F_T_MIN_OVER_TP: p.T_min_over_Tp = v; break;
    case LZQ_F_Y_CHI_INIT: p.Y_chi_init = v; p.has_Y_chi_init = 1; break;
    case LZQ_F_N_CHI_AT_TP: p.n_chi_at_Tp_GeV3 = v; p.has_n_chi_at_Tp = 1; break;
    case LZQ_F_DELTA_LZ: delta = v; break;
    case LZQ_F_M_MIX: m_mix = v; break;
    case LZQ_F_DPRIME: dprime = v; break;
    default: break;
  }
}

// Materialise grid point `idx`; returns P after the LZ closed form if an LZ axis is swept.
__device__ __forceinline__ double grid_point(const lzq_point& base, const GridSpec& g, int64_t idx, lzq_point& p) {
  p = base;
  double delta = __builtin_nan(""), m_mix = __builtin_nan(""), dprime = __builtin_nan("");
  bool has_delta = false, has_mix = false;
  for (int a = 0; a < g.n_axes; ++a) {
    int64_t c = (idx / g.stride[a]) % g.n[a];
    double v = g.values[a][c];
    set_field(p, g.field[a], v, delta, m_mix, dprime);
    has_delta |= g.field[a] == LZQ_F_DELTA_LZ;
    has_mix |= g.field[a] == LZQ_F_M_MIX;
  }
  if (has_mix) delta = m_mix * m_mix / (2.0 * pymax(p.v_w, 1e-12) * fabs(dprime));  // PAPER eq.(8)
  if (has_mix || has_delta) p.P_chi_to_B = p_closed_form(delta);                     // fpy:183-184
  return p.P_chi_to_B;
}

// ---------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------
// Block-level table staging of the dense kernels: the exp table into LDS, and with LZQ_ZLDS
// (an ablation build) the default grid's z nodes too; runtime grids (NZ = 0) keep theirs global.
#if LZQ_ZLDS
#define LZQ_STAGE_TABLES(NZ)                                   \
  __shared__ LdsTables lds;                                    \
  const double* tab;                                           \
  if constexpr (NZ == kNZ) {                                   \
    stage_tables<EXPV>(zt, &lds);                              \
    tab = lds.t;                                               \
    zt = lds.z;                                                \
  } else {                                                     \
    tab = stage_table<EXPV>(gtab, lds.t);                      \
  }
#else
#define LZQ_STAGE_TABLES(NZ)          \
  __shared__ double lds_tab[kTabN]; \
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
#endif

// NZ: kNZ for the reference's default z grid (the headline build, node count a compile-time
// constant), 0 for a runtime grid of nzp (padded) nodes -- see zsum_dispatch.
template <int YB, int EXPV, int NZ>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void yields_points_kernel(const lzq_point* __restrict__ pts, int64_t n,
                                                              int32_t n_y, const double* __restrict__ T_lo,
                                                              const double* __restrict__ T_hi,
                                                              const double* __restrict__ Pov,
                                                              const ZNode* __restrict__ zt, int32_t nzp,
                                                              const double* __restrict__ gtab,
                                                              lzq_yield* __restrict__ out, int truncate) {
  LZQ_STAGE_TABLES(NZ)
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  // wave index and point index formed from readfirstlane, so they live in SGPRs (a VGPR copy
  // of the 64-bit index was the kernel's only scratch spill)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t idx = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (idx >= n) return;  // wave-uniform
  {
    const lzq_point pt = pts[idx];
    const double P = Pov ? Pov[idx] : pt.P_chi_to_B;
    const double tlo = T_lo ? T_lo[idx] : pt.T_min_over_Tp * pt.T_p_GeV;  // fpy:369
    const double thi = T_hi ? T_hi[idx] : pt.T_max_over_Tp * pt.T_p_GeV;  // fpy:368
    park(slots[w], quad_setup(pt, P, tlo, thi, n_y), epilogue_pre(pt, P), lane);
  }
  point_yields<YB, EXPV, NZ>(slots, w, zt, nzp, tab, lane, truncate, out + idx);
}

template <int YB, int EXPV, int NZ>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void yields_grid_kernel(lzq_point base, GridSpec grid, int64_t start,
                                                            int64_t count, int32_t n_y,
                                                            const double* __restrict__ Pov,
                                                            const ZNode* __restrict__ zt, int32_t nzp,
                                                            const double* __restrict__ gtab,
                                                            lzq_yield* __restrict__ out, int truncate) {
  LZQ_STAGE_TABLES(NZ)
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR (see yields_points_kernel)
  const int64_t local = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (local >= count) return;
  {
    lzq_point pt;
    const double Pg = grid_point(base, grid, start + local, pt);
    const double P = Pov ? Pov[local] : Pg;
    park(slots[w], quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y),
         epilogue_pre(pt, P), lane);
  }
  point_yields<YB, EXPV, NZ>(slots, w, zt, nzp, tab, lane, truncate, out + local);
}

// ---------------------------------------------------------------------------------------
// lzq_sweep_grid_reuse: the z-sums F(y_j) depend on a grid point only through the fields of
// quad_setup's y-grid and c (I_p, beta/H, T_p, T_min/T_p, T_max/T_p, n_y).  The table kernel
// computes them once per combination of the grid's values of those fields (one wavefront per
// table, kYbTable: the dense kernel's passes, F stored instead of integrated); the reuse kernel
// then integrates every point from its table (kYbReuse).  Same operations, same lane order: Y_B
// is bit-identical to lzq_sweep_grid.  Table t: kTabHdr header doubles (the y-grid and c of the
// QuadSetup it was made for, and the z grid's (nz, z_max); a point whose own setup or grid
// differs gets NaN yields, never a wrong table), then its F values.
constexpr int kTabHdr = 6;
static_assert(kTabHdr == LZQ_REUSE_TABLE_HEADER, "include/lzq.h");

// The z grid a table is made for, as its header stores it.
struct ZKey {
  double nz, z_max;
};

__device__ __forceinline__ int64_t table_of(const GridSpec& g, int64_t idx) {
  int64_t t = 0;
  for (int a = 0; a < g.n_axes; ++a) t += ((idx / g.stride[a]) % g.n[a]) * g.tstride[a];
  return t;
}

// flat grid index of table t's representative (every other axis at its first value)
__device__ __forceinline__ int64_t table_rep(const GridSpec& g, int64_t t) {
  int64_t idx = 0;
  for (int a = 0; a < g.n_axes; ++a)
    if (g.tstride[a]) idx += ((t / g.tstride[a]) % g.n[a]) * g.stride[a];
  return idx;
}

// Table t of one wavefront: header + the F values of the point parked in the wave's slot.
template <int EXPV>
__device__ __forceinline__ void ztable_wave(WaveSlot* slots, int w, int lane, const QuadSetup& qs, const EpiPre& e,
                                            const ZNode* __restrict__ zt, int nzp, ZKey zk, const double* tab,
                                            int truncate, double* F) {
  if (lane == 0) {
    F[0] = qs.y_lo;
    F[1] = qs.y_hi;
    F[2] = (double)qs.n;
    F[3] = qs.cneg;
    F[4] = zk.nz;
    F[5] = zk.z_max;
  }
  park(slots[w], qs, e, lane);
  yb_wave<kYB, EXPV, kYbTable>(slots, w, zt, nzp, tab, truncate, nullptr, F + kTabHdr);
}

// One point integrated from its table F (NaN yields if the table was made for another y-grid).
__device__ __forceinline__ void reuse_wave(WaveSlot* slots, int w, int lane, const QuadSetup& qs, const EpiPre& e,
                                           ZKey zk, const double* __restrict__ F, lzq_yield* out) {
  // match is wave-uniform: every lane formed the same setup
  const bool match = qs.empty || (F[0] == qs.y_lo && F[1] == qs.y_hi && F[2] == (double)qs.n && F[3] == qs.cneg &&
                                  F[4] == zk.nz && F[5] == zk.z_max);
  park(slots[w], qs, e, lane);
  const double Y_B = match ? yb_wave<kYB, kExpTable, kYbReuse>(slots, w, nullptr, 0, nullptr, 0, F + kTabHdr) : 0.0;
  if (lane == 0) {
    lzq_yield o = epilogue_finish(slots[w].e, Y_B);
    if (!match) o.Y_B = o.rho_B_kg_m3 = o.DM_over_B = __builtin_nan("");
    *out = o;
  }
}

template <int EXPV>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void grid_ztable_kernel(lzq_point base, GridSpec grid,
                                                                          int64_t n_tab, int32_t n_y, int64_t tstride,
                                                                          const ZNode* __restrict__ zt, int32_t nzp,
                                                                          ZKey zk, const double* __restrict__ gtab,
                                                                          double* __restrict__ Fw, int truncate) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (t >= n_tab) return;
  lzq_point pt;
  const double P = grid_point(base, grid, table_rep(grid, t), pt);
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  ztable_wave<EXPV>(slots, w, lane, qs, epilogue_pre(pt, P), zt, nzp, zk, tab, truncate, Fw + t * tstride);
}

#ifndef LZQ_REUSE_MIN_WAVES
#define LZQ_REUSE_MIN_WAVES 8  // 8 waves/SIMD (SGPRs capped, a few spilled to VGPR lanes): +12% over 7 (tools/ablate_builds.py ... reuse)
#endif
__global__ __launch_bounds__(kBlock, LZQ_REUSE_MIN_WAVES) void grid_reuse_kernel(lzq_point base, GridSpec grid, int64_t start,
                                                           int64_t count, int32_t n_y,
                                                           const double* __restrict__ Pov, ZKey zk,
                                                           const double* __restrict__ Fw, int64_t tstride,
                                                           lzq_yield* __restrict__ out) {
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t local = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (local >= count) return;
  lzq_point pt;
  const double Pg = grid_point(base, grid, start + local, pt);
  const double P = Pov ? Pov[local] : Pg;
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  reuse_wave(slots, w, lane, qs, epilogue_pre(pt, P), zk, Fw + table_of(grid, start + local) * tstride, out + local);
}

// The same for explicit points (lzq_yields_batch_reuse): table t is made for point reps[t];
// point i integrates from table tidx[i].
template <int EXPV>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void points_ztable_kernel(const lzq_point* __restrict__ pts,
                                                                            const int64_t* __restrict__ reps,
                                                                            int64_t n_tab, int32_t n_y, int64_t tstride,
                                                                            const ZNode* __restrict__ zt, int32_t nzp,
                                                                            ZKey zk, const double* __restrict__ gtab,
                                                                            double* __restrict__ Fw, int truncate) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (t >= n_tab) return;
  const lzq_point pt = pts[reps[t]];
  const double P = pt.P_chi_to_B;
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  ztable_wave<EXPV>(slots, w, lane, qs, epilogue_pre(pt, P), zt, nzp, zk, tab, truncate, Fw + t * tstride);
}

__global__ __launch_bounds__(kBlock, LZQ_REUSE_MIN_WAVES) void points_reuse_kernel(const lzq_point* __restrict__ pts, int64_t n,
                                                             int32_t n_y, const double* __restrict__ Pov, ZKey zk,
                                                             const int32_t* __restrict__ tidx,
                                                             const double* __restrict__ Fw, int64_t tstride,
                                                             lzq_yield* __restrict__ out) {
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t idx = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (idx >= n) return;
  const lzq_point pt = pts[idx];
  const double P = Pov ? Pov[idx] : pt.P_chi_to_B;
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  reuse_wave(slots, w, lane, qs, epilogue_pre(pt, P), zk, Fw + (int64_t)tidx[idx] * tstride, out + idx);
}

// fpy:158-165, one lane per y value
template <int EXPV>
__global__ __launch_bounds__(kBlock) void aov_kernel(lzq_point pt, const double* __restrict__ ys, int64_t n,
                                                    const ZNode* __restrict__ zt, int32_t nzp,
                                                    const double* __restrict__ gtab, double* __restrict__ out) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = i < n;
  const double y = live ? ys[i] : 0.0;
  QuadSetup s = quad_setup(pt, pt.P_chi_to_B, 1.0, 1.0, LZQ_NY_MIN);
  double expy = exp_sc(pymax(pymin(y, 50.0), -50.0));
  double c2[1] = {((s.cneg * expy) * kLog2E) * c2_scale<EXPV>()}, F[1];
  zsum_dispatch<1, EXPV>(zt, nzp, tab, c2, F);
  if (live) out[i] = (y > 50.0) ? 0.0 : (s.pref0 * expy) * F[0];
}

// fpy:207-212 build_tables, first half: A/V at the nt knots Ts = linspace(T_lo, T_hi, nt)
// (main() uses n = 800) of main()'s window (fpy:368-369) or the given one, np.maximum(Av, 0),
// one wavefront per point (lane i takes knots i, i+64, ...), into the point's 4 nt doubles.  The
// spline is fitted by lzq_ode.hip's ode_spline_kernel.
template <int EXPV>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void ode_aov_table_kernel(const lzq_point* __restrict__ pts,
                                                                               int64_t n, int32_t nt,
                                                                               const ZNode* __restrict__ zt, int32_t nzp,
                                                                               const double* __restrict__ gtab,
                                                                               const double* __restrict__ Tlo,
                                                                               const double* __restrict__ Thi,
                                                                               double* __restrict__ ws, int truncate) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int64_t idx = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (idx >= n) return;  // wave-uniform
  const lzq_point pt = pts[idx];
  // every per-point value is wave-uniform: pinned in SGPRs (readfirstlane) so that the z-loop
  // keeps its VGPRs (without this 12 VGPRs spilled around every z-loop)
  const double Tp = uniform(pt.T_p_GeV), B = uniform(pt.beta_over_H);
  const double T_lo = uniform(Tlo ? Tlo[idx] : pt.T_min_over_Tp * Tp);
  const double T_hi = uniform(Thi ? Thi[idx] : pt.T_max_over_Tp * Tp);
  const double stepT = uniform((T_hi - T_lo) / (double)(nt - 1));
  const QuadSetup s = quad_setup(pt, 0.0, 1.0, 1.0, LZQ_NY_MIN);  // only pref0 / cneg are used
  const double pref0 = uniform(s.pref0), cneg = uniform(s.cneg);
  const int64_t ws_pt = 4 * (int64_t)nt;
  double* w = ws + idx * ws_pt;
  for (int base = 0; base < nt; base += kWaveSize) {
    const int i = base + lane;
    const int ii = i < nt ? i : nt - 1;
    const double T = linspace_at(T_lo, T_hi, stepT, ii, nt);
    const double y = y_of_T(T, Tp, B);
    const double expy = exp_sc(pymax(pymin(y, 50.0), -50.0));  // fpy:161
    double c2[1] = {((cneg * expy) * kLog2E) * c2_scale<EXPV>()}, F[1];
    zsum_dispatch<1, EXPV>(zt, nzp, tab, c2, F, truncate);
    const double Av = (y > 50.0) ? 0.0 : (pref0 * expy) * F[0];  // fpy:159-165
    if (i < nt) w[i < nt - 1 ? 4 * i + 3 : ws_pt - 1] = pymax(Av, 0.0);
  }
}

// fpy:222-223 (J_chi_flux fpy:122-123), one lane per T
__global__ __launch_bounds__(kBlock) void jchi_kernel(lzq_point pt, const double* __restrict__ Ts, int64_t n,
                                                     double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double T = Ts[i];
  out[i] = pt.incident_flux_scale *
           (0.25 * n_chi_eq(T, pt.m_chi_GeV, pt.g_chi, pt.stats) * vbar_chi(T, pt.m_chi_GeV));
}

// fpy:183-184
__global__ __launch_bounds__(kBlock) void p_closed_form_kernel(const double* __restrict__ lam, int64_t n,
                                                              double* __restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) P[i] = p_closed_form(lam[i]);
}

}  // namespace lzq

// =========================================================================================
// host side: z tables, error plumbing, C ABI
// =========================================================================================
namespace {

thread_local char g_err[512] = "";
std::mutex g_mu;
constexpr int kMaxDevices = 64;
// per device: the default grid's [LZQ_NZ] ZNode followed by the kTabN-entry exp table
lzq::ZNode* g_dev_tab[kMaxDevices] = {nullptr};
uint64_t g_exp2tab[lzq::kTabN];  // lzq::tab_entry_bits layout
bool g_exp_ready = false;
int g_exp_variant = lzq::kExpTable;
int g_truncate = 0;  // LZQ_TUNE_TRUNCATE

const double* exp_table(int dev) { return reinterpret_cast<const double*>(g_dev_tab[dev] + LZQ_NZ); }

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define LZQ_HIP(call)                                                                         \
  do {                                                                                        \
    hipError_t e_ = (call);                                                                   \
    if (e_ != hipSuccess) return fail(LZQ_EHIP, "%s: %s", #call, hipGetErrorString(e_));      \
  } while (0)

// One z grid of AoverVKernel(..., z_max, nz) (fpy:141-156) on the host: z = linspace(0, z_max, nz),
// the verbatim cancelling gamma4, and the trapezoid weights omega_k = z_k^2 e^{-z_k} (d_{k-1} +
// d_k)/2 with d = diff(z) (np.trapezoid, fpy:164, as a weighted sum).  libm exp/pow; built once
// per grid.
struct HostZGrid {
  int32_t nz = 0;
  double z_max = 0.0;
  std::vector<double> z, g4, omega;
  bool monotone = true;  // g4 non-decreasing (the truncation's binary search needs it)
};

int build_ztable(int32_t nz, double z_max, HostZGrid& h) {
  if (nz < 0) return fail(LZQ_EINVAL, "Number of samples, %d, must be non-negative.", nz);  // np.linspace
  if (nz > LZQ_NZ_MAX) return fail(LZQ_EINVAL, "nz = %d exceeds LZQ_NZ_MAX (%d)", nz, LZQ_NZ_MAX);
  if (!(z_max >= 0.0) || !isfinite(z_max))
    return fail(LZQ_EINVAL, "z_max = %g: the z grid must be finite and >= 0 (fpy:154)", z_max);
  h.nz = nz;
  h.z_max = z_max;
  h.z.assign(nz, 0.0);
  h.g4.assign(nz, 0.0);
  h.omega.assign(nz, 0.0);
  if (nz == 1) h.z[0] = 0.0;  // np.linspace(0, z_max, 1) = [0.]
  if (nz >= 2) {
    const double step = (z_max - 0.0) / (double)(nz - 1);
    for (int k = 0; k < nz; ++k)  // np.linspace (numpy's step == 0 branch when z_max underflows the step)
      h.z[k] = (k == nz - 1) ? z_max : (step == 0.0 ? ((double)k / (double)(nz - 1)) * z_max : (double)k * step) + 0.0;
  }
  std::vector<double> w(nz);
  for (int k = 0; k < nz; ++k) {
    const double z = h.z[k];
    const double ez = exp(-z);
    const double zz = z * z;
    h.g4[k] = 6.0 - ez * (((pow(z, 3.0) + 3.0 * zz) + 6.0 * z) + 6.0);
    w[k] = zz * ez;
    // the reference's cancelling form rounds below 0 only on grids far finer than its default
    // (z_1 < ~3e-4): exp of a positive argument there, which the inner loop does not evaluate
    if (!(h.g4[k] >= 0.0))
      return fail(LZQ_EINVAL, "gamma4[%d] = %g < 0 (nz = %d, z_max = %g): the cancelling form of fpy:156 rounds "
                  "below 0 on this grid", k, h.g4[k], nz, z_max);
    if (k > 0 && h.g4[k] < h.g4[k - 1]) h.monotone = false;
  }
  for (int k = 0; k < nz; ++k) {
    const double dl = k > 0 ? h.z[k] - h.z[k - 1] : 0.0;
    const double dr = k + 1 < nz ? h.z[k + 1] - h.z[k] : 0.0;
    h.omega[k] = w[k] * (0.5 * (dl + dr));
  }
  // zsum_dispatch: a lane is dead (zeroed) iff c2N g4_1 <= -1077 N, so a live lane has
  // |u| < 1077 N g4_max / g4_1; nodes beyond 2^51 are clamped and round away while |u| < 2^200
  if (nz >= 2 && z_max > 0.0) {
    const double g1 = h.g4[1], gmax = h.g4[nz - 1];
    if (!(g1 > 0.0) || !((double)lzq::kTabN * 1077.0 * gmax / g1 < 0x1p200))
      return fail(LZQ_EINVAL, "z grid (nz = %d, z_max = %g): gamma4[1] = %g breaks the inner loop's reduction", nz,
                  z_max, g1);
  }
  return LZQ_OK;
}

const HostZGrid& default_host_grid() {
  static HostZGrid h;
  static int rc = build_ztable(LZQ_NZ, LZQ_Z_MAX, h);
  (void)rc;  // the default grid always builds (tests/test_capi.py)
  return h;
}

void build_exp_table() {
  if (g_exp_ready) return;
  // T[j] = 2^(j/N): x87 long double exp2 (64-bit mantissa) rounded once to double, stored
  // with the pre-biased high word of lzq::tab_entry_bits
  for (int j = 0; j < lzq::kTabN; ++j) g_exp2tab[j] = lzq::tab_entry_bits(lzq::tab_exact(j), j);
  g_exp_ready = true;
}

// Device image of a grid: nzp >= max(nz, kKUnroll) nodes, a multiple of the unroll; the padding
// repeats the last g4 with omega' = 0 (an exact +0 per node).  Weights carry 2^-512 (the exp
// table's T' carries 2^+512, lzq_exp2.h).
int32_t padded_nodes(int32_t nz) {
  const int32_t u = lzq::kKUnroll;
  const int32_t n = nz > u ? nz : u;
  return (n + u - 1) / u * u;
}

void device_nodes(const HostZGrid& h, lzq::ZNode* dst) {
  const int32_t nzp = padded_nodes(h.nz);
  const double glast = h.nz > 0 ? h.g4[h.nz - 1] : 0.0;
  for (int k = 0; k < nzp; ++k)
    dst[k] = k < h.nz ? lzq::ZNode{h.g4[k], ldexp(h.omega[k], -lzq::kOmegaBias)} : lzq::ZNode{glast, 0.0};
}

int ensure_device(int* dev_out) {
  int dev = 0;
  LZQ_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return fail(LZQ_ENODEVICE, "device %d out of range", dev);
  if (dev_out) *dev_out = dev;
  if (g_dev_tab[dev]) return LZQ_OK;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_dev_tab[dev]) return LZQ_OK;
  const HostZGrid& h = default_host_grid();
  if ((int)h.g4.size() != LZQ_NZ) return fail(LZQ_EINVAL, "default z grid failed to build");
  build_exp_table();
  static_assert(sizeof(lzq::ZNode) == 2 * sizeof(double), "ZNode layout");
  static_assert(LZQ_NZ % lzq::kKUnroll == 0, "the default grid needs no padding");
  std::vector<lzq::ZNode> host(LZQ_NZ + lzq::kTabN / 2);
  device_nodes(h, host.data());
  memcpy(&host[LZQ_NZ], g_exp2tab, sizeof(g_exp2tab));
  const size_t bytes = host.size() * sizeof(lzq::ZNode);
  lzq::ZNode* d = nullptr;
  LZQ_HIP(hipMalloc(&d, bytes));
  LZQ_HIP(hipMemcpy(d, host.data(), bytes, hipMemcpyHostToDevice));
  g_dev_tab[dev] = d;
  return LZQ_OK;
}

// A z grid on a device, as the kernels take it.
struct DevZGrid {
  const lzq::ZNode* zt = nullptr;
  int32_t nzp = 0;
  bool is_default = false;  // the compile-time LZQ_NZ kernels apply
  bool monotone = true;
  lzq::ZKey key{0.0, 0.0};
};

struct ZGridEntry {
  int dev;
  int32_t nz;
  uint64_t zbits;
  lzq::ZNode* d;
  int32_t nzp;
  bool monotone;
};
std::vector<ZGridEntry> g_zgrids;  // runtime grids, uploaded on first use (guarded by g_mu)

bool is_default_grid(int32_t nz, double z_max) { return nz == LZQ_NZ && z_max == LZQ_Z_MAX; }

// The device tables of (nz, z_max) on the current device: the default grid's (lzq_init), or a
// runtime grid's, built and uploaded once per (device, nz, z_max) (a synchronous copy: call
// lzq_zgrid_init before capturing launches into a graph).
int zgrid_for(int32_t nz, double z_max, DevZGrid& g, int* dev_out) {
  int dev, rc = ensure_device(&dev);
  if (rc) return rc;
  if (dev_out) *dev_out = dev;
  g.key = lzq::ZKey{(double)nz, z_max};
  if (is_default_grid(nz, z_max)) {
    g.zt = g_dev_tab[dev];
    g.nzp = LZQ_NZ;
    g.is_default = true;
    g.monotone = default_host_grid().monotone;
    return LZQ_OK;
  }
  const uint64_t zb = __builtin_bit_cast(uint64_t, z_max);
  std::lock_guard<std::mutex> lk(g_mu);
  for (const ZGridEntry& e : g_zgrids)
    if (e.dev == dev && e.nz == nz && e.zbits == zb) {
      g.zt = e.d;
      g.nzp = e.nzp;
      g.monotone = e.monotone;
      return LZQ_OK;
    }
  HostZGrid h;
  rc = build_ztable(nz, z_max, h);
  if (rc) return rc;
  const int32_t nzp = padded_nodes(nz);
  std::vector<lzq::ZNode> host(nzp);
  device_nodes(h, host.data());
  lzq::ZNode* d = nullptr;
  LZQ_HIP(hipMalloc(&d, host.size() * sizeof(lzq::ZNode)));
  LZQ_HIP(hipMemcpy(d, host.data(), host.size() * sizeof(lzq::ZNode), hipMemcpyHostToDevice));
  g_zgrids.push_back(ZGridEntry{dev, nz, zb, d, nzp, h.monotone});
  g.zt = d;
  g.nzp = nzp;
  g.monotone = h.monotone;
  return LZQ_OK;
}

int64_t blocks_for(int64_t n, int64_t per_block) { return (n + per_block - 1) / per_block; }

constexpr int64_t kMaxGrid = 2147483647LL;

}  // namespace

int lzq_set_error(int code, const char* msg) { return fail(code, "%s", msg); }

int lzq::launch_ode_aov_tables(const lzq_point* d_points, int64_t n, const double* d_T_lo, const double* d_T_hi,
                               int32_t nt, int32_t nz, double z_max, double* d_work, hipStream_t stream) {
  if (n == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  const int64_t nb = blocks_for(n, lzq::kWavesPerBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_ode_tables: n too large");
  // The ODE tables always use the exact-underflow truncation of the z-sums: it is bit-identical
  // to the dense sum (tests/test_gpu_parity.py::test_truncation_is_bit_identical) and this path
  // is not the dense headline benchmark, so there is nothing to keep dense for.
  const int truncate = g.monotone ? 1 : 0;
  if (g_exp_variant == lzq::kExpTable)
    hipLaunchKernelGGL(lzq::ode_aov_table_kernel<lzq::kExpTable>, dim3((unsigned)nb), dim3(lzq::kBlock), 0, stream,
                       d_points, n, nt, g.zt, g.nzp, exp_table(dev), d_T_lo, d_T_hi, d_work, truncate);
  else
    hipLaunchKernelGGL(lzq::ode_aov_table_kernel<lzq::kExpPoly11>, dim3((unsigned)nb), dim3(lzq::kBlock), 0, stream,
                       d_points, n, nt, g.zt, g.nzp, exp_table(dev), d_T_lo, d_T_hi, d_work, truncate);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

extern "C" {

int lzq_abi_version(void) { return LZQ_ABI_VERSION; }

const char* lzq_last_error(void) { return g_err; }

int lzq_init(int device) { return lzq_zgrid_init(device, LZQ_NZ, LZQ_Z_MAX); }

int lzq_zgrid_init(int device, int32_t nz, double z_max) {
  int cur = 0;
  LZQ_HIP(hipGetDevice(&cur));
  if (device != cur) LZQ_HIP(hipSetDevice(device));
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, nullptr);
  if (device != cur) {
    hipError_t e = hipSetDevice(cur);
    if (e != hipSuccess && rc == LZQ_OK) return fail(LZQ_EHIP, "hipSetDevice: %s", hipGetErrorString(e));
  }
  return rc;
}

int lzq_tune(int32_t key, int32_t value) {
  if (key == LZQ_TUNE_EXP) {
    if (value != LZQ_EXP_POLY11 && value != LZQ_EXP_TABLE)
      return fail(LZQ_EINVAL, "lzq_tune: unknown exp variant %d", value);
    int prev = g_exp_variant;
    g_exp_variant = value;
    return prev;
  }
  if (key == LZQ_TUNE_TRUNCATE) {
    if (value != 0 && value != 1) return fail(LZQ_EINVAL, "lzq_tune: truncate must be 0 or 1, got %d", value);
    int prev = g_truncate;
    g_truncate = value;
    return prev;
  }
  if (key == LZQ_TUNE_ODE_LAUNCH_STEPS) {
    if (value < 6 || value > 40) return fail(LZQ_EINVAL, "lzq_tune: ode launch steps log2 must be in [6, 40], got %d", value);
    int prev = lzq::g_ode_launch_log2;
    lzq::g_ode_launch_log2 = value;
    return prev;
  }
  if (key == LZQ_TUNE_PROFILE_FLAT) {
    if (value != 0 && value != 1) return fail(LZQ_EINVAL, "lzq_tune: profile_flat must be 0 or 1, got %d", value);
    int prev = lzq::g_profile_flat;
    lzq::g_profile_flat = value;
    return prev;
  }
  if (key == LZQ_TUNE_ODE_COOP) {
    if (value != 0 && value != 1) return fail(LZQ_EINVAL, "lzq_tune: ode_coop must be 0 or 1, got %d", value);
    int prev = lzq::g_ode_coop;
    lzq::g_ode_coop = value;
    return prev;
  }
  return fail(LZQ_EINVAL, "lzq_tune: unknown key %d", key);
}

int lzq_ztables(int32_t nz, double z_max, double* z, double* gamma4, double* omega) {
  HostZGrid h;
  int rc;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    rc = build_ztable(nz, z_max, h);
  }
  if (rc) return rc;
  const size_t bytes = sizeof(double) * (size_t)nz;
  if (z && nz) memcpy(z, h.z.data(), bytes);
  if (gamma4 && nz) memcpy(gamma4, h.g4.data(), bytes);
  if (omega && nz) memcpy(omega, h.omega.data(), bytes);
  return LZQ_OK;
}

int lzq_aov_batch(const lzq_point* pt, const double* d_y, int64_t n, int32_t nz, double z_max, double* d_out,
                  void* stream) {
  if (!pt || n < 0 || (n > 0 && (!d_y || !d_out))) return fail(LZQ_EINVAL, "lzq_aov_batch: bad arguments");
  if (n == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  int64_t nb = blocks_for(n, lzq::kBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_aov_batch: n too large");
  if (g_exp_variant == lzq::kExpTable)
    hipLaunchKernelGGL(lzq::aov_kernel<lzq::kExpTable>, dim3((unsigned)nb), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, *pt, d_y, n, g.zt, g.nzp, exp_table(dev), d_out);
  else
    hipLaunchKernelGGL(lzq::aov_kernel<lzq::kExpPoly11>, dim3((unsigned)nb), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, *pt, d_y, n, g.zt, g.nzp, exp_table(dev), d_out);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int lzq_jchi_batch(const lzq_point* pt, const double* d_T, int64_t n, double* d_out, void* stream) {
  if (!pt || n < 0 || (n > 0 && (!d_T || !d_out))) return fail(LZQ_EINVAL, "lzq_jchi_batch: bad arguments");
  if (n == 0) return LZQ_OK;
  int64_t nb = blocks_for(n, lzq::kBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_jchi_batch: n too large");
  hipLaunchKernelGGL(lzq::jchi_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream, *pt, d_T, n,
                     d_out);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int lzq_yields_batch(const lzq_point* d_points, int64_t n, int32_t n_y, int32_t nz, double z_max,
                     const double* d_T_lo, const double* d_T_hi, const double* d_P, lzq_yield* d_out, void* stream) {
  if (n < 0 || (n > 0 && (!d_points || !d_out))) return fail(LZQ_EINVAL, "lzq_yields_batch: bad arguments");
  if ((d_T_lo == nullptr) != (d_T_hi == nullptr))
    return fail(LZQ_EINVAL, "lzq_yields_batch: T_lo and T_hi must both be given or both be NULL");
  if (n == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  int64_t nb = blocks_for(n, lzq::kWavesPerBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_yields_batch: n too large");
  const int trunc = g.monotone ? g_truncate : 0;
  const hipStream_t s = (hipStream_t)stream;
#define LZQ_POINTS(EXPV, NZ)                                                                                        \
  hipLaunchKernelGGL((lzq::yields_points_kernel<lzq::kYB, EXPV, NZ>), dim3((unsigned)nb), dim3(lzq::kBlock), 0, s, \
                     d_points, n, n_y, d_T_lo, d_T_hi, d_P, g.zt, g.nzp, exp_table(dev), d_out, trunc)
  if (g_exp_variant == lzq::kExpTable) {
    if (g.is_default) LZQ_POINTS(lzq::kExpTable, lzq::kNZ);
    else LZQ_POINTS(lzq::kExpTable, 0);
  } else {
    if (g.is_default) LZQ_POINTS(lzq::kExpPoly11, lzq::kNZ);
    else LZQ_POINTS(lzq::kExpPoly11, 0);
  }
#undef LZQ_POINTS
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

namespace {
// lzq_sweep_grid's argument checks and GridSpec (shared with lzq_sweep_grid_reuse)
int make_grid(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start, int64_t count,
              const lzq_yield* d_out, const char* who, lzq::GridSpec& g) {
  if (!base || n_axes < 0 || n_axes > LZQ_MAX_AXES || (n_axes > 0 && !axes) || start < 0 || count < 0 ||
      (count > 0 && !d_out))
    return fail(LZQ_EINVAL, "%s: bad arguments", who);
  memset(&g, 0, sizeof(g));
  g.n_axes = n_axes;
  int64_t total = 1;
  bool mix = false, dpr = false;
  for (int a = n_axes - 1; a >= 0; --a) {
    const int32_t f = axes[a].field;
    if (!((f >= 0 && f <= 14) || f == LZQ_F_DELTA_LZ || f == LZQ_F_M_MIX || f == LZQ_F_DPRIME))
      return fail(LZQ_EINVAL, "%s: axis %d has unknown field %d", who, a, f);
    if (axes[a].n <= 0 || !axes[a].values) return fail(LZQ_EINVAL, "%s: axis %d is empty", who, a);
    mix |= f == LZQ_F_M_MIX;
    dpr |= f == LZQ_F_DPRIME;
    g.field[a] = f;
    g.n[a] = axes[a].n;
    g.values[a] = axes[a].values;
    g.stride[a] = total;
    if (total > INT64_MAX / axes[a].n) return fail(LZQ_EINVAL, "%s: grid too large", who);
    total *= axes[a].n;
  }
  if (mix != dpr) return fail(LZQ_EINVAL, "%s: LZQ_F_M_MIX and LZQ_F_DPRIME must be swept together", who);
  if (start > total || count > total - start)
    return fail(LZQ_EINVAL, "%s: range [%lld, %lld) outside grid of %lld points", who, (long long)start,
                (long long)(start + count), (long long)total);
  if (base->regime != LZQ_THERMAL && base->regime != LZQ_NONTHERMAL)
    return fail(LZQ_EUNSUPPORTED, "%s: regime must be thermal or nonthermal (fpy:376-384)", who);
  return LZQ_OK;
}

// the fields quad_setup's y-grid and c depend on (lzq_sweep_grid_reuse's table axes)
bool ztable_field(int32_t f) {
  return f == LZQ_F_I_P || f == LZQ_F_BETA_OVER_H || f == LZQ_F_T_P || f == LZQ_F_T_MIN_OVER_TP ||
         f == LZQ_F_T_MAX_OVER_TP;
}

int64_t ztable_count(const lzq::GridSpec& g) {
  int64_t n = 1;
  for (int a = 0; a < g.n_axes; ++a)
    if (ztable_field(g.field[a])) n *= g.n[a];
  return n;
}
}  // namespace

int lzq_sweep_grid(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start, int64_t count,
                   int32_t n_y, int32_t nz, double z_max, const double* d_P, lzq_yield* d_out, void* stream) {
  lzq::GridSpec gs;
  int rc = make_grid(base, axes, n_axes, start, count, d_out, "lzq_sweep_grid", gs);
  if (rc) return rc;
  if (count == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  int64_t nb = blocks_for(count, lzq::kWavesPerBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_sweep_grid: count too large for one launch");
  const int trunc = g.monotone ? g_truncate : 0;
  const hipStream_t s = (hipStream_t)stream;
#define LZQ_GRID(EXPV, NZ)                                                                                         \
  hipLaunchKernelGGL((lzq::yields_grid_kernel<lzq::kYB, EXPV, NZ>), dim3((unsigned)nb), dim3(lzq::kBlock), 0, s,  \
                     *base, gs, start, count, n_y, d_P, g.zt, g.nzp, exp_table(dev), d_out, trunc)
  if (g_exp_variant == lzq::kExpTable) {
    if (g.is_default) LZQ_GRID(lzq::kExpTable, lzq::kNZ);
    else LZQ_GRID(lzq::kExpTable, 0);
  } else {
    if (g.is_default) LZQ_GRID(lzq::kExpPoly11, lzq::kNZ);
    else LZQ_GRID(lzq::kExpPoly11, 0);
  }
#undef LZQ_GRID
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int lzq_yields_batch_reuse(const lzq_point* d_points, int64_t n, int32_t n_y, int32_t nz, double z_max,
                           const double* d_P, const int64_t* d_rep, const int32_t* d_table_index, int64_t n_tables,
                           double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream) {
  if (n < 0 || n_tables < 0 || (n > 0 && (!d_points || !d_out || !d_rep || !d_table_index || n_tables == 0)))
    return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: bad arguments");
  const int64_t stride = (n_y > LZQ_NY_MIN ? n_y : LZQ_NY_MIN) + lzq::kTabHdr;
  if (n_tables > INT64_MAX / stride) return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: too many tables");
  if (n > 0 && (!d_work || work_doubles < n_tables * stride))
    return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: workspace of %lld doubles < %lld needed", (long long)work_doubles,
                (long long)(n_tables * stride));
  if (n == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  const int64_t nbt = blocks_for(n_tables, lzq::kWavesPerBlock), nb = blocks_for(n, lzq::kWavesPerBlock);
  if (nbt > kMaxGrid || nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: too large for one launch");
  const int trunc = g.monotone ? 1 : 0;  // bit-identical to the dense sums either way
  if (g_exp_variant == lzq::kExpTable)
    hipLaunchKernelGGL((lzq::points_ztable_kernel<lzq::kExpTable>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, d_points, d_rep, n_tables, n_y, stride, g.zt, g.nzp, g.key,
                       exp_table(dev), d_work, trunc);
  else
    hipLaunchKernelGGL((lzq::points_ztable_kernel<lzq::kExpPoly11>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, d_points, d_rep, n_tables, n_y, stride, g.zt, g.nzp, g.key,
                       exp_table(dev), d_work, trunc);
  LZQ_HIP(hipGetLastError());
  hipLaunchKernelGGL(lzq::points_reuse_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream, d_points,
                     n, n_y, d_P, g.key, d_table_index, d_work, stride, d_out);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int64_t lzq_sweep_grid_reuse_workspace(const lzq_axis* axes, int32_t n_axes, int32_t n_y) {
  if (n_axes < 0 || n_axes > LZQ_MAX_AXES || (n_axes > 0 && !axes)) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: bad arguments");
  int64_t n = 1;
  for (int a = 0; a < n_axes; ++a) {
    if (axes[a].n <= 0) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: axis %d is empty", a);
    if (ztable_field(axes[a].field)) {
      if (n > INT64_MAX / 16 / axes[a].n) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: too many tables");
      n *= axes[a].n;
    }
  }
  const int64_t ny = n_y > LZQ_NY_MIN ? n_y : LZQ_NY_MIN;
  if (n > INT64_MAX / (ny + lzq::kTabHdr)) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: too many tables");
  return n * (ny + lzq::kTabHdr);
}

// lzq_sweep_grid_reuse in its two halves: build every z-sum table of the grid (parts & 1) and
// integrate [start, start + count) from them (parts & 2).
static int sweep_grid_reuse_parts(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start,
                                  int64_t count, int32_t n_y, int32_t nz, double z_max, const double* d_P,
                                  double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream, int parts,
                                  const char* fn) {
  lzq::GridSpec gs;
  int rc = make_grid(base, axes, n_axes, start, count, d_out, fn, gs);
  if (rc) return rc;
  const int64_t need = lzq_sweep_grid_reuse_workspace(axes, n_axes, n_y);
  if (need < 0) return (int)need;
  const bool work = (parts & 1) || count > 0;
  if (work && (!d_work || work_doubles < need))
    return fail(LZQ_EINVAL, "%s: workspace of %lld doubles < %lld needed", fn, (long long)work_doubles,
                (long long)need);
  if (!(parts & 1) && count == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  const int64_t n_tab = ztable_count(gs);
  int64_t ts = 1;
  for (int a = gs.n_axes - 1; a >= 0; --a)
    if (ztable_field(gs.field[a])) {
      gs.tstride[a] = ts;
      ts *= gs.n[a];
    }
  const int64_t stride = (n_y > LZQ_NY_MIN ? n_y : LZQ_NY_MIN) + lzq::kTabHdr;
  const int64_t nbt = blocks_for(n_tab, lzq::kWavesPerBlock), nb = blocks_for(count, lzq::kWavesPerBlock);
  if (nbt > kMaxGrid || nb > kMaxGrid) return fail(LZQ_EINVAL, "%s: too large for one launch", fn);
  if (parts & 1) {
    // the tables use the exact-underflow truncation: bit-identical to the dense sums
    const int trunc = g.monotone ? 1 : 0;
    if (g_exp_variant == lzq::kExpTable)
      hipLaunchKernelGGL((lzq::grid_ztable_kernel<lzq::kExpTable>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                         (hipStream_t)stream, *base, gs, n_tab, n_y, stride, g.zt, g.nzp, g.key, exp_table(dev), d_work,
                         trunc);
    else
      hipLaunchKernelGGL((lzq::grid_ztable_kernel<lzq::kExpPoly11>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                         (hipStream_t)stream, *base, gs, n_tab, n_y, stride, g.zt, g.nzp, g.key, exp_table(dev), d_work,
                         trunc);
    LZQ_HIP(hipGetLastError());
  }
  if ((parts & 2) && count > 0) {
    hipLaunchKernelGGL(lzq::grid_reuse_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream, *base, gs,
                       start, count, n_y, d_P, g.key, d_work, stride, d_out);
    LZQ_HIP(hipGetLastError());
  }
  return LZQ_OK;
}

int lzq_sweep_grid_reuse(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start, int64_t count,
                         int32_t n_y, int32_t nz, double z_max, const double* d_P, double* d_work, int64_t work_doubles,
                         lzq_yield* d_out, void* stream) {
  if (count == 0) {  // nothing to integrate: validate only (tables need not be built)
    lzq::GridSpec g;
    return make_grid(base, axes, n_axes, start, count, d_out, "lzq_sweep_grid_reuse", g);
  }
  return sweep_grid_reuse_parts(base, axes, n_axes, start, count, n_y, nz, z_max, d_P, d_work, work_doubles, d_out,
                                stream, 3, "lzq_sweep_grid_reuse");
}

int lzq_sweep_grid_ztables(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int32_t n_y, int32_t nz,
                           double z_max, double* d_work, int64_t work_doubles, void* stream) {
  return sweep_grid_reuse_parts(base, axes, n_axes, 0, 0, n_y, nz, z_max, nullptr, d_work, work_doubles, nullptr,
                                stream, 1, "lzq_sweep_grid_ztables");
}

int lzq_sweep_grid_from_ztables(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start,
                                int64_t count, int32_t n_y, int32_t nz, double z_max, const double* d_P,
                                const double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream) {
  return sweep_grid_reuse_parts(base, axes, n_axes, start, count, n_y, nz, z_max, d_P, const_cast<double*>(d_work),
                                work_doubles, d_out, stream, 2, "lzq_sweep_grid_from_ztables");
}

int lzq_p_closed_form(const double* d_lambda, int64_t n, double* d_P, void* stream) {
  if (n < 0 || (n > 0 && (!d_lambda || !d_P))) return fail(LZQ_EINVAL, "lzq_p_closed_form: bad arguments");
  if (n == 0) return LZQ_OK;
  int64_t nb = blocks_for(n, lzq::kBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_p_closed_form: n too large");
  hipLaunchKernelGGL(lzq::p_closed_form_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream,
                     d_lambda, n, d_P);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

}  // extern "C"
