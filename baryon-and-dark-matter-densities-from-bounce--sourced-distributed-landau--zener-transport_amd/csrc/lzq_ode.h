// lzq_ode.h -- the device side shared by the ODE fallback's translation units (not ABI):
// lzq_ode.hip (tables, the sequential integrators, the quadrature form, the operators) and
// lzq_ode_tp.hip (the time-parallel integration, lzq_ode_integrate_tp).  fpy =
// /root/reference/first_principles_yields.py; the functions cite the lines they follow.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>

#include <algorithm>
#include <type_traits>

#include "../../include/lzq.h"
#include "lzq_exp2.h"
#include "lzq_internal.h"
#include "lzq_physics.h"

namespace lzq {


// ode_integrate_kernel: minimum waves per SIMD (its VGPR cap = 512 / this)
#ifndef LZQ_ODE_MIN_WAVES
#define LZQ_ODE_MIN_WAVES 2
#endif
constexpr int kOdeBlock = 256;
constexpr double kInvMplGeV = 1.0 / kMplGeV;

// ---------------------------------------------------------------------------------------
// per-point constants of rhs (one lane per point)
// ---------------------------------------------------------------------------------------
struct OdePoint {
  double m, m3, Tp, B, sig, flux, P;
  double H0;     // 1.66 sqrt(g*)                       fpy:85
  double s0;     // (2 pi^2/45) g*s                      fpy:88
  double c_rel;  // g 3 zeta3/(4 pi^2) | g zeta3/pi^2    fpy:96-99
  double c_nr;   // g (m/2pi)^1.5                        fpy:104
  double v0;     // pi max(m, 1e-20)                     fpy:117
  double sigmav, gamma_w;
  int deplete;
  double T_lo, T_hi, stepT;
  double inv_m, inv_sig, inv_v0, inv_stepT;  // reciprocals: ode_stage multiplies instead of dividing
  double inv_s0, mpl_over_h0;                // 1/s0, M_Pl/H0 (1/s and 1/(H x) as products)
  double Pf;                                 // P * flux: the source term's per-point scale
};

__device__ __forceinline__ void ode_point_recips(OdePoint& o) {
  o.inv_m = 1.0 / o.m;
  o.inv_sig = 1.0 / o.sig;
  o.inv_v0 = 1.0 / o.v0;
  o.inv_stepT = 1.0 / o.stepT;
  o.inv_s0 = 1.0 / o.s0;
  o.mpl_over_h0 = kMplGeV / o.H0;
}

__device__ __forceinline__ OdePoint ode_point(const lzq_point& pt, const lzq_ode_params& od) {
  OdePoint o;
  o.m = pt.m_chi_GeV;
  o.m3 = pt.m_chi_GeV / 3.0;
  o.Tp = pt.T_p_GeV;
  o.B = pt.beta_over_H;
  o.sig = pymax(pt.source_shape_sigma_y, 1e-6);
  o.flux = pt.incident_flux_scale;
  o.P = pt.P_chi_to_B;
  o.Pf = o.P * o.flux;
  o.H0 = 1.66 * sqrt(pt.g_star);
  o.s0 = (2.0 * (kPi * kPi) / 45.0) * pt.g_star_s;
  o.c_rel = (pt.stats == 0) ? pt.g_chi * (3.0 * kZeta3 / (4.0 * (kPi * kPi))) : pt.g_chi * (kZeta3 / (kPi * kPi));
  o.c_nr = pt.g_chi * pow(pt.m_chi_GeV / (2.0 * kPi), 1.5);
  o.v0 = kPi * pymax(pt.m_chi_GeV, 1e-20);
  o.sigmav = pymax(od.sigma_v_chi_GeV_m2, 0.0);  // fpy:279
  o.gamma_w = pymax(od.Gamma_wash_over_H, 0.0);  // fpy:284
  o.deplete = od.deplete_DM_from_source != 0;
  o.T_lo = pt.T_min_over_Tp * pt.T_p_GeV;         // fpy:369
  o.T_hi = pt.T_max_over_Tp * pt.T_p_GeV;         // fpy:368
  o.stepT = (o.T_hi - o.T_lo) / (double)(kOdeNT - 1);
  ode_point_recips(o);
  return o;
}

#ifndef LZQ_ODE_MIN_GROUP
#define LZQ_ODE_MIN_GROUP 8  // smallest cooperative segment (64: whole wavefronts only, round 2)
#endif
#ifndef LZQ_ODE_PREDICT
#define LZQ_ODE_PREDICT 1  // Radau5 collocation predictor for the Riccati Newton iteration
#endif
#ifndef LZQ_ODE_FASTMATH
#define LZQ_ODE_FASTMATH 1  // 0: IEEE division and ROCm exp in the stage function (tools/ablate_ode.py);
#endif
#ifndef LZQ_ODE_COOP
#define LZQ_ODE_COOP 1  // cooperative stage tables for group-uniform wavefronts (ode_integrate_kernel)
#endif
#ifndef LZQ_ODE_FMA
#define LZQ_ODE_FMA LZQ_ODE_FASTMATH  // fused multiply-adds in the spline, the window exponent, Newton's f
#endif

// fpy:214-218 A_over_V_T: min(max(T, T_lo), T_hi), then the PPoly of scipy (_ppoly.pyx:
// interval k with T_k <= T < T_{k+1}, T == T_hi in the last one; c3 + c2 s + c1 s^2 + c0 s^3
// accumulated in that order, powers by repeated multiplication).  nt: the table's knot count
// (the integrators read main()'s LZQ_ODE_NT tables; the operator kernel any build_tables n).
// Split into the interval search, which depends on the point only through its window (shared by
// the cooperative segments, whose points agree in it), and the cubic of one table.
struct SplineLoc {
  double s;  // T - T_k
  int k;     // interval
};

__device__ __forceinline__ SplineLoc spline_loc(const OdePoint& o, double T, int nt = kOdeNT) {
  const double Tq = pymin(pymax(T, o.T_lo), o.T_hi);
  int k = (int)((Tq - o.T_lo) * o.inv_stepT);
  k = k < 0 ? 0 : (k > nt - 2 ? nt - 2 : k);
  // the quotient can land one knot off after rounding: settle against the knots themselves
  if (Tq < linspace_at(o.T_lo, o.T_hi, o.stepT, k, nt) && k > 0) --k;
  else if (k < nt - 2 && Tq >= linspace_at(o.T_lo, o.T_hi, o.stepT, k + 1, nt)) ++k;
  return {Tq - linspace_at(o.T_lo, o.T_hi, o.stepT, k, nt), k};
}

// the cubic of one interval, c = (c0, c1, c2, c3) of the PPoly row
__device__ __forceinline__ double spline_cubic(const double (&c)[4], double s) {
  if (LZQ_ODE_FMA) return __builtin_fma(__builtin_fma(__builtin_fma(c[0], s, c[1]), s, c[2]), s, c[3]);  // Horner
  double z = s, res = c[3];
  res = res + c[2] * z;
  z = z * s;
  res = res + c[1] * z;
  z = z * s;
  res = res + c[0] * z;
  return res;
}

__device__ __forceinline__ double spline_at(const double* __restrict__ w, double s, int k) {
  const double* c = w + 4 * k;
  const double cc[4] = {c[0], c[1], c[2], c[3]};
  return spline_cubic(cc, s);
}

__device__ __forceinline__ double spline_eval(const OdePoint& o, const double* __restrict__ w, double T,
                                              int nt = kOdeNT) {
  const SplineLoc l = spline_loc(o, T, nt);
  return spline_at(w, l.s, l.k);
}


// 1/x for a positive normal x: v_rcp_f64 + two Newton steps (5 VALU; <= 1 ulp from the
// correctly rounded quotient, which costs ~10).
__device__ __forceinline__ double rcp_pos(double x) {
  if (!LZQ_ODE_FASTMATH) return 1.0 / x;
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}

// exp(v) for v <= 0 as 2^(v log2 e) with the degree-11 exp2 of lzq_exp2.h (0.63 ulp on the
// reduced argument; the one rounding of v log2 e costs |v| 2^-53 relative, < 1e-13 for
// |v| < 700, where the factor is still > 1e-304).  ~16 VALU against ~22 for ROCm's exp.
__device__ __forceinline__ double exp_nonpos(double v) {
  if (!LZQ_ODE_FASTMATH) return exp(v);
  return exp2_nonpos(v * kLog2E, 1.0);
}

// The ingredients of rhs(x, .) (fpy:270-286), which do not depend on Y:
//   dY_chi/dx = -lam (Y_chi^2 - E2) - S        lam = sigmav s/(H x), E2 = (n_eq/s)^2,
//                                               S = (deplete ? SB/s : 0)/(H x)
//   dY_B/dx   = alpha - beta Y_B               alpha = (SB/s)/(H x), beta = (gamma_w H)/(H x)
struct OdeStage {
  double lam, E2, S, alpha, beta;
  double a;  // alpha per unit P * flux (the Y_B recurrence forms P * flux * (its coefficient of a))
};

// The same with the per-point scalars factored out: alpha (and S) per unit P * flux, lam per
// unit sigma_v, beta per unit gamma_w.  Points that differ only in those scalars (and in their
// initial state) share these values -- the cooperative mode of ode_integrate_kernel computes
// them once per step for a whole wavefront.  Every stage goes through this split, so a point's
// result does not depend on which mode its wavefront ran in.  a = Av * ap: the A/V spline value
// times the rest of the source term, so points that differ also in the A/V kernel (I_p, v_w: their
// own spline tables) share ap and the spline location (s, k) and form a from their own table.
struct StageBase {
  double a, lam, E2, beta;
  double ap;  // a / Av
  double s;   // spline location of the stage's T (spline_loc)
  int k;
};

__device__ __forceinline__ StageBase ode_stage_base(const OdePoint& o, const double* __restrict__ w, double x,
                                                    double* Av_out = nullptr, int nt = kOdeNT) {
  // One division per call (1/x); every other quotient of fpy:270-286 is a product with a
  // per-point reciprocal or with powers of 1/T: 1/s = (1/T)^3 / s0 and 1/(H x) =
  // (M_Pl/H0) (1/T)^2 / x, exact rewrites of s = s0 T^3 and H = H0 T^2 / M_Pl (fpy:85, 88)
  // wherever the max(., 1e-300) guards are inactive (T > 1e-30 GeV: always on the ODE window;
  // the guarded branch divides).  Each product differs from the quotient by a few ulp, far
  // inside the 1e-11 oracle gate (tests/test_gpu_ode.py).
  const double xc = pymax(x, 1e-30);
  const double ixc = rcp_pos(xc);
  const double T = o.m * ixc;                                 // fpy:272  m / max(x, 1e-30)
  const double iT = T >= 1e-30 ? xc * o.inv_m : 1e30;         // 1 / max(T, 1e-30)
  const double H = pymax(o.H0 * T * T * kInvMplGeV, 1e-300);  // fpy:273 via fpy:85
  const double T3 = (T * T) * T;
  const double s = pymax(o.s0 * T3, 1e-300);                  // fpy:274 via fpy:88
  const double qT = o.Tp * iT;                                // fpy:275 y_of_T (fpy:126-128)
  const double y = 0.5 * o.B * (LZQ_ODE_FMA ? __builtin_fma(qT, qT, -1.0) : qT * qT - 1.0);
  const double q = y * o.inv_sig;
  const double window = exp_nonpos(-0.5 * (q * q));           // fpy:276
  double n_eq, vbar;                                          // fpy:90-120
  if (T > o.m3) {
    n_eq = o.c_rel * T3;
    vbar = 1.0;
  } else {
    n_eq = o.c_nr * (T * sqrt(T)) * exp_nonpos(-o.m * iT);
    vbar = sqrt(pymax(8.0 * T * o.inv_v0, 0.0));
  }
  const double Jb = 0.25 * n_eq * vbar;                       // fpy:222-223, J / flux
  const SplineLoc loc = spline_loc(o, T, nt);
  const double Av = spline_at(w, loc.s, loc.k);               // fpy:214-218
  if (Av_out) *Av_out = Av;
  const double SBb = Jb * window;                             // fpy:277, SB / (P flux Av)
  const bool plain = H > 1e-290 && s > 1e-290 && x == xc;     // the max() guards are inactive
  const double iT2 = iT * iT;
  const double is = plain ? (iT2 * iT) * o.inv_s0 : 1.0 / s;
  const double E = n_eq * is;                                 // fpy:280
  const double iHx = plain ? (o.mpl_over_h0 * iT2) * ixc : 1.0 / (H * x);
  StageBase b;
  b.ap = (SBb * is) * iHx;
  b.a = Av * b.ap;                                            // fpy:282, 285
  b.s = loc.s;
  b.k = loc.k;
  b.lam = s * iHx;                                            // fpy:279-281
  b.E2 = E * E;
  b.beta = H * iHx;                                           // fpy:284-285
  return b;
}

__device__ __forceinline__ OdeStage stage_scale(const OdePoint& o, const StageBase& b) {
  OdeStage st;
  st.alpha = o.Pf * b.a;
  st.S = o.deplete ? st.alpha : 0.0;
  st.lam = o.sigmav * b.lam;
  st.E2 = b.E2;
  st.beta = o.gamma_w * b.beta;
  st.a = b.a;
  return st;
}

__device__ __forceinline__ OdeStage ode_stage(const OdePoint& o, const double* __restrict__ w, double x,
                                              double* Av_out = nullptr, int nt = kOdeNT) {
  return stage_scale(o, ode_stage_base(o, w, x, Av_out, nt));
}

// The Y_chi-only stage of the Riccati equation with no source term (deplete off):
// lam = sigma_v s/(H x), E2 = (n_eq/s)^2, S = 0 -- no spline, no window (ode_stage's
// operations otherwise).  alpha / beta are not formed (Y_B comes from the quadrature).  Split
// like ode_stage into a shared base (lam per unit sigma_v, E2) and the per-point product.
__device__ __forceinline__ StageBase ode_stage_chi_base(const OdePoint& o, double x) {
  const double xc = pymax(x, 1e-30);
  const double ixc = rcp_pos(xc);
  const double T = o.m * ixc;
  const double iT = T >= 1e-30 ? xc * o.inv_m : 1e30;
  const double H = pymax(o.H0 * T * T * kInvMplGeV, 1e-300);
  const double T3 = (T * T) * T;
  const double s = pymax(o.s0 * T3, 1e-300);
  double n_eq;
  if (T > o.m3) n_eq = o.c_rel * T3;
  else n_eq = o.c_nr * (T * sqrt(T)) * exp_nonpos(-o.m * iT);
  const bool plain = H > 1e-290 && s > 1e-290 && x == xc;
  const double iT2 = iT * iT;
  const double is = plain ? (iT2 * iT) * o.inv_s0 : 1.0 / s;
  const double E = n_eq * is;
  const double iHx = plain ? (o.mpl_over_h0 * iT2) * ixc : 1.0 / (H * x);
  StageBase b;
  b.a = 0.0;
  b.ap = 0.0;
  b.s = 0.0;
  b.k = 0;
  b.lam = s * iHx;
  b.E2 = E * E;
  b.beta = 0.0;
  return b;
}

__device__ __forceinline__ OdeStage chi_scale(const OdePoint& o, const StageBase& b) {
  OdeStage st;
  st.lam = o.sigmav * b.lam;
  st.E2 = b.E2;
  st.S = 0.0;
  st.alpha = 0.0;
  st.beta = 0.0;
  st.a = 0.0;
  return st;
}

__device__ __forceinline__ OdeStage ode_stage_chi(const OdePoint& o, double x) {
  return chi_scale(o, ode_stage_chi_base(o, x));
}

// CubicSpline's check of the knots linspace(T_lo, T_hi, nt): strictly increasing.
__device__ __forceinline__ bool ode_grid_ok(double T_lo, double T_hi, double stepT, int nt = kOdeNT) {
  bool ok = true;
  double prev = linspace_at(T_lo, T_hi, stepT, 0, nt);
  for (int k = 1; k < nt; ++k) {
    const double xk = linspace_at(T_lo, T_hi, stepT, k, nt);
    ok = ok && (xk > prev);
    prev = xk;
  }
  return ok;
}

// The integrators read tables of kOdeNT knots at a fixed stride: ode_spline_kernel records the
// table's knot count in its last 4 doubles (spare: the cubics use 4 (nt - 1)), and a table built
// for another nt (lzq_ode_tables takes any) is refused per point instead of read as wrong rows.
__device__ __forceinline__ bool ode_table_ok(const double* __restrict__ w) { return w[kOdeWS - 4] == (double)kOdeNT; }

// Radau IIA, 3 stages (the method of scipy's Radau): nodes C, matrix A (row 3 = weights).
struct Radau {
  double c[3], a[3][3];
};

__device__ __forceinline__ Radau radau_tableau() {
  Radau r;
  const double s6 = sqrt(6.0);
  r.c[0] = (4.0 - s6) / 10.0;
  r.c[1] = (4.0 + s6) / 10.0;
  r.c[2] = 1.0;
  r.a[0][0] = (88.0 - 7.0 * s6) / 360.0;
  r.a[0][1] = (296.0 - 169.0 * s6) / 1800.0;
  r.a[0][2] = (-2.0 + 3.0 * s6) / 225.0;
  r.a[1][0] = (296.0 + 169.0 * s6) / 1800.0;
  r.a[1][1] = (88.0 + 7.0 * s6) / 360.0;
  r.a[1][2] = (-2.0 - 3.0 * s6) / 225.0;
  r.a[2][0] = (16.0 - s6) / 36.0;
  r.a[2][1] = (16.0 + s6) / 36.0;
  r.a[2][2] = 1.0 / 9.0;
  return r;
}

// The Newton start of a block's first step (LZQ_ODE_PRED_BLOCK), from Y_chi and the step's stages
// alone: per stage one linearised backward-Euler step over c_j h,
//   Z_j = Y0 + c_j h f_j(Y0) / (1 + 2 c_j h lam_j Y0),   f_j = -lam_j (Y0^2 - E2_j) - S_j,
// between E and Y0 where the stage relaxes (annihilation), ~Y0 + c_j h f where it does not -- so a
// stiff step converges in the peeled iterations as it does from the predictor, and the start stays
// history-free (the block's end a function of its start: lzq_ode_integrate_tp's exact stitching).
// false (start from Y0) for a non-finite guess or a sign change of a positive Y0.  Every integrator
// calls it with the same operands.
__device__ __forceinline__ bool block_guess(const Radau& R, double h, const OdeStage (&sg)[3], double Y0,
                                            double (&Z)[3]) {
  bool ok = true;
  double g[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double ch = (j == 0 ? R.c[0] : (j == 1 ? R.c[1] : R.c[2])) * h;  // (no dynamic index: scratch)
    const double f = -sg[j].lam * (Y0 * Y0 - sg[j].E2) - sg[j].S;
    const double den = 1.0 + 2.0 * (ch * sg[j].lam) * Y0;  // >= 1 for Y0 >= 0
    g[j] = Y0 + ch * f * rcp_pos(den);
    ok = ok && den > 0.0 && isfinite(g[j]) && (!(Y0 > 0.0) || g[j] > 0.0);
  }
  if (ok) {
#pragma unroll
    for (int j = 0; j < 3; ++j) Z[j] = g[j];
  }
  return ok;
}

// x = M^-1 b for the 3x3 stage matrices M = I + h A diag(d) (partial pivoting; branch-free
// selects, so the lanes of a wave stay converged).
__device__ __forceinline__ void solve3(double M[3][3], double b[3]) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int r = c + 1; r < 3; ++r) {
      const bool sw = fabs(M[r][c]) > fabs(M[c][c]);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double t = M[c][k];
        M[c][k] = sw ? M[r][k] : t;
        M[r][k] = sw ? t : M[r][k];
      }
      const double t = b[c];
      b[c] = sw ? b[r] : t;
      b[r] = sw ? t : b[r];
    }
#pragma unroll
    for (int r = c + 1; r < 3; ++r) {
      const double f = M[r][c] / M[c][c];
#pragma unroll
      for (int k = c; k < 3; ++k) M[r][k] = M[r][k] - f * M[c][k];
      b[r] = b[r] - f * b[c];
    }
  }
#pragma unroll
  for (int c = 2; c >= 0; --c) {
    double acc = b[c];
#pragma unroll
    for (int k = c + 1; k < 3; ++k) acc = acc - M[c][k] * b[k];
    b[c] = acc / M[c][c];
  }
}

// z[2] of M z = b by Cramer's rule (one division): the Y_B stage system needs only the last
// stage.  M = I + h A diag(beta), beta >= 0, is well conditioned for every h (A of Radau IIA
// has eigenvalues in the right half plane), so the cofactor form loses nothing against the
// pivoted elimination of solve3 (tests/test_gpu_ode.py: oracle at 1e-11).
__device__ __forceinline__ double solve3_last(const double (&M)[3][3], const double (&b)[3]) {
  const double c0 = M[1][0] * M[2][1] - M[1][1] * M[2][0];
  const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                     M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) + M[0][2] * c0;
  const double num = M[0][0] * (M[1][1] * b[2] - b[1] * M[2][1]) - M[0][1] * (M[1][0] * b[2] - b[1] * M[2][0]) +
                     b[0] * c0;
  return num / det;
}

// h * a_ij of the Radau matrix for one step size (formed once per step size, not per step), and h.
struct RadauH {
  double a[3][3];
  double h;
};

__device__ __forceinline__ RadauH radau_h(const Radau& R, double h) {
  RadauH r;
  r.h = h;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) r.a[i][j] = h * R.a[i][j];
  return r;
}

// x = M^-1 b by the adjugate (one division for all three components), for the Newton stage
// systems M = I - hA diag(jf) of the Riccati equation: well conditioned like the Y_B system
// (jf = -2 lam Z <= 0 near the solution), so the cofactor form loses nothing against pivoted
// elimination (tests/test_gpu_ode.py: oracle at 1e-11, stiff cases at 1e-10 of converged).
#ifndef LZQ_ODE_ADJFMA
#define LZQ_ODE_ADJFMA 1  // the adjugate, determinant and products as explicit fmas (the file builds with -ffp-contract=off)
#endif
struct Adj3 {
  double a[3][3];  // adjugate of M
  double id;       // 1 / det M
};
__device__ __forceinline__ Adj3 adj3(const double (&M)[3][3]) {
  Adj3 r;
  if (LZQ_ODE_ADJFMA) {
#define FMA __builtin_fma
    r.a[0][0] = FMA(M[1][1], M[2][2], -(M[1][2] * M[2][1]));
    r.a[0][1] = FMA(M[0][2], M[2][1], -(M[0][1] * M[2][2]));
    r.a[0][2] = FMA(M[0][1], M[1][2], -(M[0][2] * M[1][1]));
    r.a[1][0] = FMA(M[1][2], M[2][0], -(M[1][0] * M[2][2]));
    r.a[1][1] = FMA(M[0][0], M[2][2], -(M[0][2] * M[2][0]));
    r.a[1][2] = FMA(M[0][2], M[1][0], -(M[0][0] * M[1][2]));
    r.a[2][0] = FMA(M[1][0], M[2][1], -(M[1][1] * M[2][0]));
    r.a[2][1] = FMA(M[0][1], M[2][0], -(M[0][0] * M[2][1]));
    r.a[2][2] = FMA(M[0][0], M[1][1], -(M[0][1] * M[1][0]));
    r.id = 1.0 / FMA(M[0][0], r.a[0][0], FMA(M[0][1], r.a[1][0], M[0][2] * r.a[2][0]));
#undef FMA
  } else {
    r.a[0][0] = M[1][1] * M[2][2] - M[1][2] * M[2][1];
    r.a[0][1] = M[0][2] * M[2][1] - M[0][1] * M[2][2];
    r.a[0][2] = M[0][1] * M[1][2] - M[0][2] * M[1][1];
    r.a[1][0] = M[1][2] * M[2][0] - M[1][0] * M[2][2];
    r.a[1][1] = M[0][0] * M[2][2] - M[0][2] * M[2][0];
    r.a[1][2] = M[0][2] * M[1][0] - M[0][0] * M[1][2];
    r.a[2][0] = M[1][0] * M[2][1] - M[1][1] * M[2][0];
    r.a[2][1] = M[0][1] * M[2][0] - M[0][0] * M[2][1];
    r.a[2][2] = M[0][0] * M[1][1] - M[0][1] * M[1][0];
    r.id = 1.0 / (M[0][0] * r.a[0][0] + M[0][1] * r.a[1][0] + M[0][2] * r.a[2][0]);
  }
  return r;
}
__device__ __forceinline__ void adj3_apply(const Adj3& A, double (&b)[3]) {
  double x[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    x[i] = LZQ_ODE_ADJFMA ? __builtin_fma(A.a[i][0], b[0], __builtin_fma(A.a[i][1], b[1], A.a[i][2] * b[2])) * A.id
                          : (A.a[i][0] * b[0] + A.a[i][1] * b[1] + A.a[i][2] * b[2]) * A.id;
  b[0] = x[0];
  b[1] = x[1];
  b[2] = x[2];
}
__device__ __forceinline__ void solve3_adj(const double (&M)[3][3], double (&b)[3]) { adj3_apply(adj3(M), b); }

// Y_B's Radau step as an affine map (LZQ_ODE_YBREC): the stage system (I + hA diag(beta)) Z =
// Y_B 1 + hA alpha, alpha_j = P flux a_j, gives by Cramer's rule Z_3 = c Y_B + P flux d with
// c = (w0 + w1 + w2)/det and d = sum_j (sum_i w_i hA_ij) a_j / det, w_i the cofactors of the last
// column's numerator (solve3_last's).  c and d depend on the point only through Gamma_wash (beta)
// and the stage bases, so a cooperative segment with one Gamma_wash forms them once per step
// for all its lanes; every mode forms them with these operations, so the result does not depend
// on the mode.
struct YbW {
  double W[3], id;  // d = (sum_j W_j a_j) id: a lane whose a_j differ from the segment's forms its own d (yb_d)
};
struct YbCD {
  double c, d;
};
struct YbRec {
  double c, d;
  double W[3], id;
};
__device__ __forceinline__ double yb_d(const YbW& r, const double (&a)[3]) {
  double d = 0.0;
#pragma unroll
  for (int j = 0; j < 3; ++j) d = __builtin_fma(r.W[j], a[j], d);
  return d * r.id;
}
__device__ __forceinline__ YbRec yb_rec(const RadauH& hA, const double (&beta)[3], const double (&a)[3]) {
  double M[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) M[i][j] = __builtin_fma(hA.a[i][j], beta[j], i == j ? 1.0 : 0.0);
  const double w0 = M[1][0] * M[2][1] - M[1][1] * M[2][0];
  const double w1 = M[0][1] * M[2][0] - M[0][0] * M[2][1];
  const double w2 = M[0][0] * M[1][1] - M[0][1] * M[1][0];
  const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                     M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) + M[0][2] * w0;
  YbRec r;
  r.id = 1.0 / det;
#pragma unroll
  for (int j = 0; j < 3; ++j) r.W[j] = __builtin_fma(w2, hA.a[2][j], __builtin_fma(w1, hA.a[1][j], w0 * hA.a[0][j]));
  r.c = ((w0 + w1) + w2) * r.id;
  r.d = yb_d(YbW{{r.W[0], r.W[1], r.W[2]}, r.id}, a);
  return r;
}
__device__ __forceinline__ YbRec yb_rec(const RadauH& hA, const OdeStage (&st)[3]) {
  const double beta[3] = {st[0].beta, st[1].beta, st[2].beta}, a[3] = {st[0].a, st[1].a, st[2].a};
  return yb_rec(hA, beta, a);
}

// One Radau step for both equations (hA = h * A of the step); false when the Y_chi Newton
// iteration fails.  The stage sums are explicit fmas (hA_ij * f_j + acc); only the last stage
// of each equation is the step's result, so the linear cases form only what they need.
// Newton starting values for the next step's Riccati stages: the previous step's collocation
// polynomial (through Y at its start and its three stage values, nodes 0, c1, c2, 1) evaluated
// at 1 + c_j (Lagrange weights, mpmath): the standard Radau5 predictor.
static __constant__ double kRadauPred[3][4] = {
    {-0x1.94f343c8b1118p-1, 0x1.6c62e7ee47cd1p+0, -0x1.98b0a4fff4ae1p+0, 0x1.f6c75ef60569bp+0},
    {-0x1.337d989041bbbp+3, 0x1.0879f93eee39dp+4, -0x1.c2e1b2531e4efp+3, 0x1.056b586583971p+3},
    {-0x1.9000000000000p+4, 0x1.51cdd7dde1522p+5, -0x1.07232d3336a77p+5, 0x1.0aaaaaaaaaaabp+4}};

// A^-1 of the Radau IIA matrix (mpmath, rounded once) and the products of its off-diagonal pairs
// that the transformed Newton system's adjugate needs (LZQ_ODE_TNEWTON):
// [a12 a21, a02 a21, a01 a12, a12 a20, a02 a20, a02 a10, a10 a21, a01 a20, a01 a10].
static __constant__ double kRadauAinv[3][3] = {
    {0x1.9cc470a049097p+1, 0x1.2af7915ab4027p+0, -0x1.034624ce046cap-2},
    {-0x1.c8aefbe08d347p+1, 0x1.8cee3d7edbda3p-1, 0x1.0d9e56004de7fp+0},
    {0x1.620bd700c2c3ep+2, -0x1.e20bd700c2c3ep+2, 0x1.4000000000000p+2}};
static __constant__ double kRadauAinvP[9] = {-0x1.fbb0962b0c0cap+2, 0x1.e8360f1027593p+0, 0x1.3adf0cf78af17p+0,
                                      0x1.74e16b2ae518ap+2,  -0x1.6692fca92522fp+0, 0x1.ce862a552e616p-1,
                                      0x1.adf74aa6f6bf3p+4,  0x1.9d782ab97a58ap+2,  -0x1.0aaaaaaaaaaabp+2};
// fma(z, a, c) with the constant a as the SGPR operand, three-address (no copy of the addend)
__device__ __forceinline__ double fma_s(double z, double a, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(z), "s"(a), "v"(c));
  return r;
}

// fma(k, -a, p) for two constants a, p: a (wave-uniform) as the one SGPR operand with its negate
// modifier, p in a VGPR, three-address.  Written as __builtin_fma the compiler picks v_fmac_f64,
// which overwrites its addend, and copies p into the destination first (a v_mov_b64 per entry per
// Newton iteration); the value is the same fma.
__device__ __forceinline__ double fma_neg_s(double k, double a, double p) {
  double r;
  asm("v_fma_f64 %0, %1, -%2, %3" : "=v"(r) : "v"(k), "s"(a), "v"(p));
  return r;
}

#ifndef LZQ_ODE_TNEWTON
#define LZQ_ODE_TNEWTON 1  // the Riccati Newton iteration in the transformed form (constant off-diagonals)
#endif
#ifndef LZQ_ODE_NEWTON_RCP
#define LZQ_ODE_NEWTON_RCP 1  // the Newton solve's 1/det by rcp_pos (5 VALU) instead of the IEEE quotient (~14)
#endif

// Zs: in, Newton starting stages when `guess` (else Ychi for all three); out, the converged
// stages (the next predictor's data).  A predicted start that does not converge is retried
// from Ychi, so the predictor can only save iterations, never lose a step.
#ifndef LZQ_ODE_PEEL
#define LZQ_ODE_PEEL 1  // the first two Newton iterations (and the Y_B solve) as one straight-line block
#endif
#ifndef LZQ_ODE_NEWTON2
#define LZQ_ODE_NEWTON2 1  // the peeled pair of Newton iterations always both applied (no iterate selects)
#endif
#ifndef LZQ_ODE_SIMPLIFIED
#define LZQ_ODE_SIMPLIFIED 1  // the peeled pair's second iteration reuses the first one's adjugate and 1/det
#endif
#ifndef LZQ_ODE_KD
#define LZQ_ODE_KD 1  // the step index as a carried exact double (no 64-bit integer conversion per step)
#endif
#ifndef LZQ_ODE_NOSPLITVAR
#define LZQ_ODE_NOSPLITVAR 1  // waves with no split step in the launch run an integrator variant without the split paths
#endif
#ifndef LZQ_ODE_LINFAST
#define LZQ_ODE_LINFAST 1  // one fma per regular step on linear cooperative waves (sigma_v = 0, no depletion)
#endif
#ifndef LZQ_ODE_YBREC
#define LZQ_ODE_YBREC 1  // Y_B by its affine step map (yb_rec), shared per cooperative segment
#endif
#ifndef LZQ_ODE_RICVAR
#define LZQ_ODE_RICVAR 1  // whole-wave cooperative split-free waves run ode_riccati_kernel (compact rows, uniform constants)
#endif
#ifndef LZQ_ODE_RICTAB
#define LZQ_ODE_RICTAB 1  // table-varying whole waves too, through ode_riccati_kernel<., true> (round 6; RicRowT)
#endif
#ifndef LZQ_ODE_RICSEG
#define LZQ_ODE_RICSEG 1  // split-free waves of uniform 32/16/8-lane segments through ode_riccati_kernel<0, false, true>
#endif
#ifndef LZQ_ODE_ROWS
#define LZQ_ODE_ROWS 1  // linear waves read their run's shared row table when given one (lzq_ode_integrate_rows)
#endif
#ifndef LZQ_ODE_ROWS_ASYNC
#define LZQ_ODE_ROWS_ASYNC 0  // 1: row-table waves fetch the next block into LDS (global_load_lds) while a block steps (measured slower)
#endif
#ifndef LZQ_ODE_ROWS_COPY
#define LZQ_ODE_ROWS_COPY 4  // row staging: loads in flight per lane (a divisor of LZQ_ODE_ROWS_BLOCK / 64)
#endif
#ifndef LZQ_ODE_ROWS_BLOCK
#define LZQ_ODE_ROWS_BLOCK 256   // row-table waves stage 2x this many rows per block (LZQ_ODE_ROWS_ASYNC: two buffers of it)
#endif
#ifndef LZQ_ODE_PRED_BLOCK
// The Radau5 predictor is not used on steps k = 0 (mod LZQ_ODE_PRED_BLOCK): every block of that
// many steps starts its Newton iteration from Y_chi, so a block's end state is a function of its
// start (Y_chi, Y_B) alone -- what lzq_ode_integrate_tp's exact stitching needs.  Every integrator
// applies the rule on the absolute step index, so all modes stay bit-identical.  (A power of two.)
#define LZQ_ODE_PRED_BLOCK 64
#endif

__device__ __forceinline__ bool pred_step(int64_t k) { return (k & (LZQ_ODE_PRED_BLOCK - 1)) != 0; }
#ifndef LZQ_RIC_MIN_WAVES
#define LZQ_RIC_MIN_WAVES 4  // ode_riccati_kernel: minimum waves per SIMD (its VGPR cap = 512 / this)
#endif

template <bool kWithYB = true>
__device__ __forceinline__ bool radau_step(const RadauH& hA, const OdeStage (&st)[3], double& Ychi, double& YB,
                                           double (&Zs)[3], bool guess) {
  // Y_B: (I + hA diag(beta)) Z = YB + hA alpha, exactly; Z_3 = Y_B(x + h)
  auto yb_step = [&]() {
    double M[3][3], b[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double acc = YB;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        acc = __builtin_fma(hA.a[i][j], st[j].alpha, acc);
        M[i][j] = __builtin_fma(hA.a[i][j], st[j].beta, i == j ? 1.0 : 0.0);
      }
      b[i] = acc;
    }
    return solve3_last(M, b);
  };
  // Y_chi: Z_i = Y + h sum_j a_ij f_j(Z_j), f_j(Z) = -lam_j (Z^2 - E2_j) - S_j; one Newton
  // iteration on Z, true when its correction is below 1e-15 of the stages
  const double Y0 = Ychi;
#if LZQ_ODE_TNEWTON && LZQ_ODE_FASTMATH
  // Transformed Newton system: (I - hA diag(jf)) g = -(Z - Y0 - hA f) times h (hA)^-1 is
  //   (A^-1 - diag(h jf)) g = h f - A^-1 (Z - Y0),
  // whose matrix keeps A^-1's constant off-diagonals (kRadauAinv) and changes only on the diagonal,
  // A^-1_jj + 2 h lam_j Z_j: its adjugate is one fma per entry against constant products
  // (kRadauAinvP), and the h-scaled stage data h lam_j, 2 h lam_j, h S_j are formed once per step.
  // Same fixed point (the stage equations), ~20 FP64 instructions fewer per iteration than
  // forming I - hA diag(jf) and its full adjugate.
  double hl[3], hl2[3], hS[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    hl[j] = hA.h * st[j].lam;
    hl2[j] = 2.0 * hl[j];
    hS[j] = hA.h * st[j].S;
  }
  // the iteration matrix's adjugate and 1/det, kept for a simplified iteration (LZQ_ODE_SIMPLIFIED)
  struct NewtonJ {
    double b[3][3], id;
  };
  auto newton_j = [&](double (&Z)[3], NewtonJ& J, const bool reuse, bool& near) {
#define FMA __builtin_fma
    double d[3], r[3], k[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      r[j] = FMA(-hl[j], FMA(Z[j], Z[j], -st[j].E2), -hS[j]);  // h f_j
      d[j] = Z[j] - Y0;
      k[j] = FMA(hl2[j], Z[j], kRadauAinv[j][j]);              // A^-1_jj - h jf_j
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
      r[i] = FMA(-kRadauAinv[i][2], d[2], FMA(-kRadauAinv[i][1], d[1], FMA(-kRadauAinv[i][0], d[0], r[i])));
    if (!reuse) {
      // adjugate of [[k0, a01, a02], [a10, k1, a12], [a20, a21, k2]] (a_ij = A^-1_ij, products constant)
      J.b[0][0] = FMA(k[1], k[2], -kRadauAinvP[0]), J.b[0][1] = fma_neg_s(k[2], kRadauAinv[0][1], kRadauAinvP[1]);
      J.b[0][2] = fma_neg_s(k[1], kRadauAinv[0][2], kRadauAinvP[2]), J.b[1][0] = fma_neg_s(k[2], kRadauAinv[1][0], kRadauAinvP[3]);
      J.b[1][1] = FMA(k[0], k[2], -kRadauAinvP[4]), J.b[1][2] = fma_neg_s(k[0], kRadauAinv[1][2], kRadauAinvP[5]);
      J.b[2][0] = fma_neg_s(k[1], kRadauAinv[2][0], kRadauAinvP[6]), J.b[2][1] = fma_neg_s(k[0], kRadauAinv[2][1], kRadauAinvP[7]);
      J.b[2][2] = FMA(k[0], k[1], -kRadauAinvP[8]);
      // 1/det only scales the correction: a reciprocal within 1 ulp leaves the fixed point (the
      // stage equations) as it is and changes the iterates by rounding
      const double den = FMA(k[0], J.b[0][0], FMA(kRadauAinv[0][1], J.b[1][0], kRadauAinv[0][2] * J.b[2][0]));
      J.id = LZQ_ODE_NEWTON_RCP ? rcp_pos(den) : 1.0 / den;
    }
    double g[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) g[i] = FMA(J.b[i][0], r[0], FMA(J.b[i][1], r[1], J.b[i][2] * r[2])) * J.id;
#undef FMA
    // running maxima from +0 of |.| (never NaN on the left): fmax is pymax here, one v_max_f64
    double dmax = 0.0, zmax = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      Z[i] = Z[i] + g[i];
      dmax = fmax(dmax, fabs(g[i]));
      zmax = fmax(zmax, fabs(Z[i]));
    }
    near = !(dmax > 1e-3 * zmax);
    return !(dmax > 1e-15 * zmax);
  };
  NewtonJ J;
  bool near = false;
  auto newton = [&](double (&Z)[3]) { return newton_j(Z, J, false, near); };
#else
  auto newton = [&](double (&Z)[3]) {
    double M[3][3], g[3];
    double f[3], jf[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      f[j] = LZQ_ODE_FMA ? __builtin_fma(-st[j].lam, __builtin_fma(Z[j], Z[j], -st[j].E2), -st[j].S)
                         : -st[j].lam * (Z[j] * Z[j] - st[j].E2) - st[j].S;
      jf[j] = -st[j].lam * (2.0 * Z[j]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double acc = Z[i] - Y0;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        acc = __builtin_fma(-hA.a[i][j], f[j], acc);
        M[i][j] = __builtin_fma(-hA.a[i][j], jf[j], i == j ? 1.0 : 0.0);
      }
      g[i] = -acc;
    }
#if LZQ_ODE_FASTMATH
    solve3_adj(M, g);
#else
    solve3(M, g);
#endif
    double dmax = 0.0, zmax = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      Z[i] = Z[i] + g[i];
      dmax = fmax(dmax, fabs(g[i]));
      zmax = fmax(zmax, fabs(Z[i]));
    }
    return !(dmax > 1e-15 * zmax);
  };
#endif
  auto accept = [&](const double (&Z)[3]) {
    Zs[0] = Z[0];
    Zs[1] = Z[1];
    Zs[2] = Z[2];
    Ychi = Z[2];
  };
  const bool nonlinear = st[0].lam != 0.0 || st[1].lam != 0.0 || st[2].lam != 0.0;
  if (!nonlinear) {  // f_j = -S_j: Z_3 = Y - sum_j hA_3j S_j
    if (kWithYB) YB = yb_step();
    double acc = Ychi;
#pragma unroll
    for (int j = 0; j < 3; ++j) acc = __builtin_fma(-hA.a[2][j], st[j].S, acc);
    Ychi = acc;
    return true;
  }
  for (int attempt = guess ? 0 : 1; attempt < 2; ++attempt) {
    double Z[3] = {attempt == 0 ? Zs[0] : Y0, attempt == 0 ? Zs[1] : Y0, attempt == 0 ? Zs[2] : Y0};
    int it = 0;
#if LZQ_ODE_PEEL
    if (attempt == (guess ? 0 : 1)) {
      // the first two iterations (and Y_B's independent solve) in one basic block, so the
      // scheduler interleaves their dependent chains; the second is applied only if the first
      // did not converge -- the same iterates as the loop below, bit for bit
      if (kWithYB) YB = yb_step();
#if LZQ_ODE_NEWTON2
      // both iterations always apply: a step that converged at the first takes the second's
      // (below 1e-15 relative) correction too, so no selects between the two iterates are needed
      const bool c1 = newton(Z);
#if LZQ_ODE_SIMPLIFIED && LZQ_ODE_TNEWTON && LZQ_ODE_FASTMATH
      // Once the first correction is below 1e-3 of the stages (the predicted start, almost every
      // step), the second iteration reuses the first one's matrix (simplified Newton): its
      // correction is then the first one's residual error to first order either way, so the
      // acceptance test reads the same quantity, and the accepted iterate differs by
      // O(1e-3 x that error), far below rounding when the test passes.  A large first correction
      // (a start far from the solution) keeps the full iteration: a stale matrix there can carry
      // the iterate into the other, unstable root's basin.  Per lane, so a point's iterates do not
      // depend on its wavefront.
      const bool reuse = near;
      const bool c2 = newton_j(Z, J, reuse, near);
#else
      const bool c2 = newton(Z);
#endif
      if (c1 || c2) {
        accept(Z);
        return true;
      }
#else
      double Z2[3];
      const bool c1 = newton(Z);
      Z2[0] = Z[0];
      Z2[1] = Z[1];
      Z2[2] = Z[2];
      const bool c2 = newton(Z2);
      if (c1) {
        accept(Z);
        return true;
      }
      if (c2) {
        accept(Z2);
        return true;
      }
      Z[0] = Z2[0];
      Z[1] = Z2[1];
      Z[2] = Z2[2];
#endif
      it = 2;
    }
#else
    if (kWithYB && attempt == (guess ? 0 : 1)) YB = yb_step();
#endif
    for (; it < 40; ++it) {
      if (newton(Z)) {
        accept(Z);
        return true;
      }
    }
  }
  return false;
}

// fpy:385-417 on the ODE path, one lane per point.
// The first x in (x0, x1) at which ode_stage's T = m * (1/x) is no longer > m/3 (the branch of
// n_chi_eq / vbar_chi, fpy:100, 111), +inf if there is none: a few ulp steps from m/(m/3).
__device__ __forceinline__ double branch_x(const OdePoint& o, double x0, double x1) {
  auto rel = [&](double x) { return o.m * (1.0 / pymax(x, 1e-30)) > o.m3; };
  double xg = o.m / o.m3;
  if (!(xg > x0 && xg < x1 + 1.0)) return INFINITY;
  int guard = 0;
  if (rel(xg)) {
    while (rel(xg) && ++guard < 64) xg = nextafter(xg, INFINITY);
  } else {
    while (!rel(nextafter(xg, -INFINITY)) && ++guard < 64) xg = nextafter(xg, -INFINITY);
  }
  return (x0 < xg && xg < x1) ? xg : INFINITY;
}

// Continuation state (OdeState != nullptr): see ode_integrate_kernel (lzq_ode.hip).
struct OdeState {
  double Ychi, YB, Yp, Z[3];
  int32_t status, have;  // status: kOdeInProgress while steps remain
};
constexpr int32_t kOdeInProgress = 64;

__device__ __forceinline__ double ode_uniform(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

}  // namespace lzq

// lzq_ode.hip: the sequential integration of a batch (continuation launches of every variant),
// the fallback of lzq_ode_integrate_tp for the points it does not stitch (skip mask).
int lzq_ode_launch_sequential(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                              const int32_t* d_tidx, const double* d_work, int64_t max_steps, lzq_yield* d_out,
                              int32_t* d_status, hipStream_t s, const char* fn, const int32_t* d_skip);
// hipError_t -> LZQ_EHIP with the message in lzq_last_error
int lzq_ode_hip_check(hipError_t e, const char* what);
// the workspace / n checks of the ODE entry points (LZQ_EINVAL)
int lzq_ode_check_ws(int64_t n, const double* d_work, int64_t work_doubles, const char* fn,
                     int64_t per_table = LZQ_ODE_WS_PER_POINT);
