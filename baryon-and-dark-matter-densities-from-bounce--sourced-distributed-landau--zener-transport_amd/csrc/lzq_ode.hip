// lzq_ode.hip -- the reference's ODE fallback (fpy = /root/reference/first_principles_yields.py,
// lines 200-219 build_tables / A_over_V_T, 270-286 rhs, 385-417 main) for batches of points.
//
//   1. ode_aov_table_kernel (lzq_kernels.hip): A/V at the 800 T-knots, one wavefront per point;
//   2. ode_spline_kernel: scipy CubicSpline(bc_type='not-a-knot') of those knots, one lane per
//      point (Thomas elimination of the slope system, then the PPoly coefficients);
//   3. ode_integrate_kernel: the reference's Radau IIA (3 stages, order 5) on uniform steps
//      h <= max_step (fpy:404), one lane per point, state in registers.  The two equations
//      decouple: Y_B is linear (each step is one 3x3 solve); Y_chi is a Riccati equation
//      (Newton on the 3x3 stage system with its exact Jacobian; a linear update when
//      sigma_v = 0).  tests/golden/golden_ode.json: the reference's own Radau output sits
//      within ~1e-14 of its converged solution, so a fixed-step Radau reproduces it.
//
// The ingredients of rhs follow fpy:270-286 in the reference's operation order, with T**3 as
// (T*T)*T and T**1.5 as T*sqrt(T) (<= 2 ulp from pow; the device pow is ~100 VALU).
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
int g_ode_coop = 1;          // lzq_tune(LZQ_TUNE_ODE_COOP)
int g_ode_launch_log2 = 24;  // lzq_tune(LZQ_TUNE_ODE_LAUNCH_STEPS): <= 2^24 Radau steps per launch
int g_ode_tp_interval = 64;  // lzq_tune(LZQ_TUNE_ODE_TP_INTERVAL): steps per lzq_ode_integrate_tp interval
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
__constant__ double kRadauPred[3][4] = {
    {-0x1.94f343c8b1118p-1, 0x1.6c62e7ee47cd1p+0, -0x1.98b0a4fff4ae1p+0, 0x1.f6c75ef60569bp+0},
    {-0x1.337d989041bbbp+3, 0x1.0879f93eee39dp+4, -0x1.c2e1b2531e4efp+3, 0x1.056b586583971p+3},
    {-0x1.9000000000000p+4, 0x1.51cdd7dde1522p+5, -0x1.07232d3336a77p+5, 0x1.0aaaaaaaaaaabp+4}};

// A^-1 of the Radau IIA matrix (mpmath, rounded once) and the products of its off-diagonal pairs
// that the transformed Newton system's adjugate needs (LZQ_ODE_TNEWTON):
// [a12 a21, a02 a21, a01 a12, a12 a20, a02 a20, a02 a10, a10 a21, a01 a20, a01 a10].
__constant__ double kRadauAinv[3][3] = {
    {0x1.9cc470a049097p+1, 0x1.2af7915ab4027p+0, -0x1.034624ce046cap-2},
    {-0x1.c8aefbe08d347p+1, 0x1.8cee3d7edbda3p-1, 0x1.0d9e56004de7fp+0},
    {0x1.620bd700c2c3ep+2, -0x1.e20bd700c2c3ep+2, 0x1.4000000000000p+2}};
__constant__ double kRadauAinvP[9] = {-0x1.fbb0962b0c0cap+2, 0x1.e8360f1027593p+0, 0x1.3adf0cf78af17p+0,
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

// ---------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------
// fpy:207-212 build_tables, second half: scipy CubicSpline(Ts, Av, bc_type='not-a-knot')
// (scipy/interpolate/_cubic.py), one lane per point.  The slope system is solved by Thomas
// elimination (scipy: banded LU with partial pivoting; equal to rounding); the forward sweep
// parks (c', d') in the c0/c1 slots of the point's workspace.
__global__ __launch_bounds__(kOdeBlock) void ode_spline_kernel(const lzq_point* __restrict__ pts, int64_t n,
                                                               int32_t nt, const double* __restrict__ Tlo,
                                                               const double* __restrict__ Thi,
                                                               double* __restrict__ ws, int32_t* __restrict__ status) {
  const int64_t i = (int64_t)blockIdx.x * kOdeBlock + threadIdx.x;
  if (i >= n) return;
  const lzq_point pt = pts[i];
  const double T_lo = Tlo ? Tlo[i] : pt.T_min_over_Tp * pt.T_p_GeV;
  const double T_hi = Thi ? Thi[i] : pt.T_max_over_Tp * pt.T_p_GeV;
  const int N = nt;
  const int64_t ws_pt = 4 * (int64_t)N;  // the point's 4 nt doubles; A/V at the last knot in the last one
  const double stepT = (T_hi - T_lo) / (double)(N - 1);
  double* w = ws + i * ws_pt;
  auto X = [&](int k) { return linspace_at(T_lo, T_hi, stepT, k, N); };
  auto Yk = [&](int k) { return k < N - 1 ? w[4 * k + 3] : w[ws_pt - 1]; };
  if (!ode_grid_ok(T_lo, T_hi, stepT, N)) {
    if (status) status[i] = LZQ_ODE_BAD_GRID;
    return;
  }
  // forward sweep
  double dxm1 = X(1) - X(0), slm1 = (Yk(1) - Yk(0)) / dxm1;  // dx[k-1], slope[k-1]
  double cpm1, dpm1;
  {
    const double dx1 = X(2) - X(1), sl1 = (Yk(2) - Yk(1)) / dx1;
    const double d = X(2) - X(0);
    const double r = ((dxm1 + 2.0 * d) * dx1 * slm1 + (dxm1 * dxm1) * sl1) / d;
    cpm1 = d / dx1;
    dpm1 = r / dx1;
    w[0] = cpm1;
    w[1] = dpm1;
  }
  // (the sweeps read the knot values kSplCh rows ahead: one row at a time, each load waited behind
  // the previous row's stores, ~0.3 us per row -- 0.46 ms per 800-knot table; same operations)
  constexpr int kSplCh = 8;
  double yk = Yk(1);
  for (int k0 = 1; k0 < N - 1; k0 += kSplCh) {
    double yn[kSplCh];
#pragma unroll
    for (int i = 0; i < kSplCh; ++i) yn[i] = k0 + i < N - 1 ? Yk(k0 + i + 1) : 0.0;
#pragma unroll
    for (int i = 0; i < kSplCh; ++i) {
      const int k = k0 + i;
      if (k < N - 1) {
        const double dxk = X(k + 1) - X(k), slk = (yn[i] - yk) / dxk;
        const double a = dxk, b = 2.0 * (dxm1 + dxk), c = dxm1;
        const double r = 3.0 * (dxk * slm1 + dxm1 * slk);
        const double den = b - a * cpm1;
        cpm1 = c / den;
        dpm1 = (r - a * dpm1) / den;
        w[4 * k + 0] = cpm1;
        w[4 * k + 1] = dpm1;
        dxm1 = dxk;
        slm1 = slk;
        yk = yn[i];
      }
    }
  }
  // last row (not-a-knot): (x[-1]-x[-3]) s[-2] + dx[-2] s[-1] = b[-1]
  double s_next;
  {
    const double dx2 = X(N - 2) - X(N - 3), sl2 = (Yk(N - 2) - Yk(N - 3)) / dx2;  // dx[-2], slope[-2]
    const double d = X(N - 1) - X(N - 3);
    const double r = ((dxm1 * dxm1) * sl2 + (2.0 * d + dxm1) * dx2 * slm1) / d;
    s_next = (r - d * dpm1) / (dx2 - d * cpm1);
  }
  // back substitution, forming the PPoly coefficients of interval k on the way
  const double y_last = w[ws_pt - 1];
  double yk1 = y_last;  // Y at knot k + 1
  for (int k0 = N - 2; k0 >= 0; k0 -= kSplCh) {
    double rc[kSplCh], rd[kSplCh], ry[kSplCh];
#pragma unroll
    for (int i = 0; i < kSplCh; ++i) {
      const int k = k0 - i;
      rc[i] = k >= 0 ? w[4 * k + 0] : 0.0;
      rd[i] = k >= 0 ? w[4 * k + 1] : 0.0;
      ry[i] = k >= 0 ? w[4 * k + 3] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < kSplCh; ++i) {
      const int k = k0 - i;
      if (k >= 0) {
        const double sk = rd[i] - rc[i] * s_next;
        const double dxk = X(k + 1) - X(k);
        const double slk = (yk1 - ry[i]) / dxk;
        const double t = (sk + s_next - 2.0 * slk) / dxk;
        w[4 * k + 0] = t / dxk;
        w[4 * k + 1] = (slk - sk) / dxk - t;
        w[4 * k + 2] = sk;
        s_next = sk;
        yk1 = ry[i];
      }
    }
  }
  w[ws_pt - 4] = (double)N;  // the table's knot count, in its spare doubles (ode_table_ok)
  if (status) status[i] = LZQ_ODE_OK;
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

// tidx (optional): point i reads the spline table at ws[tidx[i] * kOdeWS] (tables shared by
// points with the same A/V kernel and window, lzq_ode_integrate_shared); NULL: its own, ws[i].
// kChiOnly (lzq_ode_quadrature, sigma_v != 0 points): Y_B is already in out[i] from the
// quadrature (exact for every sigma_v: its equation is linear); step only the Riccati equation
// of Y_chi, with ode_stage_chi when there is no source term.  Points with sigma_v = 0 return
// at once (the quadrature has done both).
// Continuation (OdeState != nullptr): the launch advances every point by the steps
// [k_lo, k_lo + k_cnt) of its fixed-step sequence only, carrying (Y_chi, Y_B, the predictor's
// previous start and stages) between launches in HBM, so a window of any length runs as a
// series of bounded launches (lzq_ode_launches); the arithmetic of every step is the single
// launch's, so the result is bit-identical to one launch over [0, N).
struct OdeState {
  double Ychi, YB, Yp, Z[3];
  int32_t status, have;  // status: kOdeInProgress while steps remain
};
constexpr int32_t kOdeInProgress = 64;

// kLin: the variant for linear cooperative waves (see lin_wave below); every launch runs both
// variants, each stepping only its own wavefronts (the other variant's return at once), so the
// linear waves' tight loop does not share a register allocation with the Riccati Newton path.
template <bool kChiOnly, bool kLin = false, bool kNoSplit = false>
__global__ __launch_bounds__(kOdeBlock, LZQ_ODE_MIN_WAVES) void ode_integrate_kernel(const lzq_point* __restrict__ pts,
                                                                  const lzq_ode_params* __restrict__ ode, int64_t n,
                                                                  const int32_t* __restrict__ tidx,
                                                                  const double* __restrict__ ws, int64_t max_steps,
                                                                  lzq_yield* __restrict__ out,
                                                                  int32_t* __restrict__ status, int coop_on,
                                                                  int64_t k_lo, int64_t k_cnt,
                                                                  OdeState* __restrict__ state,
                                                                  const int32_t* __restrict__ skip) {
  __shared__ StageBase s_base[kOdeBlock / 64][64][3];  // cooperative mode
  // shared Y_B step maps, (c, d) and the cofactor weights in separate arrays: the linear waves'
  // tight loop streams 16-B (c, d) rows
  __shared__ YbCD s_rcd[LZQ_ODE_YBREC && !kChiOnly ? kOdeBlock / 64 : 1][64];
  __shared__ YbW s_rw[LZQ_ODE_YBREC && !kChiOnly ? kOdeBlock / 64 : 1][64];
  // Lanes past the end of the batch are clones of their wavefront's first point (they compute
  // it again and write nothing), so a partial wavefront -- a single CLI point included -- is
  // still full and can run cooperatively.
  const int64_t wave0 = (int64_t)blockIdx.x * kOdeBlock + (threadIdx.x & ~63);
  if (wave0 >= n) return;
  const int64_t i_self = (int64_t)blockIdx.x * kOdeBlock + threadIdx.x;
  const bool real = i_self < n;
  const int64_t i = real ? i_self : wave0;
  if (skip && skip[i]) return;  // integrated by lzq_ode_integrate_tp's iteration
  const bool cont = state != nullptr, first = !cont || k_lo == 0;
  if (cont && !first && state[i].status != kOdeInProgress) return;  // finished in an earlier launch
  const lzq_point pt = pts[i];
  const OdePoint o = ode_point(pt, ode[i]);
  if (kChiOnly && first && (o.sigmav == 0.0 || (status && status[i] != LZQ_ODE_NOT_LINEAR))) {
    if (cont && real) state[i].status = LZQ_ODE_OK;  // nothing to step (the quadrature did it)
    return;
  }
  const double* w = ws + (tidx ? (int64_t)tidx[i] : i) * (int64_t)kOdeWS;
  const double nan = __builtin_nan("");
  lzq_yield r = {nan, nan, nan, nan, nan, pt.P_chi_to_B};
  int st = ode_grid_ok(o.T_lo, o.T_hi, o.stepT) ? (ode_table_ok(w) ? LZQ_ODE_OK : LZQ_ODE_BAD_TABLE) : LZQ_ODE_BAD_GRID;
  const double m = o.m, T_p = o.Tp;
  const double x0 = m / o.T_hi, x1 = m / pymax(o.T_lo, 1e-30);  // fpy:387-388
  double Ychi;                                                   // fpy:389-399
  if (pt.regime == LZQ_NONTHERMAL) {
    if (pt.has_Y_chi_init) Ychi = pt.Y_chi_init;
    else if (pt.has_n_chi_at_Tp) Ychi = pt.n_chi_at_Tp_GeV3 / pymax(s_entropy(T_p, pt.g_star_s), 1e-300);
    else Ychi = 1.0e-12;
  } else {  // thermal, and the fallback branch fpy:398-399 (no UnboundLocalError on this path)
    Ychi = n_chi_eq(o.T_hi, m, pt.g_chi, pt.stats) / s_entropy(o.T_hi, pt.g_star_s);
  }
  double YB = kChiOnly ? out[i].Y_B : 0.0;
#ifdef LZQ_ODE_COOP_DEBUG
  double dbg_coop = -1.0;
#endif
  const double x_p = m / pymax(T_p, 1e-30);
  const double max_step = pymin(pymin(fabs(x1 - x0) / 20000.0, x_p / 1000.0), 5e-4);  // fpy:403-404
  double steps = 0.0;
  if (st == LZQ_ODE_OK) {
    if (!(max_step > 0.0)) st = LZQ_ODE_BAD_STEP;
    else {
      steps = ceil(fabs(x1 - x0) / max_step);
      if (!(steps <= (double)max_steps)) st = LZQ_ODE_TOO_MANY_STEPS;
    }
  }
  bool finished = true;  // this launch ends the point (continuation: else its state is saved)
  if ((kLin || kNoSplit) && st != LZQ_ODE_OK) return;  // the general variant reports it (its wave is not linear)
  if (st == LZQ_ODE_OK) {
    const int64_t N = (int64_t)steps;
    const int64_t k_begin = cont ? k_lo : 0;
    const int64_t k_stop = cont ? (k_lo + k_cnt < N ? k_lo + k_cnt : N) : N;
    finished = k_stop >= N;
    const double h = (x1 - x0) / (double)N;
    const Radau R = radau_tableau();
    // n_chi_eq / vbar_chi switch formula at the strict T > m/3 (fpy:100, 111): the rhs jumps at
    // the first x whose T (ode_stage's m * (1/x)) is not > m/3.  The step that straddles it is
    // split there, ending one ulp before it, so no stage sees both branches (the oracle does
    // the same with its own T; tests/golden/golden_ode_stiff.json).
    const double xb = branch_x(o, x0, x1);
    const double xb_below = nextafter(xb, -INFINITY);  // where a split step's first part ends
    const RadauH hA = radau_h(R, h);
    const bool riccati = LZQ_ODE_PREDICT && !kLin && o.sigmav != 0.0;  // kLin: sigma_v = 0 on every lane
    double Zs[3] = {Ychi, Ychi, Ychi}, Yp = Ychi;  // previous step's start and stages (predictor)
    bool have = false, done = false;
    if (!first) {  // continue from the previous launch's state
      const OdeState sv = state[i];
      Ychi = sv.Ychi;
      YB = sv.YB;
      Yp = sv.Yp;
      Zs[0] = sv.Z[0];
      Zs[1] = sv.Z[1];
      Zs[2] = sv.Z[2];
      have = sv.have != 0;
    }
    // Cooperative mode (a full wavefront whose points agree in everything ode_stage_base (or
    // ode_stage_chi_base: kChiOnly, the same deplete flag) reads:
    // they differ at most in P, flux, sigma_v, Gamma_wash, deplete and the initial state, as in
    // sweeps over those axes): lane l evaluates the stage ingredients of step kb + l for the
    // whole wavefront into LDS, then every lane integrates those 64 steps of its own point from
    // them.  The ingredients of a step are computed once instead of 64 times; the arithmetic is
    // the same (ode_stage = stage_scale(ode_stage_base)), so results are bit-identical to the
    // per-lane mode.  Split steps (the T = m/3 branch) always evaluate their own stages.
    // Sub-groups: a wave whose aligned G-lane segments (G = 32, 16, 8) are each uniform, though
    // the wave is not (sweeps with fewer than 64 points per stage key, e.g. many m_chi values),
    // runs the same scheme per segment: lane l of a segment evaluates step kb + l of ITS
    // segment's key into its own LDS row, and the segment integrates blocks of G steps from its G
    // rows (segments may differ in N and h; they never touch each other's rows).
    // Table-varying segments (round 4): points that agree in all of that but the A/V kernel
    // (I_p, v_w: each has its own spline table) share the rows too; the rows then carry a / Av
    // and the spline location (StageBase ap, s, k), and each lane forms a = Av * ap from its own
    // table -- the operations ode_stage_base performs, so still the per-lane bits.
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int G = 0;             // cooperative segment width (0: per-lane)
    bool tab_vary = false;  // the segment's points read different spline tables
    if (LZQ_ODE_COOP && coop_on && __ballot(1) == ~0ull) {
      for (int g = 64; g >= LZQ_ODE_MIN_GROUP && G == 0; g >>= 1) {
        auto same = [g](double v) {  // bit-equal to the value of the first lane of the g-segment
          const uint64_t b = __builtin_bit_cast(uint64_t, v);
          return b == __builtin_bit_cast(uint64_t, __shfl(v, 0, g));
        };
        const bool eq = same(o.m) && same(o.Tp) && same(o.B) && same(o.sig) && same(o.H0) && same(o.s0) &&
                        same(o.c_rel) && same(o.c_nr) && same(o.v0) && same(o.T_lo) && same(o.T_hi) &&
                        (!kChiOnly || same((double)o.deplete));
        if (__all(eq)) {
          G = g;
          tab_vary = !__all(same(__builtin_bit_cast(double, w)));
        }
      }
#ifdef LZQ_ODE_COOP_DEBUG
      dbg_coop = (double)G + (tab_vary ? 0.5 : 0.0);
#endif
    }
    const bool coop = G > 0;
    const int seg = lane & ~(G - 1);  // first LDS row of this lane's segment (G > 0)
    // this lane's a of a shared row's stage (its own table in a table-varying segment)
    auto row_a = [&](const StageBase& b) -> double { return tab_vary ? spline_at(w, b.s, b.k) * b.ap : b.a; };
    // Y_B's step maps shared by the segment when it has one Gamma_wash (LZQ_ODE_YBREC)
    bool rec_shared = false;
    if (LZQ_ODE_YBREC && !kChiOnly && coop) {
      const uint64_t gb = __builtin_bit_cast(uint64_t, o.gamma_w);
      rec_shared = __all(gb == __builtin_bit_cast(uint64_t, __shfl(o.gamma_w, 0, G)));
    }
    // Linear waves (LZQ_ODE_LINFAST): with sigma_v = 0 on every lane, Y_chi's Radau step is
    // radau_step's linear branch, Z_3 = Y - sum_j hA_3j S_j with S_j = P flux a_j when depleting and
    // +0 otherwise (then Y_chi is unchanged, exactly), and Y_B's is the segment's shared map: a
    // regular step is one fma on the LDS row (+ three with depletion) -- the general path's
    // operations on the same values, hence the same bits.  Split steps take the general path.
    const bool lin_wave = LZQ_ODE_LINFAST && LZQ_ODE_YBREC && !kChiOnly && rec_shared && __all(o.sigmav == 0.0);
    if (lin_wave != kLin) return;  // the other variant of this launch steps this wavefront
    const bool lin_fast = kLin;
    // Linear waves: the first split step (xk < xb <= xk + h), found once.  x_k's rounding error is
    // far below h, so it can only be within a step of (xb - x0)/h: the predicate is checked on a
    // few candidates around it (a lane whose x scale would make the rounding comparable to h
    // takes every step on the general path, k_split = -1).  The general path takes that step and
    // the next (a rounding may split two consecutive steps); the rest run as the tight loop.
    int64_t k_split = INT64_MAX;
    // whether the previous step was split: a continuation launch starts with the single launch's
    // value, the predicate of step k_begin - 1 (else a launch boundary right after a split step
    // would send the next -- possibly split again -- step through the tight loop)
    bool prev_split = false;
    if (k_begin > 0) {
      const double xq = x0 + (double)(k_begin - 1) * h;
      prev_split = xq < xb && xb <= xq + h;
    }
    if ((lin_fast || LZQ_ODE_NOSPLITVAR) && xb < INFINITY) {  // branch_x: +inf when no step splits
      const double kf = floor((xb - x0) / h);
      const double margin = 2.0 + floor(8.0 * __DBL_EPSILON__ * (fabs(x0) + fabs(x1)) / h);
      if (!(margin <= 16.0)) {
        k_split = -1;
      } else if (kf - margin < (double)N && kf + margin >= 0.0) {  // false for NaN
        const int64_t c0 = kf - margin > 0.0 ? (int64_t)(kf - margin) : 0;
        const int64_t c1 = kf + margin < (double)(N - 1) ? (int64_t)(kf + margin) : N - 1;
#pragma nounroll
        for (int64_t c = c0; c <= c1; ++c) {
          const double xc = x0 + (double)c * h;
          if (xc < xb && xb <= xc + h) {
            k_split = c;
            break;
          }
        }
      }
    }
    // Split-free waves (LZQ_ODE_NOSPLITVAR): when no lane of the wave has a split step in this
    // launch's range (the window does not reach T = m/3, or the split lies in another
    // continuation launch), the <kNoSplit> variant steps the wave: the same operations with the
    // split paths compiled out, whose mere presence costs ~11% of a stiff / Riccati step
    // (register pressure).  Both variants evaluate the same wave-uniform predicate.
    if (!kLin && LZQ_ODE_NOSPLITVAR) {
      const bool lane_ns = k_split == INT64_MAX || (k_split >= 0 && (k_split + 1 < k_begin || k_split >= k_stop));
      if (__all(lane_ns) != kNoSplit) return;
      // whole-wave cooperative, one table, one Gamma_wash: ode_riccati_kernel steps it, split steps
      // included unless the x rounding makes the split search unreliable (k_split = -1: every step
      // takes the general path here) -- LZQ_ODE_RICVAR; the same predicate there, on the same values
      if (LZQ_ODE_RICVAR && !kChiOnly && G == 64 && !tab_vary && rec_shared && __all(k_split != -1)) return;
    }
    const int64_t block = coop ? G : N;
    for (int64_t kb = k_begin; kb < k_stop; kb += block) {
      const int64_t kend = kb + block < k_stop ? kb + block : k_stop;
      if (coop) {
        const int64_t kl = kb + (lane - seg);
        if (kl < kend) {
          const double xk = x0 + (double)kl * h;
          StageBase bs[3];
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            bs[j] = (kChiOnly && !o.deplete) ? ode_stage_chi_base(o, xk + R.c[j] * h)
                                             : ode_stage_base(o, w, xk + R.c[j] * h);
            s_base[wv][lane][j] = bs[j];
          }
          if (LZQ_ODE_YBREC && !kChiOnly && rec_shared) {
            // beta_j as stage_scale forms it (Gamma_wash * base), a_j the base: the step map (its d
            // is this lane's; a table-varying segment's lanes form theirs from W and id)
            const double beta[3] = {o.gamma_w * bs[0].beta, o.gamma_w * bs[1].beta, o.gamma_w * bs[2].beta};
            const double a[3] = {bs[0].a, bs[1].a, bs[2].a};
            const YbRec yr = yb_rec(hA, beta, a);
            s_rcd[LZQ_ODE_YBREC && !kChiOnly ? wv : 0][lane] = {yr.c, yr.d};
            s_rw[LZQ_ODE_YBREC && !kChiOnly ? wv : 0][lane] = {{yr.W[0], yr.W[1], yr.W[2]}, yr.id};
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      int64_t k = kb;
      double kd = (double)kb;  // (double)k, carried: an exact double counter instead of a 64-bit conversion per step
      while (k < kend && !done) {
        if (lin_fast && !prev_split) {
          // the block's regular steps up to its next split step in one tight loop
          const int64_t kg = k_split < 0 ? k : (k_split >= k && k_split < kend ? k_split : kend);
          const int nf = (int)(kg - k);
          if (nf > 0) {
            const int r0 = seg + (int)(k - kb);
            const YbCD* rr = &s_rcd[LZQ_ODE_YBREC && !kChiOnly ? wv : 0][r0];
            const YbW* rw = &s_rw[LZQ_ODE_YBREC && !kChiOnly ? wv : 0][r0];
            if (tab_vary) {  // each step's a_j from this lane's table, then its own d
              // T falls with x, so the rows' spline intervals run from the first row's stage 0
              // down to the last row's stage 2; when they are one interval (the rule on long
              // windows), this lane's four coefficients are read once for the run instead of per
              // stage (spline_at's operations on the same values)
              const int k_hi = s_base[wv][r0][0].k, k_lo = s_base[wv][r0 + nf - 1][2].k;
              double cc[4] = {0.0, 0.0, 0.0, 0.0};
              if (k_hi == k_lo) {
#pragma unroll
                for (int q = 0; q < 4; ++q) cc[q] = w[4 * k_hi + q];
              }
              for (int jj = 0; jj < nf; ++jj) {
                double a[3];
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                  const StageBase& b = s_base[wv][r0 + jj][j];
                  a[j] = (k_hi == k_lo ? spline_cubic(cc, b.s) : spline_at(w, b.s, b.k)) * b.ap;
                }
                YB = __builtin_fma(rr[jj].c, YB, o.Pf * yb_d(rw[jj], a));
                if (o.deplete) {
                  double acc = Ychi;
#pragma unroll
                  for (int j = 0; j < 3; ++j) acc = __builtin_fma(-hA.a[2][j], o.Pf * a[j], acc);
                  Ychi = acc;
                }
              }
            } else if (o.deplete) {
              for (int jj = 0; jj < nf; ++jj) {
                YB = __builtin_fma(rr[jj].c, YB, o.Pf * rr[jj].d);
                double acc = Ychi;
#pragma unroll
                for (int j = 0; j < 3; ++j) acc = __builtin_fma(-hA.a[2][j], o.Pf * s_base[wv][r0 + jj][j].a, acc);
                Ychi = acc;
              }
            } else {
              // the rows in batches of 8: their LDS reads are independent of Y_B, so all eight are
              // issued before the chain of fmas needs the first
              int jj = 0;
              for (; jj + 8 <= nf; jj += 8) {
                YbCD q[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) q[u] = rr[jj + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) YB = __builtin_fma(q[u].c, YB, o.Pf * q[u].d);
              }
              for (; jj < nf; ++jj) YB = __builtin_fma(rr[jj].c, YB, o.Pf * rr[jj].d);
            }
            k = kg;
            kd = (double)kg;
          }
          if (k >= kend) break;
        }
        const double xk = x0 + (LZQ_ODE_KD ? kd : (double)k) * h;
        // (kNoSplit: no step of this launch splits on any lane of the wave -- the split paths compile away)
        const bool split = !kNoSplit && xk < xb && xb <= xk + h;  // the last stage (x = xk + h) would see the other branch
        const double xa = split ? xb_below : xk + h;
        double YB_prev = YB;
        bool ok = true;
        const double Ystart = Ychi;
        bool use_guess = false;
        if (riccati && have && !split && pred_step(k)) {
          // the Riccati stage system has a second (unstable, other-sign) root: a predicted start
          // is used only when it stays within 25% of Y_chi, where Newton converges to the same
          // root as from Y_chi itself (an extrapolation across a fast transient can overshoot)
          double g[3];
          use_guess = true;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            g[j] = fma_s(Zs[2], kRadauPred[j][3], fma_s(Zs[1], kRadauPred[j][2],
                                                        fma_s(Zs[0], kRadauPred[j][1], kRadauPred[j][0] * Yp)));
            use_guess = use_guess && fabs(g[j] - Ychi) <= 0.25 * fabs(Ychi);
          }
#pragma unroll
          for (int j = 0; j < 3; ++j) Zs[j] = g[j];
        }
        if (xa > xk) {
          const double hs = split ? xa - xk : h;
          OdeStage sg[3];
          if (coop && !split) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              StageBase b = s_base[wv][seg + (k - kb)][j];
              if (!(kChiOnly && !o.deplete)) b.a = row_a(b);
              sg[j] = (kChiOnly && !o.deplete) ? chi_scale(o, b) : stage_scale(o, b);
            }
          } else {
#pragma unroll
            for (int j = 0; j < 3; ++j)
              sg[j] = (kChiOnly && !o.deplete) ? ode_stage_chi(o, xk + R.c[j] * hs) : ode_stage(o, w, xk + R.c[j] * hs);
          }
          if (riccati && !split && !pred_step(k)) use_guess = block_guess(R, hs, sg, Ychi, Zs);
          if (LZQ_ODE_YBREC && !kChiOnly) {  // Y_B by its step map, then Y_chi alone
            YbCD r;
            if (rec_shared && !split) {
              r = s_rcd[LZQ_ODE_YBREC && !kChiOnly ? wv : 0][seg + (k - kb)];
              if (tab_vary) {
                const double a[3] = {sg[0].a, sg[1].a, sg[2].a};
                r.d = yb_d(s_rw[LZQ_ODE_YBREC && !kChiOnly ? wv : 0][seg + (k - kb)], a);
              }
            } else {
              const YbRec yr = yb_rec(split ? radau_h(R, hs) : hA, sg);
              r = {yr.c, yr.d};
            }
            YB = __builtin_fma(r.c, YB, o.Pf * r.d);
            ok = radau_step<false>(split ? radau_h(R, hs) : hA, sg, Ychi, YB, Zs, use_guess);
          } else {
            ok = radau_step<!kChiOnly>(split ? radau_h(R, hs) : hA, sg, Ychi, YB, Zs, use_guess);
          }
        }
        if (ok && split && xk + h > xb) {
          const double hs = (xk + h) - xb;
          OdeStage sg[3];
          YB_prev = YB;
#pragma unroll
          for (int j = 0; j < 3; ++j)
            sg[j] = (kChiOnly && !o.deplete) ? ode_stage_chi(o, xb + R.c[j] * hs) : ode_stage(o, w, xb + R.c[j] * hs);
          if (LZQ_ODE_YBREC && !kChiOnly) {
            const YbRec r = yb_rec(radau_h(R, hs), sg);  // the split step's second part
            YB = __builtin_fma(r.c, YB, o.Pf * r.d);
            ok = radau_step<false>(radau_h(R, hs), sg, Ychi, YB, Zs, false);
          } else {
            ok = radau_step<!kChiOnly>(radau_h(R, hs), sg, Ychi, YB, Zs, false);
          }
        }
        have = !split;   // the predictor needs a full regular step behind it
        prev_split = split;
        Yp = Ystart;
        if (!ok) {
          YB = YB_prev;  // report the state at the start of the failed step, like sol.y[:, -1] (fpy:408-410)
          st = LZQ_ODE_NEWTON;
          done = true;
        }
        ++k;
        kd += 1.0;
      }
      if (coop) __builtin_amdgcn_wave_barrier();  // every lane is done with this block's table
    }
    if (done) finished = true;
    if (!finished && real) {  // save the state for the next launch
      OdeState sv;
      sv.Ychi = Ychi;
      sv.YB = YB;
      // the predictor's data (only sigma_v != 0 lanes read it; kLin's have sigma_v = 0)
      sv.Yp = kLin ? Ychi : Yp;
      sv.Z[0] = kLin ? Ychi : Zs[0];
      sv.Z[1] = kLin ? Ychi : Zs[1];
      sv.Z[2] = kLin ? Ychi : Zs[2];
      sv.status = kOdeInProgress;
      sv.have = !kLin && have ? 1 : 0;
      state[i] = sv;
    }
  }
  if (!finished) return;
  if (cont && real) state[i].status = st;
  if (st == LZQ_ODE_OK || st == LZQ_ODE_NEWTON) {  // fpy:412-417
    const double nB0 = YB * kS0M3, nDM0 = Ychi * kS0M3;
    r.Y_B = YB;
    r.Y_chi = Ychi;
    r.rho_B_kg_m3 = nB0 * kMProtonKg;
    r.rho_DM_kg_m3 = nDM0 * (m * kGeVToKg);
    r.DM_over_B = r.rho_DM_kg_m3 / pymax(r.rho_B_kg_m3, 1e-300);
  }
#ifdef LZQ_ODE_COOP_DEBUG
  r.P_used = dbg_coop;  // debug builds only: the cooperative segment width G (64 = whole wave), 0 = per-lane
#endif
  if (!real) return;
  out[i] = r;
  if (status) status[i] = st;
}

// ---------------------------------------------------------------------------------------
// ode_riccati_kernel (LZQ_ODE_RICVAR): the <kNoSplit> variant's steps for its most common wave,
// a whole 64-lane cooperative segment (G = 64) on one spline table with one Gamma_wash and no
// split step in the launch -- the Riccati sweeps over sigma_v, P, flux, deplete (and m_chi
// once grouped).  Every lane of such a wave agrees in everything ode_stage_base reads, so those
// per-point constants, the window, N, h, hA and the table pointer are wave-uniform and live in
// SGPRs (readfirstlane); the LDS rows hold only what a lane's step reads (lam, E2, a per stage
// and the Y_B step map: 88 B instead of 216 B per step); and the per-lane and split paths are
// not compiled in.  That is what keeps the kernel at LZQ_RIC_MIN_WAVES waves per SIMD against the
// general variant's 2 (VGPRs and LDS both): a step is a serial Newton chain, and more waves hide
// its latency.  The operations are the general path's, in the same order (ode_stage_base,
// stage_scale's products, yb_rec, radau_step<false>), so the bits are the same
// (tests/test_gpu_ode.py mode-independence tests).  Every launch runs every variant; each steps
// only its own waves.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ double ode_uniform(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

struct RicRow {
  double lam[3], E2[3], a[3];  // StageBase lam, E2, a of the step's three stages
};

#ifndef LZQ_RIC_KRELOAD
#define LZQ_RIC_KRELOAD 1  // ode_riccati_kernel's lean loop reloads the predictor constants per step (SGPR room)
#endif
#ifndef LZQ_RIC_V4
#define LZQ_RIC_V4 1  // ric_newton's dmax without the +0 start (same tests; see there)
#endif
#ifndef LZQ_RIC_LEAN
#define LZQ_RIC_LEAN 1  // ode_riccati_kernel's regular steps through ric_step (round 6): radau_step<false>'s operations, lean registers
#endif

// ode_riccati_kernel's cooperative fill of one row (step at xk): the stage bases, beta_j and the
// Y_B step map, with the operations of the kernel's inline fill (ode_stage_base, yb_rec on
// radau_h(R, h)).  Out of line: the fill runs once per 64 steps, and inlined its constants (the
// exponential's and the spline's) and temporaries were hoisted across the step loop, where they
// took the registers the Newton iteration needs (spills in the hot loop).
__device__ __noinline__ void ric_fill(const OdePoint* ou, const double* __restrict__ wu, double xk, double h,
                                      RicRow* row, double* bt, YbCD* rcd) {
  const Radau R = radau_tableau();
#pragma unroll 1
  for (int j = 0; j < 3; ++j) {
    const double cj = j == 0 ? R.c[0] : (j == 1 ? R.c[1] : R.c[2]);
    const StageBase bs = ode_stage_base(*ou, wu, xk + cj * h);
    row->lam[j] = bs.lam;
    row->E2[j] = bs.E2;
    row->a[j] = bs.a;
    bt[j] = ou->gamma_w * bs.beta;
  }
  const double beta[3] = {bt[0], bt[1], bt[2]}, a[3] = {row->a[0], row->a[1], row->a[2]};
  const YbRec yr = yb_rec(radau_h(R, h), beta, a);
  *rcd = {yr.c, yr.d};
}

// radau_step<false>'s transformed Newton iteration (newton_j) for ode_riccati_kernel: the same
// operations in the same order, with the six off-diagonal constant products of the adjugate held in
// VGPRs (pv, pinned once per launch) instead of copied from SGPRs into a VGPR per entry per iteration
// (fma_neg_s takes one constant as its SGPR operand, the other must be a VGPR).
// pv = kRadauAinvP[1, 2, 3, 5, 6, 7].
struct RicJ {
  double b[3][3], id;
};
template <bool kDep>
__device__ __forceinline__ bool ric_newton(double (&Z)[3], double Y0, const double (&hl)[3], const double (&hl2)[3],
                                           const double (&hS)[3], const double (&E2)[3], const double (&pv)[6],
                                           RicJ& J, const bool reuse, bool& near) {
#define FMA __builtin_fma
  double d[3], r[3], k[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    // without depletion hS_j = h * (+0) = +0, and fma(a, b, -0) rounds a * b exactly as the product
    // does (zero products keep their sign: +0 + -0 = +0, -0 + -0 = -0): the same r_j
    r[j] = kDep ? FMA(-hl[j], FMA(Z[j], Z[j], -E2[j]), -hS[j]) : -hl[j] * FMA(Z[j], Z[j], -E2[j]);
    d[j] = Z[j] - Y0;
    k[j] = FMA(hl2[j], Z[j], kRadauAinv[j][j]);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
    r[i] = FMA(-kRadauAinv[i][2], d[2], FMA(-kRadauAinv[i][1], d[1], FMA(-kRadauAinv[i][0], d[0], r[i])));
  if (!reuse) {
    J.b[0][0] = FMA(k[1], k[2], -kRadauAinvP[0]), J.b[0][1] = fma_neg_s(k[2], kRadauAinv[0][1], pv[0]);
    J.b[0][2] = fma_neg_s(k[1], kRadauAinv[0][2], pv[1]), J.b[1][0] = fma_neg_s(k[2], kRadauAinv[1][0], pv[2]);
    J.b[1][1] = FMA(k[0], k[2], -kRadauAinvP[4]), J.b[1][2] = fma_neg_s(k[0], kRadauAinv[1][2], pv[3]);
    J.b[2][0] = fma_neg_s(k[1], kRadauAinv[2][0], pv[4]), J.b[2][1] = fma_neg_s(k[0], kRadauAinv[2][1], pv[5]);
    J.b[2][2] = FMA(k[0], k[1], -kRadauAinvP[8]);
    const double den = FMA(k[0], J.b[0][0], FMA(kRadauAinv[0][1], J.b[1][0], kRadauAinv[0][2] * J.b[2][0]));
    J.id = LZQ_ODE_NEWTON_RCP ? rcp_pos(den) : 1.0 / den;
  }
  double g[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) g[i] = FMA(J.b[i][0], r[0], FMA(J.b[i][1], r[1], J.b[i][2] * r[2])) * J.id;
#undef FMA
  double zmax = 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    Z[i] = Z[i] + g[i];
    zmax = fmax(zmax, fabs(Z[i]));
  }
  // newton_j's dmax = fmax(fmax(fmax(+0, |g0|), |g1|), |g2|) without the +0: the two differ only when
  // all three corrections are NaN (+0 there, NaN here), and both then fail "dmax > c zmax" (zmax >= 0),
  // so near and the convergence test are the same
  const double dmax = LZQ_RIC_V4 ? fmax(fmax(fabs(g[0]), fabs(g[1])), fabs(g[2]))
                                 : fmax(fmax(fmax(0.0, fabs(g[0])), fabs(g[1])), fabs(g[2]));
  near = !(dmax > 1e-3 * zmax);
  return !(dmax > 1e-15 * zmax);
}

// radau_step<false>(hA, sg, Ychi, YB, Zs, guess) for ode_riccati_kernel's regular steps, from the
// step's scaled stage data (lam_j, E2_j, S_j) and h; hA2 = hA.a[2][*] for the linear branch.  The
// same branches and iterates: the linear update, the peeled pair (the second simplified when the
// first correction was small), then -- only for a lane whose pair did not converge -- full
// iterations up to the 40th, and from Y_chi once more when the start was predicted.
// kDep = false: a wave with no depleting lane (S_j = +0 on every lane): the linear branch leaves
// Y_chi as it is (fma(-hA, +0, Y) = Y + -0 = Y, exactly) and hS is not formed (ric_newton).
template <bool kDep>
__device__ __forceinline__ bool ric_step(double h, const double (&hA2)[3], const double (&lam)[3],
                                         const double (&E2)[3], const double (&S)[3], const double (&pv)[6],
                                         double& Ychi, double (&Zs)[3], bool guess) {
  const bool nonlinear = lam[0] != 0.0 || lam[1] != 0.0 || lam[2] != 0.0;
  if (!nonlinear) {
    if (kDep) {
      double acc = Ychi;
#pragma unroll
      for (int j = 0; j < 3; ++j) acc = __builtin_fma(-hA2[j], S[j], acc);
      Ychi = acc;
    }
    return true;
  }
  const double Y0 = Ychi;
  double hl[3], hl2[3], hS[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    hl[j] = h * lam[j];
    hl2[j] = 2.0 * hl[j];
    hS[j] = kDep ? h * S[j] : 0.0;
  }
  double Z[3] = {guess ? Zs[0] : Y0, guess ? Zs[1] : Y0, guess ? Zs[2] : Y0};
  RicJ J;
  bool near = false;
  const bool c1 = ric_newton<kDep>(Z, Y0, hl, hl2, hS, E2, pv, J, false, near);
  const bool reuse = near;
  const bool c2 = ric_newton<kDep>(Z, Y0, hl, hl2, hS, E2, pv, J, reuse, near);
  bool ok = c1 || c2;
  if (!ok) {  // rare: radau_step's loop after the peeled pair, and its second attempt from Y0
#pragma nounroll
    for (int it = 2; it < 40 && !ok; ++it) ok = ric_newton<kDep>(Z, Y0, hl, hl2, hS, E2, pv, J, false, near);
    if (!ok && guess) {
      Z[0] = Y0;
      Z[1] = Y0;
      Z[2] = Y0;
#pragma nounroll
      for (int it = 0; it < 40 && !ok; ++it) ok = ric_newton<kDep>(Z, Y0, hl, hl2, hS, E2, pv, J, false, near);
    }
  }
  if (ok) {
    Zs[0] = Z[0];
    Zs[1] = Z[1];
    Zs[2] = Z[2];
    Ychi = Z[2];
  }
  return ok;
}

// kPhase: a wave whose split step (the T = m/3 branch) lies in this launch's range runs in three
// passes -- 0: the regular steps before it, 1: the split step and the next (ode_integrate_kernel's
// split-step code, each lane forming its own stages: two steps, so registers do not matter),
// 2: the regular steps after it -- with its state handed on in OdeState; so the regular-step
// kernels (0, 2) carry no split code.  A wave with no split in range runs in pass 0 alone.
template <int kPhase>
__global__ __launch_bounds__(kOdeBlock, kPhase == 1 ? 1 : LZQ_RIC_MIN_WAVES) void ode_riccati_kernel(
    const lzq_point* __restrict__ pts, const lzq_ode_params* __restrict__ ode, int64_t n,
    const int32_t* __restrict__ tidx, const double* __restrict__ ws, int64_t max_steps, lzq_yield* __restrict__ out,
    int32_t* __restrict__ status, int coop_on, int64_t k_lo, int64_t k_cnt, OdeState* __restrict__ state,
    const int32_t* __restrict__ skip) {
  __shared__ RicRow s_row[kOdeBlock / 64][64];
  __shared__ YbCD s_rcd[kOdeBlock / 64][64];
  __shared__ OdePoint s_pt[kOdeBlock / 64];
  __shared__ double s_beta[kOdeBlock / 64][64][3];  // the fill's beta_j (Gamma_wash * base)

  if (!LZQ_ODE_RICVAR || !LZQ_ODE_COOP || !coop_on) return;
  // --- the classification of ode_integrate_kernel<false, false, true>, on the same values ---
  const int64_t wave0 = (int64_t)blockIdx.x * kOdeBlock + (threadIdx.x & ~63);
  if (wave0 >= n) return;
  const int64_t i_self = (int64_t)blockIdx.x * kOdeBlock + threadIdx.x;
  const bool real = i_self < n;
  const int64_t i = real ? i_self : wave0;
  if (skip && skip[i]) return;
  const bool cont = state != nullptr, first = kPhase == 0 && (!cont || k_lo == 0);
  if (kPhase > 0 && !cont) return;  // passes 1 and 2 continue from pass 0's state
  if (cont && !first && state[i].status != kOdeInProgress) return;
  const lzq_point pt = pts[i];
  const OdePoint o = ode_point(pt, ode[i]);
  const double* w = ws + (tidx ? (int64_t)tidx[i] : i) * (int64_t)kOdeWS;
  if (!ode_grid_ok(o.T_lo, o.T_hi, o.stepT) || !ode_table_ok(w)) return;  // the general variant reports it
  const double m = o.m, T_p = o.Tp;
  const double x0 = m / o.T_hi, x1 = m / pymax(o.T_lo, 1e-30);
  const double x_p = m / pymax(T_p, 1e-30);
  const double max_step = pymin(pymin(fabs(x1 - x0) / 20000.0, x_p / 1000.0), 5e-4);
  if (!(max_step > 0.0)) return;
  const double steps = ceil(fabs(x1 - x0) / max_step);
  if (!(steps <= (double)max_steps)) return;
  if (__ballot(1) != ~0ull) return;  // a lane returned above: not a whole cooperative wave
  auto same = [](double v) { return __builtin_bit_cast(uint64_t, v) == __builtin_bit_cast(uint64_t, __shfl(v, 0, 64)); };
  const bool eq = same(o.m) && same(o.Tp) && same(o.B) && same(o.sig) && same(o.H0) && same(o.s0) && same(o.c_rel) &&
                  same(o.c_nr) && same(o.v0) && same(o.T_lo) && same(o.T_hi);
  if (!__all(eq)) return;                                                    // G < 64
  if (!__all(same(__builtin_bit_cast(double, w)))) return;                   // tab_vary
  if (!__all(same(o.gamma_w))) return;                                       // !rec_shared
  if (LZQ_ODE_LINFAST && __all(o.sigmav == 0.0)) return;                     // lin_wave
  const int64_t N = (int64_t)steps;
  const int64_t k_begin = cont ? k_lo : 0;
  const int64_t k_stop = cont ? (k_lo + k_cnt < N ? k_lo + k_cnt : N) : N;
  const double h = (x1 - x0) / (double)N;
  const double xb = branch_x(o, x0, x1);
  int64_t k_split = INT64_MAX;
  if (xb < INFINITY) {  // ode_integrate_kernel's search, verbatim
    const double kf = floor((xb - x0) / h);
    const double margin = 2.0 + floor(8.0 * __DBL_EPSILON__ * (fabs(x0) + fabs(x1)) / h);
    if (!(margin <= 16.0)) {
      k_split = -1;
    } else if (kf - margin < (double)N && kf + margin >= 0.0) {
      const int64_t c0 = kf - margin > 0.0 ? (int64_t)(kf - margin) : 0;
      const int64_t c1 = kf + margin < (double)(N - 1) ? (int64_t)(kf + margin) : N - 1;
#pragma nounroll
      for (int64_t c = c0; c <= c1; ++c) {
        const double xc = x0 + (double)c * h;
        if (xc < xb && xb <= xc + h) {
          k_split = c;
          break;
        }
      }
    }
  }
  if (!__all(k_split != -1)) return;  // x rounding comparable to h: the general variant's every-step test
  // the split step (xk < xb <= xk + h) of this wave: k_split, and k_split + 1 when a rounding splits
  // that one too (wave-uniform: x0, h and xb are); every other step is a regular one
  const int64_t ks = (int64_t)__builtin_bit_cast(uint64_t, ode_uniform(__builtin_bit_cast(double, k_split)));
  const double xbu = ode_uniform(xb), xb_below = nextafter(xbu, -INFINITY);
  // this pass's steps [pk_begin, pk_stop)
  const bool in_range = ks != INT64_MAX && !(ks + 1 < k_begin || ks >= k_stop);
  if (kPhase > 0 && !in_range) return;
  const int64_t ks_lo = ks > k_begin ? ks : k_begin, ks_hi = ks + 2 < k_stop ? ks + 2 : k_stop;
  const int64_t pk_begin = kPhase == 0 ? k_begin : (kPhase == 1 ? ks_lo : ks_hi);
  const int64_t pk_stop = kPhase == 0 ? (in_range ? ks_lo : k_stop) : (kPhase == 1 ? ks_hi : k_stop);
  // --- this wave is ours: the wave-uniform point constants in the wave's LDS slot (read by the
  // fill phase only), the window, h, hA and the table pointer in SGPRs ---
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) s_pt[wv] = o;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const OdePoint& ou = s_pt[wv];
  const double* wu = reinterpret_cast<const double*>(
      (uintptr_t)__builtin_bit_cast(uint64_t, ode_uniform(__builtin_bit_cast(double, (uint64_t)(uintptr_t)w))));
  const double x0u = ode_uniform(x0), hu = ode_uniform(h);
  const Radau R = radau_tableau();
  RadauH hA = radau_h(R, hu);
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) hA.a[a][b] = ode_uniform(hA.a[a][b]);
  // --- per-lane state (ode_integrate_kernel's) ---
  const double Pf = o.Pf, sigmav = o.sigmav;
  const int deplete = o.deplete;
  int st = LZQ_ODE_OK;
  double Ychi;
  if (pt.regime == LZQ_NONTHERMAL) {
    if (pt.has_Y_chi_init) Ychi = pt.Y_chi_init;
    else if (pt.has_n_chi_at_Tp) Ychi = pt.n_chi_at_Tp_GeV3 / pymax(s_entropy(T_p, pt.g_star_s), 1e-300);
    else Ychi = 1.0e-12;
  } else {
    Ychi = n_chi_eq(o.T_hi, m, pt.g_chi, pt.stats) / s_entropy(o.T_hi, pt.g_star_s);
  }
  double YB = 0.0;
  const bool riccati = LZQ_ODE_PREDICT && sigmav != 0.0;
  double Zs[3] = {Ychi, Ychi, Ychi}, Yp = Ychi;
  bool have = false, done = false;
  if (!first) {
    const OdeState sv = state[i];
    Ychi = sv.Ychi;
    YB = sv.YB;
    Yp = sv.Yp;
    Zs[0] = sv.Z[0];
    Zs[1] = sv.Z[1];
    Zs[2] = sv.Z[2];
    have = sv.have != 0;
  }
  const bool finished_here = pk_stop >= N;
  if (kPhase == 1) {
    // ode_integrate_kernel's steps, each lane on its own stages (ode_stage: the shared base and its
    // products; the same values the cooperative rows hold): the split step in two parts around the
    // branch point without the predictor, a regular step with it
    for (int64_t k = pk_begin; k < pk_stop && !done; ++k) {
      const double xk = x0u + (double)k * hu;
      const bool split = xk < xbu && xbu <= xk + hu;
      const double xa = split ? xb_below : xk + hu;
      double YB_prev = YB;
      bool ok = true;
      const double Ystart = Ychi;
      bool use_guess = false;
      if (riccati && have && !split && pred_step(k)) {
        double g[3];
        use_guess = true;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          g[j] = fma_s(Zs[2], kRadauPred[j][3], fma_s(Zs[1], kRadauPred[j][2],
                                                      fma_s(Zs[0], kRadauPred[j][1], kRadauPred[j][0] * Yp)));
          use_guess = use_guess && fabs(g[j] - Ychi) <= 0.25 * fabs(Ychi);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) Zs[j] = g[j];
      }
      auto part = [&](double xs, double hs, bool guess, bool block_start) {
        const RadauH hAs = radau_h(R, hs);
        OdeStage sg[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const StageBase b = ode_stage_base(ou, wu, xs + R.c[j] * hs);
          sg[j].alpha = Pf * b.a;
          sg[j].S = deplete ? sg[j].alpha : 0.0;
          sg[j].lam = sigmav * b.lam;
          sg[j].E2 = b.E2;
          sg[j].beta = ou.gamma_w * b.beta;
          sg[j].a = b.a;
        }
        const YbRec yr = yb_rec(hAs, sg);
        YB = __builtin_fma(yr.c, YB, Pf * yr.d);
        if (block_start) guess = block_guess(R, hs, sg, Ychi, Zs);
        return radau_step<false>(hAs, sg, Ychi, YB, Zs, guess);
      };
      if (xa > xk) ok = part(xk, split ? xa - xk : hu, use_guess, riccati && !split && !pred_step(k));
      if (ok && split && xk + hu > xbu) {
        YB_prev = YB;
        ok = part(xbu, (xk + hu) - xbu, false, false);
      }
      have = !split;
      Yp = Ystart;
      if (!ok) {
        YB = YB_prev;
        st = LZQ_ODE_NEWTON;
        done = true;
      }
    }
  }
  // ric_step's loop constants: hA's last row (the linear branch) and the adjugate's off-diagonal
  // constant products, pinned in VGPRs (see ric_newton)
  const double hA2[3] = {hA.a[2][0], hA.a[2][1], hA.a[2][2]};
  const bool dep_any = !__all(deplete == 0);  // wave-uniform: some lane depletes its source
  double pv[6] = {kRadauAinvP[1], kRadauAinvP[2], kRadauAinvP[3], kRadauAinvP[5], kRadauAinvP[6], kRadauAinvP[7]};
  if (LZQ_RIC_LEAN && kPhase != 1) {
#pragma unroll
    for (int q = 0; q < 6; ++q) asm volatile("" : "+v"(pv[q]));
  }
  for (int64_t kb = pk_begin; kPhase != 1 && kb < pk_stop; kb += 64) {
    const int64_t kend = kb + 64 < pk_stop ? kb + 64 : pk_stop;
    uint64_t xok = 0;
    {  // lane l: the stage ingredients and Y_B step map of step kb + l (the cooperative fill)
      const int64_t kl = kb + lane;
      if (LZQ_RIC_LEAN) {
        // the steps' x guard (xk + h > xk, wave-uniform per step) as one mask, from the fill's xk
        const double xk = x0u + (double)kl * hu;
        xok = __ballot(kl < kend && xk + hu > xk);
      }
      if (kl < kend) {
        if (LZQ_RIC_LEAN) {
          ric_fill(&s_pt[wv], wu, x0u + (double)kl * hu, hu, &s_row[wv][lane], s_beta[wv][lane], &s_rcd[wv][lane]);
        } else {
        const double xk = x0u + (double)kl * hu;
        RicRow& row = s_row[wv][lane];
        double* bt = s_beta[wv][lane];
#pragma unroll 1
        for (int j = 0; j < 3; ++j) {  // one stage at a time (the fill's register peak), parked in LDS
          const double cj = j == 0 ? R.c[0] : (j == 1 ? R.c[1] : R.c[2]);  // (a dynamic index would go to scratch)
          const StageBase bs = ode_stage_base(ou, wu, xk + cj * hu);
          row.lam[j] = bs.lam;
          row.E2[j] = bs.E2;
          row.a[j] = bs.a;
          bt[j] = ou.gamma_w * bs.beta;
        }
        const double beta[3] = {bt[0], bt[1], bt[2]}, a[3] = {row.a[0], row.a[1], row.a[2]};
        const YbRec yr = yb_rec(hA, beta, a);
        s_rcd[wv][lane] = {yr.c, yr.d};
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    double kd = (double)kb;
    // the block's predictor-free step (k = 0 mod LZQ_ODE_PRED_BLOCK) is row rz (a row past the
    // block when it has none: pass 2 starts after the split steps, unaligned): one wave-uniform
    // compare per step.  (Peeling row 0 of aligned blocks, with pass 1 run on to the next block,
    // measured slower: profiles/round5/ablate_ode_pred_block.json.)
    const int rz = (int)((-kb) & (int64_t)(LZQ_ODE_PRED_BLOCK - 1));
    // a wave with no depleting lane runs the loop without the source products (ric_step<false>)
    auto lean_steps = [&](auto dep_tag) {
    constexpr bool kDep = decltype(dep_tag)::value;
    // LZQ_RIC_V4: a uniform trip count, each lane's steps under !done (a lane whose Newton iteration
    // failed stops there, as in the loop below)
    const int nr = (int)(kend - kb);
    for (int r = 0; r < nr && (LZQ_RIC_V4 || !done); ++r) {
      // the same step as the loop below: the row is read first (its LDS latency under the
      // predictor), the x guard is the fill's mask bit, the step index needs no counter
      const RicRow row = s_row[wv][r];
      const YbCD rc = s_rcd[wv][r];
      if (done) continue;
      const double YB_prev = YB;
      const double Ystart = Ychi;
      bool use_guess = false;
      if (riccati && have && r != rz) {
        // the predictor's 12 constants are read from the constant cache each step (scalar loads
        // through an opaque pointer) instead of held in 24 SGPRs across the loop (LZQ_RIC_KRELOAD)
        const __attribute__((address_space(4))) double* kp =
            (const __attribute__((address_space(4))) double*)&kRadauPred[0][0];
        if (LZQ_RIC_KRELOAD) asm volatile("" : "+s"(kp));
        double g[3];
        use_guess = true;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          g[j] = fma_s(Zs[2], kp[4 * j + 3], fma_s(Zs[1], kp[4 * j + 2], fma_s(Zs[0], kp[4 * j + 1], kp[4 * j] * Yp)));
          use_guess = use_guess && fabs(g[j] - Ychi) <= 0.25 * fabs(Ychi);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) Zs[j] = g[j];
      }
      bool ok = true;
      if ((xok >> r) & 1) {
        double lam[3], E2[3], S[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          S[j] = kDep ? (deplete ? Pf * row.a[j] : 0.0) : 0.0;
          lam[j] = sigmav * row.lam[j];
          E2[j] = row.E2[j];
        }
        YB = __builtin_fma(rc.c, YB, Pf * rc.d);
        if (riccati && r == rz) {
          OdeStage sg[3];
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            sg[j].lam = lam[j];
            sg[j].E2 = E2[j];
            sg[j].S = S[j];
          }
          use_guess = block_guess(R, hu, sg, Ychi, Zs);
        }
        ok = ric_step<kDep>(hu, hA2, lam, E2, S, pv, Ychi, Zs, use_guess);
      }
      have = true;
      Yp = Ystart;
      if (!ok) {
        YB = YB_prev;
        st = LZQ_ODE_NEWTON;
        done = true;
      }
    }
    };
    if (LZQ_RIC_LEAN) {
      if (dep_any) lean_steps(std::true_type{});
      else lean_steps(std::false_type{});
    }
    for (int r = 0; !LZQ_RIC_LEAN && r < (int)(kend - kb) && !done; ++r) {
      const double xk = x0u + kd * hu;
      kd += 1.0;
      const double YB_prev = YB;
      const double Ystart = Ychi;
      bool use_guess = false;
      if (riccati && have && r != rz) {  // the Radau5 predictor, as ode_integrate_kernel
        double g[3];
        use_guess = true;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          g[j] = fma_s(Zs[2], kRadauPred[j][3], fma_s(Zs[1], kRadauPred[j][2],
                                                      fma_s(Zs[0], kRadauPred[j][1], kRadauPred[j][0] * Yp)));
          use_guess = use_guess && fabs(g[j] - Ychi) <= 0.25 * fabs(Ychi);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) Zs[j] = g[j];
      }
      bool ok = true;
      if (xk + hu > xk) {
        const RicRow& row = s_row[wv][r];
        OdeStage sg[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {  // stage_scale's products (beta is not read by radau_step<false>)
          sg[j].alpha = Pf * row.a[j];
          sg[j].S = deplete ? sg[j].alpha : 0.0;
          sg[j].lam = sigmav * row.lam[j];
          sg[j].E2 = row.E2[j];
          sg[j].beta = 0.0;
          sg[j].a = row.a[j];
        }
        const YbCD rc = s_rcd[wv][r];
        YB = __builtin_fma(rc.c, YB, Pf * rc.d);
        if (riccati && r == rz) use_guess = block_guess(R, hu, sg, Ychi, Zs);
        if (LZQ_RIC_LEAN) {
          const double lam[3] = {sg[0].lam, sg[1].lam, sg[2].lam}, E2[3] = {sg[0].E2, sg[1].E2, sg[2].E2},
                       S[3] = {sg[0].S, sg[1].S, sg[2].S};
          ok = ric_step<true>(hu, hA2, lam, E2, S, pv, Ychi, Zs, use_guess);
        } else {
          ok = radau_step<false>(hA, sg, Ychi, YB, Zs, use_guess);
        }
      }
      have = true;
      Yp = Ystart;
      if (!ok) {
        YB = YB_prev;
        st = LZQ_ODE_NEWTON;
        done = true;
      }
    }
    __builtin_amdgcn_wave_barrier();  // every lane is done with this block's rows
  }
  const bool finished = finished_here || done;
  if (!finished) {
    if (real) {
      OdeState sv;
      sv.Ychi = Ychi;
      sv.YB = YB;
      sv.Yp = Yp;
      sv.Z[0] = Zs[0];
      sv.Z[1] = Zs[1];
      sv.Z[2] = Zs[2];
      sv.status = kOdeInProgress;
      sv.have = have ? 1 : 0;
      state[i] = sv;
    }
    return;
  }
  if (cont && real) state[i].status = st;
  const double nan = __builtin_nan("");
  lzq_yield res = {nan, nan, nan, nan, nan, pt.P_chi_to_B};
  const double nB0 = YB * kS0M3, nDM0 = Ychi * kS0M3;  // fpy:412-417 (st is OK or NEWTON here)
  res.Y_B = YB;
  res.Y_chi = Ychi;
  res.rho_B_kg_m3 = nB0 * kMProtonKg;
  res.rho_DM_kg_m3 = nDM0 * (m * kGeVToKg);
  res.DM_over_B = res.rho_DM_kg_m3 / pymax(res.rho_B_kg_m3, 1e-300);
  if (!real) return;
  out[i] = res;
  if (status) status[i] = st;
}

// ---------------------------------------------------------------------------------------
// Time-parallel integration of a few points (lzq_ode_integrate_tp): multiple shooting.
// A point's N fixed steps are cut into M intervals of L steps; node m holds the integrator's
// state at the start of interval m (Y_chi, Y_B and the predictor's data).  Each iteration
// (1) integrates every interval from its node, one lane per interval, with the per-lane steps
// of ode_integrate_kernel (same stages, Y_B step map, Radau step, split step, predictor), and
// records the end state F_m and its derivatives D_m = dY_chi_end/dY_chi_start (the product of
// the steps' dZ_3/dY_0, the implicit function theorem on the converged stage system) and
// C_m = dY_B_end/dY_B_start (the product of the Y_B step maps' c); (2) applies Newton's update to
// the nodes: with residuals r_m = F_m - s_{m+1}, the corrections solve the linear recurrence
// d_{m+1} = D_m d_m + r_m, d_0 = 0 -- a block scan of affine maps.  Node M is the point's final
// state.  Y_B's recurrence is affine (one update makes it exact up to rounding); Y_chi's is the
// Riccati map, for which Newton converges quadratically once the nodes are close.  The fixed
// point is the sequential trajectory: at convergence every node is its interval predecessor's
// end state, so the result differs from ode_integrate_kernel's only by rounding (the nodes are
// formed as s + d instead of being carried), which the contractive or neutral dynamics keep at
// the ~1e-14 level (tests/test_gpu_ode_tp.py).  A point whose iteration does not converge within
// the budget, or one whose interval hits a Newton failure, is integrated sequentially instead.
// ---------------------------------------------------------------------------------------
// The integrator's state at the start of an interval is (Y_chi, Y_B) alone: intervals are whole
// predictor blocks (LZQ_ODE_PRED_BLOCK), whose first step does not read the predictor's data.
struct TpNode {
  double Ychi, YB;
};
struct TpEnd {  // an interval's end state from its start node, and its derivatives
  double Ychi, YB;
  double D;  // dY_chi(end) / dY_chi(start)
  double C;  // dY_B(end) / dY_B(start)
  int32_t exact;  // every step took the Radau step (0: a Newton failure was bridged, see tp_bridge)
  int32_t pad;
};
struct TpCtl {
  int64_t N, M;     // the point's steps and intervals
  int64_t L;        // its interval length (steps)
  double err;       // the last update's largest relative correction
  int32_t phase;    // kTpIter, kTpDone (converged, to be stitched), kTpExact (stitched: the result is
                    // written), kTpFallback (sequential path)
  int32_t iters;    // Newton updates applied
  int32_t riccati;  // sigma_v != 0: Y_chi's map is nonlinear (the update is safeguarded)
  int32_t pad;
};
constexpr int32_t kTpIter = 0, kTpDone = 1, kTpFallback = 2;

// ode_integrate_kernel's prologue, in its order: status, window, step count, h, initial Y_chi.
struct OdeSetup {
  OdePoint o;
  double x0, x1, h, Ychi0;
  int64_t N;
  int st;
};
__device__ __forceinline__ OdeSetup ode_setup(const lzq_point& pt, const lzq_ode_params& od, const double* w,
                                              int64_t max_steps) {
  OdeSetup S;
  S.o = ode_point(pt, od);
  const OdePoint& o = S.o;
  S.st = ode_grid_ok(o.T_lo, o.T_hi, o.stepT) ? (ode_table_ok(w) ? LZQ_ODE_OK : LZQ_ODE_BAD_TABLE) : LZQ_ODE_BAD_GRID;
  const double m = o.m, T_p = o.Tp;
  S.x0 = m / o.T_hi;
  S.x1 = m / pymax(o.T_lo, 1e-30);
  if (pt.regime == LZQ_NONTHERMAL) {
    if (pt.has_Y_chi_init) S.Ychi0 = pt.Y_chi_init;
    else if (pt.has_n_chi_at_Tp) S.Ychi0 = pt.n_chi_at_Tp_GeV3 / pymax(s_entropy(T_p, pt.g_star_s), 1e-300);
    else S.Ychi0 = 1.0e-12;
  } else {
    S.Ychi0 = n_chi_eq(o.T_hi, m, pt.g_chi, pt.stats) / s_entropy(o.T_hi, pt.g_star_s);
  }
  const double x_p = m / pymax(T_p, 1e-30);
  const double max_step = pymin(pymin(fabs(S.x1 - S.x0) / 20000.0, x_p / 1000.0), 5e-4);
  double steps = 0.0;
  if (S.st == LZQ_ODE_OK) {
    if (!(max_step > 0.0)) S.st = LZQ_ODE_BAD_STEP;
    else {
      steps = ceil(fabs(S.x1 - S.x0) / max_step);
      if (!(steps <= (double)max_steps)) S.st = LZQ_ODE_TOO_MANY_STEPS;
    }
  }
  S.N = S.st == LZQ_ODE_OK ? (int64_t)steps : 0;
  S.h = S.N > 0 ? (S.x1 - S.x0) / (double)S.N : 0.0;
  return S;
}

// dZ_3/dY_0 of a converged Riccati stage system Z = Y_0 1 + hA f(Z), f_j = -lam_j (Z_j^2 - E2_j) - S_j:
// (A^-1 + diag(2 h lam_j Z_j)) dZ = A^-1 1, the transformed Newton matrix of radau_step.
__device__ __forceinline__ double tp_dz3(double h, const OdeStage (&sg)[3], const double (&Z)[3]) {
  double k[3], q[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    k[j] = kRadauAinv[j][j] + 2.0 * (h * sg[j].lam) * Z[j];
    q[j] = (kRadauAinv[j][0] + kRadauAinv[j][1]) + kRadauAinv[j][2];
  }
  const double a01 = kRadauAinv[0][1], a02 = kRadauAinv[0][2], a10 = kRadauAinv[1][0];
  const double a12 = kRadauAinv[1][2], a20 = kRadauAinv[2][0], a21 = kRadauAinv[2][1];
  const double b20 = a10 * a21 - k[1] * a20, b21 = a01 * a20 - k[0] * a21, b22 = k[0] * k[1] - a01 * a10;
  const double b00 = k[1] * k[2] - a12 * a21, b10 = a12 * a20 - a10 * k[2];
  const double det = k[0] * b00 + a01 * b10 + a02 * b20;
  const double dz = (b20 * q[0] + b21 * q[1] + b22 * q[2]) / det;
  return isfinite(dz) ? dz : 0.0;  // overflowing stiff stages: the map contracts there
}

// One block per point: ctl, and every node at the initial state (node 0 is ode_integrate_kernel's
// start; the others are the first guess).  Points the iteration does not take (a status other
// than OK, fewer than two intervals) go to the fallback.
__global__ __launch_bounds__(256) void ode_tp_init_kernel(const lzq_point* __restrict__ pts,
                                                          const lzq_ode_params* __restrict__ ode,
                                                          const int32_t* __restrict__ tidx,
                                                          const double* __restrict__ ws, int64_t max_steps, int64_t L,
                                                          int64_t Mmax, TpNode* __restrict__ nodes,
                                                          TpCtl* __restrict__ ctl) {
  const int64_t p = blockIdx.x;
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps);
  // the point's own interval length: L steps, more when its N would need over Mmax intervals
  // (max_steps only sizes the node arrays)
  // (a whole number of predictor blocks, LZQ_ODE_PRED_BLOCK: the exact stitching needs interval starts
  // whose first step does not read the predictor)
  constexpr int64_t B = LZQ_ODE_PRED_BLOCK;
  const int64_t Lp = S.N > L * Mmax ? ((S.N + Mmax - 1) / Mmax + B - 1) / B * B : L;
  const int64_t M = S.st == LZQ_ODE_OK ? (S.N + Lp - 1) / Lp : 0;
  const bool go = S.st == LZQ_ODE_OK && M >= 2 && M <= Mmax;
  if (threadIdx.x == 0) ctl[p] = TpCtl{S.N, M, Lp, 0.0, go ? kTpIter : kTpFallback, 0, S.o.sigmav != 0.0 ? 1 : 0, 0};
  if (!go) return;
  TpNode* nd = nodes + p * (Mmax + 1);
  for (int64_t m = threadIdx.x; m <= M; m += blockDim.x)
    nd[m] = TpNode{S.Ychi0, 0.0};
}

// A Riccati step whose Newton iteration fails -- possible only from a start far above the
// trajectory, as in the first iterations -- is bridged by backward Euler at the step's end,
// Y1 = Y0 - h lam (Y1^2 - E2) - h S, whose positive root 2c / (1 + sqrt(1 + 4 h lam c)),
// c = Y0 + h lam E2 - h S, exists for every start (unconditionally stable, no iteration): the
// interval still returns an end state and a derivative to improve the nodes with, and is marked
// inexact, so the iteration cannot converge while any interval needs the bridge.
__device__ __forceinline__ double tp_bridge(double Y0, double h, const OdeStage& s3, double& dY1) {
  const double hl = h * s3.lam;
  const double c = Y0 + hl * s3.E2 - h * s3.S;
  const double q = sqrt(pymax(1.0 + 4.0 * hl * c, 0.0));
  dY1 = 1.0 / pymax(q, 1e-300);
  return 2.0 * c / (1.0 + q);
}

// The integrator's state between steps (ode_integrate_kernel's per-lane registers).
struct TpState {
  double Ychi, YB, Yp, Z[3];
  bool have;
};

// Steps [k0, k1) of the fixed-step sequence x_k = x0 + k h from state St, with ode_integrate_kernel's
// per-lane operations (stages, Y_B map, Radau step, the T = m/3 split step, the predictor); D and C
// accumulate the derivatives of the end state.  Returns false when a step needed tp_bridge.
__device__ __forceinline__ bool tp_steps(const OdePoint& o, const double* __restrict__ w, double x0, double h,
                                         double xb, double xb_below, int64_t k0, int64_t k1, TpState& St, double& D,
                                         double& C) {
  const Radau R = radau_tableau();
  const RadauH hA = radau_h(R, h);
  const bool riccati = LZQ_ODE_PREDICT && o.sigmav != 0.0;
  double Ychi = St.Ychi, YB = St.YB, Yp = St.Yp;
  double Zs[3] = {St.Z[0], St.Z[1], St.Z[2]};
  bool have = St.have, exact = true;
  double kd = (double)k0;
  for (int64_t k = k0; k < k1; ++k, kd += 1.0) {
    const double xk = x0 + kd * h;
    const bool split = xk < xb && xb <= xk + h;
    const double xa = split ? xb_below : xk + h;
    const double Ystart = Ychi;
    bool use_guess = false;
    if (riccati && have && !split && pred_step(k)) {  // the Radau5 predictor, as ode_integrate_kernel
      double gs[3];
      use_guess = true;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        gs[j] = fma_s(Zs[2], kRadauPred[j][3],
                      fma_s(Zs[1], kRadauPred[j][2], fma_s(Zs[0], kRadauPred[j][1], kRadauPred[j][0] * Yp)));
        use_guess = use_guess && fabs(gs[j] - Ychi) <= 0.25 * fabs(Ychi);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) Zs[j] = gs[j];
    }
    auto part = [&](double xs, double hs, bool guess, bool own_h, bool block_start) {
      const RadauH hAs = own_h ? radau_h(R, hs) : hA;
      OdeStage sg[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) sg[j] = ode_stage(o, w, xs + R.c[j] * hs);
      const YbRec yr = yb_rec(hAs, sg);
      YB = __builtin_fma(yr.c, YB, o.Pf * yr.d);
      C *= yr.c;
      const double Y0 = Ychi;
      if (block_start) guess = block_guess(R, hs, sg, Ychi, Zs);
      // (radau_step's convergence test reads NaN corrections as converged -- it never meets one on
      // the sequential trajectory, but a start far from it can diverge: a non-finite result, or a
      // sign change of a source-free positive Y_chi (the stage system's other root), is a failure)
      const bool src = sg[0].S != 0.0 || sg[1].S != 0.0 || sg[2].S != 0.0;
      if (radau_step<false>(hAs, sg, Ychi, YB, Zs, guess) && isfinite(Ychi) && (src || !(Y0 > 0.0) || Ychi > 0.0)) {
        const bool nonlinear = sg[0].lam != 0.0 || sg[1].lam != 0.0 || sg[2].lam != 0.0;
        if (nonlinear) D *= tp_dz3(hs, sg, Zs);
        return true;
      }
      double dY1;
      Ychi = tp_bridge(Y0, hs, sg[2], dY1);
      Zs[0] = Zs[1] = Zs[2] = Ychi;
      D *= dY1;
      return false;
    };
    bool ok = true;
    if (xa > xk) ok = part(xk, split ? xa - xk : h, use_guess, split, riccati && !split && !pred_step(k));
    if (split && xk + h > xb) ok = part(xb, (xk + h) - xb, false, true, false) && ok;
    exact = exact && ok;
    have = !split && ok;  // after a bridge the predictor has no collocation polynomial behind it
    Yp = Ystart;
  }
  St = TpState{Ychi, YB, Yp, {Zs[0], Zs[1], Zs[2]}, have};
  return exact;
}

// One lane per (point, interval): F_m, D_m, C_m from node m.
__global__ __launch_bounds__(64) void ode_tp_interval_kernel(const lzq_point* __restrict__ pts,
                                                             const lzq_ode_params* __restrict__ ode, int64_t n,
                                                             const int32_t* __restrict__ tidx,
                                                             const double* __restrict__ ws, int64_t max_steps,
                                                             int64_t L, int64_t Mmax, const TpNode* __restrict__ nodes,
                                                             TpEnd* __restrict__ ends, const TpCtl* __restrict__ ctl) {
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t p = g / Mmax, m = g - p * Mmax;
  if (p >= n) return;
  const TpCtl c = ctl[p];
  if (c.phase != kTpIter || m >= c.M) return;
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps);
  const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
  const double xb = branch_x(S.o, S.x0, S.x1);
  const TpNode nd = nodes[p * (Mmax + 1) + m];
  TpState St{nd.Ychi, nd.YB, nd.Ychi, {nd.Ychi, nd.Ychi, nd.Ychi}, false};  // (the first step reads no predictor)
  double D = 1.0, C = 1.0;
  const bool exact = tp_steps(S.o, w, S.x0, S.h, xb, nextafter(xb, -INFINITY), k0, k1, St, D, C);
  ends[p * Mmax + m] = TpEnd{St.Ychi, St.YB, D, C, exact ? 1 : 0, 0};
}

// The first guess of long Riccati windows (M >= kTpGuessMin intervals): the same integrator on kTpGuessSteps
// coarse steps of (x1 - x0) / kTpGuessSteps (one lane per point, sequential), each node then
// interpolated between the coarse points around it (Y_chi geometrically when both are positive,
// Y_B linearly).  Radau IIA is L-stable, so the coarse trajectory tracks equilibrium where the
// fine one does and freezes out near where it does: Newton starts within reach of its quadratic
// phase instead of from the constant initial value (14 -> ~5 updates on the shipped window).
constexpr int64_t kTpGuessMin = 1024, kTpGuessSteps = 256;
__global__ __launch_bounds__(256) void ode_tp_guess_kernel(const lzq_point* __restrict__ pts,
                                                           const lzq_ode_params* __restrict__ ode,
                                                           const int32_t* __restrict__ tidx,
                                                           const double* __restrict__ ws, int64_t max_steps, int64_t L,
                                                           int64_t Mmax, TpNode* __restrict__ nodes,
                                                           const TpCtl* __restrict__ ctl) {
  __shared__ double s_y[kTpGuessSteps + 1], s_b[kTpGuessSteps + 1];
  const int64_t p = blockIdx.x;
  const TpCtl c = ctl[p];
  // block-uniform; without annihilation Y_chi's map is affine and Newton needs no first guess
  if (c.phase != kTpIter || c.M < kTpGuessMin || !c.riccati) return;
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps);
  const double Hc = (S.x1 - S.x0) / (double)kTpGuessSteps;
  if (threadIdx.x == 0) {
    const double xb = branch_x(S.o, S.x0, S.x1);
    TpState St{S.Ychi0, 0.0, S.Ychi0, {S.Ychi0, S.Ychi0, S.Ychi0}, false};
    s_y[0] = S.Ychi0;
    s_b[0] = 0.0;
    for (int64_t k = 0; k < kTpGuessSteps; ++k) {
      double D = 1.0, C = 1.0;
      tp_steps(S.o, w, S.x0, Hc, xb, nextafter(xb, -INFINITY), k, k + 1, St, D, C);
      s_y[k + 1] = St.Ychi;
      s_b[k + 1] = St.YB;
    }
  }
  __syncthreads();
  TpNode* nd = nodes + p * (Mmax + 1);
  for (int64_t m = 1 + threadIdx.x; m <= c.M; m += blockDim.x) {
    const int64_t km = m * c.L < S.N ? m * c.L : S.N;  // node m's step index (node M: x1)
    const double u = (double)km / (double)S.N * (double)kTpGuessSteps;
    const int64_t j = u < (double)kTpGuessSteps ? (int64_t)u : kTpGuessSteps - 1;
    const double t = u - (double)j;
    const double y0 = s_y[j], y1 = s_y[j + 1];
    const double y = (y0 > 0.0 && y1 > 0.0) ? y0 * exp(t * log(y1 / y0)) : y0 + t * (y1 - y0);
    const double b = s_b[j] + t * (s_b[j + 1] - s_b[j]);
    if (isfinite(y) && isfinite(b)) nd[m] = TpNode{y, b};
  }
}

// Newton's update of the nodes: the corrections solve d_{m+1} = D_m d_m + r_m (r_m = F_m - s_{m+1},
// d_0 = 0) for both chains, a scan of the affine maps d -> D d + r.  Three launches, kTpBlk
// intervals per block: (1) each block scans its maps in LDS (Hillis-Steele) and stores the local
// inclusive prefixes and its aggregate; (2) each block scans the aggregates of the blocks before it
// (in LDS, at most Mmax / kTpBlk of them), applies the carry to its prefixes and updates its nodes;
// (3) one thread per point folds the blocks' largest corrections and failure flags into TpCtl.
constexpr int kTpBlk = 256;
struct TpMap {
  double A, B, Ab, Bb;  // d -> A d + B (Y_chi), d -> Ab d + Bb (Y_B)
};
__device__ __forceinline__ TpMap tp_compose(const TpMap& later, const TpMap& earlier) {  // later o earlier
  return TpMap{later.A * earlier.A, __builtin_fma(later.A, earlier.B, later.B), later.Ab * earlier.Ab,
               __builtin_fma(later.Ab, earlier.Bb, later.Bb)};
}
// inclusive block scan of kTpBlk maps (every thread of the block calls it)
__device__ __forceinline__ TpMap tp_block_scan(TpMap v, TpMap* sm) {
  const int t = threadIdx.x;
  sm[t] = v;
  __syncthreads();
  for (int off = 1; off < kTpBlk; off <<= 1) {
    const TpMap prev = t >= off ? sm[t - off] : TpMap{1.0, 0.0, 1.0, 0.0};
    __syncthreads();
    if (t >= off) v = tp_compose(v, prev);
    sm[t] = v;
    __syncthreads();
  }
  return v;
}
struct TpBlkOut {
  double err;
  int32_t fail, pad;
};

__global__ __launch_bounds__(kTpBlk) void ode_tp_scan_local_kernel(int64_t Mmax, int64_t Bmax,
                                                                   const TpNode* __restrict__ nodes,
                                                                   const TpEnd* __restrict__ ends,
                                                                   const TpCtl* __restrict__ ctl,
                                                                   TpMap* __restrict__ loc, TpMap* __restrict__ agg,
                                                                   TpBlkOut* __restrict__ bout) {
  __shared__ TpMap sm[kTpBlk];
  const int64_t p = blockIdx.y, b = blockIdx.x;
  const TpCtl c = ctl[p];
  if (c.phase != kTpIter || b * kTpBlk >= c.M) return;  // block-uniform
  const int t = threadIdx.x;
  const int64_t m = b * kTpBlk + t;
  TpMap v{1.0, 0.0, 1.0, 0.0};
  int fail = 0;
  if (m < c.M) {
    const TpEnd e = ends[p * Mmax + m];
    const TpNode q = nodes[p * (Mmax + 1) + m + 1];
    const bool fin = isfinite(e.Ychi) && isfinite(e.D) && isfinite(e.YB) && isfinite(e.C);
    fail = e.exact == 0 || !fin;
    // a non-finite end (a start far from the trajectory) moves nothing downstream this update
    v = fin ? TpMap{e.D, e.Ychi - q.Ychi, e.C, e.YB - q.YB} : TpMap{0.0, 0.0, 0.0, 0.0};
  }
  const int any_fail = __syncthreads_or(fail);
  v = tp_block_scan(v, sm);
  if (m < c.M) loc[p * Mmax + m] = v;
  if (t == kTpBlk - 1) {
    agg[p * Bmax + b] = v;
    bout[p * Bmax + b].fail = any_fail;
  }
}

__global__ __launch_bounds__(kTpBlk) void ode_tp_scan_apply_kernel(int64_t Mmax, int64_t Bmax,
                                                                   TpNode* __restrict__ nodes,
                                                                   const TpEnd* __restrict__ ends,
                                                                   const TpCtl* __restrict__ ctl,
                                                                   const TpMap* __restrict__ loc,
                                                                   const TpMap* __restrict__ agg,
                                                                   TpBlkOut* __restrict__ bout) {
  __shared__ TpMap sm[kTpBlk];
  __shared__ double s_err[kTpBlk / 64];
  const int64_t p = blockIdx.y, b = blockIdx.x;
  const TpCtl c = ctl[p];
  if (c.phase != kTpIter || b * kTpBlk >= c.M) return;  // block-uniform
  const int t = threadIdx.x;
  const int64_t nb = (c.M + kTpBlk - 1) / kTpBlk;
  // the carry into this block: the aggregates of blocks 0 .. b-1 composed (their own scan, in
  // rounds of kTpBlk when there are more blocks than threads)
  TpMap carry{1.0, 0.0, 1.0, 0.0};
  for (int64_t r0 = 0; r0 < b; r0 += kTpBlk) {
    const int64_t k = r0 + t;
    TpMap v = k < b ? agg[p * Bmax + k] : TpMap{1.0, 0.0, 1.0, 0.0};
    v = tp_block_scan(v, sm);
    const int last = (int)((b - r0 < kTpBlk ? b - r0 : kTpBlk) - 1);
    carry = tp_compose(sm[last], carry);
    __syncthreads();
  }
  (void)nb;
  const int64_t m = b * kTpBlk + t;
  double err = 0.0;
  if (m < c.M) {
    const TpMap v = loc[p * Mmax + m];
    const double d = __builtin_fma(v.A, carry.B, v.B), db = __builtin_fma(v.Ab, carry.Bb, v.Bb);  // d_{m+1}
    const TpEnd e = ends[p * Mmax + m];
    TpNode q = nodes[p * (Mmax + 1) + m + 1];
    const bool fin = isfinite(e.Ychi) && isfinite(e.D) && isfinite(e.YB) && isfinite(e.C);
    const double old = q.Ychi;
    double nv = old + d;
    // the Riccati stage system has a second root below zero: a correction never takes a positive
    // node below a quarter of the smaller of its value and its predecessor interval's (positive)
    // end (far from the solution only).  Y_chi's map is affine without annihilation (depletion may
    // take it through zero): no safeguard there.
    const double lo = 0.25 * pymin(old, fin && e.Ychi > 0.0 ? e.Ychi : old);
    if (c.riccati && old > 0.0 && !(nv >= lo)) nv = lo;
    q.Ychi = nv;
    q.YB = q.YB + db;
    nodes[p * (Mmax + 1) + m + 1] = q;
    // relative to the node, floored at 1e-290: below it the doubles approach the subnormal range,
    // whose coarser spacing no correction could resolve to the tolerance
    const double ec = fabs(d) / pymax(fabs(nv), 1e-290), eb = fabs(db) / pymax(fabs(q.YB), 1e-290);
    err = pymax(ec, eb);  // pymax keeps a NaN on the right: checked below
    if (!(ec == ec) || !(eb == eb)) err = INFINITY;
#ifdef LZQ_ODE_TP_DEBUG
    if (m == 0 || m == c.M - 1 || (m % ((c.M + 7) / 8)) == 0)
      printf("  p %lld m %lld node %.6e end %.6e D %.3e exact %d\n", (long long)p, (long long)m, old, e.Ychi, e.D,
             e.exact);
#endif
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) err = pymax(err, __shfl_xor(err, off, 64));
  if ((t & 63) == 0) s_err[t >> 6] = err;
  __syncthreads();
  if (t == 0) {
    double e_all = 0.0;
    for (int k = 0; k < kTpBlk / 64; ++k) e_all = pymax(e_all, s_err[k]);
    bout[p * Bmax + b].err = e_all;
  }
}

__global__ __launch_bounds__(64) void ode_tp_scan_finish_kernel(int64_t n, int64_t Bmax, TpCtl* __restrict__ ctl,
                                                                const TpBlkOut* __restrict__ bout, int32_t max_iters,
                                                                double tol) {
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (p >= n) return;
  TpCtl c = ctl[p];
  if (c.phase != kTpIter) return;
  const int64_t nb = (c.M + kTpBlk - 1) / kTpBlk;
  double e_all = 0.0;
  bool fail = false;
  for (int64_t b = 0; b < nb; ++b) {
    e_all = pymax(e_all, bout[p * Bmax + b].err);
    fail = fail || bout[p * Bmax + b].fail != 0;
  }
  c.iters += 1;
  c.err = e_all;
#ifdef LZQ_ODE_TP_DEBUG
  printf("tp point %lld update %d: M %lld err %.3e fail %d\n", (long long)p, c.iters, (long long)c.M, e_all, (int)fail);
#endif
  // converged: the corrections are below the tolerance and every interval took only Radau steps
  if (e_all <= tol && !fail) c.phase = kTpDone;
  else if (c.iters >= max_iters) c.phase = kTpFallback;
  ctl[p] = c;
}

// Exact stitching.  At convergence the nodes sit within a few ulps of the sequential trajectory
// but are formed as s + d, not carried, so the Newton result differs from the sequential one by
// rounding.  Because no block of LZQ_ODE_PRED_BLOCK steps uses the predictor on its first step
// (and the intervals are whole blocks), interval m's end state is a function of its start
// (Y_chi, Y_B) alone: F_m for Y_chi, G_m for Y_B (independent chains: Y_B's step map does not read
// Y_chi, Y_chi's Newton does not read Y_B).  So every interval is integrated from the 2J + 1
// candidate starts s_m + j ulp, |j| <= J (both chains side by side in one lane), and the exact
// chains are followed through the candidate tables: node 0 is exact, and if node m's exact value
// is candidate j_m, node m + 1's is F_m(candidate j_m) -- a table entry, which again is a candidate
// of node m + 1 unless the Newton node was more than J ulps off.  Following the chain is M
// dependent look-ups, done as segments of kTpSeg intervals for every entry candidate in parallel
// (ode_tp_seg_kernel), then one walk over the segments per point (ode_tp_stitch_kernel).  Each
// candidate integration performs exactly the sequential kernels' operations on that start, so a
// point whose chains stay inside the windows gets the sequential integration's bits; a point whose
// chain leaves a window, or meets a bridged step, is integrated sequentially.  Three rounds: J = 4
// (cheap, the usual case), then J = 32 and J = 256 for the points the previous did not finish (the
// Newton nodes wander from the exact chain where the dynamics is neutral, e.g. a weakly annihilating
// plateau; the last round only where its tables fit kTpCandBytes).
constexpr int kTpSeg = 64;       // intervals per stitching segment
constexpr int kTpJ1 = 4, kTpJ2 = 32, kTpJ3 = 256;
constexpr size_t kTpCandBytes = size_t(1) << 30;  // candidate tables of the J = 256 round, at most

// monotone integer key of a double (ordered like the values; -0 and +0 map to 0) and back
__device__ __forceinline__ int64_t dkey(double x) {
  const int64_t b = __builtin_bit_cast(int64_t, x);
  return b >= 0 ? b : -(b & 0x7FFFFFFFFFFFFFFFll);
}
__device__ __forceinline__ double dfromkey(int64_t k) {
  return __builtin_bit_cast(double, k >= 0 ? k : ((-k) | (int64_t)0x8000000000000000ull));
}

// One lane per (point, interval, candidate j): F_m and G_m at s_m + j ulp, b_m + j ulp (NaN for a
// start that needed a bridge).  Points already stitched (phase kTpExact) or not converged return.
constexpr int32_t kTpExact = 3;
// one (interval, candidate) of one point (out of line: the grid-stride loop around it keeps no
// values of its own live across the integration)
__device__ __noinline__ void tp_cand_one(const lzq_point* __restrict__ pts, const lzq_ode_params* __restrict__ ode,
                                         const int32_t* __restrict__ tidx, const double* __restrict__ ws,
                                         int64_t max_steps, const TpNode* __restrict__ nd, const TpCtl& c, int64_t p,
                                         int64_t m, int off, double* __restrict__ oF, double* __restrict__ oG) {
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps);
  const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
  const double y0 = dfromkey(dkey(nd->Ychi) + off), b0 = dfromkey(dkey(nd->YB) + off);
  // (k0 is a whole number of predictor blocks: the first step does not read Yp / Z / have)
  TpState St{y0, b0, y0, {y0, y0, y0}, false};
  double D = 1.0, C = 1.0;
  const double xb = branch_x(S.o, S.x0, S.x1);
  const bool exact = tp_steps(S.o, w, S.x0, S.h, xb, nextafter(xb, -INFINITY), k0, k1, St, D, C);
  *oF = exact ? St.Ychi : __builtin_nan("");
  *oG = exact ? St.YB : __builtin_nan("");
}

// kStride: a grid-stride loop around an out-of-line body (the last round, whose full grid would be
// ~10^5 blocks that mostly return at once); else one lane per item, the body inline (2 waves/SIMD).
template <int J, bool kStride>
__global__ __launch_bounds__(64) void ode_tp_cand_kernel(const lzq_point* __restrict__ pts,
                                                         const lzq_ode_params* __restrict__ ode, int64_t n,
                                                         const int32_t* __restrict__ tidx,
                                                         const double* __restrict__ ws, int64_t max_steps, int64_t Mmax,
                                                         const TpNode* __restrict__ nodes, const TpCtl* __restrict__ ctl,
                                                         double* __restrict__ candF, double* __restrict__ candG) {
  constexpr int NC = 2 * J + 1;
  for (int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x; g < n * Mmax * NC; g += (int64_t)gridDim.x * 64) {
    const int64_t p = g / (Mmax * NC), rem = g - p * (Mmax * NC), m = rem / NC;
    const int jj = (int)(rem - m * NC);
    const TpCtl c = ctl[p];
    if (c.phase == kTpDone && m < c.M) {
      const int64_t o = (p * Mmax + m) * NC + jj;
      if constexpr (kStride) {
        tp_cand_one(pts, ode, tidx, ws, max_steps, nodes + p * (Mmax + 1) + m, c, p, m, jj - J, candF + o, candG + o);
      } else {
        const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
        const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps);
        const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
        const TpNode& nd = nodes[p * (Mmax + 1) + m];
        const double y0 = dfromkey(dkey(nd.Ychi) + (jj - J)), b0 = dfromkey(dkey(nd.YB) + (jj - J));
        TpState St{y0, b0, y0, {y0, y0, y0}, false};
        double D = 1.0, C = 1.0;
        const double xb = branch_x(S.o, S.x0, S.x1);
        const bool exact = tp_steps(S.o, w, S.x0, S.h, xb, nextafter(xb, -INFINITY), k0, k1, St, D, C);
        candF[o] = exact ? St.Ychi : __builtin_nan("");
        candG[o] = exact ? St.YB : __builtin_nan("");
      }
    }
    if constexpr (!kStride) break;  // one item per lane
  }
}

// One lane per (point, segment, entry candidate of both chains): follow the chains through the
// segment's intervals; the exit candidate index at the next segment's first node (-1: the chain
// left the window or met a bridged start) and the value at the segment's end node.
template <int J>
__global__ __launch_bounds__(64) void ode_tp_seg_kernel(int64_t n, int64_t Mmax, int64_t Smax,
                                                        const TpNode* __restrict__ nodes,
                                                        const TpCtl* __restrict__ ctl,
                                                        const double* __restrict__ candF,
                                                        const double* __restrict__ candG, int32_t* __restrict__ segF,
                                                        int32_t* __restrict__ segG, double* __restrict__ lastF,
                                                        double* __restrict__ lastG) {
  constexpr int NC = 2 * J + 1;
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t p = g / (Smax * NC), rem = g - p * (Smax * NC), sg = rem / NC;
  const int jj = (int)(rem - sg * NC);
  if (p >= n) return;
  const TpCtl c = ctl[p];
  if (c.phase != kTpDone || sg * kTpSeg >= c.M) return;
  const int64_t m0 = sg * kTpSeg, m1 = m0 + kTpSeg < c.M ? m0 + kTpSeg : c.M;
  const TpNode* nd = nodes + p * (Mmax + 1);
  int jF = jj, jG = jj;
  double vF = 0.0, vG = 0.0;
  for (int64_t m = m0; m < m1; ++m) {
    const int64_t o = (p * Mmax + m) * NC;
    vF = jF >= 0 ? candF[o + jF] : __builtin_nan("");
    vG = jG >= 0 ? candG[o + jG] : __builtin_nan("");
    if (m + 1 < c.M) {  // the candidate index of node m + 1 (node M, the final state, needs none)
      const int64_t dF = dkey(vF) - dkey(nd[m + 1].Ychi) + J, dG = dkey(vG) - dkey(nd[m + 1].YB) + J;
#ifdef LZQ_ODE_TP_DEBUG
      if (jj == J && ((jF >= 0 && !(isfinite(vF) && dF >= 0 && dF < NC)) || (jG >= 0 && !(isfinite(vG) && dG >= 0 && dG < NC))))
        printf("  J %d seg %lld node %lld: offset F %lld G %lld (vF %.17g node %.17g)\n", J, (long long)sg,
               (long long)(m + 1), (long long)(dF - J), (long long)(dG - J), vF, nd[m + 1].Ychi);
#endif
      jF = (isfinite(vF) && dF >= 0 && dF < NC) ? (int)dF : -1;
      jG = (isfinite(vG) && dG >= 0 && dG < NC) ? (int)dG : -1;
    }
  }
  const int64_t o = (p * Smax + sg) * NC + jj;
  segF[o] = jF;
  segG[o] = jG;
  lastF[o] = vF;
  lastG[o] = vG;
}

// The Y_B chain on its own (round 5).  Y_B's step is affine, YB <- fma(c, YB, Pf d), with c and d
// from the step's stages alone (yb_rec): they do not depend on Y_chi.  So the Y_B candidates of an
// interval need no Newton iteration and can share the stages: one lane steps kTpGChunk of them
// with tp_steps' step / split structure and Y_B operations, and a window of +-kTpJG ulps costs a
// fraction of the J = 4 round.  A point whose Y_B chain stitches here (gdone) needs only its Y_chi
// chain in the rounds after (its Y_B chain is the one that wanders where the dynamics is neutral).
constexpr int kTpGChunk = 22;  // 3 lanes per interval for JG = 32
constexpr int kTpJG = 32;      // the Y_B round's window (a wider one cost more than it saved; J = 256 stays)
template <int JG>
__global__ __launch_bounds__(64) void ode_tp_gcand_kernel(const lzq_point* __restrict__ pts,
                                                          const lzq_ode_params* __restrict__ ode, int64_t n,
                                                          const int32_t* __restrict__ tidx,
                                                          const double* __restrict__ ws, int64_t max_steps,
                                                          int64_t Mmax, const TpNode* __restrict__ nodes,
                                                          const TpCtl* __restrict__ ctl, double* __restrict__ candG) {
  constexpr int NC = 2 * JG + 1, NCH = (NC + kTpGChunk - 1) / kTpGChunk;
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t p = g / (Mmax * NCH), rem = g - p * (Mmax * NCH), m = rem / NCH;
  const int ch = (int)(rem - m * NCH);
  if (p >= n) return;
  const TpCtl c = ctl[p];
  if (c.phase != kTpDone || m >= c.M) return;
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps);
  const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
  const int64_t bkey = dkey(nodes[p * (Mmax + 1) + m].YB);
  double yb[kTpGChunk];
#pragma unroll
  for (int i = 0; i < kTpGChunk; ++i) yb[i] = dfromkey(bkey + (ch * kTpGChunk + i - JG));
  const Radau R = radau_tableau();
  const RadauH hA = radau_h(R, S.h);
  const double xb = branch_x(S.o, S.x0, S.x1), xb_below = nextafter(xb, -INFINITY);
  auto part = [&](double xs, double hs, bool own_h) {
    const RadauH hAs = own_h ? radau_h(R, hs) : hA;
    OdeStage sg[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) sg[j] = ode_stage(S.o, w, xs + R.c[j] * hs);
    const YbRec yr = yb_rec(hAs, sg);
    const double e = S.o.Pf * yr.d;
#pragma unroll
    for (int i = 0; i < kTpGChunk; ++i) yb[i] = __builtin_fma(yr.c, yb[i], e);
  };
  double kd = (double)k0;
  for (int64_t k = k0; k < k1; ++k, kd += 1.0) {
    const double xk = S.x0 + kd * S.h;
    const bool split = xk < xb && xb <= xk + S.h;
    const double xa = split ? xb_below : xk + S.h;
    if (xa > xk) part(xk, split ? xa - xk : S.h, split);
    if (split && xk + S.h > xb) part(xb, (xk + S.h) - xb, true);
  }
  double* o = candG + (p * Mmax + m) * NC;
#pragma unroll
  for (int i = 0; i < kTpGChunk; ++i)
    if (ch * kTpGChunk + i < NC) o[ch * kTpGChunk + i] = yb[i];
}

// the Y_B chain through one segment from every entry candidate (ode_tp_seg_kernel's G half)
template <int JG>
__global__ __launch_bounds__(64) void ode_tp_gseg_kernel(int64_t n, int64_t Mmax, int64_t Smax,
                                                         const TpNode* __restrict__ nodes, const TpCtl* __restrict__ ctl,
                                                         const double* __restrict__ candG, int32_t* __restrict__ segG,
                                                         double* __restrict__ lastG) {
  constexpr int NC = 2 * JG + 1;
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t p = g / (Smax * NC), rem = g - p * (Smax * NC), sg = rem / NC;
  const int jj = (int)(rem - sg * NC);
  if (p >= n) return;
  const TpCtl c = ctl[p];
  if (c.phase != kTpDone || sg * kTpSeg >= c.M) return;
  const int64_t m0 = sg * kTpSeg, m1 = m0 + kTpSeg < c.M ? m0 + kTpSeg : c.M;
  const TpNode* nd = nodes + p * (Mmax + 1);
  int jG = jj;
  double vG = 0.0;
  for (int64_t m = m0; m < m1; ++m) {
    vG = jG >= 0 ? candG[(p * Mmax + m) * NC + jG] : __builtin_nan("");
    if (m + 1 < c.M) {
      const int64_t dG = dkey(vG) - dkey(nd[m + 1].YB) + JG;
      jG = (isfinite(vG) && dG >= 0 && dG < NC) ? (int)dG : -1;
    }
  }
  segG[(p * Smax + sg) * NC + jj] = jG;
  lastG[(p * Smax + sg) * NC + jj] = vG;
}

// the Y_B chain from node 0 through the segments: gdone[p], and its final value gyb[p]
template <int JG>
__global__ __launch_bounds__(64) void ode_tp_gstitch_kernel(int64_t n, int64_t Smax, const TpCtl* __restrict__ ctl,
                                                            const int32_t* __restrict__ segG,
                                                            const double* __restrict__ lastG,
                                                            int32_t* __restrict__ gdone, double* __restrict__ gyb) {
  constexpr int NC = 2 * JG + 1;
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (p >= n) return;
  const TpCtl c = ctl[p];
  gdone[p] = 0;
  if (c.phase != kTpDone) return;
  const int64_t nseg = (c.M + kTpSeg - 1) / kTpSeg;
  int jG = JG;
  double YB = __builtin_nan("");
  for (int64_t sg = 0; sg < nseg && jG >= 0; ++sg) {
    const int64_t o = (p * Smax + sg) * NC;
    if (sg + 1 == nseg)
      YB = lastG[o + jG];
    else
      jG = segG[o + jG];
  }
  if (jG >= 0 && isfinite(YB)) {
    gdone[p] = 1;
    gyb[p] = YB;
  }
}

// One thread per point: the chains from node 0 (candidate J, the exact start) through the
// segments; both inside their windows to the end -> the final state is the sequential one: the
// yields, skip[p] = 1, phase kTpExact.  Otherwise the point waits for the next round or the
// sequential launches.
template <int J>
__global__ __launch_bounds__(64) void ode_tp_stitch_kernel(const lzq_point* __restrict__ pts, int64_t n, int64_t Smax,
                                                           TpCtl* __restrict__ ctl, const int32_t* __restrict__ segF,
                                                           const int32_t* __restrict__ segG,
                                                           const double* __restrict__ lastF,
                                                           const double* __restrict__ lastG, lzq_yield* __restrict__ out,
                                                           int32_t* __restrict__ status, int32_t* __restrict__ skip,
                                                           const int32_t* __restrict__ gdone,
                                                           const double* __restrict__ gyb, int32_t only_gdone) {
  constexpr int NC = 2 * J + 1;
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (p >= n) return;
  TpCtl c = ctl[p];
  const bool gd = gdone[p] != 0;  // the Y_B chain stitched on its own (ode_tp_gstitch_kernel)
  if (only_gdone && !gd) return;  // a walk over tables whose Y_B half is not this round's
#ifdef LZQ_ODE_TP_DEBUG
  printf("tp point %lld: stitch round J = %d, phase %d\n", (long long)p, J, c.phase);
#endif
  if (c.phase != kTpDone) return;
  const int64_t nseg = (c.M + kTpSeg - 1) / kTpSeg;
  int jF = J, jG = J;
  double YB = 0.0, Ychi = 0.0;
  for (int64_t sg = 0; sg < nseg && jF >= 0 && (gd || jG >= 0); ++sg) {
    const int64_t o = (p * Smax + sg) * NC;
    if (sg + 1 == nseg) {
      Ychi = lastF[o + jF];
      YB = gd ? gyb[p] : lastG[o + jG];
    } else {
      const int a = segF[o + jF], b = gd ? 0 : segG[o + jG];
      jF = a;
      jG = b;
    }
  }
  if (jF < 0 || (!gd && jG < 0) || !isfinite(Ychi) || !isfinite(YB)) {
#ifdef LZQ_ODE_TP_DEBUG
    printf("tp point %lld: stitching with J = %d failed (chains %d %d, %lld segments)\n", (long long)p, J, jF, jG,
           (long long)nseg);
#endif
    return;
  }
  c.phase = kTpExact;
  ctl[p] = c;
  skip[p] = 1;
  const double m = pts[p].m_chi_GeV;
  lzq_yield r;
  const double nB0 = YB * kS0M3, nDM0 = Ychi * kS0M3;  // fpy:412-417
  r.Y_B = YB;
  r.Y_chi = Ychi;
  r.rho_B_kg_m3 = nB0 * kMProtonKg;
  r.rho_DM_kg_m3 = nDM0 * (m * kGeVToKg);
  r.DM_over_B = r.rho_DM_kg_m3 / pymax(r.rho_B_kg_m3, 1e-300);
  r.P_used = pts[p].P_chi_to_B;
  out[p] = r;
  if (status) status[p] = LZQ_ODE_OK;
}

// skip[p] from the phase (stitched points only), and the optional update counts (< 0: iterated,
// not stitched, integrated sequentially).
__global__ __launch_bounds__(64) void ode_tp_finish_kernel(int64_t n, const TpCtl* __restrict__ ctl,
                                                           int32_t* __restrict__ skip, int32_t* __restrict__ iters) {
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (p >= n) return;
  const TpCtl c = ctl[p];
  const bool done = c.phase == kTpExact;
  skip[p] = done ? 1 : 0;
  if (iters) iters[p] = done ? c.iters : -c.iters;
}

// ---------------------------------------------------------------------------------------
// Converged quadrature form of the sigma_v = 0 fallback (opt-in; lzq_ode_quadrature).
// With sigma_v = 0 both equations of rhs (fpy:270-286) are linear with known integrating
// factors: beta = gamma_w H / (H x) = gamma_w / x, so
//   Y_B(x1)   = int_{x0}^{x1} alpha(x) (x / x1)^gamma_w dx,      alpha = (SB/s)/(H x),
//   Y_chi(x1) = Y_chi(x0) - [deplete] int_{x0}^{x1} alpha(x) dx,
// exactly.  In T = m/x (dx = m/T^2 dT) the integrand is the A/V spline's cubic on each knot
// interval times smooth factors (power laws, the source window, the Boltzmann factor, the
// integrating factor), with a jump at the strict T = m/3 branch (fpy:100-111): each knot
// interval is split at that branch and into sub-intervals no wider than half the narrowest
// local scale of those factors, and integrated by 8-point Gauss-Legendre.  This is the
// converged solution of the reference's equations (tests/test_gpu_ode.py: within 1e-10 of the
// reference's own rtol-1e-12 re-solve, golden_ode.json "tight"); the default Radau path
// reproduces the reference's rtol-1e-8 integrator instead.
// ---------------------------------------------------------------------------------------
__constant__ double kGLx[8] = {-0x1.ebab1cb0acc66p-1, -0x1.97e4ab249f41ep-1, -0x1.0d129583284b4p-1,
                               -0x1.77ac94f3c7344p-3, 0x1.77ac94f3c7344p-3,  0x1.0d129583284b4p-1,
                               0x1.97e4ab249f41ep-1,  0x1.ebab1cb0acc66p-1};
__constant__ double kGLw[8] = {0x1.9ea1d04ca0393p-4, 0x1.c76fb531d2b91p-3, 0x1.413c50a255611p-2, 0x1.736360b19933fp-2,
                               0x1.736360b19933fp-2, 0x1.413c50a255611p-2, 0x1.c76fb531d2b91p-3, 0x1.9ea1d04ca0393p-4};
constexpr int kQuadMaxSub = 4096;  // per knot interval; beyond: status LZQ_ODE_UNRESOLVED
#ifndef LZQ_QUAD_UNROLL
#define LZQ_QUAD_UNROLL 1
#endif
#ifndef LZQ_QUAD_MIN_WAVES
#define LZQ_QUAD_MIN_WAVES 3
#endif

// alpha(x) dx/dT = (SB/s)/(H x) * m/T^2 at T (inside knot interval k with PPoly coefficients c,
// knot Tk), with the operations of ode_stage.
__device__ __forceinline__ double ode_alpha_dT(const OdePoint& o, const double* c, double Tk, double T) {
  const double iT = rcp_pos(T);
  const double H = pymax(o.H0 * T * T * kInvMplGeV, 1e-300);
  const double T3 = (T * T) * T;
  const double s = pymax(o.s0 * T3, 1e-300);
  const double qT = o.Tp * iT;
  const double y = 0.5 * o.B * (LZQ_ODE_FMA ? __builtin_fma(qT, qT, -1.0) : qT * qT - 1.0);
  const double q = y * o.inv_sig;
  const double window = exp_nonpos(-0.5 * (q * q));
  double n_eq, vbar;
  if (T > o.m3) {
    n_eq = o.c_rel * T3;
    vbar = 1.0;
  } else {
    n_eq = o.c_nr * (T * sqrt(T)) * exp_nonpos(-o.m * iT);
    vbar = sqrt(pymax(8.0 * T * o.inv_v0, 0.0));
  }
  const double J = o.flux * (0.25 * n_eq * vbar);
  const double sT = T - Tk;
  double z = sT, Av = c[3];
  Av = Av + c[2] * z;
  z = z * sT;
  Av = Av + c[1] * z;
  z = z * sT;
  Av = Av + c[0] * z;
  const double SB = o.P * J * Av * window;
  const double x = o.m * iT;
  return SB / (s * (H * x)) * (o.m * iT * iT);
}

// One wavefront per point; lane l takes knot intervals l, l+64, ...; a fixed xor-butterfly
// reduces the lane sums (deterministic).  tidx: shared tables as in ode_integrate_kernel.
__global__ __launch_bounds__(kOdeBlock, LZQ_QUAD_MIN_WAVES) void ode_quad_kernel(const lzq_point* __restrict__ pts,
                                                             const lzq_ode_params* __restrict__ ode, int64_t n,
                                                             const int32_t* __restrict__ tidx,
                                                             const double* __restrict__ ws, lzq_yield* __restrict__ out,
                                                             int32_t* __restrict__ status) {
  constexpr int kW = 64;
  const int lane = threadIdx.x & (kW - 1);
  const int64_t i = (int64_t)blockIdx.x * (kOdeBlock / kW) + (threadIdx.x / kW);
  if (i >= n) return;  // wave-uniform
  const lzq_point pt = pts[i];
  const OdePoint o = ode_point(pt, ode[i]);
  const double* w = ws + (tidx ? (int64_t)tidx[i] : i) * (int64_t)kOdeWS;
  const double nan = __builtin_nan("");
  lzq_yield r = {nan, nan, nan, nan, nan, pt.P_chi_to_B};
  // CubicSpline's strictly-increasing check, knots split over the lanes
  bool ok = true;
  for (int k = lane + 1; k < kOdeNT; k += kW)
    ok = ok && linspace_at(o.T_lo, o.T_hi, o.stepT, k, kOdeNT) > linspace_at(o.T_lo, o.T_hi, o.stepT, k - 1, kOdeNT);
  int st = __any(!ok) ? LZQ_ODE_BAD_GRID
                      : (!ode_table_ok(w) ? LZQ_ODE_BAD_TABLE : (o.sigmav != 0.0 ? LZQ_ODE_NOT_LINEAR : LZQ_OK));
  const double m = o.m, T_p = o.Tp;
  const double x1 = m / pymax(o.T_lo, 1e-30);  // fpy:388
  const double ix1 = 1.0 / x1;
  double Ychi;  // fpy:389-399
  if (pt.regime == LZQ_NONTHERMAL) {
    if (pt.has_Y_chi_init) Ychi = pt.Y_chi_init;
    else if (pt.has_n_chi_at_Tp) Ychi = pt.n_chi_at_Tp_GeV3 / pymax(s_entropy(T_p, pt.g_star_s), 1e-300);
    else Ychi = 1.0e-12;
  } else {
    Ychi = n_chi_eq(o.T_hi, m, pt.g_chi, pt.stats) / s_entropy(o.T_hi, pt.g_star_s);
  }
  double accB = 0.0, accC = 0.0;
  bool unresolved = false;
  if (st == LZQ_OK || st == LZQ_ODE_NOT_LINEAR) {  // Y_B's equation is linear for every sigma_v
    const double gam = o.gamma_w;
    const double Bt = o.B * T_p * T_p;
    // where the source window exp(-q^2/2), q = y(T)/sigma, y = B/2 ((T_p/T)^2 - 1), is not exactly
    // 0 in double: |q| <= 40 <=> T in [T_p / sqrt(1 + r), T_p / sqrt(1 - r)], r = 80 sigma / B
    const double rw = o.B > 0.0 ? 80.0 * o.sig / o.B : INFINITY;
    const double Tw_lo = rw < INFINITY ? T_p / sqrt(1.0 + rw) : 0.0;
    const double Tw_hi = rw < 1.0 ? T_p / sqrt(1.0 - rw) : INFINITY;
    for (int k = lane; k < kOdeNT - 1; k += kW) {
      const double Tk = linspace_at(o.T_lo, o.T_hi, o.stepT, k, kOdeNT);
      const double Tk1 = linspace_at(o.T_lo, o.T_hi, o.stepT, k + 1, kOdeNT);
      const double c[4] = {w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
      const bool split = Tk < o.m3 && o.m3 < Tk1;
      for (int part = 0; part < (split ? 2 : 1); ++part) {
        double a = (split && part == 1) ? o.m3 : Tk;
        double b = (split && part == 0) ? o.m3 : Tk1;
        // the window exp(-q^2/2), q = y(T)/sigma, y monotone in T: beyond |q| = 40 it is below
        // e^-800, i.e. exactly 0 in double -- the integral is taken over the part of [a, b] where
        // it is not (no sub-intervals wasted where the source is off, and a narrow window
        // (small sigma_y, large beta/H) gets its sub-intervals where it is)
        const double qa = 0.5 * o.B * ((T_p / a) * (T_p / a) - 1.0) * o.inv_sig;
        const double qb = 0.5 * o.B * ((T_p / b) * (T_p / b) - 1.0) * o.inv_sig;
        if (qa * qb > 0.0 && pymin(fabs(qa), fabs(qb)) > 40.0) continue;
        a = pymax(a, Tw_lo);
        b = pymin(b, Tw_hi);
        if (!(b > a)) continue;
        // narrowest local scale of the smooth factors on [a, b] (all shrink as T falls):
        // window width in T, integrating factor / power laws, Boltzmann factor below m/3
        double scale = o.sig * a * a * a / pymax(Bt, 1e-300);
        scale = pymin(scale, a / (gam + 6.0));
        if (a <= o.m3) scale = pymin(scale, a * a / m);
        const double ns = ceil((b - a) / (0.5 * scale));
        if (!(ns <= (double)kQuadMaxSub)) {  // a scale the rule would not resolve: no silent answer
          unresolved = true;
          continue;
        }
        const int nsub = ns < 1.0 ? 1 : (int)ns;
        const double hs = (b - a) / (double)nsub;
        for (int j = 0; j < nsub; ++j) {
          const double mid = a + ((double)j + 0.5) * hs;
#pragma unroll LZQ_QUAD_UNROLL
          for (int g = 0; g < 8; ++g) {
            const double T = mid + (0.5 * hs) * kGLx[g];
            const double f = (0.5 * hs * kGLw[g]) * ode_alpha_dT(o, c, Tk, T);
            const double xr = (m * rcp_pos(T)) * ix1;                       // x / x1 <= 1
            accB = __builtin_fma(f, gam == 0.0 ? 1.0 : exp_nonpos(gam * log(xr)), accB);
            accC += f;
          }
        }
      }
    }
  }
#pragma unroll
  for (int d = 1; d < kW; d <<= 1) {
    accB += __shfl_xor(accB, d, kW);
    accC += __shfl_xor(accC, d, kW);
  }
  if (__any(unresolved)) st = LZQ_ODE_UNRESOLVED;
  if (lane != 0) return;
  if (st == LZQ_ODE_NOT_LINEAR) r.Y_B = accB;  // Y_chi: the Riccati stepping (ode_integrate_kernel<true>)
  if (st == LZQ_OK) {  // fpy:412-417
    const double YB = accB;
    if (o.deplete) Ychi = Ychi - accC;
    const double nB0 = YB * kS0M3, nDM0 = Ychi * kS0M3;
    r.Y_B = YB;
    r.Y_chi = Ychi;
    r.rho_B_kg_m3 = nB0 * kMProtonKg;
    r.rho_DM_kg_m3 = nDM0 * (m * kGeVToKg);
    r.DM_over_B = r.rho_DM_kg_m3 / pymax(r.rho_B_kg_m3, 1e-300);
  }
  out[i] = r;
  if (status) status[i] = st;
}

// BoltzmannSystem.A_over_V_T / .rhs of one point at n arguments (lane per argument).
__global__ __launch_bounds__(kOdeBlock) void ode_eval_kernel(lzq_point pt, lzq_ode_params od, double T_lo,
                                                             double T_hi, int32_t nt, const double* __restrict__ w,
                                                             const double* __restrict__ T, const double* __restrict__ x,
                                                             const double* __restrict__ Y, int64_t n,
                                                             double* __restrict__ out_Av, double* __restrict__ out_dY) {
  const int64_t i = (int64_t)blockIdx.x * kOdeBlock + threadIdx.x;
  if (i >= n) return;
  OdePoint o = ode_point(pt, od);
  o.T_lo = T_lo;
  o.T_hi = T_hi;
  o.stepT = (T_hi - T_lo) / (double)(nt - 1);
  ode_point_recips(o);
  if (out_Av) out_Av[i] = spline_eval(o, w, T[i], nt);
  if (out_dY) {
    const OdeStage s = ode_stage(o, w, x[i], nullptr, nt);
    const double yc = Y[2 * i], yb = Y[2 * i + 1];
    out_dY[2 * i] = -s.lam * (yc * yc - s.E2) - s.S;
    out_dY[2 * i + 1] = s.alpha - s.beta * yb;
  }
}

}  // namespace lzq

// =========================================================================================
// C ABI
// =========================================================================================
namespace {

int64_t ode_blocks(int64_t n) { return (n + lzq::kOdeBlock - 1) / lzq::kOdeBlock; }

int hip_check(hipError_t e, const char* what);

// The fixed-step integration of a batch as continuation launches of <= 2^g_ode_launch_log2
// steps each (lzq_tune(LZQ_TUNE_ODE_LAUNCH_STEPS)): ceil(max_steps / 2^log2) launches, every
// point advancing through steps [j 2^log2, (j+1) 2^log2) of its own sequence in launch j and
// finishing in the launch that reaches its N (points done early return at once).  One launch
// when max_steps fits.  The per-point state (64 B) is stream-ordered scratch (hipMallocAsync).
template <bool kChiOnly>
int launch_integrate(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const int32_t* d_tidx,
                     const double* d_work, int64_t max_steps, lzq_yield* d_out, int32_t* d_status, hipStream_t s,
                     const char* fn, const int32_t* d_skip = nullptr) {
  const int64_t per = (int64_t)1 << lzq::g_ode_launch_log2;
  const int64_t launches = max_steps <= per ? 1 : (max_steps + per - 1) / per;
  if (launches > 65536) {
    char buf[160];
    snprintf(buf, sizeof(buf), "%s: max_steps %lld needs more than 65536 launches of 2^%d steps", fn,
             (long long)max_steps, lzq::g_ode_launch_log2);
    return lzq_set_error(LZQ_EINVAL, buf);
  }
  // every variant (ode_integrate_kernel's kLin, kNoSplit) per launch, each stepping its own
  // wavefronts; no kLin for kChiOnly (no linear waves)
  auto launch = [&](int64_t k_lo, int64_t k_cnt, lzq::OdeState* st) {
    hipLaunchKernelGGL(lzq::ode_integrate_kernel<kChiOnly>, dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0, s,
                       d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, lzq::g_ode_coop, k_lo, k_cnt,
                       st, d_skip);
    int rc = hip_check(hipGetLastError(), fn);
    if constexpr (LZQ_ODE_NOSPLITVAR) {
      if (rc != LZQ_OK) return rc;
      hipLaunchKernelGGL((lzq::ode_integrate_kernel<kChiOnly, false, true>), dim3((unsigned)ode_blocks(n)),
                         dim3(lzq::kOdeBlock), 0, s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status,
                         lzq::g_ode_coop, k_lo, k_cnt, st, d_skip);
      rc = hip_check(hipGetLastError(), fn);
      if constexpr (LZQ_ODE_RICVAR && !kChiOnly) {  // the three passes (ode_riccati_kernel)
        if (rc != LZQ_OK) return rc;
        hipLaunchKernelGGL(lzq::ode_riccati_kernel<0>, dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0, s,
                           d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, lzq::g_ode_coop, k_lo,
                           k_cnt, st, d_skip);
        rc = hip_check(hipGetLastError(), fn);
        if (rc != LZQ_OK) return rc;
        hipLaunchKernelGGL(lzq::ode_riccati_kernel<1>, dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0, s,
                           d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, lzq::g_ode_coop, k_lo,
                           k_cnt, st, d_skip);
        rc = hip_check(hipGetLastError(), fn);
        if (rc != LZQ_OK) return rc;
        hipLaunchKernelGGL(lzq::ode_riccati_kernel<2>, dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0, s,
                           d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, lzq::g_ode_coop, k_lo,
                           k_cnt, st, d_skip);
        rc = hip_check(hipGetLastError(), fn);
      }
    }
    if constexpr (LZQ_ODE_LINFAST && LZQ_ODE_YBREC && !kChiOnly) {
      if (rc != LZQ_OK) return rc;
      hipLaunchKernelGGL((lzq::ode_integrate_kernel<kChiOnly, true>), dim3((unsigned)ode_blocks(n)),
                         dim3(lzq::kOdeBlock), 0, s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status,
                         lzq::g_ode_coop, k_lo, k_cnt, st, d_skip);
      rc = hip_check(hipGetLastError(), fn);
    }
    return rc;
  };
  // one launch needs no carried state, unless the Riccati passes (ode_riccati_kernel) hand a
  // wave's state from pass to pass
  if (launches == 1 && !(LZQ_ODE_RICVAR && !kChiOnly)) return launch(0, 0, nullptr);
  lzq::OdeState* st = nullptr;
  int rc = hip_check(hipMallocAsync((void**)&st, sizeof(lzq::OdeState) * (size_t)n, s), fn);
  if (rc) return rc;
  for (int64_t j = 0; j < launches && rc == LZQ_OK; ++j) rc = launch(j * per, per, st);
  const int rf = hip_check(hipFreeAsync(st, s), fn);
  return rc ? rc : rf;
}

// lzq_ode_integrate_tp: the time-parallel iteration (ode_tp_*_kernel) for batches of <= kTpMaxPoints
// points, then the sequential launches for the points it did not finish (skip mask).  Intervals
// of g_ode_tp_interval steps, more when max_steps would need over kTpMaxIntervals of them.
constexpr int64_t kTpMaxPoints = 64;
constexpr int64_t kTpMaxIntervals = 1 << 16;
constexpr int32_t kTpMaxIters = 32;
constexpr double kTpTol = 1e-14;  // largest relative node correction of a converged iteration
int launch_integrate_tp(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const int32_t* d_tidx,
                        const double* d_work, int64_t max_steps, lzq_yield* d_out, int32_t* d_status,
                        int32_t* d_iters, hipStream_t s, const char* fn) {
  // node arrays for max_steps at the default interval length, at most kTpMaxIntervals per point
  // (a point whose N needs more takes longer intervals, ode_tp_init_kernel)
  const int64_t L = lzq::g_ode_tp_interval;
  const int64_t Mmax = std::min<int64_t>((max_steps + L - 1) / L, kTpMaxIntervals);
  if (n > kTpMaxPoints || Mmax < 2) {  // nothing to cut: the sequential path alone
    if (d_iters) {
      int rc = hip_check(hipMemsetAsync(d_iters, 0, sizeof(int32_t) * (size_t)n, s), fn);
      if (rc) return rc;
    }
    return launch_integrate<false>(d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, s, fn);
  }
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const int64_t Smax = (Mmax + lzq::kTpSeg - 1) / lzq::kTpSeg;
  const bool round3 = 2 * sizeof(double) * (size_t)n * (size_t)Mmax * (size_t)(2 * lzq::kTpJ3 + 1) <= lzq::kTpCandBytes;
  const int64_t NC2 = 2 * (round3 ? lzq::kTpJ3 : lzq::kTpJ2) + 1;
  const size_t b_nodes = up(sizeof(lzq::TpNode) * (size_t)n * (size_t)(Mmax + 1));
  const size_t b_ends = up(sizeof(lzq::TpEnd) * (size_t)n * (size_t)Mmax);
  const size_t b_ctl = up(sizeof(lzq::TpCtl) * (size_t)n);
  const size_t b_skip = up(sizeof(int32_t) * (size_t)n);
  const size_t b_cand = up(sizeof(double) * (size_t)n * (size_t)Mmax * (size_t)NC2);  // per chain
  const size_t b_segi = up(sizeof(int32_t) * (size_t)n * (size_t)Smax * (size_t)NC2);
  const size_t b_segv = up(sizeof(double) * (size_t)n * (size_t)Smax * (size_t)NC2);
  const int64_t Bmax = (Mmax + lzq::kTpBlk - 1) / lzq::kTpBlk;
  const size_t b_loc = up(sizeof(lzq::TpMap) * (size_t)n * (size_t)Mmax);
  const size_t b_agg = up(sizeof(lzq::TpMap) * (size_t)n * (size_t)Bmax);
  const size_t b_bout = up(sizeof(lzq::TpBlkOut) * (size_t)n * (size_t)Bmax);
  const size_t b_gd = up(sizeof(int32_t) * (size_t)n), b_gy = up(sizeof(double) * (size_t)n);
  char* buf = nullptr;
  int rc = hip_check(hipMallocAsync((void**)&buf, b_nodes + b_ends + b_ctl + b_skip + 2 * (b_cand + b_segi + b_segv) +
                                                       b_loc + b_agg + b_bout + b_gd + b_gy,
                                    s),
                     fn);
  if (rc) return rc;
  char* q = buf;
  auto take = [&](size_t b) {
    char* r = q;
    q += b;
    return r;
  };
  auto* nodes = reinterpret_cast<lzq::TpNode*>(take(b_nodes));
  auto* ends = reinterpret_cast<lzq::TpEnd*>(take(b_ends));
  auto* ctl = reinterpret_cast<lzq::TpCtl*>(take(b_ctl));
  auto* skip = reinterpret_cast<int32_t*>(take(b_skip));
  auto* candF = reinterpret_cast<double*>(take(b_cand));
  auto* candG = reinterpret_cast<double*>(take(b_cand));
  auto* segF = reinterpret_cast<int32_t*>(take(b_segi));
  auto* segG = reinterpret_cast<int32_t*>(take(b_segi));
  auto* lastF = reinterpret_cast<double*>(take(b_segv));
  auto* lastG = reinterpret_cast<double*>(take(b_segv));
  auto* loc = reinterpret_cast<lzq::TpMap*>(take(b_loc));
  auto* agg = reinterpret_cast<lzq::TpMap*>(take(b_agg));
  auto* bout = reinterpret_cast<lzq::TpBlkOut*>(take(b_bout));
  auto* gdone = reinterpret_cast<int32_t*>(take(b_gd));
  auto* gyb = reinterpret_cast<double*>(take(b_gy));
  hipLaunchKernelGGL(lzq::ode_tp_init_kernel, dim3((unsigned)n), dim3(256), 0, s, d_points, d_ode, d_tidx, d_work,
                     max_steps, L, Mmax, nodes, ctl);
  rc = hip_check(hipGetLastError(), fn);
  if (rc == LZQ_OK && Mmax >= lzq::kTpGuessMin) {
    hipLaunchKernelGGL(lzq::ode_tp_guess_kernel, dim3((unsigned)n), dim3(256), 0, s, d_points, d_ode, d_tidx, d_work,
                       max_steps, L, Mmax, nodes, ctl);
    rc = hip_check(hipGetLastError(), fn);
  }
  const unsigned ib = (unsigned)((n * Mmax + 63) / 64);
  for (int32_t it = 0; it < kTpMaxIters && rc == LZQ_OK; ++it) {
    hipLaunchKernelGGL(lzq::ode_tp_interval_kernel, dim3(ib), dim3(64), 0, s, d_points, d_ode, n, d_tidx, d_work,
                       max_steps, L, Mmax, nodes, ends, ctl);
    rc = hip_check(hipGetLastError(), fn);
    if (rc) break;
    hipLaunchKernelGGL(lzq::ode_tp_scan_local_kernel, dim3((unsigned)Bmax, (unsigned)n), dim3(lzq::kTpBlk), 0, s, Mmax,
                       Bmax, nodes, ends, ctl, loc, agg, bout);
    rc = hip_check(hipGetLastError(), fn);
    if (rc) break;
    hipLaunchKernelGGL(lzq::ode_tp_scan_apply_kernel, dim3((unsigned)Bmax, (unsigned)n), dim3(lzq::kTpBlk), 0, s, Mmax,
                       Bmax, nodes, ends, ctl, loc, agg, bout);
    rc = hip_check(hipGetLastError(), fn);
    if (rc) break;
    hipLaunchKernelGGL(lzq::ode_tp_scan_finish_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, Bmax, ctl,
                       bout, kTpMaxIters, kTpTol);
    rc = hip_check(hipGetLastError(), fn);
  }
  // exact stitching, J = kTpJ1 then kTpJ2 for the points the first round did not finish
  auto stitch = [&](auto Jc, bool cands) {
    constexpr int J = decltype(Jc)::value, NC = 2 * J + 1;
    constexpr bool kStride = J > 32;
    const int64_t full = (n * Mmax * NC + 63) / 64;
    const int64_t cb = kStride ? std::min<int64_t>(full, 4096) : full;
    int r = LZQ_OK;
    if (cands) {
      hipLaunchKernelGGL((lzq::ode_tp_cand_kernel<J, kStride>), dim3((unsigned)cb), dim3(64), 0, s,
                         d_points, d_ode, n, d_tidx, d_work, max_steps, Mmax, nodes, ctl, candF, candG);
      r = hip_check(hipGetLastError(), fn);
      if (r) return r;
    }
    hipLaunchKernelGGL(lzq::ode_tp_seg_kernel<J>, dim3((unsigned)((n * Smax * NC + 63) / 64)), dim3(64), 0, s, n, Mmax,
                       Smax, nodes, ctl, candF, candG, segF, segG, lastF, lastG);
    r = hip_check(hipGetLastError(), fn);
    if (r) return r;
    hipLaunchKernelGGL(lzq::ode_tp_stitch_kernel<J>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, d_points, n, Smax,
                       ctl, segF, segG, lastF, lastG, d_out, d_status, skip, (const int32_t*)gdone, (const double*)gyb,
                       (int32_t)!cands);
    return hip_check(hipGetLastError(), fn);
  };
  // the Y_B chain on its own (its candidates fit the buffers of either last round)
  auto gstitch = [&](auto Jc) {
    constexpr int JG = decltype(Jc)::value, NC = 2 * JG + 1;
    constexpr int NCH = (NC + lzq::kTpGChunk - 1) / lzq::kTpGChunk;
    hipLaunchKernelGGL(lzq::ode_tp_gcand_kernel<JG>, dim3((unsigned)((n * Mmax * NCH + 63) / 64)), dim3(64), 0, s,
                       d_points, d_ode, n, d_tidx, d_work, max_steps, Mmax, nodes, ctl, candG);
    int r = hip_check(hipGetLastError(), fn);
    if (r) return r;
    hipLaunchKernelGGL(lzq::ode_tp_gseg_kernel<JG>, dim3((unsigned)((n * Smax * NC + 63) / 64)), dim3(64), 0, s, n, Mmax,
                       Smax, nodes, ctl, candG, segG, lastG);
    r = hip_check(hipGetLastError(), fn);
    if (r) return r;
    hipLaunchKernelGGL(lzq::ode_tp_gstitch_kernel<JG>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, Smax, ctl,
                       segG, lastG, gdone, gyb);
    return hip_check(hipGetLastError(), fn);
  };
  // J = 4 for both chains; then, for the points it did not finish, the Y_B chain alone at +-32
  // ulps and the J = 4 walk again over the Y_chi candidates it has (candF is untouched); then
  // J = 32 and J = 256 for both chains (a Y_B chain already stitched is not needed there)
  if (rc == LZQ_OK) rc = hip_check(hipMemsetAsync(gdone, 0, sizeof(int32_t) * (size_t)n, s), fn);
  if (rc == LZQ_OK) rc = stitch(std::integral_constant<int, lzq::kTpJ1>(), true);
  if (rc == LZQ_OK) rc = gstitch(std::integral_constant<int, lzq::kTpJG>());
  if (rc == LZQ_OK) rc = stitch(std::integral_constant<int, lzq::kTpJ1>(), false);
  if (rc == LZQ_OK) rc = stitch(std::integral_constant<int, lzq::kTpJ2>(), true);
  if (rc == LZQ_OK && round3) rc = stitch(std::integral_constant<int, lzq::kTpJ3>(), true);
  if (rc == LZQ_OK) {
    hipLaunchKernelGGL(lzq::ode_tp_finish_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, n, ctl, skip,
                       d_iters);
    rc = hip_check(hipGetLastError(), fn);
  }
  if (rc == LZQ_OK)
    rc = launch_integrate<false>(d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, s, fn, skip);
  const int rf = hip_check(hipFreeAsync(buf, s), fn);
  return rc ? rc : rf;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return LZQ_OK;
  char buf[256];
  snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  return lzq_set_error(LZQ_EHIP, buf);
}

int check_ws(int64_t n, const double* d_work, int64_t work_doubles, const char* fn,
             int64_t per_table = LZQ_ODE_WS_PER_POINT) {
  char buf[160];
  if (n < 0 || (n > 0 && !d_work)) {
    snprintf(buf, sizeof(buf), "%s: bad arguments", fn);
    return lzq_set_error(LZQ_EINVAL, buf);
  }
  if (n > 0 && (work_doubles / per_table) < n) {
    snprintf(buf, sizeof(buf), "%s: workspace of %lld doubles < n * %lld", fn, (long long)work_doubles,
             (long long)per_table);
    return lzq_set_error(LZQ_EINVAL, buf);
  }
  if (ode_blocks(n) > 2147483647LL) {
    snprintf(buf, sizeof(buf), "%s: n too large", fn);
    return lzq_set_error(LZQ_EINVAL, buf);
  }
  return LZQ_OK;
}

}  // namespace

extern "C" {

int lzq_ode_tables(const lzq_point* d_points, int64_t n, const double* d_T_lo, const double* d_T_hi, int32_t nt,
                   int32_t nz, double z_max, const lzq_aov_params* d_aov, double* d_work, int64_t work_doubles,
                   int32_t* d_status, void* stream) {
  if (nt < 4 || nt > LZQ_ODE_NT_MAX) {
    char buf[128];
    snprintf(buf, sizeof(buf), "lzq_ode_tables: nt = %d knots outside [4, %d]", nt, LZQ_ODE_NT_MAX);
    return lzq_set_error(LZQ_EINVAL, buf);
  }
  int rc = check_ws(n, d_work, work_doubles, "lzq_ode_tables", 4 * (int64_t)nt);
  if (rc) return rc;
  if (n > 0 && !d_points) return lzq_set_error(LZQ_EINVAL, "lzq_ode_tables: bad arguments");
  if ((d_T_lo == nullptr) != (d_T_hi == nullptr))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_tables: T_lo and T_hi must both be given or both be NULL");
  if (n == 0) return LZQ_OK;
  hipStream_t s = (hipStream_t)stream;
  rc = lzq::launch_ode_aov_tables(d_points, n, d_T_lo, d_T_hi, nt, nz, z_max, d_aov, d_work, s);
  if (rc) return rc;
  hipLaunchKernelGGL(lzq::ode_spline_kernel, dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0, s, d_points, n,
                     nt, d_T_lo, d_T_hi, d_work, d_status);
  return hip_check(hipGetLastError(), "lzq_ode_tables");
}

int lzq_ode_integrate(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const double* d_work,
                      int64_t work_doubles, int64_t max_steps, lzq_yield* d_out, int32_t* d_status, void* stream) {
  int rc = check_ws(n, d_work, work_doubles, "lzq_ode_integrate");
  if (rc) return rc;
  if (n > 0 && (!d_points || !d_ode || !d_out)) return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate: bad arguments");
  if (max_steps < 0) return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate: max_steps < 0");
  if (n == 0) return LZQ_OK;
  return launch_integrate<false>(d_points, d_ode, n, nullptr, d_work, max_steps, d_out, d_status, (hipStream_t)stream,
                                 "lzq_ode_integrate");
}

int lzq_ode_integrate_shared(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                             const int32_t* d_table_index, int64_t n_tables, const double* d_work,
                             int64_t work_doubles, int64_t max_steps, lzq_yield* d_out, int32_t* d_status,
                             void* stream) {
  if (n < 0 || n_tables < 0 || (n > 0 && (!d_points || !d_ode || !d_out || !d_table_index || n_tables == 0)))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate_shared: bad arguments");
  int rc = check_ws(n_tables, d_work, work_doubles, "lzq_ode_integrate_shared");
  if (rc) return rc;
  if (max_steps < 0) return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate_shared: max_steps < 0");
  if (ode_blocks(n) > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate_shared: n too large");
  if (n == 0) return LZQ_OK;
  return launch_integrate<false>(d_points, d_ode, n, d_table_index, d_work, max_steps, d_out, d_status,
                                 (hipStream_t)stream, "lzq_ode_integrate_shared");
}

int lzq_ode_integrate_tp(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                         const int32_t* d_table_index, int64_t n_tables, const double* d_work, int64_t work_doubles,
                         int64_t max_steps, lzq_yield* d_out, int32_t* d_status, int32_t* d_iters, void* stream) {
  if (n < 0 || n_tables < 0 || max_steps < 0 || (n > 0 && (!d_points || !d_ode || !d_out)) ||
      (d_table_index && n > 0 && n_tables == 0))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate_tp: bad arguments");
  int rc = check_ws(d_table_index ? n_tables : n, d_work, work_doubles, "lzq_ode_integrate_tp");
  if (rc) return rc;
  if (n == 0) return LZQ_OK;
  return launch_integrate_tp(d_points, d_ode, n, d_table_index, d_work, max_steps, d_out, d_status, d_iters,
                             (hipStream_t)stream, "lzq_ode_integrate_tp");
}

int lzq_ode_quadrature(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                       const int32_t* d_table_index, int64_t n_tables, const double* d_work, int64_t work_doubles,
                       int64_t max_steps, lzq_yield* d_out, int32_t* d_status, void* stream) {
  if (n < 0 || n_tables < 0 || max_steps < 0 || (n > 0 && (!d_points || !d_ode || !d_out)) ||
      (d_table_index && n > 0 && n_tables == 0))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_quadrature: bad arguments");
  int rc = check_ws(d_table_index ? n_tables : n, d_work, work_doubles, "lzq_ode_quadrature");
  if (rc) return rc;
  if (n == 0) return LZQ_OK;
  const int64_t nb = (n + (lzq::kOdeBlock / 64) - 1) / (lzq::kOdeBlock / 64);
  if (nb > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_ode_quadrature: n too large");
  hipLaunchKernelGGL(lzq::ode_quad_kernel, dim3((unsigned)nb), dim3(lzq::kOdeBlock), 0, (hipStream_t)stream, d_points,
                     d_ode, n, d_table_index, d_work, d_out, d_status);
  rc = hip_check(hipGetLastError(), "lzq_ode_quadrature");
  if (rc) return rc;
  // sigma_v != 0: Y_chi's Riccati equation by the Radau stepping (Y_B from the quadrature above)
  return launch_integrate<true>(d_points, d_ode, n, d_table_index, d_work, max_steps, d_out, d_status,
                                (hipStream_t)stream, "lzq_ode_quadrature");
}

int lzq_ode_batch(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, int32_t nz, double z_max,
                  const lzq_aov_params* d_aov, double* d_work, int64_t work_doubles, int64_t max_steps,
                  lzq_yield* d_out, int32_t* d_status, void* stream) {
  int rc = lzq_ode_tables(d_points, n, nullptr, nullptr, LZQ_ODE_NT, nz, z_max, d_aov, d_work, work_doubles, d_status,
                          stream);
  if (rc) return rc;
  return lzq_ode_integrate(d_points, d_ode, n, d_work, work_doubles, max_steps, d_out, d_status, stream);
}

int lzq_ode_aov_T(const lzq_point* pt, double T_lo, double T_hi, int32_t nt, const double* d_work_point,
                  const double* d_T, int64_t n, double* d_out_Av, void* stream) {
  if (!pt || n < 0 || nt < 4 || nt > LZQ_ODE_NT_MAX || (n > 0 && (!d_work_point || !d_T || !d_out_Av)))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_aov_T: bad arguments");
  if (n == 0) return LZQ_OK;
  if (ode_blocks(n) > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_ode_aov_T: n too large");
  lzq_ode_params od = {0.0, 0.0, 0, 0};
  hipLaunchKernelGGL(lzq::ode_eval_kernel, dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0, (hipStream_t)stream,
                     *pt, od, T_lo, T_hi, nt, d_work_point, d_T, nullptr, nullptr, n, d_out_Av, nullptr);
  return hip_check(hipGetLastError(), "lzq_ode_aov_T");
}

int lzq_ode_rhs(const lzq_point* pt, const lzq_ode_params* ode, double T_lo, double T_hi, int32_t nt,
                const double* d_work_point, const double* d_x, const double* d_Y, int64_t n, double* d_out_dY,
                void* stream) {
  if (!pt || !ode || n < 0 || nt < 4 || nt > LZQ_ODE_NT_MAX || (n > 0 && (!d_work_point || !d_x || !d_Y || !d_out_dY)))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_rhs: bad arguments");
  if (n == 0) return LZQ_OK;
  if (ode_blocks(n) > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_ode_rhs: n too large");
  hipLaunchKernelGGL(lzq::ode_eval_kernel, dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0, (hipStream_t)stream,
                     *pt, *ode, T_lo, T_hi, nt, d_work_point, nullptr, d_x, d_Y, n, nullptr, d_out_dY);
  return hip_check(hipGetLastError(), "lzq_ode_rhs");
}

}  // extern "C"
