// lzq_profile.hip -- the bounce-profile LZ path (PAPER p.3 §3, eqs.(5)-(9); the reference's
// plug-in hook fpy:170-187 imports the absent `transport_from_profile` for it, fpy:173).
//
// A profile SHAPE is the bounce solution's two background fields phi(xi), Phi(xi) sampled on
// knots xi_0 < ... < xi_{K-1} (xi = r - R_0, PAPER §3.1), "interpolated as smooth functions":
// here not-a-knot cubic splines, the interpolant scipy's CubicSpline builds and fpy:212 uses
// for its own tables.  A POINT is a shape plus the couplings of eqs.(5)-(8):
//   Delta(xi) = y_B phi(xi) - y_chi Phi(xi)      eq.(5)   crossings xi*: Delta(xi*) = 0
//   Delta'*   = y_B phi'(xi*) - y_chi Phi'(xi*)  eq.(6)
//   m_mix(xi) = lambda_tr_eff phi(xi)            eq.(7)
//   delta_LZ  = m_mix(xi*)^2 / (2 v_w |Delta'*|) eq.(8), F(k) = 1;  P = 1 - exp(-2 pi delta) eq.(9)
//
// Kernels (one lane per point or per spline; every lane computes from its own inputs, so the
// results do not depend on launch geometry or batch composition):
//  * profile_spline_kernel   -- the two not-a-knot splines of a shape (scipy's banded system,
//                               Thomas elimination), coefficients [shape][interval][8] =
//                               (phi c0..c3, Phi c0..c3), ascending powers of t = xi - xi_j;
//  * profile_crossings_kernel-- eqs.(5)-(8): every sign change of the cubic Delta on every knot
//                               interval (split at its stationary points into monotone pieces,
//                               each root by safeguarded Newton to full precision);
//  * profile_propagate_kernel-- the time-ordered propagation i dpsi/dt = H psi,
//                               H = Delta(xi) sigma_z + m_mix(xi) sigma_x, xi = v_w t, through the
//                               whole profile [xi_0, xi_{K-1}], started in and projected on the
//                               chi-like second-order dressed state at the two ends (several
//                               crossings interfere coherently; for one linear crossing in a wide
//                               window this is eq.(9)).  Sixth-order Magnus: three Gauss-Legendre
//                               nodes per step, the Blanes-Casas-Ros commutator form, exact SU(2)
//                               exponential; on knot interval j, S_j = max(min_steps,
//                               ceil(steps_per_radian * (len_j / v_w) * omega_j)) uniform steps,
//                               omega_j = the largest of E = sqrt(Delta^2 + m^2) and
//                               4 sqrt(|dH/dt|) (4 / the LZ time) at 5 points of the interval
//                               (from per-shape interval records, profile_samples_kernel).  A
//                               lane keeps its interval's Delta and m coefficients, the state and
//                               the step in registers; a wave whose points share the shape stages
//                               the interval records in LDS, the next one fetched while it steps
//                               (round 5; round 3's per-block staging of whole shapes was 5% slower).
//                               Large batches launch in (shape, cost, coupling angle) order
//                               (profile_key_kernel + a radix sort).
// tests/profile_ref.py restates all three in numpy; tests/test_gpu_profile.py checks them.
#include <hip/hip_runtime.h>

#include <math.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>

#include "../../include/lzq.h"
#include "lzq_internal.h"
#include "lzq_su2.h"

int lzq_set_error(int code, const char* msg);

namespace lzq {

constexpr int kProfBlock = 256;
#ifndef LZQ_PROF_MIN_WAVES
#define LZQ_PROF_MIN_WAVES 2
#endif
#ifndef LZQ_PROF_PAIR
#define LZQ_PROF_PAIR 0  // the interval loop's Magnus steps two per iteration (state in alternating registers)
#endif
#ifndef LZQ_PROF_UNIFORM
#define LZQ_PROF_UNIFORM 1  // waves whose points share one shape read its rows through the scalar cache
#endif
#ifndef LZQ_PROF_SORT
#define LZQ_PROF_SORT 1  // keyed launch order for batches of >= kProfSortMin points (0: index order)
#endif
constexpr int64_t kProfSortMin = 16384;
constexpr int kProfCostStride = 16;  // the launch-order cost model samples every 16th knot interval
constexpr double kMaxIntervalSteps = 16777216.0;  // per knot interval; beyond: P = NaN (absurd input)
constexpr int kProfCoef = 8;                      // doubles per interval row
constexpr double kHdotRate = 4.0;  // crossing-region rate: kHdotRate / (LZ time), LZ time = |dH/dt|^-1/2

struct ProfPt {
  double yB, ychi, lam, vw;
  int32_t shape;
};

__device__ __forceinline__ ProfPt load_point(const lzq_profile_point* p) {
  return {p->y_B, p->y_chi, p->lambda_tr_eff, p->v_w, p->shape};
}

// c0 + t (c1 + t (c2 + t c3)) and derivatives (numpy order of operations, no contraction)
__device__ __forceinline__ double pp0(const double* c, double t) { return c[0] + t * (c[1] + t * (c[2] + t * c[3])); }
__device__ __forceinline__ double pp1(const double* c, double t) { return c[1] + t * (2.0 * c[2] + t * 3.0 * c[3]); }
__device__ __forceinline__ double pp2(const double* c, double t) { return 2.0 * c[2] + 6.0 * c[3] * t; }

// Delta (eq.5) and m_mix (eq.7) coefficients of interval j of the point's shape
__device__ __forceinline__ void interval_coefs(const double* __restrict__ row, const ProfPt& p, double* cD,
                                               double* cM) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double a = row[k], b = row[4 + k];
    cD[k] = p.yB * a - p.ychi * b;
    cM[k] = p.lam * a;
  }
}

// the same for the propagation (fused: D_k = fma(y_B, phi_k, -(y_chi Phi_k)), 8 VALU fewer per
// interval entry; the crossings keep interval_coefs, the restatement's operations)
__device__ __forceinline__ void interval_coefs_fma(const double* __restrict__ row, const ProfPt& p, double* cD,
                                                   double* cM) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double a = row[k], b = row[4 + k];
    cD[k] = __builtin_fma(p.yB, a, -(p.ychi * b));
    cM[k] = p.lam * a;
  }
}

// ---------------------------------------------------------------------------------------
// Splines: scipy.interpolate.CubicSpline(x, y) (bc_type='not-a-knot', n >= 4): the slope
// system of scipy/_cubic.py by Thomas elimination (scipy: banded LU; equal to rounding), then
// c0 = y_j, c1 = s_j, c2 = (slope_j - s_j)/dx_j - t, c3 = t/dx_j, t = (s_j + s_{j+1} - 2 slope_j)/dx_j.
// One lane per (shape, field); the forward sweep parks (c', d') in the row's c2/c3 slots.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kProfBlock) void profile_spline_kernel(const double* __restrict__ knots,
                                                                    const double* __restrict__ phi,
                                                                    const double* __restrict__ Phi, int32_t n_shapes,
                                                                    int32_t K, double* __restrict__ coef,
                                                                    int32_t* __restrict__ bad) {
  const int64_t lane = (int64_t)blockIdx.x * kProfBlock + threadIdx.x;
  if (lane >= 2 * (int64_t)n_shapes) return;
  const int64_t s = lane >> 1;
  const int f = (int)(lane & 1);  // 0: phi, 1: Phi
  const double* x = knots + s * K;
  const double* y = (f ? Phi : phi) + s * K;
  double* w = coef + s * (int64_t)(K - 1) * kProfCoef + 4 * f;  // row j: w[j * 8 + 0..3]
  for (int j = 0; j + 1 < K; ++j)
    if (!(x[j + 1] > x[j])) {  // CubicSpline: "x must be strictly increasing"
      if (f == 0) bad[s] = 1;
      return;
    }
  auto DX = [&](int j) { return x[j + 1] - x[j]; };
  auto SL = [&](int j) { return (y[j + 1] - y[j]) / DX(j); };
  // row 0 (not-a-knot): dx1 s0 + (x2 - x0) s1 = ((dx0 + 2d) dx1 sl0 + dx0^2 sl1) / d
  double dxm1 = DX(0), slm1 = SL(0), cp, dp;
  {
    const double dx1 = DX(1), sl1 = SL(1), d = x[2] - x[0];
    const double r = ((dxm1 + 2.0 * d) * dx1 * slm1 + (dxm1 * dxm1) * sl1) / d;
    cp = d / dx1;
    dp = r / dx1;
    w[2] = cp;
    w[3] = dp;
  }
  // rows 1..K-2: dx_k s_{k-1} + 2 (dx_{k-1} + dx_k) s_k + dx_{k-1} s_{k+1} = 3 (dx_k sl_{k-1} + dx_{k-1} sl_k)
  for (int k = 1; k < K - 1; ++k) {
    const double dxk = DX(k), slk = SL(k);
    const double a = dxk, b = 2.0 * (dxm1 + dxk), c = dxm1;
    const double r = 3.0 * (dxk * slm1 + dxm1 * slk);
    const double den = b - a * cp;
    cp = c / den;
    dp = (r - a * dp) / den;
    w[k * kProfCoef + 2] = cp;
    w[k * kProfCoef + 3] = dp;
    dxm1 = dxk;
    slm1 = slk;
  }
  // last row (not-a-knot): (x[-1] - x[-3]) s[-2] + dx[-2] s[-1] = b[-1]
  double s_next;
  {
    const double dx2 = DX(K - 3), sl2 = SL(K - 3), d = x[K - 1] - x[K - 3];
    const double r = ((dxm1 * dxm1) * sl2 + (2.0 * d + dxm1) * dx2 * slm1) / d;
    s_next = (r - d * dp) / (dx2 - d * cp);
  }
  for (int k = K - 2; k >= 0; --k) {
    double* rk = w + (int64_t)k * kProfCoef;
    const double sk = rk[3] - rk[2] * s_next;
    const double dxk = DX(k), slk = SL(k);
    const double t = (sk + s_next - 2.0 * slk) / dxk;
    rk[0] = y[k];
    rk[1] = sk;
    rk[2] = (slk - sk) / dxk - t;
    rk[3] = t / dxk;
    s_next = sk;
  }
}

// ---------------------------------------------------------------------------------------
// Crossings, eqs.(5)-(8)
// ---------------------------------------------------------------------------------------
// root of the cubic c on [a, b], where it is monotone and changes sign: secant start, Newton
// steps kept inside the shrinking bracket (bisection otherwise), to full precision
__device__ double cubic_root(const double* c, double a, double b) {
  const double fa = pp0(c, a);
  double lo = a, hi = b;
  double x = a - fa * (b - a) / (pp0(c, b) - fa);
  for (int it = 0; it < 100; ++it) {
    const double f = pp0(c, x);
    if (f == 0.0) return x;
    if ((f < 0.0) == (fa < 0.0))
      lo = x;
    else
      hi = x;
    const double d = pp1(c, x);
    double xn = d != 0.0 ? x - f / d : 0.5 * (lo + hi);
    if (!(lo < xn && xn < hi)) xn = 0.5 * (lo + hi);
    if (xn == x || hi - lo <= 4e-16 * fmax(fmax(fabs(lo), fabs(hi)), 1e-300)) return xn;
    x = xn;
  }
  return x;
}

__global__ __launch_bounds__(kProfBlock) void profile_crossings_kernel(
    const double* __restrict__ knots, const double* __restrict__ coef, int32_t n_shapes, int32_t K,
    const lzq_profile_point* __restrict__ pts, int64_t n, int32_t max_cross, double* __restrict__ o_xi, double* __restrict__ o_dp, double* __restrict__ o_m,
    double* __restrict__ o_delta, int32_t* __restrict__ o_count) {
  const int64_t i = (int64_t)blockIdx.x * kProfBlock + threadIdx.x;
  if (i >= n) return;
  const ProfPt p = load_point(pts + i);
  if (p.shape < 0 || p.shape >= n_shapes) {  // bad shape index: no crossings, count -1
    o_count[i] = -1;
    return;
  }
  const double* x = knots + (int64_t)p.shape * K;
  const double* cf = coef + (int64_t)p.shape * (K - 1) * kProfCoef;
  const double vw = fmax(p.vw, 1e-12);
  int32_t cnt = 0;
  double last = 0.0;            // sign of the last nonzero boundary value (0: none yet)
  int pj = -1;                  // a boundary zero awaiting the next sign: interval pj, local pt
  double pt = 0.0;
  double cD[4], cM[4];
  auto emit = [&](int j, double t) {
    if (cnt < max_cross) {
      double rD[4], rM[4];  // the interval's Delta / m_mix rows (j may be a pending earlier one)
      interval_coefs(cf + (int64_t)j * kProfCoef, p, rD, rM);
      const double dprime = pp1(rD, t), m = pp0(rM, t);
      const int64_t o = i * max_cross + cnt;
      o_xi[o] = x[j] + t;
      o_dp[o] = dprime;
      o_m[o] = m;
      o_delta[o] = m * m / (2.0 * vw * fabs(dprime));
    }
    ++cnt;
  };
  // a zero exactly on a piece boundary is a crossing when the last nonzero value before it and
  // the first after it differ in sign (tests/profile_ref.py crossings)
  auto boundary = [&](double v, int j, double t) {
    if (v == 0.0) {
      if (pj < 0 && last != 0.0) {
        pj = j;
        pt = t;
      }
      return;
    }
    const double sg = v > 0.0 ? 1.0 : -1.0;
    if (pj >= 0 && sg != last) emit(pj, pt);
    pj = -1;
    last = sg;
  };
  for (int j = 0; j + 1 < K; ++j) {
    interval_coefs(cf + (int64_t)j * kProfCoef, p, cD, cM);
    const double L = x[j + 1] - x[j];
    // monotone pieces: cut at the stationary points of the cubic inside (0, L)
    double cuts[4];
    int nc = 0;
    cuts[nc++] = 0.0;
    const double A = 3.0 * cD[3], B = 2.0 * cD[2], C = cD[1];
    if (A != 0.0) {
      const double disc = B * B - 4.0 * A * C;
      if (disc > 0.0) {
        const double sq = sqrt(disc);
        const double q = -0.5 * (B + copysign(sq, B));
        double r1 = q / A, r2 = C / q;
        if (r2 < r1) {
          const double tt = r1;
          r1 = r2;
          r2 = tt;
        }
        if (0.0 < r1 && r1 < L) cuts[nc++] = r1;
        if (0.0 < r2 && r2 < L) cuts[nc++] = r2;
      }
    } else if (B != 0.0) {
      const double r = -C / B;
      if (0.0 < r && r < L) cuts[nc++] = r;
    }
    cuts[nc++] = L;
    for (int k = 0; k + 1 < nc; ++k) {
      const double a = cuts[k], b = cuts[k + 1];
      const double fa = pp0(cD, a), fb = pp0(cD, b);
      boundary(fa, j, a);
      if (fa * fb < 0.0) emit(j, cubic_root(cD, a, b));
      boundary(fb, j, b);
    }
  }
  o_count[i] = cnt;
}

// ---------------------------------------------------------------------------------------
// Propagation through the profile
// ---------------------------------------------------------------------------------------
// chi-like second-order dressed state of H = D sz + m sx with time derivatives (Dd, Ddd),
// (md, mdd) (lzq_propagator.hip dressed_basis with m(t) varying; tests/profile_ref.py
// dressed_chi_like): theta = atan2(m, D)/2, theta' = (m' D - m D')/(2 E^2), eps = theta'/(2E),
// eps' = theta''/(2E) - theta' E'/(2E^2), beta = -i eps - eps'/(2E).
// (out of line: its atan2 / sincos would otherwise set the step loop's register budget)
__device__ __noinline__ void dressed_chi_like(double D, double Dd, double Ddd, double m, double md, double mdd,
                                              Cplx& u0, Cplx& u1) {
  const double E2 = D * D + m * m;
  const double E = sqrt(E2);
  const double th = 0.5 * atan2(m, D);
  double s, c;
  sincos(th, &s, &c);
  const double w = md * D - m * Dd;
  const double thd = w / (2.0 * E2);
  const double Ed = (D * Dd + m * md) / E;
  const double thdd = (mdd * D - m * Ddd) / (2.0 * E2) - w * Ed / (E2 * E);
  const double eps = thd / (2.0 * E);
  const double epsd = thdd / (2.0 * E) - thd * Ed / (2.0 * E2);
  const double br = -epsd / (2.0 * E), bi = -eps;
  const double nrm = 1.0 / sqrt(1.0 + (br * br + bi * bi));
  const Cplx p0 = {(c - s * br) * nrm, -s * bi * nrm}, p1 = {(s + c * br) * nrm, c * bi * nrm};
  const bool plus = p0.re * p0.re + p0.im * p0.im >= p1.re * p1.re + p1.im * p1.im;
  if (plus) {
    u0 = p0;
    u1 = p1;
  } else {
    u0 = {(-s - c * br) * nrm, c * bi * nrm};
    u1 = {(c - s * br) * nrm, s * bi * nrm};
  }
}

__device__ __forceinline__ void edge_state(const double* cD, const double* cM, double t, double vw, Cplx& u0,
                                           Cplx& u1) {
  const double v2 = vw * vw;
  dressed_chi_like(pp0(cD, t), vw * pp1(cD, t), v2 * pp2(cD, t), pp0(cM, t), vw * pp1(cM, t), v2 * pp2(cM, t), u0,
                   u1);
}

// One sixth-order Magnus step of H = Delta sz + m sx on [t0, t0 + h] of the current knot interval
// (cD, cM its cubics in t = xi - xi_j; dt = h / v_w the step in time): H at the three Gauss nodes
// s -+ delta, s (s = t0 + h/2 the step's midpoint, delta = sqrt(15)/10 h), the Blanes-Casas-Ros
// commutator form (the alphas lie in the x-z plane, so the commutators are cross products), the
// exact SU(2) exponential.
// For a cubic P the three alphas are exact polynomials in the midpoint (round 4; the node values
// and their differences before):
//   alpha1 = dt P(s)
//   alpha2 = sqrt15/3 dt (P(s + delta) - P(s - delta)) = dt h (P'(s) + 0.15 h^2 c3)
//   alpha3 = 10/3 dt (P(s - delta) - 2 P(s) + P(s + delta)) = 0.5 dt h^2 P''(s) = dt h^2 (c2 + 3 c3 s),
// so an interval's MagnusPoly holds their coefficients and a step evaluates 3 + 2 + 1 fmas per
// axis (35 VALU before), with no cancellation in the differences.  The polynomials are written in
// u = s / h = st + 1/2 (coefficient of u^m = that of s^m times h^m): u is exact in a double, so the
// step's midpoint does not drift however many steps an interval takes (a running s += h drifted by
// up to ~2^-53 S relative, ~1.6e-10 at S = 1.4e6, which moved the long Weber fixtures 1.6e-10 -> 4.9e-10).
struct MagnusPoly {
  double ex[4], fx[3], gx[2];  // x: alpha1, alpha2, alpha3 of m as polynomials in u
  double ez[4], fz[3], gz[2];  // z: the same of Delta
};

// dk[m] = dt h^m: the coefficient of u^m in alpha1 is dk[m] c_m, and 3 dk[3] c3 is both alpha2's u^2
// and alpha3's u coefficient, so an interval costs what the polynomials in s did
__device__ __forceinline__ void axis_poly(const double (&c)[4], const double (&dk)[4], double q, double dk2x2,
                                          double dk3x3, double (&e)[4], double (&f)[3], double (&g)[2]) {
#pragma unroll
  for (int m = 0; m < 4; ++m) e[m] = dk[m] * c[m];
  f[0] = dk[1] * __builtin_fma(q, c[3], c[1]);
  f[1] = dk2x2 * c[2];
  f[2] = dk3x3 * c[3];
  g[0] = dk[2] * c[2];
  g[1] = f[2];
}

__device__ __forceinline__ MagnusPoly magnus_poly(const double (&cD)[4], const double (&cM)[4], double L, double Sd,
                                                  double ivw) {
  MagnusPoly mp;
  // h = L / S by a refined reciprocal (<= 1 ulp from the quotient; the restatement divides): S is
  // an integer >= 1, so v_rcp_f64 + two Newton steps
  double r = __builtin_amdgcn_rcp(Sd);
  double e = __builtin_fma(-Sd, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-Sd, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double h = L * r;
  const double dt = h * ivw, dth = dt * h, dth2 = dth * h;
  const double dk[4] = {dt, dth, dth2, dth2 * h};
  const double q = 0.15 * (h * h), dk2x2 = 2.0 * dk[2], dk3x3 = 3.0 * dk[3];
  axis_poly(cM, dk, q, dk2x2, dk3x3, mp.ex, mp.fx, mp.gx);
  axis_poly(cD, dk, q, dk2x2, dk3x3, mp.ez, mp.fz, mp.gz);
  return mp;
}

// u: the step's midpoint in units of the step, st + 1/2 (exact)
__device__ __forceinline__ void magnus6_step(const MagnusPoly& mp, double u, Cplx& p0, Cplx& p1) {
#define FMA __builtin_fma
  const double x1 = FMA(FMA(FMA(mp.ex[3], u, mp.ex[2]), u, mp.ex[1]), u, mp.ex[0]);
  const double z1 = FMA(FMA(FMA(mp.ez[3], u, mp.ez[2]), u, mp.ez[1]), u, mp.ez[0]);
  const double x2 = FMA(FMA(mp.fx[2], u, mp.fx[1]), u, mp.fx[0]);
  const double z2 = FMA(FMA(mp.fz[2], u, mp.fz[1]), u, mp.fz[0]);
  const double x3 = FMA(mp.gx[1], u, mp.gx[0]);
  const double z3 = FMA(mp.gz[1], u, mp.gz[0]);
  // Lie bracket of -i a.sigma, -i b.sigma is -i (2 a x b).sigma; the alphas lie in the x-z plane.
  // C1 = [alpha1, alpha2] = (0, c, 0), c = 2 ch; C2 = -[alpha1, 2 alpha3 + C1]/60 = (z1 c/30,
  // 2 C2h, -x1 c/30); Omega = alpha1 + alpha3/12 + (L x R)/240 with L = -20 alpha1 - alpha3 + C1,
  // R = alpha2 + C2 -- carried with the factors 2 of c and C2_y folded into the constants.
  const double ch = FMA(z1, x2, -(x1 * z2));
  const double c15 = ch * (1.0 / 15.0);
  const double C2h = FMA(x1, z3, -(z1 * x3)) * (1.0 / 30.0);        // C2_y / 2
  const double Lx = FMA(-20.0, x1, -x3), Lz = FMA(-20.0, z1, -z3);  // L = (Lx, c, Lz)
  const double Rx = FMA(z1, c15, x2), Rz = FMA(-x1, c15, z2);       // R = (Rx, 2 C2h, Rz)
  const double nx = FMA(FMA(ch, Rz, -(Lz * C2h)), 1.0 / 60.0, FMA(x3, 1.0 / 12.0, x1));
  const double ny = FMA(Lz, Rx, -(Lx * Rz)) * (1.0 / 120.0);
  const double nz = FMA(FMA(Lx, C2h, -(ch * Rx)), 1.0 / 60.0, FMA(z3, 1.0 / 12.0, z1));
  double cs, sc;
  cos_sinc_step(FMA(nx, nx, FMA(ny, ny, nz * nz)), cs, sc);
  su2_apply(cs, sc * nx, sc * ny, sc * nz, p0, p1);
#undef FMA
}

// The step rule samples each knot interval at t_q = (q/4) L, q = 0..4.  The shape's values there
// -- phi, Phi, phi', Phi' -- do not depend on the point, so they are evaluated once per launch
// per (shape, interval) (profile_samples_kernel, stream-ordered scratch, staged in LDS next to the
// coefficients); a point only combines them with its couplings.
// Stored as the products the rule's quadratic forms need (round 4): per sample
// [phi^2, phi Phi, Phi^2, phi'^2, phi' Phi', Phi'^2], so a point's E^2 = D^2 + m^2 =
// (y_B^2 + lambda^2) phi^2 - 2 y_B y_chi phi Phi + y_chi^2 Phi^2 is three operations per sample.
// With them (round 5) the interval's length and its spline row, so that everything an interval
// entry reads is one 320-B RECORD per (shape, interval):
//   [q0 .. q4 samples (30)] [L = x_{j+1} - x_j] [0] [phi c0..c3, Phi c0..c3]
// and one record past the last (pad: the propagation's record fetch of the last interval reads
// the next record's q = 0 slot, unused there).
constexpr int kSampD = 6;                    // doubles per sample
constexpr int kRecL = 5 * kSampD;            // the interval length
constexpr int kRecCoef = kRecL + 2;          // the spline row (kProfCoef doubles)
constexpr int kProfRec = kRecCoef + kProfCoef;  // doubles per interval record (40)

__global__ __launch_bounds__(kProfBlock) void profile_samples_kernel(const double* __restrict__ knots,
                                                                     const double* __restrict__ coef, int64_t n_rows,
                                                                     int32_t K, double* __restrict__ samp) {
  const int64_t r = (int64_t)blockIdx.x * kProfBlock + threadIdx.x;  // row = shape * (K - 1) + interval
  if (r > n_rows) return;
  double* o = samp + r * kProfRec;
  if (r == n_rows) {  // the pad record
#pragma unroll
    for (int k = 0; k < kProfRec; ++k) o[k] = 0.0;
    return;
  }
  const int64_t s = r / (K - 1), j = r - s * (K - 1);
  const double L = knots[s * K + j + 1] - knots[s * K + j];
  const double* c = coef + r * kProfCoef;
  o[kRecL] = L;
  o[kRecL + 1] = 0.0;
#pragma unroll
  for (int k = 0; k < kProfCoef; ++k) o[kRecCoef + k] = c[k];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const double t = (0.25 * q) * L;
    const double a = pp0(c, t), b = pp0(c + 4, t), da = pp1(c, t), db = pp1(c + 4, t);
    o[kSampD * q + 0] = a * a;
    o[kSampD * q + 1] = a * b;
    o[kSampD * q + 2] = b * b;
    o[kSampD * q + 3] = da * da;
    o[kSampD * q + 4] = da * db;
    o[kSampD * q + 5] = db * db;
  }
}

// Uniform Magnus steps on one interval (tests/profile_ref.py interval_steps).  The rate is
// sampled at t_q = (q/4) L, q = 0..3, from the interval's own samples and at its end from the NEXT
// interval's q = 0 sample (the same knot, whose spline value every interval but the last takes
// from the next piece; the last takes its own q = 4): a lane walking the intervals in order carries
// that end sample over as the next interval's start, 4 new samples per interval instead of 5.
// Per sample E^2 = D^2 + m^2 and |dH/dt|^2 = D'^2 + m'^2 (D = y_B phi - y_chi Phi, m = lambda phi)
// as the quadratic forms A phi^2 + B phi Phi + C Phi^2 (and the same in phi', Phi') of the point's
// RuleForm; over the interval their maxima e2, h2, then in squares
//   W2 = max(e2, kHdotRate^2 v_w sqrt(h2)),  S = max(n_min, ceil(spr (L (1/v_w)) sqrt(W2)))
// -- max(E, kHdotRate sqrt(v_w |dH/dt|)) squared: two correctly rounded square roots, no division.
struct RuleForm {
  double A, B, C;  // y_B^2 + lambda^2, -2 y_B y_chi, y_chi^2
};

__device__ __forceinline__ RuleForm rule_form(const ProfPt& p) {
  return {__builtin_fma(p.yB, p.yB, p.lam * p.lam), (-2.0 * p.yB) * p.ychi, p.ychi * p.ychi};
}

struct Rates {
  double e2, h2;
};

__device__ __forceinline__ Rates sample_rates(const double* __restrict__ sr, const RuleForm& f) {
  return {__builtin_fma(f.A, sr[0], __builtin_fma(f.B, sr[1], f.C * sr[2])),
          __builtin_fma(f.A, sr[3], __builtin_fma(f.B, sr[4], f.C * sr[5]))};
}

// fmax for the rule: v_max_f64 as such.  fmax's lowering first quiets signalling NaNs of operands
// it cannot prove canonical (a v_max_f64 x, x for each carried or loaded value, three per interval
// entry); the rule's operands are never signalling NaNs, and for every other input v_max_f64 is
// fmax (a quiet NaN operand yields the other).
#ifndef LZQ_PROF_ASM_MAX
#define LZQ_PROF_ASM_MAX 1
#endif
__device__ __forceinline__ double rmax(double a, double b) {
  if (!LZQ_PROF_ASM_MAX) return fmax(a, b);
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ Rates rates_max(Rates u, Rates v) { return {rmax(u.e2, v.e2), rmax(u.h2, v.h2)}; }

// the end sample of interval j (of K - 1): the next interval's q = 0, or the last interval's own q = 4
__device__ __forceinline__ const double* end_sample(const double* __restrict__ sm, int j, int K) {
  return j + 2 < K ? sm + (j + 1) * kProfRec : sm + j * kProfRec + 4 * kSampD;
}

// interval j's rates from its start sample's (`start`, carried) and its q = 1..3 and end samples;
// `end` returns the end sample's rates (the next interval's start)
__device__ __forceinline__ Rates interval_rates(const double* __restrict__ sm, int j, int K, const RuleForm& f,
                                                Rates start, Rates& end) {
  const double* sr = sm + j * kProfRec;
  Rates r = start;
#pragma unroll
  for (int q = 1; q < 4; ++q) r = rates_max(r, sample_rates(sr + kSampD * q, f));
  end = sample_rates(end_sample(sm, j, K), f);
  return rates_max(r, end);
}

// The rule's square roots: the device library's sqrt is v_rsq_f64 + two Goldschmidt / Newton
// refinements, wrapped in range fix-ups (a 2^256 pre-scale below 2^-767, 0 / +inf passed through).
// When every lane's argument lies in [2^-767, DBL_MAX] the fix-ups are identities, so the bare
// sequence gives the library's bits; otherwise the wave takes the library sqrt.
#ifndef LZQ_PROF_RULE_SQRT
#define LZQ_PROF_RULE_SQRT 1
#endif
// every active lane's x in [2^-767, DBL_MAX] (NaN: no): the two compares' lane masks straight into
// SGPRs (a ballot of the C++ condition re-materialises it as a VGPR and compares that again)
#ifndef LZQ_PROF_VOTE_ASM
#define LZQ_PROF_VOTE_ASM 1
#endif
__device__ __forceinline__ bool wave_in_sqrt_range(double x) {
  if (!LZQ_PROF_VOTE_ASM) return __all(x >= 0x1p-767 && x <= 0x1.fffffffffffffp+1023);
  uint64_t lo, hi;
  asm("v_cmp_le_f64_e64 %0, %1, %2" : "=s"(lo) : "s"(0x1p-767), "v"(x));
  asm("v_cmp_ge_f64_e64 %0, %1, %2" : "=s"(hi) : "s"(0x1.fffffffffffffp+1023), "v"(x));
  return (lo & hi) == __builtin_amdgcn_read_exec();
}
__device__ __forceinline__ double rule_sqrt(double x) {
  if (LZQ_PROF_RULE_SQRT && wave_in_sqrt_range(x)) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
  }
  return sqrt(x);
}

__device__ __forceinline__ double steps_of(Rates r, double L, const ProfPt& p, double ivw, double spr, int32_t n_min) {
  const double W2 = rmax(r.e2, (kHdotRate * kHdotRate) * (p.vw * rule_sqrt(r.h2)));
  return rmax((double)n_min, ceil((spr * (L * ivw)) * rule_sqrt(W2)));
}

// interval j on its own (no carried start): the same samples and operations, the same count
__device__ __forceinline__ double interval_steps(const double* __restrict__ sm, int j, int K, const ProfPt& p,
                                                 double L, double ivw, double spr, int32_t n_min) {
  const RuleForm f = rule_form(p);
  Rates end;
  const Rates r = interval_rates(sm, j, K, f, sample_rates(sm + j * kProfRec, f), end);
  return steps_of(r, L, p, ivw, spr, n_min);
}

// Launch order.  A lane's cost is its Magnus step count, which scales as 1/v_w and with the
// couplings, so a wave of random points waits on its slowest lane in every knot interval.  For
// large batches the kernel reads its point index from a launch order; each lane still computes
// one point from its own inputs, so P is bit-identical to index order.  The estimate of a point's
// step count: the step rule on every kProfCostStride-th interval, x kProfCostStride, 4 bins per
// octave (0 = costliest).
// Launch key of the interval loop (round 4): the loop kernel steps a wave through interval j for
// its lanes' largest S_j, so lanes should agree in the whole step PROFILE, not only in the total.
// Points of one shape whose totals are close and whose couplings put Delta's zeros at the same
// places (Delta = y_B phi - y_chi Phi vanishes where phi / Phi = y_chi / y_B: the angle
// atan(y_chi / y_B)) have nearly the same S_j, so the key is (shape, cost bin, angle bin), radix
// sorted (stable) -- tools/profile_order_model.py: executed / useful lane-steps 1.31 with the cost
// bins alone, 1.16 with this key, on tools/bench_profile.py's workload.
// Round 6: 6 cost bins per octave, and the angle bins walked up in one cost bin and down in the
// next (boustrophedon), so a wave that straddles two cost bins holds neighbouring angles, not
// the two ends of the range: the model's 1.131 -> 1.102 (tools/profile_order_model.py).
constexpr int kAngleBins = 256;
#ifndef LZQ_PROF_KEY_SERP
#define LZQ_PROF_KEY_SERP 1
#endif
#ifndef LZQ_PROF_KEY_BINS
#define LZQ_PROF_KEY_BINS 6
#endif
constexpr double kKeyBinsPerOctave = LZQ_PROF_KEY_BINS;  // 128 bins: saturate at 2^21 steps per point
__global__ __launch_bounds__(kProfBlock) void profile_key_kernel(const double* __restrict__ knots, int32_t n_shapes,
                                                                 int32_t K, const lzq_profile_point* __restrict__ pts,
                                                                 int64_t n, double spr, int32_t n_min,
                                                                 const double* __restrict__ samp,
                                                                 uint32_t* __restrict__ keys, int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * kProfBlock + threadIdx.x;
  if (i >= n) return;
  const ProfPt p = load_point(pts + i);
  double st = 0.0;
  const bool valid = p.vw > 0.0 && p.shape >= 0 && p.shape < n_shapes;
  if (valid) {
    auto cost = [&](const double* __restrict__ x, const double* __restrict__ sm) {
      const double ivw = 1.0 / p.vw;
      double c = 0.0;
      for (int j = 0; j + 1 < K; j += kProfCostStride) c += interval_steps(sm, j, K, p, x[j + 1] - x[j], ivw, spr, n_min);
      return c * kProfCostStride;
    };
    const int64_t s0 = __builtin_amdgcn_readfirstlane(p.shape), sl = p.shape;  // scalar loads when uniform
    st = (LZQ_PROF_UNIFORM && __all(p.shape == s0)) ? cost(knots + s0 * K, samp + s0 * (K - 1) * kProfRec)
                                                    : cost(knots + sl * K, samp + sl * (K - 1) * kProfRec);
  }
  const double cb = st == st ? fmin(fmax(kKeyBinsPerOctave * log2(1.0 + st), 0.0), (double)(kCostBins - 1)) : 0.0;
  const uint32_t cost = (uint32_t)((kCostBins - 1) - (int32_t)cb);  // 0 = costliest
  const double ang = atan(p.ychi / p.yB);                            // (-pi/2, pi/2); NaN for 0/0
  const double af = ang == ang ? (ang * (1.0 / 3.141592653589793) + 0.5) * kAngleBins : 0.0;
  uint32_t ab = (uint32_t)fmin(fmax(af, 0.0), (double)(kAngleBins - 1));
  if (LZQ_PROF_KEY_SERP && (cost & 1)) ab = (kAngleBins - 1) - ab;  // boustrophedon: see kKeyBinsPerOctave
  const uint32_t sh = valid ? (uint32_t)min(p.shape, 65534) : (uint32_t)min(n_shapes, 65535);  // invalid: last
  keys[i] = (sh << 15) | (cost << 8) | ab;  // shape, 7 + 8 bits
  idx[i] = (int32_t)i;
}

// An interval's entry reads the SPAN of the records from its own q = 1 sample up to the next
// record's q = 0 (its end sample): 40 doubles, 320 B, contiguous.  Offsets in the span:
constexpr int kSpanOff = kSampD;                   // the span starts at the record's q = 1
constexpr int kSpan = kProfRec;                    // doubles
constexpr int kSpQ4 = 3 * kSampD;                  // the record's own q = 4 (the last interval's end)
constexpr int kSpL = kRecL - kSpanOff;             // L
constexpr int kSpCoef = kRecCoef - kSpanOff;       // the spline row
constexpr int kSpNext = kProfRec - kSpanOff;       // the next record's q = 0

// Interval entry from its span s: the step rule's count (rates carried in `start`), Delta / m
// coefficients and Magnus polynomials -- the operations of the round-4 loop in the same order, so
// S and every bit of the polynomials are unchanged.  All of the span is read before any branch, so
// its loads issue together.  False for a non-finite or absurd count.  S: the count as a double (an
// integer; 0 for a bad one) -- the step loop runs on the midpoint u = 1/2, 3/2, .. < S, exact in a
// double, without an integer counter.
__device__ __forceinline__ bool enter_interval(const double* __restrict__ s, bool last, const ProfPt& p,
                                               const RuleForm& rf, double ivw, double spr, int32_t n_min, Rates& start,
                                               double (&cD)[4], double (&cM)[4], MagnusPoly& mp, double& S) {
  interval_coefs_fma(s + kSpCoef, p, cD, cM);
  Rates r = start;
#pragma unroll
  for (int q = 0; q < 3; ++q) r = rates_max(r, sample_rates(s + kSampD * q, rf));
  const Rates end = sample_rates(s + (last ? kSpQ4 : kSpNext), rf);
  r = rates_max(r, end);
  start = end;
  const double L = s[kSpL];
  const double Sd = steps_of(r, L, p, ivw, spr, n_min);
  mp = magnus_poly(cD, cM, L, Sd, ivw);
  const bool good = Sd <= kMaxIntervalSteps;
  S = good ? Sd : 0.0;
  return good;
}

// The wave's LDS stage: two spans (interval j, j + 1) per wave
struct alignas(16) ProfStage {
  double span[2][kSpan];
};

// One point through the whole profile (rec: its shape's interval records).  Returns P, NaN for a
// non-finite or absurd step count (that lane takes no further steps).
//   kStaged: the wave's points share the shape and all 64 lanes are here -- the record spans go
//   through the wave's LDS stage, interval j + 1's fetched (global_load_lds, 20 lanes x 16 B) while
//   the wave steps interval j, so an entry waits on LDS, not on a trip to L2 (round 4: five
//   dependent scalar loads per entry, 24% of the waves' cycles in SQ_WAIT_ANY).
//   Otherwise each lane reads its own spans from global memory.
template <bool kStaged>
__device__ __forceinline__ double propagate_point(const double* __restrict__ rec, int32_t K, const ProfPt& p,
                                                  double spr, int32_t n_min, ProfStage* stage) {
  const int lane = (int)(threadIdx.x & 63);
  auto fetch = [&](int j, double* dst) {  // interval j's span into the stage buffer dst
    if (lane < kSpan / 2)
      __builtin_amdgcn_global_load_lds(rec + (int64_t)j * kProfRec + kSpanOff + 2 * lane, dst, 16, 0, 0);
  };
  if (kStaged) fetch(0, &stage->span[0][0]);
  const double ivw = 1.0 / p.vw;
  double cD[4], cM[4];
  interval_coefs_fma(rec + kRecCoef, p, cD, cM);
  Cplx p0, p1;
  edge_state(cD, cM, 0.0, p.vw, p0, p1);
  const RuleForm rf = rule_form(p);
  Rates start = sample_rates(rec, rf);  // interval 0's q = 0; then each interval's end is the next one's start
  bool ok = true;
  // interval j from its span s; staged: then interval j + 1's span into `next`
  auto interval = [&](int j, const double* s, double* next) {
    MagnusPoly mp;
    double S;
    ok = enter_interval(s, j + 2 == K, p, rf, ivw, spr, n_min, start, cD, cM, mp, S) && ok;
    if (kStaged && j + 2 < K) fetch(j + 1, next);
    if (!ok) S = 0.0;
    if (LZQ_PROF_PAIR) {
      double u = 0.5;
      for (; u + 1.0 < S; u += 2.0) {
        magnus6_step(mp, u, p0, p1);
        magnus6_step(mp, u + 1.0, p0, p1);
      }
      if (u < S) magnus6_step(mp, u, p0, p1);
    } else {
      for (double u = 0.5; u < S; u += 1.0) magnus6_step(mp, u, p0, p1);
    }
  };
  if constexpr (kStaged) {
    // two intervals per iteration, so each one's LDS buffer is a constant offset
    double* b0 = &stage->span[0][0];
    double* b1 = &stage->span[1][0];
    for (int j = 0; j + 1 < K; j += 2) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this interval's span has landed in LDS
      interval(j, b0, b1);
      if (j + 2 < K) {
        __builtin_amdgcn_s_waitcnt(0x0F70);
        interval(j + 1, b1, b0);
      }
    }
  } else {
    for (int j = 0; j + 1 < K; ++j) interval(j, rec + (int64_t)j * kProfRec + kSpanOff, nullptr);
  }
  if (!ok) return __builtin_nan("");
  // the last interval's row again for the end state (not kept live across the step loop)
  const double* s = kStaged ? &stage->span[(K - 2) & 1][0] : rec + (int64_t)(K - 2) * kProfRec + kSpanOff;
  interval_coefs_fma(s + kSpCoef, p, cD, cM);
  Cplx u0, u1;
  edge_state(cD, cM, s[kSpL], p.vw, u0, u1);
  const Cplx a = inner(u0, u1, p0, p1);
  const double norm = p0.re * p0.re + p0.im * p0.im + p1.re * p1.re + p1.im * p1.im;
  return 1.0 - (a.re * a.re + a.im * a.im) / norm;
}

#ifndef LZQ_PROF_STAGE
#define LZQ_PROF_STAGE 1  // 0: every wave reads its spans from global memory
#endif

// The interval loop walks every lane of a wave through the same knot interval j, so when the wave's
// points share one shape (the keyed launch order makes that the rule) the interval's records are
// the same addresses for all lanes: those waves stage them in LDS (propagate_point<true>).
// Mixed-shape and partial waves take the per-lane path; both run the same operations on the same
// values, so P does not depend on the path.
__global__ __launch_bounds__(kProfBlock, LZQ_PROF_MIN_WAVES) void profile_propagate_kernel(
    int32_t n_shapes, int32_t K, const lzq_profile_point* __restrict__ pts, int64_t n, double spr, int32_t n_min,
    const int32_t* __restrict__ order, const double* __restrict__ rec, double* __restrict__ P_out) {
  __shared__ ProfStage stage[kProfBlock / 64];
  const int64_t tid = (int64_t)blockIdx.x * kProfBlock + threadIdx.x;
  if (tid >= n) return;
  const int64_t i = order ? (int64_t)order[tid] : tid;
  const ProfPt p = load_point(pts + i);
  if (!(p.vw > 0.0) || p.shape < 0 || p.shape >= n_shapes) {  // bad wall speed or shape index
    P_out[i] = __builtin_nan("");
    return;
  }
  const int32_t sh0 = __builtin_amdgcn_readfirstlane(p.shape);
  double P;
  if (LZQ_PROF_STAGE && __builtin_amdgcn_read_exec() == ~0ull && __all(p.shape == sh0)) {
    P = propagate_point<true>(rec + (int64_t)sh0 * (K - 1) * kProfRec, K, p, spr, n_min, &stage[threadIdx.x >> 6]);
  } else {
    P = propagate_point<false>(rec + (int64_t)p.shape * (K - 1) * kProfRec, K, p, spr, n_min, nullptr);
  }
  P_out[i] = P;
}

// ---------------------------------------------------------------------------------------
// Flattened propagation (LZQ_TUNE_PROFILE_FLAT, the default).  The interval-by-interval loop
// above runs, per knot interval, the step rule and the coefficient rows for every lane and then
// max-over-the-wave Magnus steps: with ~2.2 steps per interval on typical profiles, lanes idle
// while the wave finishes its longest lane's steps, and the per-interval work is paid once per
// interval whatever a lane needs (253 VALU per useful lane-step, profiles/round3/profile_pmc.json).
// Here the step rule runs ahead of the propagation, one lane per point over all its intervals
// (profile_steps_kernel: no lane waits, and the exact step totals order the launch), and the
// propagation is ONE loop of Magnus steps per lane: a lane whose interval is done enters its next
// one (its Delta / m rows and step geometry, ~35 VALU) in the same iteration while the other lanes
// keep stepping.  Every lane performs exactly the interval loop's operations on its own point, so
// P is bit-identical to profile_propagate_kernel (tests/test_gpu_profile.py).
//
// Step counts: uint16 per (point, interval), [point][interval] so a lane walks one row (one 64-B
// line per 32 intervals).  0 = non-finite / absurd (P = NaN); kStepsRecompute = the count did
// not fit (the lane re-derives it from the samples).
constexpr uint16_t kStepsRecompute = 0xFFFF;

__global__ __launch_bounds__(kProfBlock) void profile_steps_kernel(const double* __restrict__ knots, int32_t n_shapes,
                                                                   int32_t K, const lzq_profile_point* __restrict__ pts,
                                                                   int64_t n, double spr, int32_t n_min,
                                                                   const double* __restrict__ samp,
                                                                   uint16_t* __restrict__ steps,
                                                                   int32_t* __restrict__ bins, int32_t* __restrict__ hist) {
  __shared__ int32_t lh[kCostBins];
  if (bins)
    for (int t = threadIdx.x; t < kCostBins; t += kProfBlock) lh[t] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kProfBlock + threadIdx.x;
  if (i < n) {
    const ProfPt p = load_point(pts + i);
    double tot = 0.0;
    if (p.vw > 0.0 && p.shape >= 0 && p.shape < n_shapes) {
      const double* x = knots + (int64_t)p.shape * K;
      const double* sm = samp + (int64_t)p.shape * (K - 1) * kProfRec;
      uint16_t* row = steps + i * (int64_t)(K - 1);
      const double ivw = 1.0 / p.vw;
      const RuleForm rf = rule_form(p);
      Rates start = sample_rates(sm, rf);
      for (int j = 0; j + 1 < K; ++j) {
        Rates end;
        const double Sd = steps_of(interval_rates(sm, j, K, rf, start, end), x[j + 1] - x[j], p, ivw, spr, n_min);
        start = end;
        row[j] = !(Sd <= kMaxIntervalSteps) ? (uint16_t)0 : (Sd < (double)kStepsRecompute ? (uint16_t)Sd : kStepsRecompute);
        tot += Sd;
      }
    }
    if (bins) {
      const double key = tot == tot ? fmin(fmax(4.0 * log2(1.0 + tot), 0.0), (double)(kCostBins - 1)) : 0.0;
      const int32_t b = (kCostBins - 1) - (int32_t)key;
      bins[i] = b;
      atomicAdd(&lh[b], 1);
    }
  }
  if (!bins) return;
  __syncthreads();
  for (int t = threadIdx.x; t < kCostBins; t += kProfBlock)
    if (lh[t]) atomicAdd(&hist[t], lh[t]);
}

__global__ __launch_bounds__(kProfBlock, LZQ_PROF_MIN_WAVES) void profile_flat_kernel(
    const double* __restrict__ knots, const double* __restrict__ coef, int32_t n_shapes, int32_t K,
    const lzq_profile_point* __restrict__ pts, int64_t n, double spr, int32_t n_min, const int32_t* __restrict__ order,
    const double* __restrict__ samp, const uint16_t* __restrict__ steps, double* __restrict__ P_out) {
  const int64_t tid = (int64_t)blockIdx.x * kProfBlock + threadIdx.x;
  if (tid >= n) return;
  const int64_t i = order ? (int64_t)order[tid] : tid;
  const ProfPt p = load_point(pts + i);
  if (!(p.vw > 0.0) || p.shape < 0 || p.shape >= n_shapes) {  // bad wall speed or shape index
    P_out[i] = __builtin_nan("");
    return;
  }
  const double* x = knots + (int64_t)p.shape * K;
  const double* cf = coef + (int64_t)p.shape * (K - 1) * kProfCoef;
  const double* sm = samp + (int64_t)p.shape * (K - 1) * kProfRec;
  const uint16_t* srow = steps + i * (int64_t)(K - 1);
  const double ivw = 1.0 / p.vw;
  double cD[4], cM[4];
  interval_coefs_fma(cf, p, cD, cM);
  Cplx p0, p1;
  edge_state(cD, cM, 0.0, p.vw, p0, p1);
  // interval j's step count and Magnus polynomials; false for a non-finite / absurd count (P = NaN)
  int S = 0;
  MagnusPoly mp;
  double smid = 0.0;  // the current step's midpoint, in steps
  auto enter = [&](int j) -> bool {
    const double L = x[j + 1] - x[j];
    const uint16_t sr = srow[j];
    const double Sd = sr == kStepsRecompute ? interval_steps(sm, j, K, p, L, ivw, spr, n_min) : (double)sr;
    if (sr == 0 || !(Sd <= kMaxIntervalSteps)) return false;
    S = (int)Sd;
    mp = magnus_poly(cD, cM, L, Sd, ivw);
    smid = 0.5;
    return true;
  };
  bool ok = enter(0);
  int j = 0, st = 0;
  while (ok) {
    if (st == S) {  // this lane's interval is done: enter the next one (the others keep stepping)
      if (++j == K - 1) break;
      interval_coefs_fma(cf + j * kProfCoef, p, cD, cM);
      ok = enter(j);
      if (!ok) break;
      st = 0;
    }
    magnus6_step(mp, smid, p0, p1);
    smid += 1.0;
    ++st;
  }
  if (!ok) {
    P_out[i] = __builtin_nan("");
    return;
  }
  Cplx u0, u1;
  edge_state(cD, cM, x[K - 1] - x[K - 2], p.vw, u0, u1);
  const Cplx a = inner(u0, u1, p0, p1);
  const double norm = p0.re * p0.re + p0.im * p0.im + p1.re * p1.re + p1.im * p1.im;
  P_out[i] = 1.0 - (a.re * a.re + a.im * a.im) / norm;
}

int g_profile_flat = 0;  // lzq_tune(LZQ_TUNE_PROFILE_FLAT): the interval loop is the default

}  // namespace lzq

namespace {
bool shape_args_ok(const double* knots, const double* coef, int32_t n_shapes, int32_t K) {
  return knots && coef && n_shapes > 0 && K >= 4;
}

constexpr int64_t kStepsScratchBytes = int64_t(1) << 29;  // per slice of the flattened propagation

// The flattened propagation in slices of points whose step-count rows fit kStepsScratchBytes: per
// slice the step rule (+ the longest-first order for slices of >= kProfSortMin points) and the
// Magnus loop, all stream-ordered.
int profile_flat_launch(const double* d_knots, const double* d_coef, int32_t n_shapes, int32_t K,
                        const lzq_profile_point* d_points, int64_t n, double spr, int32_t n_min, const double* samp,
                        double* d_P, hipStream_t st) {
  const int64_t row = 2 * (int64_t)(K - 1);
  const int64_t per = std::max<int64_t>(1024, std::min<int64_t>(n, kStepsScratchBytes / row));
  const int64_t m_max = std::min(per, n);
  char* ws = nullptr;
  const size_t bytes = (size_t)m_max * (size_t)row + sizeof(int32_t) * (size_t)(2 * m_max + 2 * lzq::kCostBins) + 256;
  hipError_t e = hipMallocAsync((void**)&ws, bytes, st);
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  uint16_t* steps = reinterpret_cast<uint16_t*>(ws);
  int32_t* bins = reinterpret_cast<int32_t*>(ws + (((size_t)m_max * (size_t)row + 255) & ~(size_t)255));
  int32_t *ord = bins + m_max, *hist = ord + m_max, *offs = hist + lzq::kCostBins;
  int rc = LZQ_OK;
  for (int64_t s0 = 0; s0 < n && rc == LZQ_OK && e == hipSuccess; s0 += per) {
    const int64_t m = std::min(per, n - s0);
    const int64_t nb = (m + lzq::kProfBlock - 1) / lzq::kProfBlock;
    const bool sort = LZQ_PROF_SORT && m >= lzq::kProfSortMin;
    if (sort) e = hipMemsetAsync(hist, 0, sizeof(int32_t) * lzq::kCostBins, st);
    if (e != hipSuccess) break;
    hipLaunchKernelGGL(lzq::profile_steps_kernel, dim3((unsigned)nb), dim3(lzq::kProfBlock), 0, st, d_knots, n_shapes, K,
                       d_points + s0, m, spr, n_min, samp, steps, sort ? bins : nullptr, sort ? hist : nullptr);
    if (sort) rc = lzq::launch_bin_order(bins, hist, offs, m, ord, st);
    if (rc != LZQ_OK) break;
    hipLaunchKernelGGL(lzq::profile_flat_kernel, dim3((unsigned)nb), dim3(lzq::kProfBlock), 0, st, d_knots, d_coef,
                       n_shapes, K, d_points + s0, m, spr, n_min, sort ? (const int32_t*)ord : nullptr, samp,
                       (const uint16_t*)steps, d_P + s0);
    e = hipGetLastError();
  }
  const hipError_t ef = hipFreeAsync(ws, st);
  if (rc != LZQ_OK) return rc;
  if (e == hipSuccess) e = ef;
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  return LZQ_OK;
}
}  // namespace

extern "C" int lzq_profile_splines(const double* d_knots, const double* d_phi, const double* d_Phi, int32_t n_shapes,
                                   int32_t n_knots, double* d_coef, int32_t* d_bad, void* stream) {
  if (!d_knots || !d_phi || !d_Phi || !d_coef || !d_bad || n_shapes <= 0 || n_knots < 4)
    return lzq_set_error(LZQ_EINVAL, "lzq_profile_splines: bad arguments (need n_shapes > 0, n_knots >= 4, "
                                     "non-null buffers)");
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(d_bad, 0, sizeof(int32_t) * (size_t)n_shapes, st);
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  const int64_t lanes = 2 * (int64_t)n_shapes;
  hipLaunchKernelGGL(lzq::profile_spline_kernel, dim3((unsigned)((lanes + lzq::kProfBlock - 1) / lzq::kProfBlock)),
                     dim3(lzq::kProfBlock), 0, st, d_knots, d_phi, d_Phi, n_shapes, n_knots, d_coef, d_bad);
  e = hipGetLastError();
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  return LZQ_OK;
}

extern "C" int lzq_profile_crossings(const double* d_knots, const double* d_coef, int32_t n_shapes, int32_t n_knots,
                                     const lzq_profile_point* d_points, int64_t n, int32_t max_cross, double* d_xi,
                                     double* d_dprime, double* d_m_mix, double* d_delta, int32_t* d_count,
                                     void* stream) {
  if (!shape_args_ok(d_knots, d_coef, n_shapes, n_knots) || n < 0 || max_cross < 0 ||
      (n > 0 && (!d_points || !d_count || (max_cross > 0 && (!d_xi || !d_dprime || !d_m_mix || !d_delta)))))
    return lzq_set_error(LZQ_EINVAL, "lzq_profile_crossings: bad arguments (need n_shapes > 0, n_knots >= 4, "
                                     "n >= 0, max_cross >= 0, non-null buffers)");
  if (n == 0) return LZQ_OK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(lzq::profile_crossings_kernel, dim3((unsigned)((n + lzq::kProfBlock - 1) / lzq::kProfBlock)),
                     dim3(lzq::kProfBlock), 0, st, d_knots, d_coef, n_shapes, n_knots, d_points, n, max_cross, d_xi, d_dprime,
                     d_m_mix, d_delta, d_count);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  return LZQ_OK;
}

extern "C" int lzq_lz_propagate_profile(const double* d_knots, const double* d_coef, int32_t n_shapes,
                                        int32_t n_knots, const lzq_profile_point* d_points, int64_t n,
                                        double steps_per_radian, int32_t min_steps, double* d_P, void* stream) {
  if (!shape_args_ok(d_knots, d_coef, n_shapes, n_knots) || n < 0 || !(steps_per_radian >= 0.5) ||
      !(steps_per_radian <= 1000.0) || min_steps < 1 || min_steps > 1000000 || (n > 0 && (!d_points || !d_P)))
    return lzq_set_error(LZQ_EINVAL, "lzq_lz_propagate_profile: bad arguments (need n_shapes > 0, n_knots >= 4, "
                                     "n >= 0, 0.5 <= steps_per_radian <= 1000, 1 <= min_steps <= 1e6)");
  if (n == 0) return LZQ_OK;
  if (n > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_lz_propagate_profile: n too large");
  hipStream_t st = (hipStream_t)stream;
  // the shapes' step-rule samples: stream-ordered scratch
  const int64_t rows = (int64_t)n_shapes * (n_knots - 1);
  double* samp = nullptr;
  hipError_t e = hipMallocAsync((void**)&samp, sizeof(double) * lzq::kProfRec * (size_t)(rows + 1), st);
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  hipLaunchKernelGGL(lzq::profile_samples_kernel, dim3((unsigned)((rows + 1 + lzq::kProfBlock - 1) / lzq::kProfBlock)),
                     dim3(lzq::kProfBlock), 0, st, d_knots, d_coef, rows, n_knots, samp);
  if (lzq::g_profile_flat) {
    const int rc2 = profile_flat_launch(d_knots, d_coef, n_shapes, n_knots, d_points, n, steps_per_radian, min_steps,
                                        samp, d_P, st);
    const hipError_t ef = hipFreeAsync(samp, st);
    if (rc2 != LZQ_OK) return rc2;
    if (ef != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(ef));
    return LZQ_OK;
  }
  const int64_t nb = (n + lzq::kProfBlock - 1) / lzq::kProfBlock;
  // launch order (profile_key_kernel): keys and indices, their sorted copies and the radix sort's
  // temporary storage in one scratch
  char* ws = nullptr;
  const int32_t* order = nullptr;
  int rc = LZQ_OK;
  if (LZQ_PROF_SORT && n >= lzq::kProfSortMin) {
    size_t tmp_bytes = 0;
    // sort only the key bits in use: the shape field needs bits for n_shapes + 1 values (invalid last)
    int end_bit = 15;
    while (end_bit < 31 && (int64_t(1) << (end_bit - 15)) <= std::min<int64_t>(n_shapes, 65535)) ++end_bit;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, end_bit, st);
    const size_t arr = ((size_t)n * 4 + 255) & ~(size_t)255;
    if (e == hipSuccess) e = hipMallocAsync((void**)&ws, 4 * arr + tmp_bytes, st);
    if (e == hipSuccess) {
      uint32_t* keys = (uint32_t*)ws;
      uint32_t* keys_sorted = (uint32_t*)(ws + arr);
      int32_t* idx = (int32_t*)(ws + 2 * arr);
      int32_t* ord = (int32_t*)(ws + 3 * arr);
      hipLaunchKernelGGL(lzq::profile_key_kernel, dim3((unsigned)nb), dim3(lzq::kProfBlock), 0, st, d_knots, n_shapes,
                         n_knots, d_points, n, steps_per_radian, min_steps, (const double*)samp, keys, idx);
      e = hipGetLastError();
      if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs((void*)(ws + 4 * arr), tmp_bytes, (const uint32_t*)keys, keys_sorted,
                                               (const int32_t*)idx, ord, (int)n, 0, end_bit, st);
      order = ord;
    }
  }
  if (e == hipSuccess && rc == LZQ_OK) {
    hipLaunchKernelGGL(lzq::profile_propagate_kernel, dim3((unsigned)nb), dim3(lzq::kProfBlock), 0, st, n_shapes,
                       n_knots, d_points, n, steps_per_radian, min_steps, order, (const double*)samp, d_P);
    e = hipGetLastError();
  }
  if (ws) {
    const hipError_t ef = hipFreeAsync(ws, st);
    if (e == hipSuccess) e = ef;
  }
  const hipError_t ef = hipFreeAsync(samp, st);
  if (e == hipSuccess) e = ef;
  if (rc != LZQ_OK) return rc;
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  return LZQ_OK;
}
