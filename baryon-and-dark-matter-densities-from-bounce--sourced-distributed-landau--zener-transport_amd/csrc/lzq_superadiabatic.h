// lzq_superadiabatic.h -- superadiabatic frames of a two-level crossing, shared
// device code of the LZ propagator.  Not ABI.  tests/lz_ref.py (sa_levels, sa_to_frame,
// sa_from_frame, sa_phase, sa_core_tau) restates every function here.
//
// Units: alpha = |dD/dt| of the cell, tau = sqrt(alpha) t, Dh = D/sqrt(alpha) = sg tau (sg = +-1),
// mh = m/sqrt(alpha).  Iterated adiabatic frames (Berry's superadiabatic iteration):
//   level j: H_j = e_j sz + g_j sigma_a,  a = x for even j, y for odd j,  e_0 = Dh, g_0 = mh;
//   V_j = exp(-i theta_j sy) (even j) or exp(+i theta_j sx) (odd j), theta_j = atan2(g_j, e_j)/2,
//   diagonalises it; in the next frame e_{j+1} = sqrt(e_j^2 + g_j^2) and the coupling is
//   g_{j+1} = -theta_j' (even j) or +theta_j' (odd j).
// Far from the crossing the couplings fall like g_j ~ mh E^-(2j+1): a state is followed in the
// frame of order N (psi = V_0 .. V_{N-1} phi) with phi's components only picking up
// exp(-+ i int e_N dtau), and the error is the first neglected angle, |theta_N| at the inner end
// of the stretch (measured against a converged ODE solve for N = 6 .. 10; tests/lz_ref.py).
// theta_j' needs the j-th derivative of the level-0 data, so the levels run on truncated Taylor
// series ("jets") in tau of length N.  The half-angles come from cos 2theta = e/r and
// sin 2theta = g/r with r = e_{j+1} (already computed): no atan2, no sincos.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>

#include "lzq_su2.h"

namespace lzq {

// The frame and phase algebra below is checked against the numpy restatement at tolerances, not bit
// for bit, so its products and sums may contract to fma (the library builds with -ffp-contract=off
// for the oracle-matched quadrature); reset to off at the end of this header.
#ifndef LZQ_SA_CONTRACT
#define LZQ_SA_CONTRACT 1
#endif
#if LZQ_SA_CONTRACT
#pragma clang fp contract(fast)
#endif

constexpr int kSALevels = 10;      // frame order outside a Magnus core (rotations V_0 .. V_9)
constexpr double kSATol = 1e-11;   // core edge: first neglected angle |theta_10| <= this
constexpr double kSAC = 3.2e5;     // |theta_10| <= kSAC mh / E^21 (fitted; conservative for mh > 1)
constexpr int kSAFarLevels = 6;    // the outer end of a follow stretch, when that order is enough:
constexpr double kSAFarC = 80.0;   //   |theta_6| <= kSAFarC mh / E^13 (fitted) <= kSATol / 10

// 1/x for the frame and phase algebra (x: energies, their squares and the like, normal doubles far
// from the range limits).  On the device v_rcp_f64 + two Newton steps (<= 1 ulp from the
// quotient, ~4 VALU where the IEEE division takes ~10; the follow kernel divides ~130 times per
// cell); the host build (tests/test_superadiabatic_host.py) divides.
#ifndef LZQ_SA_FASTDIV
#define LZQ_SA_FASTDIV 1
#endif
__host__ __device__ __forceinline__ double sa_rcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && LZQ_SA_FASTDIV
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
#else
  return 1.0 / x;
#endif
}

// 1/sqrt(x) for the same quantities: v_rsq_f64 + two Newton steps r += r (1 - x r^2) / 2 (~1 ulp).
// A square root and a reciprocal of the same number then cost one such chain (sqrt(x) = x rsqrt(x),
// 1/x = rsqrt(x)^2) instead of the IEEE square root's refinement followed by sa_rcp's: the frame
// levels are a dependent chain of these, so their latency is the follow kernel's (LZQ_SA_RSQRT).
#ifndef LZQ_SA_RSQRT
#define LZQ_SA_RSQRT 1
#endif
__host__ __device__ __forceinline__ double sa_rsqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && LZQ_SA_FASTDIV
  double r = __builtin_amdgcn_rsq(x);
  double e = __builtin_fma(-(x * r), r, 1.0);
  r = __builtin_fma(0.5 * r, e, r);
  e = __builtin_fma(-(x * r), r, 1.0);
  return __builtin_fma(0.5 * r, e, r);
#else
  return 1.0 / sqrt(x);
#endif
}

// cos theta, sin theta from cos 2theta = c2, sin 2theta = s2 >= 0 (theta in [0, pi/2]) or any
// s2 with c2 > 0, without cancellation
__host__ __device__ __forceinline__ void half_angle(double c2, double s2, bool pos, double& c, double& s) {
#if LZQ_SA_RSQRT
  const double x = 0.5 * (pos ? 1.0 + c2 : 1.0 - c2);  // in [1/2, 1]
  const double rr = sa_rsqrt(x);
  const double big = x * rr, small = s2 * (0.5 * rr);
  c = pos ? big : small;
  s = pos ? small : big;
#else
  if (pos) {
    c = sqrt(0.5 * (1.0 + c2));
    s = s2 * (0.5 * sa_rcp(c));
  } else {
    s = sqrt(0.5 * (1.0 - c2));
    c = s2 * (0.5 * sa_rcp(s));
  }
#endif
}

// The frame rotation U = V_0 V_1 .. V_{N-1} accumulated as it is built: an SU(2) element
// [[a, -conj(b)], [b, conj(a)]], so 4 doubles instead of every level's (cos, sin).
struct SU2 {
  Cplx a, b;
};

// U <- U V_j with V_j = [[c, -s], [s, c]] (even j) or [[c, i s], [i s, c]] (odd j)
template <bool kEven>
__host__ __device__ __forceinline__ void su2_right_mul(SU2& u, double c, double s) {
  Cplx na, nb;
  if constexpr (kEven) {  // V = (a2 = c, b2 = s): a = a1 c - conj(b1) s, b = b1 c + conj(a1) s
    na = {u.a.re * c - u.b.re * s, u.a.im * c + u.b.im * s};
    nb = {u.b.re * c + u.a.re * s, u.b.im * c - u.a.im * s};
  } else {  // V = (a2 = c, b2 = i s): a = a1 c - conj(b1) i s, b = b1 c + conj(a1) i s
    na = {u.a.re * c - u.b.im * s, u.a.im * c - u.b.re * s};
    nb = {u.b.re * c + u.a.im * s, u.b.im * c + u.a.re * s};
  }
  u.a = na;
  u.b = nb;
}

// Generic levels J0 + J .. of jets e, g of length M - J (in place).  Accumulates the frame
// rotation into u (kRot) and stores ev[lev] = e_{lev+1}, gv[lev] = g_lev (kEG).
template <int M, int J, int J0, bool kRot, bool kEG>
__host__ __device__ __forceinline__ void sa_chain(double (&e)[M], double (&g)[M], SU2& u, double* ev, double* gv) {
  if constexpr (J < M) {
    constexpr int n = M - J;
    constexpr int lev = J0 + J;
    double q[n];  // e^2 + g^2, later its square root (e_{lev+1}); symmetric sums: half the terms
#pragma unroll
    for (int l = 0; l < n; ++l) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; 2 * i < l; ++i) acc = __builtin_fma(e[i], e[l - i], __builtin_fma(g[i], g[l - i], acc));
      acc += acc;
      if (l % 2 == 0) acc = __builtin_fma(e[l / 2], e[l / 2], __builtin_fma(g[l / 2], g[l / 2], acc));
      q[l] = acc;
    }
#if LZQ_SA_RSQRT
    const double ir = sa_rsqrt(q[0]);
    const double r0 = q[0] * ir;
#else
    const double r0 = sqrt(q[0]);
    const double ir = sa_rcp(r0);
#endif
    if constexpr (kRot) {
      double c, s;
      half_angle(e[0] * ir, g[0] * ir, e[0] >= 0.0, c, s);
      su2_right_mul<lev % 2 == 0>(u, c, s);
    }
    if constexpr (kEG) {
      ev[lev] = r0;
      gv[lev] = g[0];
    }
    if constexpr (n > 1) {
      // theta' = (e g' - g e') / (2 q): w = num / q, g_next = -+ w / 2
#if LZQ_SA_RSQRT
      const double iq = ir * ir;
#else
      const double iq = sa_rcp(q[0]);
#endif
      double w[n - 1];
#pragma unroll
      for (int l = 0; l < n - 1; ++l) {
        // num_l = sum_{i + j = l + 1} j (e_i g_j - g_i e_j); the pairs (i, j), (j, i) with i, j >= 1
        // combine to (j - i) (e_i g_j - g_i e_j)
        double acc = (double)(l + 1) * __builtin_fma(e[0], g[l + 1], -(g[0] * e[l + 1]));
#pragma unroll
        for (int i = 1; 2 * i < l + 1; ++i) {
          const double k = (double)(l + 1 - 2 * i);
          acc = __builtin_fma(k, __builtin_fma(e[i], g[l + 1 - i], -(g[i] * e[l + 1 - i])), acc);
        }
#pragma unroll
        for (int i = 0; i < l; ++i) acc = __builtin_fma(-w[i], q[l - i], acc);
        w[l] = acc * iq;
      }
      // sqrt(q) in place: r_l = (q_l - sum_{i=1}^{l-1} r_i r_{l-i}) / (2 r_0)
      const double h0 = 0.5 * ir;
      q[0] = r0;
#pragma unroll
      for (int l = 1; l < n - 1; ++l) {
        double acc = 0.0;
#pragma unroll
        for (int i = 1; 2 * i < l; ++i) acc = __builtin_fma(q[i], q[l - i], acc);
        acc += acc;
        if (l % 2 == 0) acc = __builtin_fma(q[l / 2], q[l / 2], acc);
        q[l] = (q[l] - acc) * h0;
      }
      constexpr double f = (lev % 2 == 0) ? -0.5 : 0.5;
#pragma unroll
      for (int l = 0; l < n - 1; ++l) {
        g[l] = f * w[l];
        e[l] = q[l];
      }
      sa_chain<M, J + 1, J0, kRot, kEG>(e, g, u, ev, gv);
    }
  }
}

// Levels 0 .. N-1 of the linear crossing Dh(tau0 + h) = Dh + sg h, constant mh: the frame
// rotation U = V_0 .. V_{N-1} (kRot) and ev[j] = e_{j+1}, gv[j] = g_j (kEG).  Level 0 is done in
// closed form (its jets are sparse).
template <int N, bool kRot, bool kEG>
__host__ __device__ __forceinline__ void sa_levels_linear(double Dh, double sg, double mh, SU2& u, double* ev, double* gv) {
  // q = (Dh + sg h)^2 + mh^2 = [E^2, 2 sg Dh, 1]
  const double q0 = __builtin_fma(Dh, Dh, mh * mh), q1 = 2.0 * sg * Dh;
#if LZQ_SA_RSQRT
  const double iE = sa_rsqrt(q0);
  const double E = q0 * iE;
#else
  const double E = sqrt(q0);
  const double iE = sa_rcp(E);
#endif
  if constexpr (kRot) {
    double c, s;
    half_angle(Dh * iE, mh * iE, Dh >= 0.0, c, s);
    u.a = {c, 0.0};
    u.b = {s, 0.0};
  }
  if constexpr (kEG) {
    ev[0] = E;
    gv[0] = mh;
  }
  if constexpr (N > 1) {
    constexpr int M = N - 1;
    double e[M], g[M];
    // e_1 = sqrt(q) (jet); theta_0' = w/2 with w = -mh sg / q, g_1 = -w/2
    const double h0 = 0.5 * iE;
    e[0] = E;
    if constexpr (M > 1) e[1] = q1 * h0;
#pragma unroll
    for (int l = 2; l < M; ++l) {
      double acc = 0.0;
#pragma unroll
      for (int i = 1; 2 * i < l; ++i) acc = __builtin_fma(e[i], e[l - i], acc);
      acc += acc;
      if (l % 2 == 0) acc = __builtin_fma(e[l / 2], e[l / 2], acc);
      e[l] = ((l == 2 ? 1.0 : 0.0) - acc) * h0;
    }
#if LZQ_SA_RSQRT
    const double iq = iE * iE;
#else
    const double iq = sa_rcp(q0);
#endif
    double w[M];
    w[0] = -mh * sg * iq;
#pragma unroll
    for (int l = 1; l < M; ++l) {
      double acc = -w[l - 1] * q1;
      if (l >= 2) acc = acc - w[l - 2];
      w[l] = acc * iq;
    }
#pragma unroll
    for (int l = 0; l < M; ++l) g[l] = -0.5 * w[l];
    sa_chain<M, 0, 1, kRot, kEG>(e, g, u, ev, gv);
  }
}

// P U^+ with P = diag(e^{-i ph}, e^{i ph}) = (a = e^{-i ph}, b = 0) and U^+ = (conj(a), -b)
__host__ __device__ __forceinline__ SU2 su2_phase_adj(double ph, const SU2& u) {
  const double sn = sin(ph), cs = cos(ph);
  SU2 m;
  m.a = {cs * u.a.re - sn * u.a.im, -sn * u.a.re - cs * u.a.im};   // e^{-i ph} conj(a)
  m.b = {sn * u.b.im - cs * u.b.re, -(cs * u.b.im + sn * u.b.re)};  // e^{+i ph} (-b)
  return m;
}

// u r: a = a1 a2 - conj(b1) b2, b = b1 a2 + conj(a1) b2
__host__ __device__ __forceinline__ SU2 su2_mul(const SU2& u, const SU2& r) {
  SU2 m;
  m.a = {u.a.re * r.a.re - u.a.im * r.a.im - (u.b.re * r.b.re + u.b.im * r.b.im),
         u.a.re * r.a.im + u.a.im * r.a.re - (u.b.re * r.b.im - u.b.im * r.b.re)};
  m.b = {u.b.re * r.a.re - u.b.im * r.a.im + u.a.re * r.b.re + u.a.im * r.b.im,
         u.b.re * r.a.im + u.b.im * r.a.re + u.a.re * r.b.im - u.a.im * r.b.re};
  return m;
}

// psi <- U^+ psi (diabatic -> frame), U = [[a, -conj(b)], [b, conj(a)]]
__host__ __device__ __forceinline__ void su2_apply_adj(const SU2& u, Cplx& p0, Cplx& p1) {
  // U^+ = [[conj(a), conj(b)], [-b, a]]
  const Cplx q0 = {u.a.re * p0.re + u.a.im * p0.im + u.b.re * p1.re + u.b.im * p1.im,
                   u.a.re * p0.im - u.a.im * p0.re + u.b.re * p1.im - u.b.im * p1.re};
  const Cplx q1 = {-(u.b.re * p0.re - u.b.im * p0.im) + u.a.re * p1.re - u.a.im * p1.im,
                   -(u.b.re * p0.im + u.b.im * p0.re) + u.a.re * p1.im + u.a.im * p1.re};
  p0 = q0;
  p1 = q1;
}

// psi <- U psi (frame -> diabatic)
__host__ __device__ __forceinline__ void su2_apply_mat(const SU2& u, Cplx& p0, Cplx& p1) {
  const Cplx q0 = {u.a.re * p0.re - u.a.im * p0.im - (u.b.re * p1.re + u.b.im * p1.im),
                   u.a.re * p0.im + u.a.im * p0.re - (u.b.re * p1.im - u.b.im * p1.re)};
  const Cplx q1 = {u.b.re * p0.re - u.b.im * p0.im + u.a.re * p1.re + u.a.im * p1.im,
                   u.b.re * p0.im + u.b.im * p0.re + u.a.re * p1.im - u.a.im * p1.re};
  p0 = q0;
  p1 = q1;
}

// Core half-width in tau: out to E = sqrt(tau^2 + mh^2) where kSAC max(mh, kSAMFloor) / E^21
// = kSATol, at least 1.  The following error is an amplitude ~ |theta_10| ~ mh / E^21, and for
// small mh the conversion probability is P ~ pi mh^2, so its relative error ~ 1/E^21 would grow as
// mh shrinks: the floor keeps it <= ~1e-10 (E >= 5.4) however small the coupling.
constexpr double kSAMFloor = 0.05;
__host__ __device__ __forceinline__ double sa_core_tau(double mh) {
  const double Ec = pow(kSAC * fmax(mh, kSAMFloor) / kSATol, 1.0 / (2.0 * kSALevels + 1.0));
  return sqrt(fmax(Ec * Ec - mh * mh, 1.0));
}

// G(x) = int_0^x sqrt(t^2 + m^2) dt
__host__ __device__ __forceinline__ double wkb_G(double x, double m) {
  return 0.5 * (x * sqrt(x * x + m * m) + (m > 0.0 ? m * m * asinh(x / m) : 0.0));
}

// T(x0) = int_{|x0|}^inf dx / (x^2 + m^2)^{5/2}: closed form, or its series in u = m^2/x0^2 where
// the closed form cancels (u < 1e-3; truncation ~u^4).
__host__ __device__ __forceinline__ double tail_T(double x0, double m) {
  x0 = fabs(x0);
  const double u = (m * m) / (x0 * x0);
  if (u < 1e-3) {
    const double ix2 = 1.0 / (x0 * x0);
    return (0.25 - u * (5.0 / 12.0 - u * (35.0 / 64.0 - u * (21.0 / 32.0)))) * ix2 * ix2;
  }
  const double E = sqrt(x0 * x0 + m * m);
  const double m2 = m * m;
  return (2.0 - x0 * (2.0 * x0 * x0 + 3.0 * m2) / (E * E * E)) / (3.0 * m2 * m2);
}

// int_ta^tb e_4 dtau on one side of a crossing (1 <= |ta|, |tb|; tests/lz_ref.py sa_phase): the
// WKB phase G, the leading dressed-energy term mh^2/(8E^5) in closed form (tail_T), and the rest,
// e_4 - E - mh^2/(8E^5) = O(E^-9) (differences e_{j+1} - e_j = g_j^2/(e_j + e_{j+1}), no
// cancellation), by 4-point Gauss-Legendre in u = 1/|tau|.  e_5 - e_4 < 1e-12 beyond the core.
__host__ __device__ __forceinline__ double sa_phase(double ta, double tb, double mh) {
  constexpr double gx[4] = {-0.8611363115940526, -0.3399810435848563, 0.3399810435848563, 0.8611363115940526};
  constexpr double gw[4] = {0.3478548451374538, 0.6521451548625461, 0.6521451548625461, 0.3478548451374538};
  const double base = wkb_G(tb, mh) - wkb_G(ta, mh);
  const double lead = mh * mh * 0.125 * fabs(tail_T(ta, mh) - tail_T(tb, mh));
  const double u1 = 1.0 / fabs(ta), u2 = 1.0 / fabs(tb);
  const double ulo = fmin(u1, u2), uhi = fmax(u1, u2);
  const double half = 0.5 * (uhi - ulo), mid = 0.5 * (uhi + ulo);
  double acc = 0.0;
#ifndef LZQ_SA_PHASE_UNROLL
#define LZQ_SA_PHASE_UNROLL 1  // the 4 Gauss points one after another (2, 4: side by side, tools/ablate_prop.py)
#endif
#pragma unroll LZQ_SA_PHASE_UNROLL
  for (int k = 0; k < 4; ++k) {
    const double u = __builtin_fma(half, gx[k], mid);
    const double iu = sa_rcp(u);
    SU2 unused;
    double ev[4], gv[4];
    sa_levels_linear<4, false, true>(iu, 1.0, mh, unused, ev, gv);
    const double E = ev[0];
    const double i01 = sa_rcp(E + ev[1]);
    const double d1 = gv[1] * gv[1] * i01;
    const double d2 = gv[2] * gv[2] * sa_rcp(ev[1] + ev[2]);
    const double d3 = gv[3] * gv[3] * sa_rcp(ev[2] + ev[3]);
    const double E5 = E * E * E * E * E;
    const double f = d3 + d2 - mh * mh * d1 * (0.125 * sa_rcp(E5) * i01);
    acc = __builtin_fma(gw[k], f * (iu * iu), acc);
  }
  return base + lead + half * acc;
}

// The frame at -tau from the frame at +tau: U(-tau) = -sz U(tau) sx exactly (H(-tau) = sx H(tau) sx
// and the jets' derivatives flip sign with tau; checked bit for bit on the restatement), i.e.
// (a, b) -> (conj(b), conj(a)).
__host__ __device__ __forceinline__ SU2 sa_reflect(const SU2& u) {
  SU2 r;
  r.a = {u.b.re, -u.b.im};
  r.b = {u.a.re, -u.a.im};
  return r;
}

// Transfer matrices of superadiabatic following (tests/lz_ref.py sa_follow) on both sides of a
// cell's core [-tau_c, tau_c]: ML from tl (< -tau_c) to -tau_c when has_left (stored at out[0..3]
// as (a.re, a.im, b.re, b.im) as soon as it is built, so it holds no registers while MR is), MR from
// tau_c to tr (> tau_c) when has_right (out[4..7]), each U(tb) diag(e^{-i ph}, e^{i ph}) U(ta)^+ with U the frame
// rotation of order kSALevels (kSAFarLevels at an outer end where that is enough) and
// ph = int e dtau (sa_phase).  Error ~ |theta_10| at the inner end.  They do not depend on the
// state, so lz_follow_kernel computes them ahead of the propagation.  The core-edge frame is
// computed once (the one at -tau_c by sa_reflect), and one frame per loop iteration: two side by
// side (they are independent) would need ~250 VGPRs.
#ifndef LZQ_FOLLOW_PAIR
#define LZQ_FOLLOW_PAIR 0  // 1: the two outer frames (and phases) side by side after the core's (tools/ablate_prop.py)
#endif
__host__ __device__ __forceinline__ SU2 sa_frame(double tau, double sg, double mh, bool outer) {
  const double Ef2 = tau * tau + mh * mh, Ef4 = Ef2 * Ef2, Ef12 = Ef4 * Ef4 * Ef4;
  const bool far6 = outer && kSAFarC * fmax(mh, kSAMFloor) <= 0.1 * kSATol * Ef12 * sqrt(Ef2);
  SU2 u;
  if (far6)
    sa_levels_linear<kSAFarLevels, true, false>(sg * tau, sg, mh, u, nullptr, nullptr);
  else
    sa_levels_linear<kSALevels, true, false>(sg * tau, sg, mh, u, nullptr, nullptr);
  return u;
}
__host__ __device__ __forceinline__ void sa_store(const SU2& m, double* out) {
  out[0] = m.a.re, out[1] = m.a.im, out[2] = m.b.re, out[3] = m.b.im;
}
__host__ __device__ __forceinline__ void sa_cell_follow(double mh, double sg, double tl, double tr, double tau_c,
                                                        bool has_left, bool has_right, double* out) {
#if LZQ_FOLLOW_PAIR
  if (!(has_left || has_right)) return;
  const SU2 uc = sa_frame(tau_c, sg, mh, false);
  // both outer stretches in one straight block (the compiler interleaves the independent chains);
  // a side that is absent evaluates the other's arguments and is not stored
  const double ta = has_left ? tl : tr, tb = has_right ? tr : tl;
  const SU2 ua = sa_frame(ta, sg, mh, true), ub = sa_frame(tb, sg, mh, true);
  const double pa = sa_phase(ta, -tau_c, mh), pb = sa_phase(tau_c, tb, mh);
  if (has_left) sa_store(su2_mul(sa_reflect(uc), su2_phase_adj(pa, ua)), out);
  if (has_right) sa_store(su2_mul(ub, su2_phase_adj(pb, uc)), out + 4);
#else
  SU2 uc;
#ifndef LZQ_FOLLOW_JOB_UNROLL
#define LZQ_FOLLOW_JOB_UNROLL 1  // 3: the three frames straight-line (tools/ablate_follow.sh)
#endif
#pragma unroll LZQ_FOLLOW_JOB_UNROLL
  for (int job = 0; job < 3; ++job) {
    if ((job == 0 && !(has_left || has_right)) || (job == 1 && !has_left) || (job == 2 && !has_right)) continue;
    const double tau = job == 0 ? tau_c : (job == 1 ? tl : tr);
    const double Ef2 = tau * tau + mh * mh, Ef4 = Ef2 * Ef2, Ef12 = Ef4 * Ef4 * Ef4;
    const bool far6 = job > 0 && kSAFarC * fmax(mh, kSAMFloor) <= 0.1 * kSATol * Ef12 * sqrt(Ef2);
    SU2 u;
    if (far6)
      sa_levels_linear<kSAFarLevels, true, false>(sg * tau, sg, mh, u, nullptr, nullptr);
    else
      sa_levels_linear<kSALevels, true, false>(sg * tau, sg, mh, u, nullptr, nullptr);
    if (job == 0)
      uc = u;
    else if (job == 1)
      sa_store(su2_mul(sa_reflect(uc), su2_phase_adj(sa_phase(tl, -tau_c, mh), u)), out);  // U(-tau_c) P U(tl)^+
    else
      sa_store(su2_mul(u, su2_phase_adj(sa_phase(tau_c, tr, mh), uc)), out + 4);           // U(tr) P U(tau_c)^+
  }
#endif
}

#if LZQ_SA_CONTRACT
#pragma clang fp contract(off)
#endif

}  // namespace lzq
