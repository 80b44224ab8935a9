// lzq_propagator.hip -- time-ordered two-level Landau-Zener propagation (north_star (1)).
//
// The reference has no propagator: it only applies the closed form P = 1 - exp(-2 pi delta)
// (fpy:183-184, PAPER eqs.(8)-(9), delta = m_mix^2 / (2 v_w |Delta'|), F = 1).  This kernel
// integrates the underlying Schroedinger equation so that profiles with several sequential
// crossings (BASELINE config C5) can be evaluated coherently; for one isolated crossing it
// reduces to the closed form (tests/test_gpu_propagator.py states the window tolerance).
//
// Model (DESIGN.md "LZ propagator"): diabatic basis (chi, B), xi = v_w t,
//   i d psi/dt = H psi,   H(xi) = [[D(xi), m_c], [m_c, -D(xi)]]
// with crossings c = 0..N-1 at xi_c (increasing).  On cell c, D(xi) = s_c |Delta'_c| (xi - xi_c),
// s_c = (-1)^c, and the coupling is m_c.  Interior cell edges b_c are where neighbouring
// linear pieces meet (D continuous, |D| maximal); the outer edges are xi_0 - W_0 and
// xi_{N-1} + W_{N-1} with W_c = K * L_c, L_c = sqrt(v_w/|Delta'_c|) * max(1, sqrt(delta_c))
// the LZ length of crossing c (delta_c = m_c^2 / (2 v_w |Delta'_c|)) and K = window_lz.  psi starts in the adiabatic state that is chi-like at the first edge; the
// result is the conversion probability 1 - |<chi-like adiabatic state | psi>|^2 at the last.
//
// Integrator, per cell c with delta_c = m_c^2 / (2 v_w |Delta'_c|):
//  * delta_c <= kDeltaAdiabatic: fourth-order Magnus (two Gauss-Legendre nodes) with the exact
//    SU(2) exponential, S_c = max(S, ceil(Phi_c * kStepsPerRadian)) uniform steps, Phi_c the
//    cell's adiabatic phase (closed form below), so wide / strongly coupled cells get the
//    steps their phase needs: for H = D sz + m sx,
//      Omega = -i (n . sigma),  n = (dt m, (sqrt3/6) dt^2 m (D2-D1), dt (D1+D2)/2)
//      U = cos|n| - i sin|n| (n/|n|) . sigma;
//  * delta_c > kDeltaAdiabatic: the crossing is adiabatic to e^{-2 pi delta} < 1e-43, and the
//    cell is propagated exactly in the adiabatic basis: amplitudes b+- pick up
//    exp(-+ i (Phi + phi_S)) with the WKB phase Phi = int E dt in closed form
//    (E = sqrt(D^2 + m^2), G(x) = [x sqrt(x^2+m^2) + m^2 asinh(x/m)]/2) and the LZ Stokes phase
//    phi_S = pi/4 + delta (ln delta - 1) + arg Gamma(1 - i delta) = 1/(12 delta) + 1/(360 delta^3)
//    + 1/(1260 delta^5) + 1/(1680 delta^7) + O(delta^-9) (Stirling series of ln Gamma(-i delta);
//    checked against mpmath, and its sign against brute-force Magnus, in
//    tests/test_propagator_math.py).
// One parameter point per lane, all state in registers.
#include <hip/hip_runtime.h>

#include <math.h>

#include "../../include/lzq.h"

namespace lzq {

constexpr int kPropBlock = 256;
constexpr double kSqrt3Over6 = 0x1.279a74590331cp-2;  // sqrt(3)/6
constexpr double kDeltaAdiabatic = 16.0;              // e^{-2 pi 16} = 2e-44
constexpr double kStepsPerRadian = 1.0;

// G(x) = int_0^x sqrt(t^2 + m^2) dt
__device__ __forceinline__ double wkb_G(double x, double m) {
  return 0.5 * (x * sqrt(x * x + m * m) + (m > 0.0 ? m * m * asinh(x / m) : 0.0));
}

struct Cplx {
  double re, im;
};

// LZ length of a crossing in xi: sqrt(v_w/|Delta'|) * max(1, sqrt(delta)).
__device__ __forceinline__ double lz_length(double m, double a, double v_w) {
  const double delta = m * m / (2.0 * v_w * a);
  return sqrt(v_w / a) * fmax(1.0, sqrt(delta));
}

// Adiabatic eigenvector of [[d, m],[m, -d]] with eigenvalue -sign * sqrt(d^2+m^2) ...
// returns the eigenvector (u0, u1) (real) of the state that is chi-like (|u0| >= |u1|).
__device__ __forceinline__ void chi_like_adiabatic(double d, double m, double& u0, double& u1) {
  // theta = atan2(m, d)/2 ; |+> = (cos t, sin t) (eigenvalue +E), |-> = (-sin t, cos t)
  double th = 0.5 * atan2(m, d);
  double c = cos(th), s = sin(th);
  if (fabs(c) >= fabs(s)) {  // |+> is chi-like
    u0 = c;
    u1 = s;
  } else {                   // |-> is chi-like
    u0 = -s;
    u1 = c;
  }
}

__global__ __launch_bounds__(kPropBlock) void lz_propagate_kernel(const double* __restrict__ m_mix,
                                                                  const double* __restrict__ dprime,
                                                                  const double* __restrict__ xi, int64_t n,
                                                                  int32_t n_cross, double v_w, double K,
                                                                  int32_t S, double* __restrict__ P_out) {
  const int64_t p = (int64_t)blockIdx.x * kPropBlock + threadIdx.x;
  if (p >= n) return;
  const double* mm = m_mix + p * n_cross;
  const double* dp = dprime + p * n_cross;
  const double* xc = xi + p * n_cross;
  const double inv_vw = 1.0 / v_w;

  // left edge of cell 0
  double a0 = fabs(dp[0]);
  double left = xc[0] - K * lz_length(mm[0], a0, v_w);
  double D_left = a0 * (left - xc[0]);  // s_0 = +1
  double u0, u1;
  chi_like_adiabatic(D_left, mm[0], u0, u1);
  Cplx p0 = {u0, 0.0}, p1 = {u1, 0.0};

  double sgn = 1.0;
  double right = left;
  for (int c = 0; c < n_cross; ++c) {
    const double ac = fabs(dp[c]);
    const double mc = mm[c];
    const double xcc = xc[c];
    if (c + 1 < n_cross) {
      const double an = fabs(dp[c + 1]);
      right = (ac * xcc + an * xc[c + 1]) / (ac + an);  // D continuous at the turning point
    } else {
      right = xcc + K * lz_length(mc, ac, v_w);
    }
    const double slope = sgn * ac;
    const double delta = mc * mc / (2.0 * v_w * ac);
    // adiabatic phase of the cell, int E dt (closed form)
    const double Phi = (wkb_G(ac * (right - xcc), mc) - wkb_G(ac * (left - xcc), mc)) / (ac * v_w);
    if (delta > kDeltaAdiabatic) {
      // exact adiabatic following through the cell (see header)
      double l0, l1, r0, r1;
      const double DL = slope * (left - xcc), DR = slope * (right - xcc);
      {
        const double th = 0.5 * atan2(mc, DL);
        l0 = cos(th);
        l1 = sin(th);
        const double tr = 0.5 * atan2(mc, DR);
        r0 = cos(tr);
        r1 = sin(tr);
      }
      // b+ = <+|psi>, b- = <-|psi>; |+> = (c, s), |-> = (-s, c)
      Cplx bp = {l0 * p0.re + l1 * p1.re, l0 * p0.im + l1 * p1.im};
      Cplx bm = {-l1 * p0.re + l0 * p1.re, -l1 * p0.im + l0 * p1.im};
      const double id = 1.0 / delta, id2 = id * id;
      const double phiS = id * (1.0 / 12.0 + id2 * (1.0 / 360.0 + id2 * (1.0 / 1260.0 + id2 * (1.0 / 1680.0))));
      double sn, cs;
      sincos(Phi + phiS, &sn, &cs);
      const Cplx bp2 = {bp.re * cs + bp.im * sn, bp.im * cs - bp.re * sn};  // * e^{-i a}
      const Cplx bm2 = {bm.re * cs - bm.im * sn, bm.im * cs + bm.re * sn};  // * e^{+i a}
      p0 = {r0 * bp2.re - r1 * bm2.re, r0 * bp2.im - r1 * bm2.im};
      p1 = {r1 * bp2.re + r0 * bm2.re, r1 * bp2.im + r0 * bm2.im};
    } else {
      const int Sc = (int)fmax((double)S, ceil(Phi * kStepsPerRadian));
      const double h = (right - left) / (double)Sc;  // step in xi
      const double dt = h * inv_vw;                  // step in t
      const double nx = dt * mc;
      for (int i = 0; i < Sc; ++i) {
        const double xm = left + ((double)i + 0.5) * h;
        const double D1 = slope * ((xm - kSqrt3Over6 * h) - xcc);
        const double D2 = slope * ((xm + kSqrt3Over6 * h) - xcc);
        const double ny = kSqrt3Over6 * dt * mc * (D2 - D1) * dt;
        const double nz = 0.5 * dt * (D1 + D2);
        const double nn = sqrt(nx * nx + ny * ny + nz * nz);
        double sn, cs;
        sincos(nn, &sn, &cs);
        const double sc = nn > 0.0 ? sn / nn : 1.0;
        const double sx = sc * nx, sy = sc * ny, sz = sc * nz;
        // U11 = cs - i sz ; U12 = -sy - i sx ; U21 = sy - i sx ; U22 = cs + i sz
        Cplx q0, q1;
        q0.re = cs * p0.re + sz * p0.im - sy * p1.re + sx * p1.im;
        q0.im = cs * p0.im - sz * p0.re - sy * p1.im - sx * p1.re;
        q1.re = sy * p0.re + sx * p0.im + cs * p1.re - sz * p1.im;
        q1.im = sy * p0.im - sx * p0.re + cs * p1.im + sz * p1.re;
        p0 = q0;
        p1 = q1;
      }
    }
    left = right;
    sgn = -sgn;
  }
  // project on the chi-like adiabatic state at the right edge of the last cell
  const int last = n_cross - 1;
  const double D_right = (sgn * -1.0) * fabs(dp[last]) * (right - xc[last]);  // sgn was flipped once more
  chi_like_adiabatic(D_right, mm[last], u0, u1);
  const double re = u0 * p0.re + u1 * p1.re;
  const double im = u0 * p0.im + u1 * p1.im;
  const double norm = p0.re * p0.re + p0.im * p0.im + p1.re * p1.re + p1.im * p1.im;
  P_out[p] = 1.0 - (re * re + im * im) / norm;
}

}  // namespace lzq

// error plumbing shared with lzq_kernels.hip (C++ linkage, not part of the C ABI)
int lzq_set_error(int code, const char* msg);

extern "C" int lzq_lz_propagate(const double* d_m_mix, const double* d_dprime, const double* d_xi, int64_t n,
                                int32_t n_cross, double v_w, double window_lz, int32_t steps_per_crossing,
                                double* d_P, void* stream) {
  if (n < 0 || n_cross <= 0 || steps_per_crossing <= 0 || !(v_w > 0.0) || !(window_lz > 0.0) ||
      (n > 0 && (!d_m_mix || !d_dprime || !d_xi || !d_P)))
    return lzq_set_error(LZQ_EINVAL, "lzq_lz_propagate: bad arguments");
  if (n == 0) return LZQ_OK;
  const int64_t nb = (n + lzq::kPropBlock - 1) / lzq::kPropBlock;
  if (nb > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_lz_propagate: n too large");
  hipLaunchKernelGGL(lzq::lz_propagate_kernel, dim3((unsigned)nb), dim3(lzq::kPropBlock), 0, (hipStream_t)stream,
                     d_m_mix, d_dprime, d_xi, n, n_cross, v_w, window_lz, steps_per_crossing, d_P);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  return LZQ_OK;
}
