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
// the LZ length of crossing c (delta_c = m_c^2 / (2 v_w |Delta'_c|)) and K = window_lz.
// psi starts in the chi-like DRESSED state of the first cell at its outer edge, and the result is
// the conversion probability 1 - |<chi-like dressed state | psi>|^2 at the last cell's outer edge.
// Dressed = second-order superadiabatic (dressed_basis below): the state that an adiabatic
// state at t -> -inf has become, up to O(eps/(alpha tau^2)^2).  Projecting on it instead of the
// plain adiabatic state removes the window's O(K^-3) error: a single crossing reproduces the
// asymptotic eq.(9) to ~2e-9 at K = 20 (1/K^5), where the adiabatic projection was 7e-5 off.
//
// Integrator, per cell c with delta_c = m_c^2 / (2 v_w |Delta'_c|):
//  * delta_c <= kDeltaAdiabatic: eighth-order Magnus with the exact SU(2) exponential on the
//    cell's CORE [xi_c - W_c, xi_c + W_c] with S_c = max(S, ceil(Phi_core * kStepsPerRadian))
//    uniform steps, Phi_core the core's adiabatic phase (closed form below).  Outside the core
//    the state is followed in the superadiabatic frame of order 10 (lzq_superadiabatic.h: ten
//    iterated adiabatic rotations built from Taylor jets), where it only picks up the frame's
//    phase; the error of that is the first neglected rotation angle at the core edge, and the
//    core ends where that falls to kSATol = 1e-11: E = (kSAC mh / kSATol)^(1/21) in units of
//    sqrt(alpha) (~4-7 LZ lengths, against 40 for round 2's second-order dressed basis).  The
//    follow stretches do not depend on the state, so lz_follow_kernel computes their SU(2)
//    transfer matrices first (one thread per point and cell) and this kernel applies them.
//    H = D(t) sz + m sx is linear in t, so its Magnus series over a step of length dt
//    centred on D is known in closed form (derived symbolically: Dyson series, then log):
//      Omega = -i (n . sigma),  U = cos|n| - i sin|n| (n/|n|) . sigma,  D' = dD/dt, E2 = D^2 + m^2
//      n_x = m dt [1 - D'^2 dt^4/60 - D'^2 dt^6 (3D^2 + 4m^2)/1890]
//      n_y = D' m dt^3 [1/6 + dt^2 E2/90 + dt^4 (8 E2^2 - 9 D'^2)/7560]
//      n_z = D dt [1 - D'^2 m^2 dt^6/1890]                                     + O(dt^9).
//    The dt^3 terms alone are the two-node Gauss-Legendre (fourth-order) Magnus step; the dt^5
//    and dt^7 terms carry the far-field E^2 growth of its error.  tests/lz_ref.py restates it;
//    tests/test_propagator_exact.py checks it against the exact Weber solution;
//  * delta_c > kDeltaAdiabatic: the crossing is adiabatic to e^{-2 pi delta} < 1e-43, and the
//    cell is propagated exactly in its dressed basis: amplitudes b+- pick up
//    exp(-+ i (Phi + phi_S - tails)) with the WKB phase Phi = int E dt in closed form
//    (E = sqrt(D^2 + m^2), G(x) = [x sqrt(x^2+m^2) + m^2 asinh(x/m)]/2) and the LZ Stokes phase
//    phi_S = pi/4 + delta (ln delta - 1) + arg Gamma(1 - i delta) = 1/(12 delta) + 1/(360 delta^3)
//    + 1/(1260 delta^5) + 1/(1680 delta^7) + O(delta^-9) (Stirling series of ln Gamma(-i delta);
//    checked against mpmath, and its sign against brute-force Magnus, in
//    tests/test_propagator_math.py).  phi_S is the whole line's dressed-energy correction; its
//    leading part int theta'^2/(2E) dt = (m^2 alpha/8) int dD/E^5 (= 1/(12 delta) over the line)
//    has the pieces beyond the cell's two edges removed ("tails", tail_T below).
// One parameter point per lane, all state in registers.
#include <hip/hip_runtime.h>

#include <math.h>

#include <algorithm>

#include "../../include/lzq.h"
#include "lzq_internal.h"
#include "lzq_su2.h"
#include "lzq_superadiabatic.h"

namespace lzq {

constexpr int kPropBlock = 256;
#ifndef LZQ_PROP_UNROLL
#define LZQ_PROP_UNROLL 3  // step-loop unroll: ILP across steps (A/B: 1 -> 3 = -12%, tools/ablate_prop.py)
#endif
#ifndef LZQ_PROP_MIN_WAVES
#define LZQ_PROP_MIN_WAVES 2  // 217 VGPRs with the 3-step unroll, no spills (3 waves/SIMD: 168 VGPRs, spills; same time)
#endif
#ifndef LZQ_FOLLOW_SPLIT
#define LZQ_FOLLOW_SPLIT 0  // 1: lz_follow_split_kernel (three frame jobs on three wavefronts; measured slower)
#endif
#ifndef LZQ_FOLLOW_MIN_WAVES
#define LZQ_FOLLOW_MIN_WAVES 1  // lz_follow_kernel's occupancy floor (tools/ablate_prop.py)
#endif
constexpr double kDeltaAdiabatic = 16.0;              // e^{-2 pi 16} = 2e-44
constexpr double kStepsPerRadian = 6.0;              // Magnus steps per radian of adiabatic phase in a core
constexpr double kMaxCellSteps = 16777216.0;         // per-cell Magnus steps beyond this: P = NaN (bad input)

// LZ length of a crossing in xi: sqrt(v_w/|Delta'|) * max(1, sqrt(delta)).
__device__ __forceinline__ double lz_length(double m, double a, double v_w) {
  const double delta = m * m / (2.0 * v_w * a);
  return sqrt(v_w / a) * fmax(1.0, sqrt(delta));
}

// Second-order dressed (superadiabatic) basis of H = d sz + m sx with dd/dt = ddot (d linear in
// t).  theta = atan2(m, d)/2, |+> = (cos, sin) (eigenvalue +E), |-> = (-sin, cos),
// E = sqrt(d^2 + m^2).  Adiabatic elimination of the coupling theta' between the adiabatic
// amplitudes, to second order in eps = theta'/(2E) = -m ddot/(4E^3):
//   |+~> = N (|+> + beta |->),  |-~> = N (|-> - conj(beta) |+>),
//   beta = -i eps - eps'/(2E),  eps' = 3 m ddot^2 d / (4 E^5),  N = (1 + |beta|^2)^-1/2
// (orthonormal exactly).  tests/lz_ref.py dressed_basis restates it.
struct Dressed {
  Cplx p0, p1;  // |+~>
  Cplx q0, q1;  // |-~>
};

__device__ __forceinline__ Dressed dressed_basis(double d, double ddot, double m) {
  const double th = 0.5 * atan2(m, d);
  double s, c;
  sincos(th, &s, &c);
  const double E = sqrt(d * d + m * m);
  const double iE = 1.0 / E, iE2 = iE * iE;
  const double eps = -m * ddot * 0.25 * iE2 * iE;
  const double epsd = 0.75 * m * ddot * ddot * d * iE2 * iE2 * iE;
  const double br = -0.5 * epsd * iE, bi = -eps;
  const double nrm = 1.0 / sqrt(1.0 + br * br + bi * bi);
  Dressed r;
  r.p0 = {(c - s * br) * nrm, -s * bi * nrm};
  r.p1 = {(s + c * br) * nrm, c * bi * nrm};
  r.q0 = {(-s - c * br) * nrm, c * bi * nrm};
  r.q1 = {(c - s * br) * nrm, s * bi * nrm};
  return r;
}

// The chi-like dressed state (|<chi|.>| >= 1/sqrt2): start state and final projection.
__device__ __forceinline__ void chi_like_dressed(double d, double ddot, double m, Cplx& u0, Cplx& u1) {
  const Dressed b = dressed_basis(d, ddot, m);
  const bool plus = b.p0.re * b.p0.re + b.p0.im * b.p0.im >= b.p1.re * b.p1.re + b.p1.im * b.p1.im;
  u0 = plus ? b.p0 : b.q0;
  u1 = plus ? b.p1 : b.q1;
}

#ifndef LZQ_PROP_POLY
#define LZQ_PROP_POLY 1  // 0: the Magnus vector from D and E^2 per step (round 3; tools/ablate_prop.py)
#endif

#ifndef LZQ_PROP_CORE
#define LZQ_PROP_CORE 1  // 0: Magnus over every whole cell (round-1 scheme; tools/ablate_prop.py)
#endif

// Core of a delta <= 16 cell in xi: [xc - W, xc + W], W = tau_c v_w / sqrt(alpha)
__device__ __forceinline__ double core_halfwidth(double m, double a, double v_w) {
  if (!LZQ_PROP_CORE) return INFINITY;
  const double sa = sqrt(a * v_w);
  return sa_core_tau(m / sa) * v_w / sa;
}

// ---------------------------------------------------------------------------------------
// Launch order.  A lane's cost is its Magnus step count, which its cells' cores set (C5 slice:
// ~170-280 steps per delta <= 16 cell, none in the closed-form cells; round 2's 40-LZ-length
// cores took 1000-1200 for delta <= 1 and up to ~6e4 for 1 < delta <= 16).  In index order
// a wave waits on its slowest lane in every cell and the launch ends on a few long waves.  So,
// for large batches, the points are first binned by their step count (the per-cell counts
// lz_follow_kernel stores), the bins laid out longest-first (a counting sort: LDS histograms, one
// scan, a scatter), and the kernel reads its point index from that order.  Every point is still
// computed by one lane from its own inputs, so P is bit-identical to index order; only the
// order within a bin depends on the scatter's atomics.
// ---------------------------------------------------------------------------------------
#ifndef LZQ_PROP_SORT
#define LZQ_PROP_SORT 1  // 0: index order (tools/ablate_prop.py)
#endif
constexpr int64_t kSortMinPoints = 16384;  // below this the three extra launches do not pay

constexpr int kFollowDoubles = 11;  // per (point, cell): two SU(2) matrices, the core's edges, its steps

// bin (0 = costliest) of every point + the histogram of bins.  A point's cost is the sum of its
// cells' Magnus step counts, which lz_follow_kernel (launched first) has stored per cell at + 10
// (a closed-form cell, -1 there, counts as a few steps' work; NaN: the point is returned as NaN).
__global__ __launch_bounds__(kPropBlock) void lz_cost_kernel(const double* __restrict__ vw, int64_t n,
                                                             int32_t n_cross, double v_w0,
                                                             const double* __restrict__ follow,
                                                             int32_t* __restrict__ bins, int32_t* __restrict__ hist) {
  __shared__ int32_t lh[kCostBins];
  for (int t = threadIdx.x; t < kCostBins; t += kPropBlock) lh[t] = 0;
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * kPropBlock + threadIdx.x;
  if (p < n) {
    const double v_w = vw ? vw[p] : v_w0;
    double st = __builtin_nan("");  // a bad wall speed: the follow kernel wrote nothing for this point
    if (v_w > 0.0) {
      st = 0.0;
      const double* f = follow + p * n_cross * kFollowDoubles + 10;
      for (int c = 0; c < n_cross; ++c) {
        const double Sd = f[c * kFollowDoubles];
        st += Sd < 0.0 ? 4.0 : Sd;
      }
    }
    // non-finite or absurd inputs (the kernel returns NaN at once) go with the cheapest
    const double key = st == st ? fmin(fmax(4.0 * log2(1.0 + st), 0.0), (double)(kCostBins - 1)) : 0.0;
    const int32_t b = (kCostBins - 1) - (int32_t)key;
    bins[p] = b;
    atomicAdd(&lh[b], 1);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kCostBins; t += kPropBlock)
    if (lh[t]) atomicAdd(&hist[t], lh[t]);
}

// exclusive prefix sum of the histogram (one block)
__global__ void lz_bin_scan_kernel(const int32_t* __restrict__ hist, int32_t* __restrict__ offs) {
  if (threadIdx.x == 0) {
    int32_t acc = 0;
    for (int b = 0; b < kCostBins; ++b) {
      offs[b] = acc;
      acc += hist[b];
    }
  }
}

// order[offs[bin] + rank] = p (rank within the bin from LDS counters + one global reservation
// per bin and block)
__global__ __launch_bounds__(kPropBlock) void lz_scatter_kernel(const int32_t* __restrict__ bins, int64_t n,
                                                                int32_t* __restrict__ offs,
                                                                int32_t* __restrict__ order) {
  __shared__ int32_t cnt[kCostBins], base[kCostBins];
  for (int t = threadIdx.x; t < kCostBins; t += kPropBlock) cnt[t] = 0;
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * kPropBlock + threadIdx.x;
  int32_t b = 0, r = 0;
  if (p < n) {
    b = bins[p];
    r = atomicAdd(&cnt[b], 1);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kCostBins; t += kPropBlock) base[t] = cnt[t] ? atomicAdd(&offs[t], cnt[t]) : 0;
  __syncthreads();
  if (p < n) order[base[b] + r] = (int32_t)p;
}


// Per-cell data of every (point, cell), one thread each: everything about a cell that does not
// depend on the state.  Cell c's edges are computed with the propagate kernel's own expressions
// (so bit-identical).  A delta <= 16 cell gets the superadiabatic transfer matrices of the
// stretches left and right of its core at follow[(p n_cross + c) 11 + 0..3 / 4..7] as (a.re,
// a.im, b.re, b.im), the core's edges cl, cr at + 8, 9 and its Magnus step count at + 10 (NaN for
// an absurd count).  A delta > 16 cell gets its closed-form adiabatic transfer matrix (dressed
// bases, WKB + Stokes phase, header) at + 0..3 and -1 at + 10.
__global__ __launch_bounds__(kPropBlock, LZQ_FOLLOW_MIN_WAVES) void lz_follow_kernel(const double* __restrict__ m_mix,
                                                               const double* __restrict__ dprime,
                                                               const double* __restrict__ xi,
                                                               const double* __restrict__ vw, int64_t n,
                                                               int32_t n_cross, double v_w0, double K, int32_t S,
                                                               double* __restrict__ follow) {
  const int64_t t = (int64_t)blockIdx.x * kPropBlock + threadIdx.x;
  if (t >= n * n_cross) return;
  const int64_t p = t / n_cross;
  const int c = (int)(t - p * n_cross);
  const double v_w = vw ? vw[p] : v_w0;
  if (!(v_w > 0.0)) return;  // the propagate kernel writes NaN for this point
  const double* mm = m_mix + p * n_cross;
  const double* dp = dprime + p * n_cross;
  const double* xc = xi + p * n_cross;
  const double ac = fabs(dp[c]), mc = mm[c], xcc = xc[c];
  double left, right;
  if (c == 0) {
    left = xc[0] - K * lz_length(mm[0], fabs(dp[0]), v_w);
  } else {
    const double ap = fabs(dp[c - 1]);
    left = (ap * xc[c - 1] + ac * xcc) / (ap + ac);
  }
  if (c + 1 < n_cross) {
    const double an = fabs(dp[c + 1]);
    right = (ac * xcc + an * xc[c + 1]) / (ac + an);
  } else {
    right = xcc + K * lz_length(mc, ac, v_w);
  }
  const double delta = mc * mc / (2.0 * v_w * ac);
  const double sg = (c % 2 == 0) ? 1.0 : -1.0;
  double* out = follow + (p * n_cross + c) * kFollowDoubles;
  if (delta > kDeltaAdiabatic) {
    // exact adiabatic following through the cell, in its dressed basis (header): the WKB phase
    // int E dt (closed form) + the Stokes phase - the dressed-energy tails beyond the edges
    const double slope = sg * ac;
    const double Phi = (wkb_G(ac * (right - xcc), mc) - wkb_G(ac * (left - xcc), mc)) / (ac * v_w);
    const double DL = slope * (left - xcc), DR = slope * (right - xcc);
    const double ddot = slope * v_w;
    const Dressed L = dressed_basis(DL, ddot, mc), R = dressed_basis(DR, ddot, mc);
    const double id = 1.0 / delta, id2 = id * id;
    const double phiS = id * (1.0 / 12.0 + id2 * (1.0 / 360.0 + id2 * (1.0 / 1260.0 + id2 * (1.0 / 1680.0))));
    const double tails = 0.125 * mc * mc * ac * v_w * (tail_T(DL, mc) + tail_T(DR, mc));
    // [R.p R.q] diag(e^{-i ph}, e^{i ph}) [L.p L.q]^+; a dressed basis is an SU(2) element with
    // first column |+~>
    const SU2 m = su2_mul({R.p0, R.p1}, su2_phase_adj(Phi + phiS - tails, {L.p0, L.p1}));
    out[0] = m.a.re, out[1] = m.a.im, out[2] = m.b.re, out[3] = m.b.im;
    out[10] = -1.0;
    return;
  }
  const double W = core_halfwidth(mc, ac, v_w);  // INFINITY without cores (LZQ_PROP_CORE=0)
  const double cl = fmax(left, xcc - W), cr = fmin(right, xcc + W);
  const double Phic = (wkb_G(ac * (cr - xcc), mc) - wkb_G(ac * (cl - xcc), mc)) / (ac * v_w);
  const double Sd = fmax((double)S, ceil(Phic * kStepsPerRadian));
  const double inv_vw = 1.0 / v_w;
  const double sa = sqrt(ac * v_w), mh = mc / sa;
  const double tau_c = W * sa * inv_vw;
  out[8] = cl;
  out[9] = cr;
  out[10] = Sd <= kMaxCellSteps ? Sd : __builtin_nan("");  // non-finite or absurd input: P = NaN
  const bool has_left = left < cl, has_right = cr < right;
  sa_cell_follow(mh, sg, sa * (left - xcc) * inv_vw, sa * (right - xcc) * inv_vw, tau_c, has_left, has_right, out);
}

// lz_follow_kernel with a cell's three frame jobs on three wavefronts (round 6, LZQ_FOLLOW_SPLIT):
// a block takes 64 cells; wave 0 forms each cell's core-edge frame U(tau_c) (and the header:
// edges, step count, or the closed form of an adiabatic cell), wave 1 the left stretch's outer
// frame and phase, wave 2 the right one's; after a block barrier waves 1 and 2 combine them with
// the core frame from LDS and store ML / MR.  sa_cell_follow's operations per job, so the same
// matrices; what changes is that a lane carries one frame chain at a time instead of three
// (its registers: more waves per SIMD to hide the chains' latency) and a wave runs one kind of
// job (no has_left / has_right predication across the three).
constexpr int kFollowCells = 64;
#ifndef LZQ_FOLLOW_SPLIT_WAVES
#define LZQ_FOLLOW_SPLIT_WAVES 4  // lz_follow_split_kernel's waves per SIMD (its VGPR cap = 512 / this)
#endif
__global__ __launch_bounds__(3 * kFollowCells) __attribute__((amdgpu_waves_per_eu(LZQ_FOLLOW_SPLIT_WAVES)))
void lz_follow_split_kernel(
    const double* __restrict__ m_mix, const double* __restrict__ dprime, const double* __restrict__ xi,
    const double* __restrict__ vw, int64_t n, int32_t n_cross, double v_w0, double K, int32_t S,
    double* __restrict__ follow) {
  struct Geo {
    double tl, tr, tau_c, mh;
    int32_t sides;  // bit 0: the left stretch, bit 1: the right one
  };
  __shared__ SU2 s_uc[kFollowCells];
  __shared__ Geo s_geo[kFollowCells];
  const int lane = threadIdx.x & 63, job = threadIdx.x >> 6;  // job: wave-uniform
  const int64_t t = (int64_t)blockIdx.x * kFollowCells + lane;
  const int c = t < n * n_cross ? (int)(t % n_cross) : 0;
  const double sg = (c % 2 == 0) ? 1.0 : -1.0;
  double* out = follow + t * kFollowDoubles;
  if (job == 0) {  // the cell's geometry (lz_follow_kernel's, verbatim), the header and the core frame
    Geo geo{0.0, 0.0, 0.0, 0.0, 0};
    const int64_t p = t / n_cross;
    const double v_w = t < n * n_cross ? (vw ? vw[p] : v_w0) : 0.0;
    if (t < n * n_cross && v_w > 0.0) {  // (the propagate kernel writes NaN for a bad wall speed)
      const double* mm = m_mix + p * n_cross;
      const double* dp = dprime + p * n_cross;
      const double* xc = xi + p * n_cross;
      const double ac = fabs(dp[c]), mc = mm[c], xcc = xc[c];
      double left, right;
      if (c == 0) {
        left = xc[0] - K * lz_length(mm[0], fabs(dp[0]), v_w);
      } else {
        const double ap = fabs(dp[c - 1]);
        left = (ap * xc[c - 1] + ac * xcc) / (ap + ac);
      }
      if (c + 1 < n_cross) {
        const double an = fabs(dp[c + 1]);
        right = (ac * xcc + an * xc[c + 1]) / (ac + an);
      } else {
        right = xcc + K * lz_length(mc, ac, v_w);
      }
      const double delta = mc * mc / (2.0 * v_w * ac);
      if (delta > kDeltaAdiabatic) {
        const double slope = sg * ac;
        const double Phi = (wkb_G(ac * (right - xcc), mc) - wkb_G(ac * (left - xcc), mc)) / (ac * v_w);
        const double DL = slope * (left - xcc), DR = slope * (right - xcc);
        const double ddot = slope * v_w;
        const Dressed L = dressed_basis(DL, ddot, mc), R = dressed_basis(DR, ddot, mc);
        const double id = 1.0 / delta, id2 = id * id;
        const double phiS = id * (1.0 / 12.0 + id2 * (1.0 / 360.0 + id2 * (1.0 / 1260.0 + id2 * (1.0 / 1680.0))));
        const double tails = 0.125 * mc * mc * ac * v_w * (tail_T(DL, mc) + tail_T(DR, mc));
        const SU2 m = su2_mul({R.p0, R.p1}, su2_phase_adj(Phi + phiS - tails, {L.p0, L.p1}));
        out[0] = m.a.re, out[1] = m.a.im, out[2] = m.b.re, out[3] = m.b.im;
        out[10] = -1.0;
      } else {
        const double W = core_halfwidth(mc, ac, v_w);
        const double cl = fmax(left, xcc - W), cr = fmin(right, xcc + W);
        const double Phic = (wkb_G(ac * (cr - xcc), mc) - wkb_G(ac * (cl - xcc), mc)) / (ac * v_w);
        const double Sd = fmax((double)S, ceil(Phic * kStepsPerRadian));
        const double inv_vw = 1.0 / v_w;
        const double sa = sqrt(ac * v_w);
        geo.mh = mc / sa;
        geo.tau_c = W * sa * inv_vw;
        geo.tl = sa * (left - xcc) * inv_vw;
        geo.tr = sa * (right - xcc) * inv_vw;
        geo.sides = (left < cl ? 1 : 0) | (cr < right ? 2 : 0);
        out[8] = cl;
        out[9] = cr;
        out[10] = Sd <= kMaxCellSteps ? Sd : __builtin_nan("");
      }
    }
    s_geo[lane] = geo;
  }
  __syncthreads();
  const Geo geo = s_geo[lane];
  // wave 0: the core frame; waves 1, 2: the outer frame and the phase of their stretch
  const bool mine = job == 0 ? geo.sides != 0 : ((geo.sides >> (job - 1)) & 1) != 0;
  SU2 u{};
  double ph = 0.0;
  if (mine) {
    if (job == 0) {
      s_uc[lane] = sa_frame(geo.tau_c, sg, geo.mh, false);
    } else {
      const double tau = job == 1 ? geo.tl : geo.tr;
      u = sa_frame(tau, sg, geo.mh, true);
      ph = job == 1 ? sa_phase(geo.tl, -geo.tau_c, geo.mh) : sa_phase(geo.tau_c, geo.tr, geo.mh);
    }
  }
  __syncthreads();
  if (mine && job > 0) {
    const SU2 uc = s_uc[lane];
    if (job == 1) sa_store(su2_mul(sa_reflect(uc), su2_phase_adj(ph, u)), out);  // U(-tau_c) P U(tl)^+
    else sa_store(su2_mul(u, su2_phase_adj(ph, uc)), out + 4);                   // U(tr) P U(tau_c)^+
  }
}

__global__ __launch_bounds__(kPropBlock, LZQ_PROP_MIN_WAVES) void lz_propagate_kernel(const double* __restrict__ m_mix,
                                                                  const double* __restrict__ dprime,
                                                                  const double* __restrict__ xi,
                                                                  const double* __restrict__ vw, int64_t n,
                                                                  int32_t n_cross, double v_w0, double K,
                                                                  int32_t S, const int32_t* __restrict__ order,
                                                                  const double* __restrict__ follow,
                                                                  double* __restrict__ P_out) {
  const int64_t tid = (int64_t)blockIdx.x * kPropBlock + threadIdx.x;
  if (tid >= n) return;
  const int64_t p = order ? (int64_t)order[tid] : tid;
  const double v_w = vw ? vw[p] : v_w0;  // per-point wall speed (lzq_lz_propagate_v) or the batch's
  if (!(v_w > 0.0)) {
    P_out[p] = __builtin_nan("");
    return;
  }
  const double* mm = m_mix + p * n_cross;
  const double* dp = dprime + p * n_cross;
  const double* xc = xi + p * n_cross;
  const double inv_vw = 1.0 / v_w;

  // left edge of cell 0
  double a0 = fabs(dp[0]);
  double left = xc[0] - K * lz_length(mm[0], a0, v_w);
  double D_left = a0 * (left - xc[0]);  // s_0 = +1
  Cplx p0, p1;
  chi_like_dressed(D_left, a0 * v_w, mm[0], p0, p1);

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
    const double* Mc = follow + (p * n_cross + c) * kFollowDoubles;  // lz_follow_kernel's cell data
    const double Sd = Mc[10];
    if (Sd < 0.0) {
      su2_apply_mat({{Mc[0], Mc[1]}, {Mc[2], Mc[3]}}, p0, p1);  // closed-form adiabatic cell
    } else {
      // Magnus on the core, superadiabatic following on either side of it
      const double cl = Mc[8], cr = Mc[9];
      if (!(Sd <= kMaxCellSteps)) {  // non-finite or absurd input (bounded for any valid one)
        P_out[p] = __builtin_nan("");
        return;
      }
      if (left < cl) su2_apply_mat({{Mc[0], Mc[1]}, {Mc[2], Mc[3]}}, p0, p1);
      const int Sc = (int)Sd;
      const double h = (cr - cl) / (double)Sc;  // step in xi
      const double dt = h * inv_vw;                  // step in t
      // per-cell coefficients of the eighth-order Magnus vector (header)
      const double ddot = slope * v_w, dd2 = ddot * ddot, m2 = mc * mc;
      const double dt2 = dt * dt, dt4 = dt2 * dt2;
      const double ax = 1.0 - dd2 * dt4 * (1.0 / 60.0);
      const double bx = dd2 * dt4 * dt2 * (1.0 / 1890.0);
      const double cxm = dt * mc, m2x4 = 4.0 * m2;
      const double cy = ddot * mc * dt * dt2, ey1 = dt2 * (1.0 / 90.0), ey2 = dt4 * (1.0 / 7560.0);
      const double dd2x9 = 9.0 * dd2;
      const double cz = dt * (1.0 - bx * m2);
      // The step as fused multiply-adds (the file builds with -ffp-contract=off for the
      // oracle-matching kernels, so contraction is spelled out): 63 VALU per step where the
      // separate products and sums took 84.
#define FMA __builtin_fma
#if LZQ_PROP_POLY
      // Round 4: n as polynomials in the step's midpoint D = D0 + i dD (D linear in xi):
      //   n_x = kx0 + kx2 D^2,  n_y = ky0 + ky2 D^2 + ky4 D^4,  n_z = cz D
      // (the header's coefficients expanded in E^2 = D^2 + m^2 once per cell), 7 VALU for the
      // Magnus vector where the expressions above take 15.
      const double D0 = slope * ((cl - xcc) + 0.5 * h), dD = slope * h;
      const double kx0 = cxm * FMA(-bx, m2x4, ax), kx2 = -3.0 * cxm * bx;
      const double ky0 = cy * FMA(ey2, FMA(8.0 * m2, m2, -dd2x9), FMA(ey1, m2, 1.0 / 6.0));
      const double ky2 = cy * FMA(16.0 * ey2, m2, ey1), ky4 = 8.0 * cy * ey2;
      auto step = [&](int i) {
        const double D = FMA((double)i, dD, D0);
        const double D2 = D * D;
        const double nx = FMA(kx2, D2, kx0);
        const double ny = FMA(FMA(ky4, D2, ky2), D2, ky0);
        const double nz = cz * D;
        double cs, sc;  // cos|n| and sin|n|/|n|, both functions of |n|^2
        cos_sinc_short(FMA(nx, nx, FMA(ny, ny, nz * nz)), cs, sc);
        su2_apply(cs, sc * nx, sc * ny, sc * nz, p0, p1);
      };
#else
      auto step = [&](int i) {
        const double xm = FMA((double)i + 0.5, h, cl);
        const double D = slope * (xm - xcc);
        const double D2 = D * D, E2 = D2 + m2;
        const double nx = cxm * FMA(-bx, FMA(3.0, D2, m2x4), ax);
        const double ny = cy * FMA(ey2, FMA(8.0 * E2, E2, -dd2x9), FMA(ey1, E2, 1.0 / 6.0));
        const double nz = cz * D;
        double cs, sc;  // cos|n| and sin|n|/|n|, both functions of |n|^2
        cos_sinc(FMA(nx, nx, FMA(ny, ny, nz * nz)), cs, sc);
        su2_apply(cs, sc * nx, sc * ny, sc * nz, p0, p1);
      };
#endif
      // unrolled by hand: the polynomial's inline asm (fma3) is convergent, which rules out
      // the compiler's runtime unrolling
      int i = 0;
      for (; i + LZQ_PROP_UNROLL <= Sc; i += LZQ_PROP_UNROLL) {
#pragma unroll
        for (int u = 0; u < LZQ_PROP_UNROLL; ++u) step(i + u);
      }
      for (; i < Sc; ++i) step(i);
#undef FMA
      if (cr < right) su2_apply_mat({{Mc[4], Mc[5]}, {Mc[6], Mc[7]}}, p0, p1);
    }
    left = right;
    sgn = -sgn;
  }
  // project on the chi-like dressed state at the right edge of the last cell
  const int last = n_cross - 1;
  const double slope_last = -sgn * fabs(dp[last]);  // sgn was flipped once more
  Cplx u0, u1;
  chi_like_dressed(slope_last * (right - xc[last]), slope_last * v_w, mm[last], u0, u1);
  const Cplx a = inner(u0, u1, p0, p1);
  const double re = a.re, im = a.im;
  const double norm = p0.re * p0.re + p0.im * p0.im + p1.re * p1.re + p1.im * p1.im;
  P_out[p] = 1.0 - (re * re + im * im) / norm;
}

}  // namespace lzq

// error plumbing shared with lzq_kernels.hip (C++ linkage, not part of the C ABI)
int lzq_set_error(int code, const char* msg);

namespace {
// Cell data take 88 B per (point, cell): batches are run in slices of at most this many
// (point, cell) pairs (704 MiB).
constexpr int64_t kFollowMaxPairs = (int64_t)1 << 23;

int propagate_slice(const double* d_m_mix, const double* d_dprime, const double* d_xi, const double* d_v_w, int64_t n,
                    int32_t n_cross, double v_w, double window_lz, int32_t steps_per_crossing, double* d_P,
                    hipStream_t st) {
  const int64_t nb = (n + lzq::kPropBlock - 1) / lzq::kPropBlock;
  // stream-ordered scratch (calls on different streams stay independent): the follow matrices,
  // then the longest-first launch order (see lz_cost_kernel) for large batches
  const bool sort = LZQ_PROP_SORT && n >= lzq::kSortMinPoints;
  const size_t follow_bytes = (size_t)(n * n_cross) * lzq::kFollowDoubles * sizeof(double);
  const size_t sort_bytes = sort ? (size_t)(2 * n + 2 * lzq::kCostBins) * sizeof(int32_t) : 0;
  char* ws = nullptr;
  {
    hipError_t e = hipMallocAsync((void**)&ws, follow_bytes + sort_bytes, st);
    if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  }
  double* follow = (double*)ws;
  const int32_t* order = nullptr;
  hipError_t e = hipSuccess;
  {
    if (LZQ_FOLLOW_SPLIT) {
      const int64_t nf = (n * n_cross + lzq::kFollowCells - 1) / lzq::kFollowCells;
      hipLaunchKernelGGL(lzq::lz_follow_split_kernel, dim3((unsigned)nf), dim3(3 * lzq::kFollowCells), 0, st, d_m_mix,
                         d_dprime, d_xi, d_v_w, n, n_cross, v_w, window_lz, steps_per_crossing, follow);
    } else {
      const int64_t nf = (n * n_cross + lzq::kPropBlock - 1) / lzq::kPropBlock;
      hipLaunchKernelGGL(lzq::lz_follow_kernel, dim3((unsigned)nf), dim3(lzq::kPropBlock), 0, st, d_m_mix, d_dprime,
                         d_xi, d_v_w, n, n_cross, v_w, window_lz, steps_per_crossing, follow);
    }
  }
  if (sort) {
    int32_t* iw = (int32_t*)(ws + follow_bytes);
    int32_t *bins = iw, *ord = iw + n, *hist = iw + 2 * n, *offs = hist + lzq::kCostBins;
    e = hipMemsetAsync(hist, 0, lzq::kCostBins * sizeof(int32_t), st);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(lzq::lz_cost_kernel, dim3((unsigned)nb), dim3(lzq::kPropBlock), 0, st, d_v_w, n, n_cross, v_w,
                         follow, bins, hist);
      hipLaunchKernelGGL(lzq::lz_bin_scan_kernel, dim3(1), dim3(64), 0, st, hist, offs);
      hipLaunchKernelGGL(lzq::lz_scatter_kernel, dim3((unsigned)nb), dim3(lzq::kPropBlock), 0, st, bins, n, offs,
                         ord);
      order = ord;
    }
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(lzq::lz_propagate_kernel, dim3((unsigned)nb), dim3(lzq::kPropBlock), 0, st, d_m_mix, d_dprime,
                       d_xi, d_v_w, n, n_cross, v_w, window_lz, steps_per_crossing, order, follow, d_P);
    e = hipGetLastError();
  }
  if (ws) {
    const hipError_t ef = hipFreeAsync(ws, st);
    if (e == hipSuccess) e = ef;
  }
  if (e != hipSuccess) return lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
  return LZQ_OK;
}

int propagate_launch(const double* d_m_mix, const double* d_dprime, const double* d_xi, const double* d_v_w, int64_t n,
                     int32_t n_cross, double v_w, double window_lz, int32_t steps_per_crossing, double* d_P,
                     void* stream) {
  if (n == 0) return LZQ_OK;
  if (n > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_lz_propagate: n too large (int32 point order)");
  const int64_t slice = std::max<int64_t>(1, kFollowMaxPairs / n_cross);
  for (int64_t s0 = 0; s0 < n; s0 += slice) {
    const int64_t k = std::min(slice, n - s0);
    const int rc = propagate_slice(d_m_mix + s0 * n_cross, d_dprime + s0 * n_cross, d_xi + s0 * n_cross,
                                   d_v_w ? d_v_w + s0 : nullptr, k, n_cross, v_w, window_lz, steps_per_crossing,
                                   d_P + s0, (hipStream_t)stream);
    if (rc != LZQ_OK) return rc;
  }
  return LZQ_OK;
}

}  // namespace

// Longest-first launch order from per-point cost bins (0 = costliest) and their histogram
// (lzq_internal.h; shared with lzq_profile.hip): the scan and scatter kernels above.
int lzq::launch_bin_order(const int32_t* bins, const int32_t* hist, int32_t* offs, int64_t n, int32_t* order,
                          hipStream_t st) {
  const int64_t nb = (n + lzq::kPropBlock - 1) / lzq::kPropBlock;
  hipLaunchKernelGGL(lzq::lz_bin_scan_kernel, dim3(1), dim3(64), 0, st, hist, offs);
  hipLaunchKernelGGL(lzq::lz_scatter_kernel, dim3((unsigned)nb), dim3(lzq::kPropBlock), 0, st, bins, n, offs, order);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LZQ_OK : lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
}

namespace {
bool propagate_args_ok(int64_t n, int32_t n_cross, double window_lz, int32_t steps_per_crossing) {
  return n >= 0 && n_cross > 0 && steps_per_crossing > 0 && steps_per_crossing <= 1000000 && window_lz > 0.0 &&
         window_lz <= 200.0;
}
}  // namespace

extern "C" int lzq_lz_propagate(const double* d_m_mix, const double* d_dprime, const double* d_xi, int64_t n,
                                int32_t n_cross, double v_w, double window_lz, int32_t steps_per_crossing,
                                double* d_P, void* stream) {
  if (!propagate_args_ok(n, n_cross, window_lz, steps_per_crossing) || !(v_w > 0.0) ||
      (n > 0 && (!d_m_mix || !d_dprime || !d_xi || !d_P)))
    return lzq_set_error(LZQ_EINVAL, "lzq_lz_propagate: bad arguments (need n >= 0, n_cross > 0, "
                                     "0 < steps_per_crossing <= 1e6, v_w > 0, 0 < window_lz <= 200)");
  return propagate_launch(d_m_mix, d_dprime, d_xi, nullptr, n, n_cross, v_w, window_lz, steps_per_crossing, d_P,
                          stream);
}

extern "C" int lzq_lz_propagate_v(const double* d_m_mix, const double* d_dprime, const double* d_xi,
                                  const double* d_v_w, int64_t n, int32_t n_cross, double window_lz,
                                  int32_t steps_per_crossing, double* d_P, void* stream) {
  if (!propagate_args_ok(n, n_cross, window_lz, steps_per_crossing) ||
      (n > 0 && (!d_m_mix || !d_dprime || !d_xi || !d_v_w || !d_P)))
    return lzq_set_error(LZQ_EINVAL, "lzq_lz_propagate_v: bad arguments (need n >= 0, n_cross > 0, "
                                     "0 < steps_per_crossing <= 1e6, 0 < window_lz <= 200, d_v_w)");
  return propagate_launch(d_m_mix, d_dprime, d_xi, d_v_w, n, n_cross, 1.0, window_lz, steps_per_crossing, d_P,
                          stream);
}
