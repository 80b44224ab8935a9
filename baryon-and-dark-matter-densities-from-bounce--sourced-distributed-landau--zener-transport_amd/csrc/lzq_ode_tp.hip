// lzq_ode_tp.hip -- lzq_ode_integrate_tp: the reference's ODE fallback (fpy:270-286, 385-417)
// for a few points, parallel in time (multiple shooting, then the exact chains stitched through
// candidate starts), bit-identical to the sequential integration of lzq_ode.hip.  The device
// helpers (stages, Radau step, predictor) are lzq_ode.h's, shared with the sequential kernels.
#include "lzq_ode.h"

namespace lzq {

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
// verified: the point's window and table already passed these checks (ode_tp_init_kernel took it:
// ctl.phase != kTpFallback), so the knot-by-knot grid check (~800 comparisons per lane) is skipped;
// every other value is formed as in the checked call.
__device__ __forceinline__ OdeSetup ode_setup(const lzq_point& pt, const lzq_ode_params& od, const double* w,
                                              int64_t max_steps, bool verified = false) {
  OdeSetup S;
  S.o = ode_point(pt, od);
  const OdePoint& o = S.o;
  S.st = verified ? LZQ_ODE_OK
                  : (ode_grid_ok(o.T_lo, o.T_hi, o.stepT) ? (ode_table_ok(w) ? LZQ_ODE_OK : LZQ_ODE_BAD_TABLE)
                                                          : LZQ_ODE_BAD_GRID);
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

// A regular step's stage data for one point (round 6): what tp_steps reads of its three stages
// (ode_stage: lam, E2, S) and of Y_B's step map (yb_rec: c, d), formed by ode_tp_rows_kernel once per
// call -- the stages depend on the point and x only, not on the state -- instead of in every
// interval integration, candidate and update.  The same functions on the same x, so the same bits.
// Layout per point: step k at (k mod L) * Mmax + k / L (the lanes of an interval launch, one
// interval each, read consecutive rows); only points whose interval length is L (ctl.L) use them.
struct TpRow {
  double lam[3], E2[3], S[3], c, d;
};
constexpr size_t kTpRowBytes = size_t(1) << 31;  // row tables of one call, at most (else stages inline)
#ifndef LZQ_ODE_TP_FUSE
#define LZQ_ODE_TP_FUSE 1  // a Newton update in two launches instead of four (same operations)
#endif
#ifndef LZQ_ODE_TP_ROWS
#define LZQ_ODE_TP_ROWS 1  // 0: every step forms its stages inline (the round-5 path; same bits)
#endif

__global__ __launch_bounds__(256) void ode_tp_rows_kernel(const lzq_point* __restrict__ pts,
                                                          const lzq_ode_params* __restrict__ ode, int64_t n,
                                                          const int32_t* __restrict__ tidx,
                                                          const double* __restrict__ ws, int64_t max_steps, int64_t L,
                                                          int64_t Mmax, const TpCtl* __restrict__ ctl,
                                                          TpRow* __restrict__ rows) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = Mmax * L;
  const int64_t p = g / per, rem = g - p * per;
  if (p >= n) return;
  const TpCtl c = ctl[p];
  const int64_t r = rem / Mmax, m = rem - r * Mmax, k = m * L + r;  // lanes: consecutive intervals
  if (c.phase != kTpIter || c.L != L || k >= c.N) return;
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps, true);
  const Radau R = radau_tableau();
  const RadauH hA = radau_h(R, S.h);
  const double xk = S.x0 + (double)k * S.h;  // tp_steps' x_k (its step counter is an exact double)
  OdeStage sg[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) sg[j] = ode_stage(S.o, w, xk + R.c[j] * S.h);
  const YbRec yr = yb_rec(hA, sg);
  TpRow row;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    row.lam[j] = sg[j].lam;
    row.E2[j] = sg[j].E2;
    row.S[j] = sg[j].S;
  }
  row.c = yr.c;
  row.d = yr.d;
  rows[p * per + rem] = row;  // (a split step's row is formed too, and not read: tp_steps splits it)
}

// Steps [k0, k1) of the fixed-step sequence x_k = x0 + k h from state St, with ode_integrate_kernel's
// per-lane operations (stages, Y_B map, Radau step, the T = m/3 split step, the predictor); D and C
// accumulate the derivatives of the end state.  Returns false when a step needed tp_bridge.
// rows (optional): the TpRow of step k0 of an interval, the next steps' rows `stride` apart (the
// point's table at (k mod L) * Mmax + k / L: stride Mmax), for the regular steps.
__device__ __forceinline__ bool tp_steps(const OdePoint& o, const double* __restrict__ w, double x0, double h,
                                         double xb, double xb_below, int64_t k0, int64_t k1, TpState& St, double& D,
                                         double& C, const TpRow* __restrict__ rows = nullptr, int64_t stride = 0) {
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
      double yc, yd;
      if (rows && !own_h) {  // a regular step: its stage data from the row table
        const TpRow& rw = rows[(k - k0) * stride];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          sg[j].lam = rw.lam[j];
          sg[j].E2 = rw.E2[j];
          sg[j].S = rw.S[j];
        }
        yc = rw.c;
        yd = rw.d;
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) sg[j] = ode_stage(o, w, xs + R.c[j] * hs);
        const YbRec yr = yb_rec(hAs, sg);
        yc = yr.c;
        yd = yr.d;
      }
      YB = __builtin_fma(yc, YB, o.Pf * yd);
      C *= yc;
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
                                                             TpEnd* __restrict__ ends, const TpCtl* __restrict__ ctl,
                                                             const TpRow* __restrict__ rows) {
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t p = g / Mmax, m = g - p * Mmax;
  if (p >= n) return;
  const TpCtl c = ctl[p];
  if (c.phase != kTpIter || m >= c.M) return;
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps, true);
  const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
  const double xb = branch_x(S.o, S.x0, S.x1);
  const TpNode nd = nodes[p * (Mmax + 1) + m];
  TpState St{nd.Ychi, nd.YB, nd.Ychi, {nd.Ychi, nd.Ychi, nd.Ychi}, false};  // (the first step reads no predictor)
  double D = 1.0, C = 1.0;
  const TpRow* rp = rows && c.L == L ? rows + p * Mmax * L + m : nullptr;  // interval m's first row
  const bool exact = tp_steps(S.o, w, S.x0, S.h, xb, nextafter(xb, -INFINITY), k0, k1, St, D, C, rp, Mmax);
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
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps, true);
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

// (LZQ_ODE_TP_FUSE) the interval integration and the block-local scan in one launch: thread t of
// block b integrates interval b kTpBlk + t (ode_tp_interval_kernel's body), then the block scans.
__global__ __launch_bounds__(kTpBlk) void ode_tp_interval_scan_kernel(
    const lzq_point* __restrict__ pts, const lzq_ode_params* __restrict__ ode, const int32_t* __restrict__ tidx,
    const double* __restrict__ ws, int64_t max_steps, int64_t L, int64_t Mmax, int64_t Bmax,
    const TpNode* __restrict__ nodes, TpEnd* __restrict__ ends, const TpCtl* __restrict__ ctl,
    const TpRow* __restrict__ rows, TpMap* __restrict__ loc, TpMap* __restrict__ agg, TpBlkOut* __restrict__ bout) {
  __shared__ TpMap sm[kTpBlk];
  const int64_t p = blockIdx.y, b = blockIdx.x;
  const TpCtl c = ctl[p];
  if (c.phase != kTpIter || b * kTpBlk >= c.M) return;  // block-uniform
  const int t = threadIdx.x;
  const int64_t m = b * kTpBlk + t;
  TpEnd e{0.0, 0.0, 0.0, 0.0, 0, 0};
  if (m < c.M) {
    const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
    const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps, true);
    const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
    const double xb = branch_x(S.o, S.x0, S.x1);
    const TpNode nd = nodes[p * (Mmax + 1) + m];
    TpState St{nd.Ychi, nd.YB, nd.Ychi, {nd.Ychi, nd.Ychi, nd.Ychi}, false};
    double D = 1.0, C = 1.0;
    const TpRow* rp = rows && c.L == L ? rows + p * Mmax * L + m : nullptr;
    const bool exact = tp_steps(S.o, w, S.x0, S.h, xb, nextafter(xb, -INFINITY), k0, k1, St, D, C, rp, Mmax);
    e = TpEnd{St.Ychi, St.YB, D, C, exact ? 1 : 0, 0};
    ends[p * Mmax + m] = e;
  }
  TpMap v{1.0, 0.0, 1.0, 0.0};
  int fail = 0;
  if (m < c.M) {
    const TpNode q = nodes[p * (Mmax + 1) + m + 1];
    const bool fin = isfinite(e.Ychi) && isfinite(e.D) && isfinite(e.YB) && isfinite(e.C);
    fail = e.exact == 0 || !fin;
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

// ticket (LZQ_ODE_TP_FUSE, else nullptr): per point, the blocks of this update that are done; the
// last one folds the point's block results into TpCtl (tp_finish_update, what
// ode_tp_scan_finish_kernel does in its own launch) and resets the count for the next update.
__device__ __forceinline__ void tp_finish_update(int64_t p, int64_t Bmax, TpCtl* __restrict__ ctl,
                                                 const TpBlkOut* __restrict__ bout, int32_t max_iters, double tol);
__global__ __launch_bounds__(kTpBlk) void ode_tp_scan_apply_kernel(int64_t Mmax, int64_t Bmax,
                                                                   TpNode* __restrict__ nodes,
                                                                   const TpEnd* __restrict__ ends,
                                                                   TpCtl* __restrict__ ctl,
                                                                   const TpMap* __restrict__ loc,
                                                                   const TpMap* __restrict__ agg,
                                                                   TpBlkOut* __restrict__ bout,
                                                                   int32_t* __restrict__ ticket, int32_t max_iters,
                                                                   double tol) {
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
    if (ticket) {
      // release this block's bout store, count it; the last block acquires the others' and folds
      const int32_t done = __hip_atomic_fetch_add(&ticket[p], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (done == (int32_t)(nb - 1)) {
        tp_finish_update(p, Bmax, ctl, bout, max_iters, tol);
        __hip_atomic_store(&ticket[p], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

__device__ __forceinline__ void tp_finish_update(int64_t p, int64_t Bmax, TpCtl* __restrict__ ctl,
                                                 const TpBlkOut* __restrict__ bout, int32_t max_iters, double tol);
__global__ __launch_bounds__(64) void ode_tp_scan_finish_kernel(int64_t n, int64_t Bmax, TpCtl* __restrict__ ctl,
                                                                const TpBlkOut* __restrict__ bout, int32_t max_iters,
                                                                double tol) {
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (p >= n) return;
  if (ctl[p].phase != kTpIter) return;
  tp_finish_update(p, Bmax, ctl, bout, max_iters, tol);
}
// fold point p's block errors and failure flags into its TpCtl (the update count, converged ->
// kTpDone, out of updates -> kTpFallback)
__device__ __forceinline__ void tp_finish_update(int64_t p, int64_t Bmax, TpCtl* __restrict__ ctl,
                                                 const TpBlkOut* __restrict__ bout, int32_t max_iters, double tol) {
  TpCtl c = ctl[p];
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
                                         int64_t m, int off, double* __restrict__ oF, double* __restrict__ oG,
                                         const TpRow* __restrict__ rp, int64_t stride) {
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps, true);
  const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
  const double y0 = dfromkey(dkey(nd->Ychi) + off), b0 = dfromkey(dkey(nd->YB) + off);
  // (k0 is a whole number of predictor blocks: the first step does not read Yp / Z / have)
  TpState St{y0, b0, y0, {y0, y0, y0}, false};
  double D = 1.0, C = 1.0;
  const double xb = branch_x(S.o, S.x0, S.x1);
  const bool exact = tp_steps(S.o, w, S.x0, S.h, xb, nextafter(xb, -INFINITY), k0, k1, St, D, C, rp, stride);
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
                                                         double* __restrict__ candF, double* __restrict__ candG,
                                                         const TpRow* __restrict__ rows, int64_t L) {
  constexpr int NC = 2 * J + 1;
  for (int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x; g < n * Mmax * NC; g += (int64_t)gridDim.x * 64) {
    const int64_t p = g / (Mmax * NC), rem = g - p * (Mmax * NC), m = rem / NC;
    const int jj = (int)(rem - m * NC);
    const TpCtl c = ctl[p];
    if (c.phase == kTpDone && m < c.M) {
      const int64_t o = (p * Mmax + m) * NC + jj;
      const TpRow* rp = rows && c.L == L ? rows + p * Mmax * L + m : nullptr;  // interval m's first row
      if constexpr (kStride) {
        tp_cand_one(pts, ode, tidx, ws, max_steps, nodes + p * (Mmax + 1) + m, c, p, m, jj - J, candF + o, candG + o, rp,
                    Mmax);
      } else {
        const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
        const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps, true);
        const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
        const TpNode& nd = nodes[p * (Mmax + 1) + m];
        const double y0 = dfromkey(dkey(nd.Ychi) + (jj - J)), b0 = dfromkey(dkey(nd.YB) + (jj - J));
        TpState St{y0, b0, y0, {y0, y0, y0}, false};
        double D = 1.0, C = 1.0;
        const double xb = branch_x(S.o, S.x0, S.x1);
        const bool exact = tp_steps(S.o, w, S.x0, S.h, xb, nextafter(xb, -INFINITY), k0, k1, St, D, C, rp, Mmax);
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
                                                          const TpCtl* __restrict__ ctl, double* __restrict__ candG,
                                                          const TpRow* __restrict__ rows, int64_t L) {
  constexpr int NC = 2 * JG + 1, NCH = (NC + kTpGChunk - 1) / kTpGChunk;
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t p = g / (Mmax * NCH), rem = g - p * (Mmax * NCH), m = rem / NCH;
  const int ch = (int)(rem - m * NCH);
  if (p >= n) return;
  const TpCtl c = ctl[p];
  if (c.phase != kTpDone || m >= c.M) return;
  const double* w = ws + (tidx ? (int64_t)tidx[p] : p) * (int64_t)kOdeWS;
  const OdeSetup S = ode_setup(pts[p], ode[p], w, max_steps, true);
  const int64_t k0 = m * c.L, k1 = k0 + c.L < S.N ? k0 + c.L : S.N;
  const int64_t bkey = dkey(nodes[p * (Mmax + 1) + m].YB);
  double yb[kTpGChunk];
#pragma unroll
  for (int i = 0; i < kTpGChunk; ++i) yb[i] = dfromkey(bkey + (ch * kTpGChunk + i - JG));
  const Radau R = radau_tableau();
  const RadauH hA = radau_h(R, S.h);
  const double xb = branch_x(S.o, S.x0, S.x1), xb_below = nextafter(xb, -INFINITY);
  const TpRow* rp = rows && c.L == L ? rows + p * Mmax * L + m : nullptr;  // interval m's first row
  int64_t k = k0;
  auto part = [&](double xs, double hs, bool own_h) {
    double yc, yd;
    if (rp && !own_h) {  // a regular step: Y_B's map from the row table
      const TpRow& rw = rp[(k - k0) * Mmax];
      yc = rw.c;
      yd = rw.d;
    } else {
      const RadauH hAs = own_h ? radau_h(R, hs) : hA;
      OdeStage sg[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) sg[j] = ode_stage(S.o, w, xs + R.c[j] * hs);
      const YbRec yr = yb_rec(hAs, sg);
      yc = yr.c;
      yd = yr.d;
    }
    const double e = S.o.Pf * yd;
#pragma unroll
    for (int i = 0; i < kTpGChunk; ++i) yb[i] = __builtin_fma(yc, yb[i], e);
  };
  double kd = (double)k0;
  for (; k < k1; ++k, kd += 1.0) {
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

}  // namespace lzq

namespace {

int hip_check(hipError_t e, const char* what) { return lzq_ode_hip_check(e, what); }
int check_ws(int64_t n, const double* d_work, int64_t work_doubles, const char* fn) {
  return lzq_ode_check_ws(n, d_work, work_doubles, fn);
}

template <bool kChiOnly>
int launch_integrate(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const int32_t* d_tidx,
                     const double* d_work, int64_t max_steps, lzq_yield* d_out, int32_t* d_status, hipStream_t s,
                     const char* fn, const int32_t* d_skip = nullptr) {
  static_assert(!kChiOnly, "lzq_ode_integrate_tp steps both equations");
  return lzq_ode_launch_sequential(d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, s, fn, d_skip);
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
  // the regular steps' stage rows (TpRow), when the tables of the call fit kTpRowBytes
  const size_t rows_raw = sizeof(lzq::TpRow) * (size_t)n * (size_t)Mmax * (size_t)L;
  const bool use_rows = LZQ_ODE_TP_ROWS && rows_raw <= lzq::kTpRowBytes;
  const size_t b_rows = use_rows ? up(rows_raw) : 0;
  const size_t b_tk = up(sizeof(int32_t) * (size_t)n);
  char* buf = nullptr;
  int rc = hip_check(hipMallocAsync((void**)&buf, b_nodes + b_ends + b_ctl + b_skip + 2 * (b_cand + b_segi + b_segv) +
                                                       b_loc + b_agg + b_bout + b_gd + b_gy + b_rows + b_tk,
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
  auto* rows = use_rows ? reinterpret_cast<lzq::TpRow*>(take(b_rows)) : nullptr;
  auto* ticket = reinterpret_cast<int32_t*>(take(b_tk));
  hipLaunchKernelGGL(lzq::ode_tp_init_kernel, dim3((unsigned)n), dim3(256), 0, s, d_points, d_ode, d_tidx, d_work,
                     max_steps, L, Mmax, nodes, ctl);
  rc = hip_check(hipGetLastError(), fn);
  if (rc == LZQ_OK && Mmax >= lzq::kTpGuessMin) {
    hipLaunchKernelGGL(lzq::ode_tp_guess_kernel, dim3((unsigned)n), dim3(256), 0, s, d_points, d_ode, d_tidx, d_work,
                       max_steps, L, Mmax, nodes, ctl);
    rc = hip_check(hipGetLastError(), fn);
  }
  if (rc == LZQ_OK && use_rows) {
    hipLaunchKernelGGL(lzq::ode_tp_rows_kernel, dim3((unsigned)((n * Mmax * L + 255) / 256)), dim3(256), 0, s,
                       d_points, d_ode, n, d_tidx, d_work, max_steps, L, Mmax, ctl, rows);
    rc = hip_check(hipGetLastError(), fn);
  }
  const unsigned ib = (unsigned)((n * Mmax + 63) / 64);
  // one Newton update: LZQ_ODE_TP_FUSE, two launches (intervals + local scans, then the carries,
  // the node update and -- in the point's last block -- the convergence fold); else four
  if (rc == LZQ_OK && LZQ_ODE_TP_FUSE) rc = hip_check(hipMemsetAsync(ticket, 0, sizeof(int32_t) * (size_t)n, s), fn);
  for (int32_t it = 0; it < kTpMaxIters && rc == LZQ_OK; ++it) {
    if (LZQ_ODE_TP_FUSE) {
      hipLaunchKernelGGL(lzq::ode_tp_interval_scan_kernel, dim3((unsigned)Bmax, (unsigned)n), dim3(lzq::kTpBlk), 0, s,
                         d_points, d_ode, d_tidx, d_work, max_steps, L, Mmax, Bmax, nodes, ends, ctl, rows, loc, agg,
                         bout);
      rc = hip_check(hipGetLastError(), fn);
      if (rc) break;
      hipLaunchKernelGGL(lzq::ode_tp_scan_apply_kernel, dim3((unsigned)Bmax, (unsigned)n), dim3(lzq::kTpBlk), 0, s,
                         Mmax, Bmax, nodes, ends, ctl, loc, agg, bout, ticket, kTpMaxIters, kTpTol);
      rc = hip_check(hipGetLastError(), fn);
      continue;
    }
    hipLaunchKernelGGL(lzq::ode_tp_interval_kernel, dim3(ib), dim3(64), 0, s, d_points, d_ode, n, d_tidx, d_work,
                       max_steps, L, Mmax, nodes, ends, ctl, rows);
    rc = hip_check(hipGetLastError(), fn);
    if (rc) break;
    hipLaunchKernelGGL(lzq::ode_tp_scan_local_kernel, dim3((unsigned)Bmax, (unsigned)n), dim3(lzq::kTpBlk), 0, s, Mmax,
                       Bmax, nodes, ends, ctl, loc, agg, bout);
    rc = hip_check(hipGetLastError(), fn);
    if (rc) break;
    hipLaunchKernelGGL(lzq::ode_tp_scan_apply_kernel, dim3((unsigned)Bmax, (unsigned)n), dim3(lzq::kTpBlk), 0, s, Mmax,
                       Bmax, nodes, ends, ctl, loc, agg, bout, (int32_t*)nullptr, kTpMaxIters, kTpTol);
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
                         d_points, d_ode, n, d_tidx, d_work, max_steps, Mmax, nodes, ctl, candF, candG, rows, L);
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
                       d_points, d_ode, n, d_tidx, d_work, max_steps, Mmax, nodes, ctl, candG, rows, L);
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

}  // namespace

extern "C" {

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

}  // extern "C"
