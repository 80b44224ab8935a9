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
//
// The device helpers (per-point constants, stages, the Radau step) live in lzq_ode.h, shared with
// lzq_ode_tp.hip (the time-parallel integration of a few points).
#include "lzq_ode.h"

namespace lzq {
int g_ode_coop = 1;          // lzq_tune(LZQ_TUNE_ODE_COOP)
int g_ode_launch_log2 = 24;  // lzq_tune(LZQ_TUNE_ODE_LAUNCH_STEPS): <= 2^24 Radau steps per launch
int g_ode_tp_interval = 64;  // lzq_tune(LZQ_TUNE_ODE_TP_INTERVAL): steps per lzq_ode_integrate_tp interval
int g_ode_table_wide = 3;    // lzq_tune(LZQ_TUNE_ODE_TABLE_WIDE): few tables built wide (1: A/V, 2: spline)

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

// ode_spline_kernel's table, one wavefront per point (round 6): for batches of few tables (the
// CLI's single point, a sweep's shared tables), where one lane per point leaves the table build a
// serial chain of ~800 global-memory rows.  Per knot, everything but the two short recurrences is
// independent: the lanes form 64 knots' (a, b, c, r) of the slope system (and, going back, their
// PPoly coefficients) side by side; lane 0 runs only the forward elimination (den, c', d') and the
// back substitution (s_k = d'_k - c'_k s_{k+1}).  Every value is formed by the same operations on
// the same operands as in ode_spline_kernel (dx[k-1] and slope[k-1] recomputed from the knots, as
// that kernel computed them one row earlier), so the table is the same, bit for bit.
constexpr int kSplWaves = 4;  // points (wavefronts) per block
__global__ __launch_bounds__(64 * kSplWaves) void ode_spline_wave_kernel(const lzq_point* __restrict__ pts, int64_t n,
                                                                         int32_t nt, const double* __restrict__ Tlo,
                                                                         const double* __restrict__ Thi,
                                                                         double* __restrict__ ws,
                                                                         int32_t* __restrict__ status) {
  __shared__ double s_abcr[kSplWaves][4][64];
  __shared__ double s_s[kSplWaves][65];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * kSplWaves + wv;
  if (i >= n) return;  // wave-uniform
  const lzq_point pt = pts[i];
  const double T_lo = Tlo ? Tlo[i] : pt.T_min_over_Tp * pt.T_p_GeV;
  const double T_hi = Thi ? Thi[i] : pt.T_max_over_Tp * pt.T_p_GeV;
  const int N = nt;
  const int64_t ws_pt = 4 * (int64_t)N;
  const double stepT = (T_hi - T_lo) / (double)(N - 1);
  double* w = ws + i * ws_pt;
  auto X = [&](int k) { return linspace_at(T_lo, T_hi, stepT, k, N); };
  auto Yk = [&](int k) { return k < N - 1 ? w[4 * k + 3] : w[ws_pt - 1]; };
  // ode_grid_ok, its comparisons spread over the lanes
  bool ok = true;
  for (int k = 1 + lane; k < N; k += 64) ok = ok && (X(k) > X(k - 1));
  if (!__all(ok)) {
    if (lane == 0 && status) status[i] = LZQ_ODE_BAD_GRID;
    return;
  }
  auto sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  double* A = s_abcr[wv][0];
  double* Bv = s_abcr[wv][1];
  double* Cv = s_abcr[wv][2];
  double* Rv = s_abcr[wv][3];
  // first row (lane 0, as ode_spline_kernel)
  double cpm1 = 0.0, dpm1 = 0.0;
  if (lane == 0) {
    const double dxm1 = X(1) - X(0), slm1 = (Yk(1) - Yk(0)) / dxm1;
    const double dx1 = X(2) - X(1), sl1 = (Yk(2) - Yk(1)) / dx1;
    const double d = X(2) - X(0);
    const double r = ((dxm1 + 2.0 * d) * dx1 * slm1 + (dxm1 * dxm1) * sl1) / d;
    cpm1 = d / dx1;
    dpm1 = r / dx1;
    w[0] = cpm1;
    w[1] = dpm1;
  }
  // forward sweep over rows 1 .. N-2, 64 at a time
  for (int k0 = 1; k0 < N - 1; k0 += 64) {
    const int k = k0 + lane;
    if (k < N - 1) {
      const double dxm1 = X(k) - X(k - 1), slm1 = (Yk(k) - Yk(k - 1)) / dxm1;
      const double dxk = X(k + 1) - X(k), slk = (Yk(k + 1) - Yk(k)) / dxk;
      A[lane] = dxk;
      Bv[lane] = 2.0 * (dxm1 + dxk);
      Cv[lane] = dxm1;
      Rv[lane] = 3.0 * (dxk * slm1 + dxm1 * slk);
    }
    sync();
    if (lane == 0) {
      const int nk = N - 1 - k0 < 64 ? N - 1 - k0 : 64;
      for (int j = 0; j < nk; ++j) {
        const double a = A[j];
        const double den = Bv[j] - a * cpm1;
        cpm1 = Cv[j] / den;
        dpm1 = (Rv[j] - a * dpm1) / den;
        w[4 * (k0 + j) + 0] = cpm1;
        w[4 * (k0 + j) + 1] = dpm1;
      }
    }
    sync();
  }
  // last row (not-a-knot) and back substitution (lane 0), the coefficients of 64 intervals at a
  // time (all lanes)
  double s_next = 0.0;
  if (lane == 0) {
    const double dxm1 = X(N - 1) - X(N - 2), slm1 = (Yk(N - 1) - Yk(N - 2)) / dxm1;  // dx[-1], slope[-1]
    const double dx2 = X(N - 2) - X(N - 3), sl2 = (Yk(N - 2) - Yk(N - 3)) / dx2;    // dx[-2], slope[-2]
    const double d = X(N - 1) - X(N - 3);
    const double r = ((dxm1 * dxm1) * sl2 + (2.0 * d + dxm1) * dx2 * slm1) / d;
    s_next = (r - d * dpm1) / (dx2 - d * cpm1);
    s_s[wv][64] = s_next;
  }
  double* Sv = s_s[wv];
  for (int top = N - 2; top >= 0; top -= 64) {
    const int nk = top + 1 < 64 ? top + 1 : 64;  // knots top, top-1, ..., top-nk+1 (slot j: knot top - j)
    if (lane == 0) {
      // Sv[64] holds s of knot top + 1
      double sn = Sv[64];
      for (int j = 0; j < nk; ++j) {
        const int k = top - j;
        const double sk = w[4 * k + 1] - w[4 * k + 0] * sn;
        Sv[j] = sk;
        sn = sk;
      }
    }
    sync();
    if (lane < nk) {
      const int k = top - lane;
      const double sk = Sv[lane], sn = lane == 0 ? Sv[64] : Sv[lane - 1];
      const double dxk = X(k + 1) - X(k);
      const double slk = (Yk(k + 1) - w[4 * k + 3]) / dxk;
      const double t = (sk + sn - 2.0 * slk) / dxk;
      w[4 * k + 0] = t / dxk;
      w[4 * k + 1] = (slk - sk) / dxk - t;
      w[4 * k + 2] = sk;
    }
    sync();
    if (lane == 0) Sv[64] = Sv[nk - 1];
    sync();
  }
  if (lane == 0) {
    w[ws_pt - 4] = (double)N;
    if (status) status[i] = LZQ_ODE_OK;
  }
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

// kLin: the variant for linear cooperative waves (see lin_wave below); every launch runs both
// variants, each stepping only its own wavefronts (the other variant's return at once), so the
// linear waves' tight loop does not share a register allocation with the Riccati Newton path.
#ifndef LZQ_ODE_GEN_RICSTEP
#define LZQ_ODE_GEN_RICSTEP 1  // the general variant's regular Riccati steps through ric_step (round 6)
#endif
template <bool kDep>
__device__ bool ric_step(double h, const double (&hA2)[3], const double (&lam)[3], const double (&E2)[3],
                         const double (&S)[3], const double (&pv)[6], double& Ychi, double (&Zs)[3], bool guess);

// Shared stage-row tables (round 6, lzq_ode_rows): Y_B's step maps (c, d) of every step of a
// run -- points of the launch order equal in the cooperative fields, spline table and Gamma_wash
// (engine.ode_runs) -- computed once per run by ode_rows_kernel instead of once per wavefront by
// the cooperative fill.  ode_integrate_kernel<kLin> reads a run's rows for a wave only after
// checking that the wave is that one run and that the run's representative point agrees with
// every lane in all the fill reads (the cooperative fields, table, Gamma_wash, step count).
struct OdeRows {
  const int32_t* run_of;   // [n] each point's run, -1: none
  const int64_t* run_rep;  // [n_runs] a point of each run
  const int64_t* row_off;  // [n_runs + 1] the first row of each run (run r: row_off[r+1] - row_off[r] rows)
  const YbCD* rows;        // nullptr: no row tables (every wave fills its own rows)
  int64_t n_runs, cap;     // runs; rows the buffer holds
};

template <bool kChiOnly, bool kLin = false, bool kNoSplit = false>
__global__ __launch_bounds__(kOdeBlock, LZQ_ODE_MIN_WAVES) void ode_integrate_kernel(const lzq_point* __restrict__ pts,
                                                                  const lzq_ode_params* __restrict__ ode, int64_t n,
                                                                  const int32_t* __restrict__ tidx,
                                                                  const double* __restrict__ ws, int64_t max_steps,
                                                                  lzq_yield* __restrict__ out,
                                                                  int32_t* __restrict__ status, int coop_on,
                                                                  int64_t k_lo, int64_t k_cnt,
                                                                  OdeState* __restrict__ state,
                                                                  const int32_t* __restrict__ skip, OdeRows rws) {
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
      if (LZQ_ODE_RICVAR && !kChiOnly && G == 64 && (!tab_vary || LZQ_ODE_RICTAB) && rec_shared &&
          __all(k_split != -1))
        return;
      // and waves of narrower uniform segments, one table and one Gamma_wash each:
      // ode_riccati_kernel<., false, true> (LZQ_ODE_RICSEG)
      if (LZQ_ODE_RICVAR && LZQ_ODE_RICSEG && !kChiOnly && G > 0 && G < 64 && !tab_vary && rec_shared &&
          __all(k_split != -1))
        return;
    }
    // Row tables (OdeRows): a whole linear wave of one run, no depletion (its rows would need the
    // stage a_j too), whose run's representative agrees with every lane in the fill's inputs --
    // the cooperative fields, table and Gamma_wash, bit for bit, and the step count -- reads the
    // run's rows instead of filling its own (the same values: ode_rows_kernel's operations are the
    // fill's).  Regular steps off the tight loop (after a split) then form their stages per lane.
    const YbCD* rrow = nullptr;
    if (kLin && LZQ_ODE_ROWS && rws.rows && G == 64) {
      const int32_t ru = rws.run_of[i];
      if (__all(ru >= 0 && (int64_t)ru < rws.n_runs && ru == __shfl(ru, 0, 64) && !o.deplete)) {
        const int64_t rep = rws.run_rep[ru], r0 = rws.row_off[ru], r1 = rws.row_off[ru + 1];
        bool ok = rep >= 0 && rep < n && r0 >= 0 && r1 - r0 == N && r1 <= rws.cap;
        if (__all(ok)) {
          const OdePoint q = ode_point(pts[rep], ode[rep]);
          auto eqb = [](double a, double b) {
            return __builtin_bit_cast(uint64_t, a) == __builtin_bit_cast(uint64_t, b);
          };
          ok = eqb(q.m, o.m) && eqb(q.Tp, o.Tp) && eqb(q.B, o.B) && eqb(q.sig, o.sig) && eqb(q.H0, o.H0) &&
               eqb(q.s0, o.s0) && eqb(q.c_rel, o.c_rel) && eqb(q.c_nr, o.c_nr) && eqb(q.v0, o.v0) &&
               eqb(q.T_lo, o.T_lo) && eqb(q.T_hi, o.T_hi) && eqb(q.gamma_w, o.gamma_w) &&
               (tidx ? tidx[rep] == tidx[i] : rep == i);
          if (__all(ok)) rrow = rws.rows + r0;
        }
      }
    }
    // Row-table waves stage their run's rows in their wave's s_base slot (unused by them: their
    // stages are per lane off the tight loop), kOdeRowBlk rows per block in two buffers: block
    // i + 1's rows are fetched straight into LDS (global_load_lds, 16 B per lane, no registers)
    // while block i steps, so the global latency is off the step chain.
    // (LZQ_ODE_ROWS_ASYNC = 0: one buffer of twice the rows, staged through registers, 4 loads in flight)
    constexpr int kOdeRowBlk = LZQ_ODE_ROWS_ASYNC ? LZQ_ODE_ROWS_BLOCK : 2 * LZQ_ODE_ROWS_BLOCK;
    static_assert(sizeof(s_base[0]) >= (LZQ_ODE_ROWS_ASYNC ? 2 : 1) * kOdeRowBlk * sizeof(YbCD),
                  "row buffers exceed the s_base slot");
    static_assert(kOdeRowBlk % 64 == 0, "row blocks are whole wavefront fetches");
    YbCD* const s_rows = reinterpret_cast<YbCD*>(&s_base[wv][0][0]);
    const bool rowblk = kLin && LZQ_ODE_ROWS && rrow;
    const int64_t block = rowblk ? kOdeRowBlk : (coop ? G : N);
    // rows kf .. kf + kOdeRowBlk - 1 (those < k_stop) into dst; lane l's row of each 64 lands at dst + 64 j + l
    auto fetch_rows = [&](int64_t kf, YbCD* dst) {
#pragma unroll
      for (int j = 0; j < kOdeRowBlk / 64; ++j)
        if (kf + 64 * j + lane < k_stop)
          __builtin_amdgcn_global_load_lds(rrow + kf + 64 * j + lane, dst + 64 * j, 16, 0, 0);
    };
    if (LZQ_ODE_ROWS_ASYNC && rowblk) fetch_rows(k_begin, s_rows);
    YbCD* s_cur = s_rows;  // row-table waves: this block's buffer
    for (int64_t kb = k_begin; kb < k_stop; kb += block) {
      const int64_t kend = kb + block < k_stop ? kb + block : k_stop;
      if (rowblk && !LZQ_ODE_ROWS_ASYNC) {
        // groups of LZQ_ODE_ROWS_COPY loads, all issued before the group's first store (the empty
        // asm consumes the whole group; guarded per row, the compiler waited on each load before
        // its store); rows past the run's end read its last row, into LDS slots no step reads
#pragma unroll
        for (int g = 0; g < kOdeRowBlk / 64; g += LZQ_ODE_ROWS_COPY) {
          YbCD t[LZQ_ODE_ROWS_COPY];
#pragma unroll
          for (int j = 0; j < LZQ_ODE_ROWS_COPY; ++j) {
            const int64_t kr = kb + lane + 64 * (g + j);
            t[j] = rrow[kr < k_stop ? kr : k_stop - 1];
          }
#pragma unroll
          for (int j = 0; j < LZQ_ODE_ROWS_COPY; ++j) asm volatile("" : "+v"(t[j].c), "+v"(t[j].d));
#pragma unroll
          for (int j = 0; j < LZQ_ODE_ROWS_COPY; ++j) s_rows[lane + 64 * (g + j)] = t[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else if (rowblk) {
        s_cur = s_rows + (((kb - k_begin) / kOdeRowBlk) & 1) * kOdeRowBlk;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this block's rows have landed in LDS
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the next block's rows into the other buffer (its last reader was the previous block, whose
        // steps ended at that block's closing wave barrier)
        if (kb + kOdeRowBlk < k_stop) fetch_rows(kb + kOdeRowBlk, s_rows + kOdeRowBlk - (s_cur - s_rows));
      } else if (coop) {
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
            const YbCD* rr = rowblk ? &s_cur[k - kb] : &s_rcd[LZQ_ODE_YBREC && !kChiOnly ? wv : 0][r0];
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
              // issued before the chain of fmas needs the first (reading the next batch ahead of
              // the current one's fmas measured the same, profiles/round6/ablate_ode_lin_pipe.json)
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
          if (coop && !split && !rowblk) {  // (row tables: no stage bases in LDS)
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
            if (rowblk && !split) {
              r = s_cur[k - kb];
            } else if (rec_shared && !split) {
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
            if (LZQ_ODE_GEN_RICSTEP && !split) {  // the same operations through ric_step (see there)
              double lam[3], E2[3], S[3];
#pragma unroll
              for (int j = 0; j < 3; ++j) {
                lam[j] = sg[j].lam;
                E2[j] = sg[j].E2;
                S[j] = sg[j].S;
              }
              const double hA2[3] = {hA.a[2][0], hA.a[2][1], hA.a[2][2]};
              const double pv[6] = {kRadauAinvP[1], kRadauAinvP[2], kRadauAinvP[3],
                                    kRadauAinvP[5], kRadauAinvP[6], kRadauAinvP[7]};
              ok = ric_step<true>(h, hA2, lam, E2, S, pv, Ychi, Zs, use_guess);
            } else {
              ok = radau_step<false>(split ? radau_h(R, hs) : hA, sg, Ychi, YB, Zs, use_guess);
            }
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

// Row r of run q (lzq_ode_rows): Y_B's step map of step r of the run's representative point, with
// the cooperative fill's operations (ode_integrate_kernel above: x_k, the stage bases, beta_j =
// Gamma_wash * base, yb_rec with the step's hA; h from the run's step count as the integrator
// forms it).  One lane per row; runs over blockIdx.y, grid-strided.
__global__ __launch_bounds__(kOdeBlock) void ode_rows_kernel(const lzq_point* __restrict__ pts,
                                                             const lzq_ode_params* __restrict__ ode, int64_t n,
                                                             const int32_t* __restrict__ tidx,
                                                             const double* __restrict__ ws,
                                                             const int64_t* __restrict__ run_rep,
                                                             const int64_t* __restrict__ row_off, int64_t n_runs,
                                                             YbCD* __restrict__ rows, int64_t cap) {
  const int64_t k = (int64_t)blockIdx.x * kOdeBlock + threadIdx.x;
  for (int64_t q = blockIdx.y; q < n_runs; q += gridDim.y) {
    const int64_t r0 = row_off[q], N = row_off[q + 1] - r0, i = run_rep[q];
    if (k >= N || i < 0 || i >= n || r0 < 0 || r0 + k >= cap) continue;
    const OdePoint o = ode_point(pts[i], ode[i]);
    const double* w = ws + (tidx ? (int64_t)tidx[i] : i) * (int64_t)kOdeWS;
    const double m = o.m;
    const double x0 = m / o.T_hi, x1 = m / pymax(o.T_lo, 1e-30);
    const double h = (x1 - x0) / (double)N;
    const Radau R = radau_tableau();
    const RadauH hA = radau_h(R, h);
    const double xk = x0 + (double)k * h;
    double beta[3], a[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const StageBase b = ode_stage_base(o, w, xk + R.c[j] * h);
      beta[j] = o.gamma_w * b.beta;
      a[j] = b.a;
    }
    const YbRec yr = yb_rec(hA, beta, a);
    rows[r0 + k] = {yr.c, yr.d};
  }
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

struct RicRow {
  double lam[3], E2[3], a[3];  // StageBase lam, E2, a of the step's three stages
};

#ifndef LZQ_RIC_KRELOAD
#define LZQ_RIC_KRELOAD 1  // ode_riccati_kernel's lean loop reloads the predictor constants per step (SGPR room)
#endif
#ifndef LZQ_RIC_TAB_MIN_WAVES
#define LZQ_RIC_TAB_MIN_WAVES 3  // its rows take 38 KB of LDS per 4-wave block: 3 blocks per CU
#endif
#ifndef LZQ_RIC_IP
#define LZQ_RIC_IP 2  // ode_riccati_kernel's lean steps through ric_step_ip (round 6; see there); 2: have / Yp outside the joins
#endif
#ifndef LZQ_RIC_KPTR
#define LZQ_RIC_KPTR 1  // the predictor table's address hoisted out of the step loop (see there)
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

// ode_riccati_kernel<., kTab = true> (LZQ_ODE_RICTAB, round 6): whole waves whose points agree in
// everything but the A/V kernel (I_p, v_w: a spline table each), the table-varying waves the
// general variant stepped.  A row then holds what every lane shares -- lam, E2, the spline location
// (s, k) and a / Av (ap) of each stage, and the Y_B step map's c, W, id (which do not depend on a)
// -- and each lane forms a_j = Av(own table; s_j, k_j) * ap_j and d = yb_d(W, a) itself: the
// general variant's row_a / stage_scale / yb_d on the same values, so the same bits.
struct RicRowT {
  double lam[3], E2[3], ap[3], s[3];
  double W[3], id, c;
  int k[3];
};

__device__ __noinline__ void ric_fill_tab(const OdePoint* ou, const double* __restrict__ wu, double xk, double h,
                                          RicRowT* row, double* bt) {
  const Radau R = radau_tableau();
#pragma unroll 1
  for (int j = 0; j < 3; ++j) {
    const double cj = j == 0 ? R.c[0] : (j == 1 ? R.c[1] : R.c[2]);
    const StageBase bs = ode_stage_base(*ou, wu, xk + cj * h);
    row->lam[j] = bs.lam;
    row->E2[j] = bs.E2;
    row->ap[j] = bs.ap;
    row->s[j] = bs.s;
    row->k[j] = bs.k;
    bt[j] = ou->gamma_w * bs.beta;
  }
  const double beta[3] = {bt[0], bt[1], bt[2]}, none[3] = {0.0, 0.0, 0.0};  // d is each lane's
  const YbRec yr = yb_rec(radau_h(R, h), beta, none);
  row->W[0] = yr.W[0];
  row->W[1] = yr.W[1];
  row->W[2] = yr.W[2];
  row->id = yr.id;
  row->c = yr.c;
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

// ric_step with the iterate kept in Zs itself (LZQ_RIC_IP): the start is guess ? g : Y0 (g: the
// predictor's or block_guess's stages), Newton updates Zs in place, and on success Ychi = Zs[2] --
// the values ric_step leaves in Zs and Ychi.  A failed step leaves Zs holding the last iterate
// where ric_step kept g, but its lane is done (no later step or saved state reads Zs), so every
// value that is read is the same.  The linear branch takes g as ric_step's Zs = g did.
template <bool kDep>
__device__ __forceinline__ bool ric_step_ip(double h, const double (&hA2)[3], const double (&lam)[3],
                                            const double (&E2)[3], const double (&S)[3], const double (&pv)[6],
                                            double& Ychi, double (&Zs)[3], const double (&g)[3], bool guess) {
  const bool nonlinear = lam[0] != 0.0 || lam[1] != 0.0 || lam[2] != 0.0;
  if (!nonlinear) {
#pragma unroll
    for (int j = 0; j < 3; ++j) Zs[j] = g[j];
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
    Zs[j] = guess ? g[j] : Y0;
  }
  RicJ J;
  bool near = false;
  const bool c1 = ric_newton<kDep>(Zs, Y0, hl, hl2, hS, E2, pv, J, false, near);
  const bool reuse = near;
  const bool c2 = ric_newton<kDep>(Zs, Y0, hl, hl2, hS, E2, pv, J, reuse, near);
  bool ok = c1 || c2;
  if (!ok) {
#pragma nounroll
    for (int it = 2; it < 40 && !ok; ++it) ok = ric_newton<kDep>(Zs, Y0, hl, hl2, hS, E2, pv, J, false, near);
    if (!ok && guess) {
      Zs[0] = Y0;
      Zs[1] = Y0;
      Zs[2] = Y0;
#pragma nounroll
      for (int it = 0; it < 40 && !ok; ++it) ok = ric_newton<kDep>(Zs, Y0, hl, hl2, hS, E2, pv, J, false, near);
    }
  }
  if (ok) Ychi = Zs[2];
  return ok;
}

// kPhase: a wave whose split step (the T = m/3 branch) lies in this launch's range runs in three
// passes -- 0: the regular steps before it, 1: the split step and the next (ode_integrate_kernel's
// split-step code, each lane forming its own stages: two steps, so registers do not matter),
// 2: the regular steps after it -- with its state handed on in OdeState; so the regular-step
// kernels (0, 2) carry no split code.  A wave with no split in range runs in pass 0 alone.
template <int kPhase, bool kTab = false, bool kSeg = false>
__global__ __launch_bounds__(kOdeBlock, kPhase == 1 ? 1 : (kTab || kSeg ? LZQ_RIC_TAB_MIN_WAVES : LZQ_RIC_MIN_WAVES)) void
ode_riccati_kernel(const lzq_point* __restrict__ pts, const lzq_ode_params* __restrict__ ode, int64_t n,
                   const int32_t* __restrict__ tidx, const double* __restrict__ ws, int64_t max_steps,
                   lzq_yield* __restrict__ out, int32_t* __restrict__ status, int coop_on, int64_t k_lo, int64_t k_cnt,
                   OdeState* __restrict__ state, const int32_t* __restrict__ skip) {
  __shared__ RicRow s_row[kOdeBlock / 64][kTab ? 1 : 64];
  __shared__ YbCD s_rcd[kOdeBlock / 64][kTab ? 1 : 64];
  __shared__ RicRowT s_rowt[kOdeBlock / 64][kTab ? 64 : 1];
  __shared__ OdePoint s_pt[kOdeBlock / 64][kSeg ? 64 / LZQ_ODE_MIN_GROUP : 1];  // kSeg: one per segment
  __shared__ double s_beta[kOdeBlock / 64][64][3];  // the fill's beta_j (Gamma_wash * base)
  static_assert(!kSeg || !kTab, "segment waves: one table per segment");

  if (!LZQ_ODE_RICVAR || !LZQ_ODE_COOP || !coop_on) return;
  if (kSeg && !LZQ_ODE_RICSEG) return;
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
  const double* w = ws + (tidx ? (int64_t)tidx[i] : i) * (int64_t)kOdeWS;
  // Two of the wave-uniform exits below, taken first (before the point's constants, ~40 us per
  // 2.6e5 points in each of this kernel's launches): a linear wave (sigma_v = 0 on every lane:
  // ode_integrate_kernel<kLin>'s) and, for whole waves, one of the other table class.  Evaluated on
  // the lanes still here; with one missing the ballot below returns anyway, so neither exits a wave
  // this kernel would step.
  if (LZQ_ODE_LINFAST && __all(pymax(ode[i].sigma_v_chi_GeV_m2, 0.0) == 0.0)) return;
  if (!kSeg) {
    const uint64_t wb = (uint64_t)(uintptr_t)w;
    if (__all(wb == __builtin_bit_cast(uint64_t, __shfl(__builtin_bit_cast(double, wb), 0, 64))) == kTab) return;
  }
  const lzq_point pt = pts[i];
  const OdePoint o = ode_point(pt, ode[i]);
  if (!ode_grid_ok(o.T_lo, o.T_hi, o.stepT) || !ode_table_ok(w)) return;  // the general variant reports it
  const double m = o.m, T_p = o.Tp;
  const double x0 = m / o.T_hi, x1 = m / pymax(o.T_lo, 1e-30);
  const double x_p = m / pymax(T_p, 1e-30);
  const double max_step = pymin(pymin(fabs(x1 - x0) / 20000.0, x_p / 1000.0), 5e-4);
  if (!(max_step > 0.0)) return;
  const double steps = ceil(fabs(x1 - x0) / max_step);
  if (!(steps <= (double)max_steps)) return;
  if (__ballot(1) != ~0ull) return;  // a lane returned above: not a whole cooperative wave
  // G: the widest aligned segments (64, 32, 16, 8 lanes) that are each uniform in the stage key --
  // ode_integrate_kernel's cooperative width, found the same way; this kernel takes G = 64 (kSeg
  // false) or 8 <= G < 64 (kSeg), on one table and one Gamma_wash per segment
  int G = 0;
  for (int g = 64; g >= LZQ_ODE_MIN_GROUP && G == 0; g >>= 1) {
    auto same_g = [g](double v) {
      return __builtin_bit_cast(uint64_t, v) == __builtin_bit_cast(uint64_t, __shfl(v, 0, g));
    };
    const bool eq = same_g(o.m) && same_g(o.Tp) && same_g(o.B) && same_g(o.sig) && same_g(o.H0) && same_g(o.s0) &&
                    same_g(o.c_rel) && same_g(o.c_nr) && same_g(o.v0) && same_g(o.T_lo) && same_g(o.T_hi);
    if (__all(eq)) G = g;
    if (!kSeg) break;  // only G = 64 is this variant's
  }
  if (kSeg ? !(G > 0 && G < 64) : G != 64) return;
  auto same = [G](double v) { return __builtin_bit_cast(uint64_t, v) == __builtin_bit_cast(uint64_t, __shfl(v, 0, G)); };
  if (__all(same(__builtin_bit_cast(double, w))) == kTab) return;            // tab_vary: the kTab kernel's
  if (kTab && !LZQ_ODE_RICTAB) return;
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
  // (kSeg: the segment's own, per lane; so are the passes' ranges below, and a segment with no split
  // step in range leaves passes 1 and 2 at once)
  const int64_t ks = kSeg ? k_split : (int64_t)__builtin_bit_cast(uint64_t, ode_uniform(__builtin_bit_cast(double, k_split)));
  const double xbu = kSeg ? xb : ode_uniform(xb), xb_below = nextafter(xbu, -INFINITY);
  // this pass's steps [pk_begin, pk_stop)
  const bool in_range = ks != INT64_MAX && !(ks + 1 < k_begin || ks >= k_stop);
  if (kPhase > 0 && !in_range) return;
  const int64_t ks_lo = ks > k_begin ? ks : k_begin, ks_hi = ks + 2 < k_stop ? ks + 2 : k_stop;
  const int64_t pk_begin = kPhase == 0 ? k_begin : (kPhase == 1 ? ks_lo : ks_hi);
  const int64_t pk_stop = kPhase == 0 ? (in_range ? ks_lo : k_stop) : (kPhase == 1 ? ks_hi : k_stop);
  // --- this wave is ours: the wave-uniform point constants in the wave's LDS slot (read by the
  // fill phase only), the window, h, hA and the table pointer in SGPRs ---
  // (kSeg: per segment -- the segment's point in its LDS slot; the window, h, hA and the table each
  // lane's own, which equal its segment leader's bit for bit, in VGPRs)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int seg = kSeg ? (lane & ~(G - 1)) : 0;  // the segment's first lane: its rows are seg .. seg + G - 1
  if (lane == seg) s_pt[wv][kSeg ? seg / G : 0] = o;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const OdePoint& ou = s_pt[wv][kSeg ? seg / G : 0];
  const double* wu = kSeg ? w : reinterpret_cast<const double*>(
      (uintptr_t)__builtin_bit_cast(uint64_t, ode_uniform(__builtin_bit_cast(double, (uint64_t)(uintptr_t)w))));
  const double x0u = kSeg ? x0 : ode_uniform(x0), hu = kSeg ? h : ode_uniform(h);
  const Radau R = radau_tableau();
  RadauH hA = radau_h(R, hu);
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) hA.a[a][b] = kSeg ? hA.a[a][b] : ode_uniform(hA.a[a][b]);
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
          const StageBase b = ode_stage_base(ou, kTab ? w : wu, xs + R.c[j] * hs);
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
  int kc = -1;                             // kTab: the spline interval held in cc
  double cc[4] = {0.0, 0.0, 0.0, 0.0};
  // (kSeg: blocks of G steps; k_begin, hence kb, is the same on every lane, each segment's range
  // ends at its own pk_stop -- a segment past it takes no steps while the others run on)
  const int64_t blk = kSeg ? (int64_t)G : 64;
  for (int64_t kb = pk_begin; kPhase != 1 && (kSeg ? __any(kb < pk_stop) : kb < pk_stop); kb += blk) {
    const int64_t kend = kb + blk < pk_stop ? kb + blk : pk_stop;
    uint64_t xok = 0;
    {  // lane l: the stage ingredients and Y_B step map of step kb + l (the cooperative fill)
      const int64_t kl = kb + (lane - seg);
      if (LZQ_RIC_LEAN) {
        // the steps' x guard (xk + h > xk, wave-uniform per step) as one mask, from the fill's xk
        const double xk = x0u + (double)kl * hu;
        xok = __ballot(kl < kend && xk + hu > xk);
      }
      if (kl < kend) {
        if (kTab) {
          ric_fill_tab(&ou, wu, x0u + (double)kl * hu, hu, &s_rowt[wv][lane], s_beta[wv][lane]);
        } else if (LZQ_RIC_LEAN) {
          ric_fill(&ou, wu, x0u + (double)kl * hu, hu, &s_row[wv][lane], s_beta[wv][lane], &s_rcd[wv][lane]);
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
    // LZQ_RIC_KPTR: the predictor table's address formed once per block of steps (two SGPRs), so a
    // step's reload is the constants' own scalar loads, not a GOT load and then them
    const __attribute__((address_space(4))) double* kp_loop =
        (const __attribute__((address_space(4))) double*)&kRadauPred[0][0];
    if (LZQ_RIC_KPTR) asm volatile("" : "+s"(kp_loop));  // opaque: not re-formed in the loop
    // a wave with no depleting lane runs the loop without the source products (ric_step<false>)
    auto lean_steps = [&](auto dep_tag) {
    constexpr bool kDep = decltype(dep_tag)::value;
    // LZQ_RIC_V4: a uniform trip count, each lane's steps under !done (a lane whose Newton iteration
    // failed stops there, as in the loop below)
    const int nr = kend > kb ? (int)(kend - kb) : 0;  // kSeg: this segment's steps in the block
    if (LZQ_RIC_IP || kTab || kSeg) {
      // the same steps with the loop-carried values written once each (ric_step_ip): the predictor
      // and block_guess fill g, the iterate lives in Zs, Y_B is committed only on success and the
      // status once after the loop (a lane done here failed here) -- the loop below copied Y_chi,
      // Y_B, the stages and the status between registers at every step's joins
      const bool done0 = done;
      const int nr_loop = kSeg ? G : nr;  // a uniform trip count (kSeg: a segment past its nr skips)
      for (int r = 0; r < nr_loop; ++r) {
        const RicRow row = s_row[wv][kTab ? 0 : seg + r];
        const YbCD rc = s_rcd[wv][kTab ? 0 : seg + r];
        if (done || (kSeg && r >= nr)) continue;
        bool use_guess = false;
        double g[3] = {Zs[0], Zs[1], Zs[2]};  // Zs as it stands unless a guess replaces it
        // a lane that is not done has taken steps 0 .. r - 1 of this block, so have = have || r > 0
        if (riccati && (LZQ_RIC_IP < 2 || r > 0 || have) && (LZQ_RIC_IP >= 2 || have) && r != rz) {
          const __attribute__((address_space(4))) double* kp = kp_loop;
          if (LZQ_RIC_KRELOAD) asm volatile("" : "+s"(kp));
          use_guess = true;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            g[j] = fma_s(Zs[2], kp[4 * j + 3], fma_s(Zs[1], kp[4 * j + 2], fma_s(Zs[0], kp[4 * j + 1], kp[4 * j] * Yp)));
            use_guess = use_guess && fabs(g[j] - Ychi) <= 0.25 * fabs(Ychi);
          }
        }
        const double Ystart = Ychi;
        if (LZQ_RIC_IP >= 2) Yp = Ystart;  // the predictor has read the previous one
        bool ok = true;
        if ((xok >> (seg + r)) & 1) {
          double lam[3], E2[3], S[3];
          double YBn;
          if constexpr (kTab) {
            // this lane's a_j from its own table at the row's (shared) spline location: the interval's
            // four coefficients are reloaded only when k changes (wave-uniform; spline_at's
            // operations on the same values), d from the row's W, id
            const RicRowT& rw = s_rowt[wv][r];
            double a[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const int kj = __builtin_amdgcn_readfirstlane(rw.k[j]);
              if (kj != kc) {
                kc = kj;
#pragma unroll
                for (int q = 0; q < 4; ++q) cc[q] = w[4 * kj + q];
              }
              a[j] = spline_cubic(cc, rw.s[j]) * rw.ap[j];
              S[j] = kDep ? (deplete ? Pf * a[j] : 0.0) : 0.0;
              lam[j] = sigmav * rw.lam[j];
              E2[j] = rw.E2[j];
            }
            const double d = yb_d(YbW{{rw.W[0], rw.W[1], rw.W[2]}, rw.id}, a);
            YBn = __builtin_fma(rw.c, YB, Pf * d);
          } else {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              S[j] = kDep ? (deplete ? Pf * row.a[j] : 0.0) : 0.0;
              lam[j] = sigmav * row.lam[j];
              E2[j] = row.E2[j];
            }
            YBn = __builtin_fma(rc.c, YB, Pf * rc.d);
          }
          if (riccati && r == rz) {
            OdeStage sg[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              sg[j].lam = lam[j];
              sg[j].E2 = E2[j];
              sg[j].S = S[j];
            }
            use_guess = block_guess(R, hu, sg, Ychi, g);
          }
          ok = ric_step_ip<kDep>(hu, hA2, lam, E2, S, pv, Ychi, Zs, g, use_guess);
          if (ok) YB = YBn;
        } else {
#pragma unroll
          for (int j = 0; j < 3; ++j) Zs[j] = g[j];
        }
        if (LZQ_RIC_IP < 2) {
          have = true;
          Yp = Ystart;
        }
        done = !ok;
      }
      if (LZQ_RIC_IP >= 2 && nr > 0 && !done0) have = true;
      if (done && !done0) st = LZQ_ODE_NEWTON;
      return;
    }
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
        const __attribute__((address_space(4))) double* kp = LZQ_RIC_KPTR ? kp_loop
            : (const __attribute__((address_space(4))) double*)&kRadauPred[0][0];
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
// lzq_ode_tables: up to this many tables take ode_spline_wave_kernel (a wavefront each); more, one
// lane each (ode_spline_kernel: the serial chains of 64 tables share a wavefront's issue)
constexpr int64_t kSplineWaveMax = 4096;

int hip_check(hipError_t e, const char* what);

// The fixed-step integration of a batch as continuation launches of <= 2^g_ode_launch_log2
// steps each (lzq_tune(LZQ_TUNE_ODE_LAUNCH_STEPS)): ceil(max_steps / 2^log2) launches, every
// point advancing through steps [j 2^log2, (j+1) 2^log2) of its own sequence in launch j and
// finishing in the launch that reaches its N (points done early return at once).  One launch
// when max_steps fits.  The per-point state (64 B) is stream-ordered scratch (hipMallocAsync).
template <bool kChiOnly>
int launch_integrate(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const int32_t* d_tidx,
                     const double* d_work, int64_t max_steps, lzq_yield* d_out, int32_t* d_status, hipStream_t s,
                     const char* fn, const int32_t* d_skip = nullptr, const lzq::OdeRows* rows = nullptr) {
  const int64_t per = (int64_t)1 << lzq::g_ode_launch_log2;
  const lzq::OdeRows rw = rows ? *rows : lzq::OdeRows{nullptr, nullptr, nullptr, nullptr, 0, 0};
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
                       st, d_skip, rw);
    int rc = hip_check(hipGetLastError(), fn);
    if constexpr (LZQ_ODE_NOSPLITVAR) {
      if (rc != LZQ_OK) return rc;
      hipLaunchKernelGGL((lzq::ode_integrate_kernel<kChiOnly, false, true>), dim3((unsigned)ode_blocks(n)),
                         dim3(lzq::kOdeBlock), 0, s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status,
                         lzq::g_ode_coop, k_lo, k_cnt, st, d_skip, rw);
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
        // the table-varying waves' three passes (none for one point: its wave is clones of it)
        if (LZQ_ODE_RICTAB && n > 1) {
          if (rc != LZQ_OK) return rc;
          hipLaunchKernelGGL((lzq::ode_riccati_kernel<0, true>), dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0,
                             s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, lzq::g_ode_coop, k_lo,
                             k_cnt, st, d_skip);
          rc = hip_check(hipGetLastError(), fn);
          if (rc != LZQ_OK) return rc;
          hipLaunchKernelGGL((lzq::ode_riccati_kernel<1, true>), dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0,
                             s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, lzq::g_ode_coop, k_lo,
                             k_cnt, st, d_skip);
          rc = hip_check(hipGetLastError(), fn);
          if (rc != LZQ_OK) return rc;
          hipLaunchKernelGGL((lzq::ode_riccati_kernel<2, true>), dim3((unsigned)ode_blocks(n)), dim3(lzq::kOdeBlock), 0,
                             s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, lzq::g_ode_coop, k_lo,
                             k_cnt, st, d_skip);
          rc = hip_check(hipGetLastError(), fn);
        }
        if (LZQ_ODE_RICSEG && n > 1) {  // uniform 32/16/8-lane segments (a one-point wave is one whole segment)
          if (rc != LZQ_OK) return rc;
          hipLaunchKernelGGL((lzq::ode_riccati_kernel<0, false, true>), dim3((unsigned)ode_blocks(n)),
                             dim3(lzq::kOdeBlock), 0, s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status,
                             lzq::g_ode_coop, k_lo, k_cnt, st, d_skip);
          rc = hip_check(hipGetLastError(), fn);
          if (rc != LZQ_OK) return rc;
          hipLaunchKernelGGL((lzq::ode_riccati_kernel<1, false, true>), dim3((unsigned)ode_blocks(n)),
                             dim3(lzq::kOdeBlock), 0, s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status,
                             lzq::g_ode_coop, k_lo, k_cnt, st, d_skip);
          rc = hip_check(hipGetLastError(), fn);
          if (rc != LZQ_OK) return rc;
          hipLaunchKernelGGL((lzq::ode_riccati_kernel<2, false, true>), dim3((unsigned)ode_blocks(n)),
                             dim3(lzq::kOdeBlock), 0, s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status,
                             lzq::g_ode_coop, k_lo, k_cnt, st, d_skip);
          rc = hip_check(hipGetLastError(), fn);
        }
      }
    }
    if constexpr (LZQ_ODE_LINFAST && LZQ_ODE_YBREC && !kChiOnly) {
      if (rc != LZQ_OK) return rc;
      hipLaunchKernelGGL((lzq::ode_integrate_kernel<kChiOnly, true>), dim3((unsigned)ode_blocks(n)),
                         dim3(lzq::kOdeBlock), 0, s, d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status,
                         lzq::g_ode_coop, k_lo, k_cnt, st, d_skip, rw);
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

int lzq_ode_launch_sequential(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                              const int32_t* d_tidx, const double* d_work, int64_t max_steps, lzq_yield* d_out,
                              int32_t* d_status, hipStream_t s, const char* fn, const int32_t* d_skip) {
  return launch_integrate<false>(d_points, d_ode, n, d_tidx, d_work, max_steps, d_out, d_status, s, fn, d_skip);
}
int lzq_ode_hip_check(hipError_t e, const char* what) { return hip_check(e, what); }
int lzq_ode_check_ws(int64_t n, const double* d_work, int64_t work_doubles, const char* fn, int64_t per_table) {
  return check_ws(n, d_work, work_doubles, fn, per_table);
}

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
  if (n <= kSplineWaveMax && (lzq::g_ode_table_wide & 2))  // few tables: a wavefront per table (same bits)
    hipLaunchKernelGGL(lzq::ode_spline_wave_kernel, dim3((unsigned)((n + lzq::kSplWaves - 1) / lzq::kSplWaves)),
                       dim3(64 * lzq::kSplWaves), 0, s, d_points, n, nt, d_T_lo, d_T_hi, d_work, d_status);
  else
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

int lzq_ode_rows(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const int32_t* d_table_index,
                 int64_t n_tables, const double* d_work, int64_t work_doubles, const int64_t* d_run_rep,
                 const int64_t* d_row_off, int64_t n_runs, int64_t max_run_rows, double* d_rows,
                 int64_t rows_doubles, void* stream) {
  if (n < 0 || n_tables < 0 || n_runs < 0 || max_run_rows < 0 || rows_doubles < 0 ||
      (n_runs > 0 && (!d_points || !d_ode || !d_run_rep || !d_row_off || !d_rows || n == 0)) ||
      (d_table_index && n > 0 && n_tables == 0))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_rows: bad arguments");
  int rc = check_ws(d_table_index ? n_tables : n, d_work, work_doubles, "lzq_ode_rows");
  if (rc) return rc;
  if (n_runs == 0 || max_run_rows == 0) return LZQ_OK;
  const int64_t bx = (max_run_rows + lzq::kOdeBlock - 1) / lzq::kOdeBlock;
  if (bx > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_ode_rows: max_run_rows too large");
  const unsigned by = (unsigned)(n_runs < 65535 ? n_runs : 65535);  // runs beyond: grid-strided
  hipLaunchKernelGGL(lzq::ode_rows_kernel, dim3((unsigned)bx, by), dim3(lzq::kOdeBlock), 0, (hipStream_t)stream,
                     d_points, d_ode, n, d_table_index, d_work, d_run_rep, d_row_off, n_runs, (lzq::YbCD*)d_rows,
                     rows_doubles / 2);
  return hip_check(hipGetLastError(), "lzq_ode_rows");
}

int lzq_ode_integrate_rows(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                           const int32_t* d_table_index, int64_t n_tables, const double* d_work,
                           int64_t work_doubles, int64_t max_steps, const int32_t* d_run_of,
                           const int64_t* d_run_rep, const int64_t* d_row_off, int64_t n_runs,
                           const double* d_rows, int64_t rows_doubles, lzq_yield* d_out, int32_t* d_status,
                           void* stream) {
  if (n < 0 || n_tables < 0 || n_runs < 0 || rows_doubles < 0 ||
      (n > 0 && (!d_points || !d_ode || !d_out || !d_table_index || n_tables == 0)) ||
      (n_runs > 0 && (!d_run_of || !d_run_rep || !d_row_off || !d_rows)))
    return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate_rows: bad arguments");
  int rc = check_ws(n_tables, d_work, work_doubles, "lzq_ode_integrate_rows");
  if (rc) return rc;
  if (max_steps < 0) return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate_rows: max_steps < 0");
  if (ode_blocks(n) > 2147483647LL) return lzq_set_error(LZQ_EINVAL, "lzq_ode_integrate_rows: n too large");
  if (n == 0) return LZQ_OK;
  const lzq::OdeRows rows{d_run_of, d_run_rep, d_row_off, n_runs > 0 ? (const lzq::YbCD*)d_rows : nullptr, n_runs,
                          rows_doubles / 2};
  return launch_integrate<false>(d_points, d_ode, n, d_table_index, d_work, max_steps, d_out, d_status,
                                 (hipStream_t)stream, "lzq_ode_integrate_rows", nullptr, &rows);
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
