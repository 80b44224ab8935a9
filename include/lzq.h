/*
 * lzq.h -- C ABI of the MI355X-native bounce-sourced Landau-Zener yield engine.
 *
 * Drop-in boundary for the hot path of /root/reference/first_principles_yields.py ("fpy"):
 *
 *   fpy:141-165  AoverVKernel(..., z_max, nz) / A_over_V_y -> lzq_aov_batch (any z grid: nz, z_max)
 *   fpy:231-267  integrate_YB_by_quadrature           -> lzq_yields_batch (out->Y_B), lzq_sweep_grid
 *   fpy:372-384, fpy:413-417  Y_chi + densities        -> lzq_yields_batch / lzq_sweep_grid epilogue
 *   fpy:170-187  LZ plug-in closed form (fpy:183-184)  -> lzq_p_closed_form
 *   fpy:222-223 + fpy:122-123  J_chi (diagnostics)     -> lzq_jchi_batch
 *   (no reference counterpart; north_star (1))        -> lzq_lz_propagate
 *   fpy:200-219, 270-286, 385-417  ODE fallback        -> lzq_ode_tables / _integrate / _batch,
 *                                                         lzq_ode_integrate_shared, lzq_ode_quadrature,
 *                                                         lzq_ode_aov_T, lzq_ode_rhs
 *
 * Conventions (all entry points):
 *   - plain C types only; device buffers are raw device pointers, `stream` is a hipStream_t
 *     passed as void* (NULL = the null stream) and must belong to the current HIP device;
 *   - the caller owns every buffer; the library never frees caller memory; launches are
 *     asynchronous on `stream` (no host synchronisation inside the launch functions once
 *     lzq_init has run for the device);
 *   - return 0 on success, a negative LZQ_E* code on failure; lzq_last_error() returns a
 *     thread-local message for the last failure on the calling thread; no C++ exception
 *     crosses the boundary;
 *   - results are deterministic: each point is reduced by one wavefront in a fixed order, so
 *     they do not depend on launch geometry, batch composition or the number of GPUs.
 */
#ifndef LZQ_H
#define LZQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LZQ_ABI_VERSION 3   /* 3: optional lzq_aov_params on the A/V-evaluating entry points */
#define LZQ_NZ 1200          /* fpy:142 nz default, used unchanged at fpy:197 */
#define LZQ_Z_MAX 30.0       /* fpy:142 z_max default */
#define LZQ_NZ_MAX (1 << 22) /* largest z grid accepted (64 MB of device nodes) */
#define LZQ_NY_MAIN 8000     /* fpy:374 */
#define LZQ_NY_MIN 2000      /* fpy:246 */

enum lzq_status {
  LZQ_OK = 0,
  LZQ_EINVAL = -1,       /* bad argument (null pointer, n < 0, unknown field, ...)        */
  LZQ_EHIP = -2,         /* a HIP runtime call failed (message has the HIP error string)  */
  LZQ_EUNSUPPORTED = -3, /* configuration outside the fast quadrature path (fpy:372)       */
  LZQ_ENODEVICE = -4
};

/* chi statistics (fpy:96: str(stats).lower().startswith("ferm")) */
enum lzq_stats { LZQ_FERMION = 0, LZQ_BOSON = 1 };
/* regime (fpy:376-384); LZQ_REGIME_OTHER ("auto") has no branch in the reference, which
 * raises UnboundLocalError; the engine returns NaN yields for such points. */
enum lzq_regime { LZQ_THERMAL = 0, LZQ_NONTHERMAL = 1, LZQ_REGIME_OTHER = 2 };

/* One parameter point: the fpy `Config` fields (fpy:44-79) read by the fast path.
 * Optional[float] fields carry has_* flags.  136 bytes, 8-byte aligned. */
typedef struct lzq_point {
  double m_chi_GeV;            /* field  0 */
  double g_chi;                /* field  1 (int in fpy; used as a float factor) */
  double T_p_GeV;              /* field  2 */
  double beta_over_H;          /* field  3 */
  double v_w;                  /* field  4 */
  double I_p;                  /* field  5 */
  double g_star;               /* field  6 */
  double g_star_s;             /* field  7 */
  double P_chi_to_B;           /* field  8 */
  double source_shape_sigma_y; /* field  9 */
  double incident_flux_scale;  /* field 10 */
  double T_max_over_Tp;        /* field 11 */
  double T_min_over_Tp;        /* field 12 */
  double Y_chi_init;           /* field 13 (valid iff has_Y_chi_init) */
  double n_chi_at_Tp_GeV3;     /* field 14 (valid iff has_n_chi_at_Tp) */
  int32_t stats;               /* enum lzq_stats  */
  int32_t regime;              /* enum lzq_regime */
  int32_t has_Y_chi_init;
  int32_t has_n_chi_at_Tp;
} lzq_point;

/* The A/V kernel's own parameters: AoverVKernel(I_p, beta_over_H, T_p, v_w, g_star, z_max, nz)
 * (fpy:141-151).  BoltzmannSystem builds self.aov from cfg (fpy:197), but it is a separate public
 * object: integrate_YB_by_quadrature (fpy:261), build_tables (fpy:211) and S_B_T (fpy:228) take
 * A/V from self.aov while the y-grid, T(y), H, s, J and window come from self.cfg (fpy:234-262).
 * Entry points that take an optional lzq_aov_params block use it for the A/V constants
 * pref0 = (I_p/2)(beta/max(v_w, 1e-12)), beta = beta_over_H H_std(T_p, g_star), and c = -I_p/6
 * (fpy:146-151, 162-163); NULL = the point's own fields (self.aov built from cfg).  40 bytes. */
typedef struct lzq_aov_params {
  double I_p;          /* fpy:143 */
  double beta_over_H;  /* fpy:144 */
  double T_p_GeV;      /* fpy:145 (AoverVKernel's T_p) */
  double v_w;          /* fpy:146 (max(., 1e-12) applied) */
  double g_star;       /* fpy:147 */
} lzq_aov_params;

/* Per-point yield record: the `final` block of yields_out.json (fpy:425-427) + P_used
 * (fpy:424).  48 bytes; tables of these are what the multi-GPU all-gather moves. */
typedef struct lzq_yield {
  double Y_B, Y_chi, rho_B_kg_m3, rho_DM_kg_m3, DM_over_B, P_used;
} lzq_yield;

/* Sweep axis fields.  0..14 address the double fields of lzq_point in declaration order.
 * Derived LZ fields set P_chi_to_B through the closed form (fpy:183-184, PAPER eq.(9)):
 *   LZQ_F_DELTA_LZ           : P = clamp(1 - exp(-2 pi max(delta, 0)), 0, 1)
 *   LZQ_F_M_MIX, LZQ_F_DPRIME: delta = m_mix^2 / (2 max(v_w,1e-12) |Delta'|) (PAPER eq.(8), F = 1)
 * Axis values live in device memory. */
enum lzq_field {
  LZQ_F_M_CHI = 0, LZQ_F_G_CHI = 1, LZQ_F_T_P = 2, LZQ_F_BETA_OVER_H = 3, LZQ_F_V_W = 4,
  LZQ_F_I_P = 5, LZQ_F_G_STAR = 6, LZQ_F_G_STAR_S = 7, LZQ_F_P = 8, LZQ_F_SIGMA_Y = 9,
  LZQ_F_FLUX = 10, LZQ_F_T_MAX_OVER_TP = 11, LZQ_F_T_MIN_OVER_TP = 12, LZQ_F_Y_CHI_INIT = 13,
  LZQ_F_N_CHI_AT_TP = 14,
  LZQ_F_DELTA_LZ = 32, LZQ_F_M_MIX = 33, LZQ_F_DPRIME = 34
};

#define LZQ_MAX_AXES 8
typedef struct lzq_axis {
  int32_t field;          /* enum lzq_field */
  int32_t n;              /* number of values (> 0) */
  const double* values;   /* device pointer, n doubles */
} lzq_axis;

/* ---- library / device management ---------------------------------------------------- */
int lzq_abi_version(void);
const char* lzq_last_error(void);
/* The z grid.  Every entry point that evaluates A/V (fpy:158-165) takes the grid of the
 * reference operator AoverVKernel(I_p, beta_over_H, T_p, v_w, g_star, z_max=30.0, nz=1200)
 * (fpy:141-156) as (int32 nz, double z_max): z = linspace(0, z_max, nz), the cancelling gamma4
 * of fpy:156 verbatim, the trapezoid of fpy:164.  (LZQ_NZ, LZQ_Z_MAX) is the grid main() uses
 * (fpy:197) and runs the compile-time-sized headline kernels; any other grid is built on the
 * host and uploaded once per (device, nz, z_max) on first use (a synchronous copy), then kept.
 * 0 <= nz <= LZQ_NZ_MAX (nz < 0 is numpy's ValueError) and 0 <= z_max < inf; nz <= 1 or z_max = 0
 * give A/V = 0 exactly, as numpy's trapezoid of <= 1 node / zero width does.  Refused with
 * LZQ_EINVAL although numpy accepts them (documented parity gaps):
 *   - z_max < 0: linspace(0, z_max, nz) runs backwards and the trapezoid of fpy:164 changes sign;
 *   - a grid so fine that the cancelling gamma4 of fpy:156 rounds below 0 (the reference then
 *     exponentiates positive arguments) or stops being non-decreasing (rounding noise of a few ulp
 *     of 6.0 at the first nodes): z_1 below ~1e-3, i.e. nz >~ 2e4 on [0, 1] or >~ 1e5 on [0, 30]. */
/* Builds and uploads the default z tables (fpy:154-156) and the exp table for `device`.  Called
 * lazily by every entry point; call it up front before capturing launches into a graph. */
int lzq_init(int device);
/* The same for the grid (nz, z_max) (lzq_init = lzq_zgrid_init(device, LZQ_NZ, LZQ_Z_MAX)). */
int lzq_zgrid_init(int device, int32_t nz, double z_max);
/* Host copies of the z tables of the grid (nz, z_max): z (fpy:154), gamma4 (fpy:156) and the
 * quadrature weights omega_k = z_k^2 e^{-z_k} * (trapezoid weight of node k); nz entries each
 * (any pointer may be NULL). */
int lzq_ztables(int32_t nz, double z_max, double* z, double* gamma4, double* omega);

/* Tuning knobs for ablations (process-wide, not thread-safe against concurrent launches).
 * LZQ_TUNE_EXP selects the inner-loop exponential: LZQ_EXP_TABLE (default; 2^(j/N) LDS table,
 * N = 2^LZQ_TABBITS = 8192, + degree-2 minimax polynomial in completed-square form, <= 1.73e-14 relative) or
 * LZQ_EXP_POLY11 (degree-11 minimax polynomial, 0.6 ulp).  Results agree to ~1e-14 relative.
 * Returns the previous value. */
/* LZQ_TUNE_TRUNCATE (0 = dense, the default; 1 = on): stop each wave's z-sum at the first
 * node beyond which every lane's term is below 2^-1080, where it can no longer change the
 * FP64 accumulator.  Results are bit-identical to the dense sum; fewer nodes are executed.
 * The headline benchmark is dense and reports this mode separately. */
/* LZQ_TUNE_ODE_COOP (1 = on, the default; 0 = off): the ODE integrator's cooperative mode,
 * where a full wavefront of points that differ only in P, flux, sigma_v, Gamma_wash, deplete
 * and the initial state evaluates each step's stage ingredients once for the whole wavefront.
 * Results are bit-identical either way (tests/test_gpu_ode.py). */
/* LZQ_TUNE_ODE_LAUNCH_STEPS (value = log2 of the steps per launch, 6..40; default 24): the ODE
 * integrator runs a batch as continuation launches of at most 2^value fixed Radau steps each,
 * ceil(max_steps / 2^value) launches (<= 65536), the per-point state carried between them in
 * stream-ordered scratch (64 B per point), so any window the reference accepts completes in
 * bounded launches.  Results are bit-identical for every value (tests/test_gpu_ode.py). */
/* LZQ_TUNE_PROFILE_FLAT (1 = on; 0 = off, the default): lzq_lz_propagate_profile's flattened
 * propagation (the step rule for all of a point's knot intervals ahead of the propagation, then one
 * loop of Magnus steps per lane, a lane entering its next interval while the others step) or the
 * interval-by-interval loop in keyed launch order (measured faster).  P is
 * bit-identical either way (tests/test_gpu_profile.py). */
/* LZQ_TUNE_ODE_TP_INTERVAL (steps, a multiple of 64 in [64, 2^20]; default 64): the interval length of
 * lzq_ode_integrate_tp's multiple shooting (longer for a point whose window would need over 65536
 * intervals). */
/* LZQ_TUNE_ODE_TABLE_WIDE (bit mask, default 3 = both; 0 = off): lzq_ode_tables for few tables
 * (<= 4096) spreads each table wide -- bit 0: the A/V knots over 64-knot wavefronts instead of one
 * wavefront per table; bit 1: the spline's per-knot work over a wavefront's lanes around its two
 * recurrences instead of one lane per table.  The tables are bit-identical either way
 * (tests/test_gpu_ode_tp.py). */
enum lzq_tune_key { LZQ_TUNE_EXP = 0, LZQ_TUNE_TRUNCATE = 1, LZQ_TUNE_ODE_COOP = 2, LZQ_TUNE_ODE_LAUNCH_STEPS = 3,
                    LZQ_TUNE_PROFILE_FLAT = 4, LZQ_TUNE_ODE_TP_INTERVAL = 5, LZQ_TUNE_ODE_TABLE_WIDE = 6 };
enum lzq_exp_variant { LZQ_EXP_POLY11 = 0, LZQ_EXP_TABLE = 1 };
int lzq_tune(int32_t key, int32_t value);

/* ---- hot path -------------------------------------------------------------------------- */
/* fpy:158-165: out[i] = A_over_V_y(y[i]) for the kernel AoverVKernel(I_p, beta_over_H, T_p, v_w,
 * g_star, z_max, nz): aov (host struct) if non-NULL, else point *pt's fields (pt may then be NULL
 * only if aov is not; no other field of *pt is read). */
int lzq_aov_batch(const lzq_point* pt, const lzq_aov_params* aov, const double* d_y, int64_t n, int32_t nz,
                  double z_max, double* d_out, void* stream);

/* fpy:222-223: out[i] = BoltzmannSystem.J_chi(T[i]) for point *pt (diagnostics table). */
int lzq_jchi_batch(const lzq_point* pt, const double* d_T, int64_t n, double* d_out, void* stream);

/* fpy:231-267 + fpy:372-384 + fpy:413-417 for n explicit points (device AoS array).
 * d_T_lo / d_T_hi: optional per-point integration range (NULL: main()'s
 * T_lo = T_min_over_Tp*T_p, T_hi = T_max_over_Tp*T_p, fpy:367-369).
 * d_P: optional per-point P override (NULL: point.P_chi_to_B), e.g. lzq_lz_propagate output.
 * n_y: y-grid size as passed to integrate_YB_by_quadrature (fpy:374 uses 8000; raised to
 * LZQ_NY_MIN as fpy:246).  (nz, z_max): the A/V kernel's z grid (fpy:141-142; main(): LZQ_NZ,
 * LZQ_Z_MAX).  d_aov: optional [n] device lzq_aov_params, point i's A/V kernel (bs.aov replaced,
 * fpy:261); NULL = each point's own fields (fpy:197), the headline kernels. */
int lzq_yields_batch(const lzq_point* d_points, int64_t n, int32_t n_y, int32_t nz, double z_max,
                     const double* d_T_lo, const double* d_T_hi, const double* d_P, const lzq_aov_params* d_aov,
                     lzq_yield* d_out, void* stream);

/* Cartesian sweep: points [start, start+count) of the grid base x axes[0] x ... x
 * axes[n_axes-1] (C order: last axis fastest), generated on device from the flat index.
 * d_P: optional [count] per-point P override (e.g. lzq_lz_propagate output for multi-crossing
 * profiles, config C5); it takes precedence over P_chi_to_B and the LZ axes. */
int lzq_sweep_grid(const lzq_point* base, const lzq_axis* axes, int32_t n_axes,
                   int64_t start, int64_t count, int32_t n_y, int32_t nz, double z_max, const double* d_P,
                   lzq_yield* d_out, void* stream);

/* lzq_sweep_grid with the z-sums shared -- a separate mode, NOT the dense headline path
 * (SURVEY §8d allows separable reuse only as such).  The z-sums F(y_j) = sum_k omega_k
 * exp(c(y_j) gamma4_k) of fpy:160-165 depend on a point only through I_p, beta_over_H, T_p_GeV,
 * T_min_over_Tp, T_max_over_Tp (its y-grid and c, fpy:141-156, 234-247) and n_y: they are
 * computed once per combination of the grid's values of those fields (each table = the dense
 * kernel's passes for the combination's first grid point, into d_work), then every point of
 * [start, start+count) is integrated from its table.  Yields are bit-identical to
 * lzq_sweep_grid (same operations, same lane order).  d_work: >= lzq_sweep_grid_reuse_workspace
 * doubles (tables x (max(n_y, LZQ_NY_MIN) + LZQ_REUSE_TABLE_HEADER)); a negative return is an
 * error code.  A table's header records the y grid, c and the z grid (nz, z_max) it was made
 * for: a point integrated from a table of another setup or z grid gets NaN yields. */
#define LZQ_REUSE_TABLE_HEADER 6
int64_t lzq_sweep_grid_reuse_workspace(const lzq_axis* axes, int32_t n_axes, int32_t n_y);
/* The same for n explicit points: d_rep[n_tables] (int64) names one point per table, whose
 * I_p, beta_over_H, T_p_GeV, T_min_over_Tp, T_max_over_Tp the table is made for;
 * d_table_index[n] (int32) gives each point's table.  main()'s window only (no T_lo/T_hi
 * overrides).  d_work >= n_tables * (max(n_y, LZQ_NY_MIN) + LZQ_REUSE_TABLE_HEADER) doubles.  A point
 * whose y-grid or c differs from its table's gets NaN yields.  Bit-identical to lzq_yields_batch. */
int lzq_yields_batch_reuse(const lzq_point* d_points, int64_t n, int32_t n_y, int32_t nz, double z_max,
                           const double* d_P, const int64_t* d_rep, const int32_t* d_table_index, int64_t n_tables,
                           double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream);
int lzq_sweep_grid_reuse(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start, int64_t count,
                         int32_t n_y, int32_t nz, double z_max, const double* d_P, double* d_work,
                         int64_t work_doubles, lzq_yield* d_out, void* stream);

/* lzq_sweep_grid_reuse in two halves, so a sweep evaluated in chunks (or shards) builds its
 * z-sum tables once: lzq_sweep_grid_ztables writes every table of the grid into d_work (the
 * whole grid's, independent of any range); lzq_sweep_grid_from_ztables integrates points
 * [start, start+count) from tables built by it for the same base, axes and n_y (and exponential
 * variant).  Together they are lzq_sweep_grid_reuse, bit for bit. */
int lzq_sweep_grid_ztables(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int32_t n_y, int32_t nz,
                           double z_max, double* d_work, int64_t work_doubles, void* stream);
int lzq_sweep_grid_from_ztables(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start,
                                int64_t count, int32_t n_y, int32_t nz, double z_max, const double* d_P,
                                const double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream);

/* fpy:183-184: P[i] = clamp(1 - exp(-2 pi max(lambda[i], 0)), 0, 1) (naive 1-exp kept). */
int lzq_p_closed_form(const double* d_lambda, int64_t n, double* d_P, void* stream);

/* ---- ODE fallback (fpy:200-219, 270-286, 385-417) -------------------------------------- */
/* Configurations with sigma_v != 0, Gamma_wash != 0 or depletion leave the fast path
 * (fpy:372) for the reference's Boltzmann ODE.  These three Config fields ride next to the
 * lzq_point of each point. */
typedef struct lzq_ode_params {
  double sigma_v_chi_GeV_m2;       /* fpy:279 (max(., 0) applied) */
  double Gamma_wash_over_H;        /* fpy:284 (max(., 0) applied) */
  int32_t deplete_DM_from_source;  /* fpy:282 */
  int32_t reserved;                /* 0 */
} lzq_ode_params;                  /* 24 bytes */

#define LZQ_ODE_NT 800             /* fpy:207 build_tables(n=800), the n main() uses (fpy:387) */
#define LZQ_ODE_WS_PER_POINT 3200  /* workspace doubles per point (spline coefficients): 4 x LZQ_ODE_NT */
#define LZQ_ODE_NT_MAX (1 << 20)   /* largest build_tables n accepted */
enum lzq_ode_status {
  LZQ_ODE_OK = 0,
  LZQ_ODE_BAD_GRID = 1,       /* T grid not strictly increasing: CubicSpline raises ValueError */
  LZQ_ODE_BAD_STEP = 2,       /* max_step <= 0 (zero-width x range): solve_ivp raises ValueError */
  LZQ_ODE_TOO_MANY_STEPS = 3, /* more than max_steps integration steps: not attempted */
  LZQ_ODE_NOT_LINEAR = 5,     /* internal to lzq_ode_quadrature: Y_chi still to be stepped */
  LZQ_ODE_BAD_TABLE = 7,      /* the point's spline table was not built by lzq_ode_tables with
                                 nt = LZQ_ODE_NT (the integrators' knot count; NaN yields) */
  LZQ_ODE_UNRESOLVED = 6,     /* lzq_ode_quadrature: a knot interval needs more than 4096
                                 Gauss sub-intervals to resolve its scales (NaN yields) */
  LZQ_ODE_NEWTON = 4          /* a Radau stage system did not converge: the yields are the
                                 state at the start of the failed step (fpy:408-410 reports
                                 sol.y[:, -1] after a failed solve) */
};

/* BoltzmannSystem.build_tables(T_lo, T_hi, n=nt) (fpy:207-212) with self.aov = AoverVKernel(...,
 * z_max, nz) for n points, at per-point windows d_T_lo/d_T_hi ([n] each) or, both NULL, main()'s
 * window T_lo = T_min_over_Tp T_p, T_hi = T_max_over_Tp T_p (fpy:368-369, what lzq_ode_integrate
 * needs): A/V at linspace(T_lo, T_hi, nt) (the quadrature kernels' z-sum on the grid (nz, z_max))
 * and its not-a-knot cubic spline (scipy CubicSpline), into d_work[i * 4 nt ...] (work_doubles >=
 * n * 4 nt; 4 <= nt <= LZQ_ODE_NT_MAX).  The integrators (lzq_ode_integrate*, lzq_ode_quadrature)
 * read tables of nt = LZQ_ODE_NT knots, main()'s build_tables (fpy:387), on any z grid: a table
 * records its nt in its last 4 (spare) doubles, and a point whose table holds another nt gets
 * LZQ_ODE_BAD_TABLE (NaN yields) from them.
 * d_status (optional, [n] int32): LZQ_ODE_BAD_GRID for a window CubicSpline rejects.  d_aov:
 * optional [n] device lzq_aov_params, the A/V kernel of each point's table (bs.aov replaced:
 * y(T) from the point, A/V from the block, fpy:211); NULL = the point's own fields. */
int lzq_ode_tables(const lzq_point* d_points, int64_t n, const double* d_T_lo, const double* d_T_hi, int32_t nt,
                   int32_t nz, double z_max, const lzq_aov_params* d_aov, double* d_work, int64_t work_doubles,
                   int32_t* d_status, void* stream);

/* fpy:385-417 on built tables: Y_chi(x1), Y_B(x1) of rhs (fpy:270-286) from x0 = m/T_hi to
 * x1 = m/max(T_lo, 1e-30), Y(x0) = (Y_chi0 of fpy:389-399, 0), by the reference's method
 * (3-stage Radau IIA) on uniform steps h = (x1 - x0)/ceil(|x1 - x0|/max_step) <= max_step of
 * fpy:404, one point per lane; then the densities epilogue.  The steps run as continuation
 * launches of <= 2^24 steps (LZQ_TUNE_ODE_LAUNCH_STEPS), so max_steps only caps the work: points
 * needing more than max_steps steps are not integrated (status LZQ_ODE_TOO_MANY_STEPS, NaN
 * yields; max_steps <= 65536 x the launch size); so are
 * points whose T grid CubicSpline would reject (LZQ_ODE_BAD_GRID).  A Newton failure
 * (LZQ_ODE_NEWTON) stops the point and reports the state reached.  d_status: optional [n]
 * int32 output (enum lzq_ode_status). */
int lzq_ode_integrate(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const double* d_work,
                      int64_t work_doubles, int64_t max_steps, lzq_yield* d_out, int32_t* d_status,
                      void* stream);

/* lzq_ode_integrate with tables shared between points: point i reads the spline table at
 * d_work[d_table_index[i] * LZQ_ODE_WS_PER_POINT] (0 <= d_table_index[i] < n_tables, the
 * caller's contract; work_doubles >= n_tables * LZQ_ODE_WS_PER_POINT).  A table depends only
 * on the A/V kernel and the window of fpy:141-156, 207-212 -- (I_p, beta_over_H, T_p_GeV, v_w,
 * g_star, T_min_over_Tp, T_max_over_Tp) -- so points equal in those fields (a sweep over P,
 * flux, sigma_v, Gamma_wash, m_chi, ...) share one lzq_ode_tables row; the results are
 * bit-identical to lzq_ode_integrate with per-point tables. */
int lzq_ode_integrate_shared(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                             const int32_t* d_table_index, int64_t n_tables, const double* d_work,
                             int64_t work_doubles, int64_t max_steps, lzq_yield* d_out, int32_t* d_status,
                             void* stream);

/* Shared step-row tables for linear sweeps (sigma_v = 0, no depletion; round 6; no reference
 * counterpart -- a re-use of fpy:270-286's per-step quantities across points).  A run is a set
 * of points equal in everything Y_B's Radau step map reads but P and the flux: the stage fields
 * of the A/V spline, m_chi, g_chi, g_star_s, source_shape_sigma_y, stats, the table and
 * Gamma_wash.  lzq_ode_rows writes run q's N_q step maps (c, d: Y_B' = c Y_B + P flux d, 16 B a
 * step) from its representative point d_run_rep[q] into d_rows (as doubles) from row
 * d_row_off[q] on, N_q = d_row_off[q + 1] - d_row_off[q] = the point's step count (ceil(|x1 -
 * x0| / max_step), fpy:403-404); max_run_rows >= every N_q; rows past rows_doubles / 2 are not
 * written.  lzq_ode_integrate_rows is lzq_ode_integrate_shared whose linear wavefronts read their
 * run's rows (d_run_of[i]: point i's run, -1 none) instead of forming their own -- only after
 * checking, per wavefront, that it is one run whose representative equals each point in all the
 * rows depend on, bit for bit, and whose row count is the point's step count (otherwise, and for
 * every other wavefront, lzq_ode_integrate_shared's path).  Results are bit-identical to
 * lzq_ode_integrate_shared. */
int lzq_ode_rows(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, const int32_t* d_table_index,
                 int64_t n_tables, const double* d_work, int64_t work_doubles, const int64_t* d_run_rep,
                 const int64_t* d_row_off, int64_t n_runs, int64_t max_run_rows, double* d_rows,
                 int64_t rows_doubles, void* stream);
int lzq_ode_integrate_rows(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                           const int32_t* d_table_index, int64_t n_tables, const double* d_work,
                           int64_t work_doubles, int64_t max_steps, const int32_t* d_run_of,
                           const int64_t* d_run_rep, const int64_t* d_row_off, int64_t n_runs,
                           const double* d_rows, int64_t rows_doubles, lzq_yield* d_out, int32_t* d_status,
                           void* stream);

/* lzq_ode_integrate / lzq_ode_integrate_shared (d_table_index NULL: table i for point i) for a
 * FEW points on long windows -- the CLI's single point -- integrated parallel in time: each
 * point's N fixed steps are cut into intervals of LZQ_TUNE_ODE_TP_INTERVAL steps, every interval
 * is integrated from a guess of its start state on its own lane (the same per-step operations),
 * and Newton's method on the interval boundaries (multiple shooting; the corrections by a scan of
 * the intervals' linearised maps) iterates the guesses to within a few ulps of the sequential
 * trajectory; then every interval is integrated from the candidate starts around its converged
 * node and the exact chains are followed through those tables from the exact initial state (no
 * integrator uses the predictor on the first step of a 64-step block, so an interval's end is a
 * function of its start values alone).  A point's latency drops from N serial steps to (a few
 * iterations + the candidate pass) x (one interval), and its result is lzq_ode_integrate's, BIT FOR
 * BIT (tests/test_gpu_ode_tp.py).  A point whose iteration does not converge to 1e-14 within 32
 * updates, whose exact chain leaves the candidate windows (+-256 ulps), or whose status is not OK,
 * takes the sequential integration (the same bits again, at the sequential cost); so does every
 * point of a batch of more than 64.  d_iters (optional, [n] int32): the Newton updates of a point
 * that was stitched; 0: not iterated, -k: iterated k updates, then integrated sequentially.
 * Blocks nothing: the iteration count is fixed (32 rounds of two launches; a converged point's
 * later launches return at once), so the call is stream-ordered like lzq_ode_integrate.
 * Scratch (stream-ordered, hipMallocAsync, freed by the call): with L = LZQ_TUNE_ODE_TP_INTERVAL
 * and M = min(ceil(max_steps / L), 65536) intervals per point, about n M (72 + 32 (2J + 1)) bytes
 * for the nodes, ends, scans and the two chains' candidate tables, J = 256 when those fit 1 GiB
 * (else 32), plus n M L 88 bytes of the regular steps' stage rows when they fit 2 GiB (else the
 * stages are formed inline).  max_steps only sizes it: pass the batch's longest step count
 * (Engine.ode does), not a generous cap -- e.g. n = 64 with max_steps = 2^22 asks ~4.7 GB. */
int lzq_ode_integrate_tp(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                         const int32_t* d_table_index, int64_t n_tables, const double* d_work, int64_t work_doubles,
                         int64_t max_steps, lzq_yield* d_out, int32_t* d_status, int32_t* d_iters, void* stream);

/* Quadrature form of the fallback (opt-in; not the reference's method).  Y_B's equation of
 * fpy:270-286 is linear with integrating factor (x/x1)^Gamma_wash for every sigma_v, so
 * Y_B(x1) = int alpha(x) (x/x1)^Gamma_wash dx, alpha = (SB/s)/(H x), exactly; with
 * sigma_v = 0 so is Y_chi's: Y_chi(x1) = Y_chi(x0) - [deplete] int alpha(x) dx.  Both are
 * integrated over the built spline tables (knot intervals split at T = m/3 and into
 * sub-intervals below the window / integrating-factor / Boltzmann scales, 8-point
 * Gauss-Legendre), one wavefront per point: the converged solution of the reference's
 * equations (the reference's own rtol-1e-8 Radau sits up to ~2e-8 from it on wide windows).
 * For sigma_v != 0 points Y_chi's Riccati equation is then stepped alone by the Radau
 * integrator (max_steps as lzq_ode_integrate; without a source term its stages need neither
 * the spline nor the window).  d_table_index: optional shared tables as in
 * lzq_ode_integrate_shared (NULL: table i for point i). */
int lzq_ode_quadrature(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n,
                       const int32_t* d_table_index, int64_t n_tables, const double* d_work, int64_t work_doubles,
                       int64_t max_steps, lzq_yield* d_out, int32_t* d_status, void* stream);

/* lzq_ode_tables (nt = LZQ_ODE_NT, main()'s window, the z grid (nz, z_max), d_aov as there) +
 * lzq_ode_integrate (d_status may be NULL). */
int lzq_ode_batch(const lzq_point* d_points, const lzq_ode_params* d_ode, int64_t n, int32_t nz, double z_max,
                  const lzq_aov_params* d_aov, double* d_work, int64_t work_doubles, int64_t max_steps,
                  lzq_yield* d_out, int32_t* d_status, void* stream);

/* BoltzmannSystem.A_over_V_T (fpy:214-218) and .rhs (fpy:270-286) of ONE point (host structs)
 * whose nt-knot tables for the window (T_lo, T_hi) are at d_work_point (4 nt doubles, from
 * lzq_ode_tables): out_Av[i] = A_over_V_T(T[i]); out_dY[2i..2i+1] = rhs(x[i], (Y[2i], Y[2i+1])). */
int lzq_ode_aov_T(const lzq_point* pt, double T_lo, double T_hi, int32_t nt, const double* d_work_point,
                  const double* d_T, int64_t n, double* d_out_Av, void* stream);
int lzq_ode_rhs(const lzq_point* pt, const lzq_ode_params* ode, double T_lo, double T_hi, int32_t nt,
                const double* d_work_point, const double* d_x, const double* d_Y, int64_t n, double* d_out_dY,
                void* stream);

/* ---- Landau-Zener propagator (north_star (1); no reference counterpart) --------------- */
/* Coherent two-level propagation through n_cross sequential linear avoided crossings per
 * point: i dpsi/dt = H(t) psi, H = [[D(xi), m_c],[m_c, -D(xi)]], xi = v_w t, D piecewise linear
 * with slope (-1)^c |Delta'_c| through crossing c at xi_c (continuous at the turning points
 * between crossings).  The outer half-windows are window_lz LZ lengths of the first/last
 * crossing (L = sqrt(v_w/|Delta'|) max(1, sqrt(delta))).  Each cell with delta <= 16 takes
 * max(steps_per_crossing, 6 x the adiabatic phase in radians of its core) eighth-order Magnus
 * steps (exact SU(2) exponentials) on a core around its crossing (~5-7 LZ lengths: out to where
 * the first neglected angle of the order-10 superadiabatic frame falls to 1e-11) and follows the
 * state in that frame outside it, so the step count is bounded for any crossing spacing; cells
 * with delta > 16 are propagated in closed form.  Arrays are [n][n_cross] row-major device
 * buffers (xi increasing per point).  0 < window_lz <= 200, 0 < steps_per_crossing <= 1e6 (else
 * LZQ_EINVAL); a point whose inputs are not finite gets P = NaN.  Output d_P[n]: conversion
 * probability 1 - |<chi-like dressed state | psi_end>|^2, psi_start = chi-like dressed state,
 * where "dressed" = second-order superadiabatic state of the outer cell (the adiabatic state
 * carried in from / out to infinity).  For one crossing this is 1 - exp(-2 pi delta)
 * (fpy:183-184, PAPER eq.(9)) to <= 1e-8 relative at window_lz = 20 for any steps_per_crossing;
 * DESIGN.md §4.4 states the window / step tolerances (the C5 default is steps_per_crossing = 64).
 * Scratch from hipMallocAsync on `stream`, freed stream-ordered: 80 bytes per (point, crossing)
 * for the follow matrices (lz_follow_kernel; batches beyond 2^23 pairs run in slices) and, for
 * n >= 16384 points, 8n bytes for the longest-first launch order (points binned by their step
 * count, a counting sort in three small kernels); d_P is bit-identical to index order.
 * n < 2^31. */
int lzq_lz_propagate(const double* d_m_mix, const double* d_dprime, const double* d_xi,
                     int64_t n, int32_t n_cross, double v_w, double window_lz,
                     int32_t steps_per_crossing, double* d_P, void* stream);

/* lzq_lz_propagate with a per-point wall speed d_v_w[n] (sweeps over v_w with crossings); a
 * point whose v_w is not > 0 gets P = NaN. */
int lzq_lz_propagate_v(const double* d_m_mix, const double* d_dprime, const double* d_xi, const double* d_v_w,
                       int64_t n, int32_t n_cross, double window_lz, int32_t steps_per_crossing, double* d_P,
                       void* stream);

/* ---- bounce-profile LZ path (PAPER p.3 §3 eqs.(5)-(9); the absent modules of fpy:173) ---- */
/* The reference's hook (fpy:170-187) imports `transport_from_profile` and calls
 * compute_prob_from_profile(csv, v_w) / compute_lambda_eff_from_profile(csv) (fpy:178-184);
 * that module is absent from the reference, so these entry points implement the paper's
 * definition of it.  A profile SHAPE is the bounce's two background fields phi(xi), Phi(xi)
 * on n_knots knots xi_0 < ... < xi_{n_knots-1} (xi = r - R_0), each a not-a-knot cubic spline
 * (scipy CubicSpline, the interpolant fpy:212 uses).  Coefficient rows: d_coef[shape][j][8] =
 * (phi c0..c3, Phi c0..c3) with value c0 + c1 t + c2 t^2 + c3 t^3, t = xi - xi_j on
 * [xi_j, xi_{j+1}].  A POINT is a shape plus the couplings of eqs.(5)-(8):
 *   Delta = y_B phi - y_chi Phi (eq.5), Delta'* (eq.6), m_mix = lambda_tr_eff phi (eq.7),
 *   delta_LZ = m_mix(xi*)^2 / (2 v_w |Delta'*|) (eq.8, F = 1), P = 1 - exp(-2 pi delta) (eq.9). */
typedef struct lzq_profile_point {
  double y_B;            /* eq.(5) */
  double y_chi;          /* eq.(5) */
  double lambda_tr_eff;  /* eq.(7) */
  double v_w;            /* eq.(8); the propagation's xi = v_w t */
  int32_t shape;         /* 0 <= shape < n_shapes (else: NaN P / count -1) */
  int32_t reserved;      /* 0 */
} lzq_profile_point;     /* 40 bytes */

/* The not-a-knot splines of n_shapes shapes: d_knots/d_phi/d_Phi [n_shapes][n_knots] (device),
 * n_knots >= 4, into d_coef [n_shapes][n_knots-1][8].  d_bad[n_shapes] (int32): 1 for a shape
 * whose knots are not strictly increasing (CubicSpline raises ValueError; its rows are not
 * written), else 0. */
int lzq_profile_splines(const double* d_knots, const double* d_phi, const double* d_Phi, int32_t n_shapes,
                        int32_t n_knots, double* d_coef, int32_t* d_bad, void* stream);

/* eqs.(5)-(8) per point: every sign change of Delta in [xi_0, xi_{n_knots-1}) (a cubic per knot
 * interval, split at its stationary points; each root by safeguarded Newton to full precision).
 * Up to max_cross crossings per point, in increasing xi, into d_xi / d_dprime (signed Delta'*) /
 * d_m_mix / d_delta_lz [n][max_cross]; d_count[n] = the number found (which may exceed
 * max_cross: the rest are not written; -1 for a bad shape index). */
int lzq_profile_crossings(const double* d_knots, const double* d_coef, int32_t n_shapes, int32_t n_knots,
                          const lzq_profile_point* d_points, int64_t n, int32_t max_cross, double* d_xi,
                          double* d_dprime, double* d_m_mix, double* d_delta_lz, int32_t* d_count, void* stream);

/* Time-ordered propagation through the whole profile (beyond the minimal estimator of eq.(8):
 * the crossings' energy dependence and their interference are kept): i dpsi/dt = H psi,
 * H = Delta(xi) sigma_z + m_mix(xi) sigma_x, xi = v_w t, from xi_0 to xi_{n_knots-1}.  psi starts
 * in the chi-like second-order dressed (superadiabatic) state of H at xi_0; d_P[n] =
 * 1 - |<chi-like dressed state at the far end | psi>|^2.  Sixth-order Magnus (three
 * Gauss-Legendre nodes, exact SU(2) exponentials), on knot interval j
 * max(min_steps, ceil(steps_per_radian x duration x max(E, 4 sqrt|dH/dt|))) uniform steps.
 * 0.5 <= steps_per_radian <= 1000 and 1 <= min_steps <= 1e6 (else LZQ_EINVAL); a point with
 * v_w <= 0, a bad shape index or more than 2^24 steps in one interval gets P = NaN.  For one
 * linear crossing in a wide window P -> eq.(9).  Accuracy: the error falls as
 * steps_per_radian^-6; at 3 it is within 9.2e-10 of the exact (Weber) solutions of
 * lzq_lz_propagate's piecewise-linear model and up to ~1e-8 on coarse smooth profiles, at 4 (the
 * package default) <= ~1e-9. 
 * n < 2^31. */
int lzq_lz_propagate_profile(const double* d_knots, const double* d_coef, int32_t n_shapes, int32_t n_knots,
                             const lzq_profile_point* d_points, int64_t n, double steps_per_radian,
                             int32_t min_steps, double* d_P, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LZQ_H */
