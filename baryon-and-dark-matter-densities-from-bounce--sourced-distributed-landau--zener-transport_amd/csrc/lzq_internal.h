// lzq_internal.h -- declarations shared between the library's translation units (not ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lzq.h"

namespace lzq {

constexpr int kOdeNT = LZQ_ODE_NT;           // fpy:207 build_tables(n=800)
constexpr int kOdeWS = LZQ_ODE_WS_PER_POINT;  // workspace doubles per point

// Per-point workspace layout (doubles): w[4k + 0..3] = PPoly c0..c3 of interval k < 799
// (value c0 s^3 + c1 s^2 + c2 s + c3, s = T - T_k); w[kOdeWS - 1] holds A/V at the last knot
// while the spline is built.

// A/V at the nt T-knots of every point (z grid (nz, z_max)) into w[4k + 3] / w[4 nt - 1] of its
// 4 nt doubles (lzq_kernels.hip: the quadrature kernels' z-sum, one wavefront per point).
// Host-side launch; sets lzq_last_error.
// d_aov (optional, [n]): the A/V kernel's own parameters per point (lzq_aov.hip).
int launch_ode_aov_tables(const lzq_point* d_points, int64_t n, const double* d_T_lo, const double* d_T_hi,
                          int32_t nt, int32_t nz, double z_max, const lzq_aov_params* d_aov, double* d_work,
                          hipStream_t stream);

// lzq_aov.hip: the quadrature / build_tables kernels with the A/V constants of a per-point
// lzq_aov_params block (fpy:141-151, 197, 211, 261), on a resolved z grid (zt, nzp; default_grid:
// the compile-time LZQ_NZ kernels) and exp table gtab.  Set lzq_last_error on failure.
struct ZNode;  // lzq_quad.h
int launch_yields_points_aov(int exp_variant, bool default_grid, const lzq_point* d_points,
                             const lzq_aov_params* d_aov, int64_t n, int32_t n_y, const double* d_T_lo,
                             const double* d_T_hi, const double* d_P, const ZNode* zt, int32_t nzp, const double* gtab,
                             lzq_yield* d_out, int truncate, hipStream_t s);
int launch_ode_aov_tables_aov(int exp_variant, const lzq_point* d_points, const lzq_aov_params* d_aov, int64_t n,
                              int32_t nt, const ZNode* zt, int32_t nzp, const double* gtab, const double* d_T_lo,
                              const double* d_T_hi, double* d_work, int truncate, hipStream_t s, int chunks = 1);

// Longest-first launch order (lzq_propagator.hip): cost bins per point (0 = costliest, kCostBins
// of them) and their histogram -> offs (kCostBins scratch) and order[n] (a counting sort: one
// scan, one scatter; stable across bins, atomics order within one).  Sets lzq_last_error.
constexpr int kCostBins = 128;  // 4 bins per octave of a point's step count
int launch_bin_order(const int32_t* bins, const int32_t* hist, int32_t* offs, int64_t n, int32_t* order,
                     hipStream_t st);

// lzq_tune(LZQ_TUNE_ODE_COOP) / (LZQ_TUNE_ODE_LAUNCH_STEPS) state, read by lzq_ode.hip's launches
extern int g_ode_coop;
extern int g_ode_launch_log2;
extern int g_ode_tp_interval;  // lzq_tune(LZQ_TUNE_ODE_TP_INTERVAL): steps per lzq_ode_integrate_tp interval
extern int g_ode_table_wide;   // lzq_tune(LZQ_TUNE_ODE_TABLE_WIDE): few ODE tables built a wavefront wide
// lzq_tune(LZQ_TUNE_PROFILE_FLAT) state, read by lzq_profile.hip's launch
extern int g_profile_flat;

}  // namespace lzq

// lzq_kernels.hip's error plumbing (thread-local message behind lzq_last_error)
int lzq_set_error(int code, const char* msg);
