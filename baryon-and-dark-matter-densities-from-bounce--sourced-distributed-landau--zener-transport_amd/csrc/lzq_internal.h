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
int launch_ode_aov_tables(const lzq_point* d_points, int64_t n, const double* d_T_lo, const double* d_T_hi,
                          int32_t nt, int32_t nz, double z_max, double* d_work, hipStream_t stream);

// Longest-first launch order (lzq_propagator.hip): cost bins per point (0 = costliest, kCostBins
// of them) and their histogram -> offs (kCostBins scratch) and order[n] (a counting sort: one
// scan, one scatter; stable across bins, atomics order within one).  Sets lzq_last_error.
constexpr int kCostBins = 128;  // 4 bins per octave of a point's step count
int launch_bin_order(const int32_t* bins, const int32_t* hist, int32_t* offs, int64_t n, int32_t* order,
                     hipStream_t st);

// lzq_tune(LZQ_TUNE_ODE_COOP) / (LZQ_TUNE_ODE_LAUNCH_STEPS) state, read by lzq_ode.hip's launches
extern int g_ode_coop;
extern int g_ode_launch_log2;
// lzq_tune(LZQ_TUNE_PROFILE_FLAT) state, read by lzq_profile.hip's launch
extern int g_profile_flat;

}  // namespace lzq

// lzq_kernels.hip's error plumbing (thread-local message behind lzq_last_error)
int lzq_set_error(int code, const char* msg);
