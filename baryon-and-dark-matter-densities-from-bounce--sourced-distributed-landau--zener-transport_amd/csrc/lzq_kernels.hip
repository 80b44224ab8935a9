// lzq_kernels.hip -- CDNA4 (gfx950) kernels + C ABI of the bounce-sourced LZ yield engine.
//
// Hot path (fpy = /root/reference/first_principles_yields.py):
//   Y_B = trapz_y[ P J(y) A/V(y) W(y) / (s H T) |dT/dy| ]          fpy:231-267
//   A/V(y) = pref(y) * trapz_z[ z^2 e^-z exp(c(y) g4(z)) ]          fpy:158-165
// with 8000 y-nodes x 1200 z-nodes per parameter point.
//
// Mapping:
//   * one 64-lane wavefront owns one parameter point; lane l takes y-nodes l, l+64, ...;
//     no barriers (besides staging the exp table) and no atomics; 16 independent wavefronts
//     per 1024-thread block, two blocks per CU (8 waves per SIMD);
//   * the point-invariant z tables {g4_k, omega'_k} (omega = z^2 e^-z x trapezoid weight,
//     scaled by 2^-512) are read with wave-uniform addresses -> scalar loads into SGPRs, so
//     every FP64 VALU op of the inner loop takes its table operand from an SGPR;
//   * the inner exp is the pre-biased 8192-entry LDS table of lzq_exp2.h: 9-10 VALU per
//     (y, z) node including the accumulate (zsum below);
//   * per-lane partial sums over its y-nodes are combined by a fixed xor-butterfly, so the
//     result is a pure function of the point: independent of launch geometry, batch
//     composition and GPU count (SURVEY §8e bit-identity across W = 1,2,4,8).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/lzq.h"
#include "lzq_exp2.h"
#include "lzq_internal.h"
#include "lzq_physics.h"

#include "lzq_quad.h"

namespace lzq {

// ---------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------
// Block-level table staging of the dense kernels: the exp table into LDS, and with LZQ_ZLDS
// (an ablation build) the default grid's z nodes too; runtime grids (NZ = 0) keep theirs global.
#if LZQ_ZLDS
#define LZQ_STAGE_TABLES(NZ)                                   \
  __shared__ LdsTables lds;                                    \
  const double* tab;                                           \
  if constexpr (NZ == kNZ) {                                   \
    stage_tables<EXPV>(zt, &lds);                              \
    tab = lds.t;                                               \
    zt = lds.z;                                                \
  } else {                                                     \
    tab = stage_table<EXPV>(gtab, lds.t);                      \
  }
#else
#define LZQ_STAGE_TABLES(NZ)          \
  __shared__ double lds_tab[kTabN]; \
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
#endif

// NZ: kNZ for the reference's default z grid (the headline build, node count a compile-time
// constant), 0 for a runtime grid of nzp (padded) nodes -- see zsum_dispatch.
template <int YB, int EXPV, int NZ>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void yields_points_kernel(const lzq_point* __restrict__ pts, int64_t n,
                                                              int32_t n_y, const double* __restrict__ T_lo,
                                                              const double* __restrict__ T_hi,
                                                              const double* __restrict__ Pov,
                                                              const ZNode* __restrict__ zt, int32_t nzp,
                                                              const double* __restrict__ gtab,
                                                              lzq_yield* __restrict__ out, int truncate) {
  LZQ_STAGE_TABLES(NZ)
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  // wave index and point index formed from readfirstlane, so they live in SGPRs (a VGPR copy
  // of the 64-bit index was the kernel's only scratch spill)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t idx = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (idx >= n) return;  // wave-uniform
  {
    const lzq_point pt = pts[idx];
    const double P = Pov ? Pov[idx] : pt.P_chi_to_B;
    const double tlo = T_lo ? T_lo[idx] : pt.T_min_over_Tp * pt.T_p_GeV;  // fpy:369
    const double thi = T_hi ? T_hi[idx] : pt.T_max_over_Tp * pt.T_p_GeV;  // fpy:368
    park(slots[w], quad_setup(pt, P, tlo, thi, n_y), epilogue_pre(pt, P), lane);
  }
  point_yields<YB, EXPV, NZ>(slots, w, zt, nzp, tab, lane, truncate, out + idx);
}

template <int YB, int EXPV, int NZ>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void yields_grid_kernel(lzq_point base, GridSpec grid, int64_t start,
                                                            int64_t count, int32_t n_y,
                                                            const double* __restrict__ Pov,
                                                            const ZNode* __restrict__ zt, int32_t nzp,
                                                            const double* __restrict__ gtab,
                                                            lzq_yield* __restrict__ out, int truncate) {
  LZQ_STAGE_TABLES(NZ)
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR (see yields_points_kernel)
  const int64_t local = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (local >= count) return;
  {
    lzq_point pt;
    const double Pg = grid_point(base, grid, start + local, pt);
    const double P = Pov ? Pov[local] : Pg;
    park(slots[w], quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y),
         epilogue_pre(pt, P), lane);
  }
  point_yields<YB, EXPV, NZ>(slots, w, zt, nzp, tab, lane, truncate, out + local);
}

// ---------------------------------------------------------------------------------------
// lzq_sweep_grid_reuse: the z-sums F(y_j) depend on a grid point only through the fields of
// quad_setup's y-grid and c (I_p, beta/H, T_p, T_min/T_p, T_max/T_p, n_y).  The table kernel
// computes them once per combination of the grid's values of those fields (one wavefront per
// table, kYbTable: the dense kernel's passes, F stored instead of integrated); the reuse kernel
// then integrates every point from its table (kYbReuse).  Same operations, same lane order: Y_B
// is bit-identical to lzq_sweep_grid.  Table t: kTabHdr header doubles (the y-grid and c of the
// QuadSetup it was made for, and the z grid's (nz, z_max); a point whose own setup or grid
// differs gets NaN yields, never a wrong table), then its F values.
constexpr int kTabHdr = 6;
static_assert(kTabHdr == LZQ_REUSE_TABLE_HEADER, "include/lzq.h");

// The z grid a table is made for, as its header stores it.
struct ZKey {
  double nz, z_max;
};

__device__ __forceinline__ int64_t table_of(const GridSpec& g, int64_t idx) {
  int64_t t = 0;
  for (int a = 0; a < g.n_axes; ++a) t += ((idx / g.stride[a]) % g.n[a]) * g.tstride[a];
  return t;
}

// flat grid index of table t's representative (every other axis at its first value)
__device__ __forceinline__ int64_t table_rep(const GridSpec& g, int64_t t) {
  int64_t idx = 0;
  for (int a = 0; a < g.n_axes; ++a)
    if (g.tstride[a]) idx += ((t / g.tstride[a]) % g.n[a]) * g.stride[a];
  return idx;
}

// Table t of one wavefront: header + the F values of the point parked in the wave's slot.
template <int EXPV>
__device__ __forceinline__ void ztable_wave(WaveSlot* slots, int w, int lane, const QuadSetup& qs, const EpiPre& e,
                                            const ZNode* __restrict__ zt, int nzp, ZKey zk, const double* tab,
                                            int truncate, double* F) {
  if (lane == 0) {
    F[0] = qs.y_lo;
    F[1] = qs.y_hi;
    F[2] = (double)qs.n;
    F[3] = qs.cneg;
    F[4] = zk.nz;
    F[5] = zk.z_max;
  }
  park(slots[w], qs, e, lane);
  yb_wave<kYB, EXPV, kYbTable>(slots, w, zt, nzp, tab, truncate, nullptr, F + kTabHdr);
}

// One point integrated from its table F (NaN yields if the table was made for another y-grid).
__device__ __forceinline__ void reuse_wave(WaveSlot* slots, int w, int lane, const QuadSetup& qs, const EpiPre& e,
                                           ZKey zk, const double* __restrict__ F, lzq_yield* out) {
  // match is wave-uniform: every lane formed the same setup
  const bool match = qs.empty || (F[0] == qs.y_lo && F[1] == qs.y_hi && F[2] == (double)qs.n && F[3] == qs.cneg &&
                                  F[4] == zk.nz && F[5] == zk.z_max);
  park(slots[w], qs, e, lane);
  const double Y_B = match ? yb_wave<kYB, kExpTable, kYbReuse>(slots, w, nullptr, 0, nullptr, 0, F + kTabHdr) : 0.0;
  if (lane == 0) {
    lzq_yield o = epilogue_finish(slots[w].e, Y_B);
    if (!match) o.Y_B = o.rho_B_kg_m3 = o.DM_over_B = __builtin_nan("");
    *out = o;
  }
}

template <int EXPV>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void grid_ztable_kernel(lzq_point base, GridSpec grid,
                                                                          int64_t n_tab, int32_t n_y, int64_t tstride,
                                                                          const ZNode* __restrict__ zt, int32_t nzp,
                                                                          ZKey zk, const double* __restrict__ gtab,
                                                                          double* __restrict__ Fw, int truncate) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (t >= n_tab) return;
  lzq_point pt;
  const double P = grid_point(base, grid, table_rep(grid, t), pt);
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  ztable_wave<EXPV>(slots, w, lane, qs, epilogue_pre(pt, P), zt, nzp, zk, tab, truncate, Fw + t * tstride);
}

#ifndef LZQ_REUSE_MIN_WAVES
#define LZQ_REUSE_MIN_WAVES 8  // 8 waves/SIMD (SGPRs capped, a few spilled to VGPR lanes): +12% over 7 (tools/ablate_builds.py ... reuse)
#endif
__global__ __launch_bounds__(kBlock, LZQ_REUSE_MIN_WAVES) void grid_reuse_kernel(lzq_point base, GridSpec grid, int64_t start,
                                                           int64_t count, int32_t n_y,
                                                           const double* __restrict__ Pov, ZKey zk,
                                                           const double* __restrict__ Fw, int64_t tstride,
                                                           lzq_yield* __restrict__ out) {
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t local = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (local >= count) return;
  lzq_point pt;
  const double Pg = grid_point(base, grid, start + local, pt);
  const double P = Pov ? Pov[local] : Pg;
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  reuse_wave(slots, w, lane, qs, epilogue_pre(pt, P), zk, Fw + table_of(grid, start + local) * tstride, out + local);
}

// The same for explicit points (lzq_yields_batch_reuse): table t is made for point reps[t];
// point i integrates from table tidx[i].
template <int EXPV>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void points_ztable_kernel(const lzq_point* __restrict__ pts,
                                                                            const int64_t* __restrict__ reps,
                                                                            int64_t n_tab, int32_t n_y, int64_t tstride,
                                                                            const ZNode* __restrict__ zt, int32_t nzp,
                                                                            ZKey zk, const double* __restrict__ gtab,
                                                                            double* __restrict__ Fw, int truncate) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (t >= n_tab) return;
  const lzq_point pt = pts[reps[t]];
  const double P = pt.P_chi_to_B;
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  ztable_wave<EXPV>(slots, w, lane, qs, epilogue_pre(pt, P), zt, nzp, zk, tab, truncate, Fw + t * tstride);
}

__global__ __launch_bounds__(kBlock, LZQ_REUSE_MIN_WAVES) void points_reuse_kernel(const lzq_point* __restrict__ pts, int64_t n,
                                                             int32_t n_y, const double* __restrict__ Pov, ZKey zk,
                                                             const int32_t* __restrict__ tidx,
                                                             const double* __restrict__ Fw, int64_t tstride,
                                                             lzq_yield* __restrict__ out) {
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t idx = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (idx >= n) return;
  const lzq_point pt = pts[idx];
  const double P = Pov ? Pov[idx] : pt.P_chi_to_B;
  const QuadSetup qs = quad_setup(pt, P, pt.T_min_over_Tp * pt.T_p_GeV, pt.T_max_over_Tp * pt.T_p_GeV, n_y);
  reuse_wave(slots, w, lane, qs, epilogue_pre(pt, P), zk, Fw + (int64_t)tidx[idx] * tstride, out + idx);
}

// fpy:158-165, one lane per y value
template <int EXPV>
__global__ __launch_bounds__(kBlock) void aov_kernel(lzq_point pt, const double* __restrict__ ys, int64_t n,
                                                    const ZNode* __restrict__ zt, int32_t nzp,
                                                    const double* __restrict__ gtab, double* __restrict__ out) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = i < n;
  const double y = live ? ys[i] : 0.0;
  QuadSetup s = quad_setup(pt, pt.P_chi_to_B, 1.0, 1.0, LZQ_NY_MIN);
  double expy = exp_sc(pymax(pymin(y, 50.0), -50.0));
  double c2[1] = {((s.cneg * expy) * kLog2E) * c2_scale<EXPV>()}, F[1];
  zsum_dispatch<1, EXPV>(zt, nzp, tab, c2, F);
  if (live) out[i] = (y > 50.0) ? 0.0 : (s.pref0 * expy) * F[0];
}

// fpy:207-212 build_tables, first half: A/V at the nt knots Ts = linspace(T_lo, T_hi, nt)
// (main() uses n = 800) of main()'s window (fpy:368-369) or the given one, np.maximum(Av, 0),
// one wavefront per point (lane i takes knots i, i+64, ...), into the point's 4 nt doubles.  The
// spline is fitted by lzq_ode.hip's ode_spline_kernel.
template <int EXPV>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void ode_aov_table_kernel(const lzq_point* __restrict__ pts,
                                                                               int64_t n, int32_t nt,
                                                                               const ZNode* __restrict__ zt, int32_t nzp,
                                                                               const double* __restrict__ gtab,
                                                                               const double* __restrict__ Tlo,
                                                                               const double* __restrict__ Thi,
                                                                               double* __restrict__ ws, int truncate,
    int chunks) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  const int lane = threadIdx.x & (kWaveSize - 1);
  // chunks > 1 (few tables, LZQ_TUNE_ODE_TABLE_WIDE): the point's 64-knot groups spread over
  // `chunks` wavefronts (group g on wave g mod chunks) -- each group's operations as with one wave
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t idx = wave / chunks;
  const int chunk = (int)(wave - idx * chunks);
  if (idx >= n) return;  // wave-uniform
  const lzq_point pt = pts[idx];
  // every per-point value is wave-uniform: pinned in SGPRs (readfirstlane) so that the z-loop
  // keeps its VGPRs (without this 12 VGPRs spilled around every z-loop)
  const double Tp = uniform(pt.T_p_GeV), B = uniform(pt.beta_over_H);
  const double T_lo = uniform(Tlo ? Tlo[idx] : pt.T_min_over_Tp * Tp);
  const double T_hi = uniform(Thi ? Thi[idx] : pt.T_max_over_Tp * Tp);
  const double stepT = uniform((T_hi - T_lo) / (double)(nt - 1));
  const QuadSetup s = quad_setup(pt, 0.0, 1.0, 1.0, LZQ_NY_MIN);  // only pref0 / cneg are used
  const double pref0 = uniform(s.pref0), cneg = uniform(s.cneg);
  const int64_t ws_pt = 4 * (int64_t)nt;
  double* w = ws + idx * ws_pt;
  for (int base = chunk * kWaveSize; base < nt; base += kWaveSize * chunks) {
    const int i = base + lane;
    const int ii = i < nt ? i : nt - 1;
    const double T = linspace_at(T_lo, T_hi, stepT, ii, nt);
    const double y = y_of_T(T, Tp, B);
    const double expy = exp_sc(pymax(pymin(y, 50.0), -50.0));  // fpy:161
    double c2[1] = {((cneg * expy) * kLog2E) * c2_scale<EXPV>()}, F[1];
    zsum_dispatch<1, EXPV>(zt, nzp, tab, c2, F, truncate);
    const double Av = (y > 50.0) ? 0.0 : (pref0 * expy) * F[0];  // fpy:159-165
    if (i < nt) w[i < nt - 1 ? 4 * i + 3 : ws_pt - 1] = pymax(Av, 0.0);
  }
}

// fpy:222-223 (J_chi_flux fpy:122-123), one lane per T
__global__ __launch_bounds__(kBlock) void jchi_kernel(lzq_point pt, const double* __restrict__ Ts, int64_t n,
                                                     double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double T = Ts[i];
  out[i] = pt.incident_flux_scale *
           (0.25 * n_chi_eq(T, pt.m_chi_GeV, pt.g_chi, pt.stats) * vbar_chi(T, pt.m_chi_GeV));
}

// fpy:183-184
__global__ __launch_bounds__(kBlock) void p_closed_form_kernel(const double* __restrict__ lam, int64_t n,
                                                              double* __restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) P[i] = p_closed_form(lam[i]);
}

}  // namespace lzq

// =========================================================================================
// host side: z tables, error plumbing, C ABI
// =========================================================================================
namespace {

thread_local char g_err[512] = "";
std::mutex g_mu;
constexpr int kMaxDevices = 64;
// per device: the default grid's [LZQ_NZ] ZNode followed by the kTabN-entry exp table
lzq::ZNode* g_dev_tab[kMaxDevices] = {nullptr};
uint64_t g_exp2tab[lzq::kTabN];  // lzq::tab_entry_bits layout
bool g_exp_ready = false;
int g_exp_variant = lzq::kExpTable;
int g_truncate = 0;  // LZQ_TUNE_TRUNCATE

const double* exp_table(int dev) { return reinterpret_cast<const double*>(g_dev_tab[dev] + LZQ_NZ); }

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define LZQ_HIP(call)                                                                         \
  do {                                                                                        \
    hipError_t e_ = (call);                                                                   \
    if (e_ != hipSuccess) return fail(LZQ_EHIP, "%s: %s", #call, hipGetErrorString(e_));      \
  } while (0)

// One z grid of AoverVKernel(..., z_max, nz) (fpy:141-156) on the host: z = linspace(0, z_max, nz),
// the verbatim cancelling gamma4, and the trapezoid weights omega_k = z_k^2 e^{-z_k} (d_{k-1} +
// d_k)/2 with d = diff(z) (np.trapezoid, fpy:164, as a weighted sum).  libm exp/pow; built once
// per grid.
struct HostZGrid {
  int32_t nz = 0;
  double z_max = 0.0;
  std::vector<double> z, g4, omega;
  bool monotone = true;  // g4 non-decreasing (the truncation's binary search needs it)
};

int build_ztable(int32_t nz, double z_max, HostZGrid& h) {
  if (nz < 0) return fail(LZQ_EINVAL, "Number of samples, %d, must be non-negative.", nz);  // np.linspace
  if (nz > LZQ_NZ_MAX) return fail(LZQ_EINVAL, "nz = %d exceeds LZQ_NZ_MAX (%d)", nz, LZQ_NZ_MAX);
  if (!(z_max >= 0.0) || !isfinite(z_max))
    return fail(LZQ_EINVAL, "z_max = %g: the z grid must be finite and >= 0 (fpy:154)", z_max);
  h.nz = nz;
  h.z_max = z_max;
  h.z.assign(nz, 0.0);
  h.g4.assign(nz, 0.0);
  h.omega.assign(nz, 0.0);
  if (nz == 1) h.z[0] = 0.0;  // np.linspace(0, z_max, 1) = [0.]
  if (nz >= 2) {
    const double step = (z_max - 0.0) / (double)(nz - 1);
    for (int k = 0; k < nz; ++k)  // np.linspace (numpy's step == 0 branch when z_max underflows the step)
      h.z[k] = (k == nz - 1) ? z_max : (step == 0.0 ? ((double)k / (double)(nz - 1)) * z_max : (double)k * step) + 0.0;
  }
  std::vector<double> w(nz);
  for (int k = 0; k < nz; ++k) {
    const double z = h.z[k];
    const double ez = exp(-z);
    const double zz = z * z;
    h.g4[k] = 6.0 - ez * (((pow(z, 3.0) + 3.0 * zz) + 6.0 * z) + 6.0);
    w[k] = zz * ez;
    // the reference's cancelling form rounds below 0 only on grids far finer than its default
    // (z_1 < ~3e-4): exp of a positive argument there, which the inner loop does not evaluate
    if (!(h.g4[k] >= 0.0))
      return fail(LZQ_EINVAL, "gamma4[%d] = %g < 0 (nz = %d, z_max = %g): the cancelling form of fpy:156 rounds "
                  "below 0 on this grid", k, h.g4[k], nz, z_max);
    if (k > 0 && h.g4[k] < h.g4[k - 1]) h.monotone = false;
  }
  // zsum_dispatch zeroes a lane whose term at node 1 underflows (c2 g4_1 <= -1077 N), which is
  // exact only if g4_1 is the smallest g4 over k >= 1: a grid whose rounded gamma4 decreases
  // anywhere (only the finest grids, where the cancelling form is noise at its first nodes) is
  // refused like the negative one above
  if (!h.monotone)
    return fail(LZQ_EINVAL, "z grid (nz = %d, z_max = %g): the cancelling gamma4 of fpy:156 is not non-decreasing on "
                "this grid (rounding noise at its first nodes)", nz, z_max);
  for (int k = 0; k < nz; ++k) {
    const double dl = k > 0 ? h.z[k] - h.z[k - 1] : 0.0;
    const double dr = k + 1 < nz ? h.z[k + 1] - h.z[k] : 0.0;
    h.omega[k] = w[k] * (0.5 * (dl + dr));
  }
  // zsum_dispatch: a lane is dead (zeroed) iff c2N g4_1 <= -1077 N, so a live lane has
  // |u| < 1077 N g4_max / g4_1; nodes beyond 2^51 are clamped and round away while |u| < 2^200
  if (nz >= 2 && z_max > 0.0) {
    const double g1 = h.g4[1], gmax = h.g4[nz - 1];
    if (!(g1 > 0.0) || !((double)lzq::kTabN * 1077.0 * gmax / g1 < 0x1p200))
      return fail(LZQ_EINVAL, "z grid (nz = %d, z_max = %g): gamma4[1] = %g breaks the inner loop's reduction", nz,
                  z_max, g1);
  }
  return LZQ_OK;
}

const HostZGrid& default_host_grid() {
  static HostZGrid h;
  static int rc = build_ztable(LZQ_NZ, LZQ_Z_MAX, h);
  (void)rc;  // the default grid always builds (tests/test_capi.py)
  return h;
}

void build_exp_table() {
  if (g_exp_ready) return;
  // T[j] = 2^(j/N): x87 long double exp2 (64-bit mantissa) rounded once to double, stored
  // with the pre-biased high word of lzq::tab_entry_bits
  for (int j = 0; j < lzq::kTabN; ++j) g_exp2tab[j] = lzq::tab_entry_bits(lzq::tab_exact(j), j);
  g_exp_ready = true;
}

// Device image of a grid: nzp >= max(nz, kKUnroll) nodes, a multiple of the unroll; the padding
// repeats the last g4 with omega' = 0 (an exact +0 per node).  Weights carry 2^-512 (the exp
// table's T' carries 2^+512, lzq_exp2.h).
int32_t padded_nodes(int32_t nz) {
  const int32_t u = lzq::kKUnroll;
  const int32_t n = nz > u ? nz : u;
  return (n + u - 1) / u * u;
}

void device_nodes(const HostZGrid& h, lzq::ZNode* dst) {
  const int32_t nzp = padded_nodes(h.nz);
  const double glast = h.nz > 0 ? h.g4[h.nz - 1] : 0.0;
  for (int k = 0; k < nzp; ++k)
    dst[k] = k < h.nz ? lzq::ZNode{h.g4[k], ldexp(h.omega[k], -lzq::kOmegaBias)} : lzq::ZNode{glast, 0.0};
}

int ensure_device(int* dev_out) {
  int dev = 0;
  LZQ_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return fail(LZQ_ENODEVICE, "device %d out of range", dev);
  if (dev_out) *dev_out = dev;
  if (g_dev_tab[dev]) return LZQ_OK;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_dev_tab[dev]) return LZQ_OK;
  const HostZGrid& h = default_host_grid();
  if ((int)h.g4.size() != LZQ_NZ) return fail(LZQ_EINVAL, "default z grid failed to build");
  build_exp_table();
  static_assert(sizeof(lzq::ZNode) == 2 * sizeof(double), "ZNode layout");
  static_assert(LZQ_NZ % lzq::kKUnroll == 0, "the default grid needs no padding");
  std::vector<lzq::ZNode> host(LZQ_NZ + lzq::kTabN / 2);
  device_nodes(h, host.data());
  memcpy(&host[LZQ_NZ], g_exp2tab, sizeof(g_exp2tab));
  const size_t bytes = host.size() * sizeof(lzq::ZNode);
  lzq::ZNode* d = nullptr;
  LZQ_HIP(hipMalloc(&d, bytes));
  LZQ_HIP(hipMemcpy(d, host.data(), bytes, hipMemcpyHostToDevice));
  g_dev_tab[dev] = d;
  return LZQ_OK;
}

// A z grid on a device, as the kernels take it.
struct DevZGrid {
  const lzq::ZNode* zt = nullptr;
  int32_t nzp = 0;
  bool is_default = false;  // the compile-time LZQ_NZ kernels apply
  bool monotone = true;
  lzq::ZKey key{0.0, 0.0};
};

struct ZGridEntry {
  int dev;
  int32_t nz;
  uint64_t zbits;
  lzq::ZNode* d;
  int32_t nzp;
  bool monotone;
};
std::vector<ZGridEntry> g_zgrids;  // runtime grids, uploaded on first use (guarded by g_mu)

bool is_default_grid(int32_t nz, double z_max) { return nz == LZQ_NZ && z_max == LZQ_Z_MAX; }

// The device tables of (nz, z_max) on the current device: the default grid's (lzq_init), or a
// runtime grid's, built and uploaded once per (device, nz, z_max) (a synchronous copy: call
// lzq_zgrid_init before capturing launches into a graph).
int zgrid_for(int32_t nz, double z_max, DevZGrid& g, int* dev_out) {
  int dev, rc = ensure_device(&dev);
  if (rc) return rc;
  if (dev_out) *dev_out = dev;
  g.key = lzq::ZKey{(double)nz, z_max};
  if (is_default_grid(nz, z_max)) {
    g.zt = g_dev_tab[dev];
    g.nzp = LZQ_NZ;
    g.is_default = true;
    g.monotone = default_host_grid().monotone;
    return LZQ_OK;
  }
  const uint64_t zb = __builtin_bit_cast(uint64_t, z_max);
  std::lock_guard<std::mutex> lk(g_mu);
  for (const ZGridEntry& e : g_zgrids)
    if (e.dev == dev && e.nz == nz && e.zbits == zb) {
      g.zt = e.d;
      g.nzp = e.nzp;
      g.monotone = e.monotone;
      return LZQ_OK;
    }
  HostZGrid h;
  rc = build_ztable(nz, z_max, h);
  if (rc) return rc;
  const int32_t nzp = padded_nodes(nz);
  std::vector<lzq::ZNode> host(nzp);
  device_nodes(h, host.data());
  lzq::ZNode* d = nullptr;
  LZQ_HIP(hipMalloc(&d, host.size() * sizeof(lzq::ZNode)));
  LZQ_HIP(hipMemcpy(d, host.data(), host.size() * sizeof(lzq::ZNode), hipMemcpyHostToDevice));
  g_zgrids.push_back(ZGridEntry{dev, nz, zb, d, nzp, h.monotone});
  g.zt = d;
  g.nzp = nzp;
  g.monotone = h.monotone;
  return LZQ_OK;
}

int64_t blocks_for(int64_t n, int64_t per_block) { return (n + per_block - 1) / per_block; }

constexpr int64_t kMaxGrid = 2147483647LL;

}  // namespace

int lzq_set_error(int code, const char* msg) { return fail(code, "%s", msg); }

int lzq::launch_ode_aov_tables(const lzq_point* d_points, int64_t n, const double* d_T_lo, const double* d_T_hi,
                               int32_t nt, int32_t nz, double z_max, const lzq_aov_params* d_aov, double* d_work,
                               hipStream_t stream) {
  if (n == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  // few tables: one wavefront per 64 knots (LZQ_TUNE_ODE_TABLE_WIDE; the same bits), else one per table
  const int chunks = ((lzq::g_ode_table_wide & 1) && n <= 4096) ? (int)((nt + lzq::kWaveSize - 1) / lzq::kWaveSize) : 1;
  const int64_t nb = blocks_for(n * chunks, lzq::kWavesPerBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_ode_tables: n too large");
  // The ODE tables always use the exact-underflow truncation of the z-sums: it is bit-identical
  // to the dense sum (tests/test_gpu_parity.py::test_truncation_is_bit_identical) and this path
  // is not the dense headline benchmark, so there is nothing to keep dense for.
  const int truncate = g.monotone ? 1 : 0;
  if (d_aov)  // the A/V kernel's own parameters (lzq_aov.hip)
    return lzq::launch_ode_aov_tables_aov(g_exp_variant, d_points, d_aov, n, nt, g.zt, g.nzp, exp_table(dev), d_T_lo,
                                          d_T_hi, d_work, truncate, stream, chunks);
  if (g_exp_variant == lzq::kExpTable)
    hipLaunchKernelGGL(lzq::ode_aov_table_kernel<lzq::kExpTable>, dim3((unsigned)nb), dim3(lzq::kBlock), 0, stream,
                       d_points, n, nt, g.zt, g.nzp, exp_table(dev), d_T_lo, d_T_hi, d_work, truncate, chunks);
  else
    hipLaunchKernelGGL(lzq::ode_aov_table_kernel<lzq::kExpPoly11>, dim3((unsigned)nb), dim3(lzq::kBlock), 0, stream,
                       d_points, n, nt, g.zt, g.nzp, exp_table(dev), d_T_lo, d_T_hi, d_work, truncate, chunks);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

extern "C" {

int lzq_abi_version(void) { return LZQ_ABI_VERSION; }

const char* lzq_last_error(void) { return g_err; }

int lzq_init(int device) { return lzq_zgrid_init(device, LZQ_NZ, LZQ_Z_MAX); }

int lzq_zgrid_init(int device, int32_t nz, double z_max) {
  int cur = 0;
  LZQ_HIP(hipGetDevice(&cur));
  if (device != cur) LZQ_HIP(hipSetDevice(device));
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, nullptr);
  if (device != cur) {
    hipError_t e = hipSetDevice(cur);
    if (e != hipSuccess && rc == LZQ_OK) return fail(LZQ_EHIP, "hipSetDevice: %s", hipGetErrorString(e));
  }
  return rc;
}

int lzq_tune(int32_t key, int32_t value) {
  if (key == LZQ_TUNE_EXP) {
    if (value != LZQ_EXP_POLY11 && value != LZQ_EXP_TABLE)
      return fail(LZQ_EINVAL, "lzq_tune: unknown exp variant %d", value);
    int prev = g_exp_variant;
    g_exp_variant = value;
    return prev;
  }
  if (key == LZQ_TUNE_TRUNCATE) {
    if (value != 0 && value != 1) return fail(LZQ_EINVAL, "lzq_tune: truncate must be 0 or 1, got %d", value);
    int prev = g_truncate;
    g_truncate = value;
    return prev;
  }
  if (key == LZQ_TUNE_ODE_LAUNCH_STEPS) {
    if (value < 6 || value > 40) return fail(LZQ_EINVAL, "lzq_tune: ode launch steps log2 must be in [6, 40], got %d", value);
    int prev = lzq::g_ode_launch_log2;
    lzq::g_ode_launch_log2 = value;
    return prev;
  }
  if (key == LZQ_TUNE_PROFILE_FLAT) {
    if (value != 0 && value != 1) return fail(LZQ_EINVAL, "lzq_tune: profile_flat must be 0 or 1, got %d", value);
    int prev = lzq::g_profile_flat;
    lzq::g_profile_flat = value;
    return prev;
  }
  if (key == LZQ_TUNE_ODE_TABLE_WIDE) {
    if (value < 0 || value > 3) return fail(LZQ_EINVAL, "lzq_tune: ode_table_wide must be in 0..3, got %d", value);
    int prev = lzq::g_ode_table_wide;
    lzq::g_ode_table_wide = value;
    return prev;
  }
  if (key == LZQ_TUNE_ODE_TP_INTERVAL) {
    if (value < 64 || value > (1 << 20) || value % 64 != 0)
      return fail(LZQ_EINVAL, "lzq_tune: ode_tp_interval must be a multiple of 64 in [64, 2^20] steps, got %d", value);
    int prev = lzq::g_ode_tp_interval;
    lzq::g_ode_tp_interval = value;
    return prev;
  }
  if (key == LZQ_TUNE_ODE_COOP) {
    if (value != 0 && value != 1) return fail(LZQ_EINVAL, "lzq_tune: ode_coop must be 0 or 1, got %d", value);
    int prev = lzq::g_ode_coop;
    lzq::g_ode_coop = value;
    return prev;
  }
  return fail(LZQ_EINVAL, "lzq_tune: unknown key %d", key);
}

int lzq_ztables(int32_t nz, double z_max, double* z, double* gamma4, double* omega) {
  HostZGrid h;
  int rc;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    rc = build_ztable(nz, z_max, h);
  }
  if (rc) return rc;
  const size_t bytes = sizeof(double) * (size_t)nz;
  if (z && nz) memcpy(z, h.z.data(), bytes);
  if (gamma4 && nz) memcpy(gamma4, h.g4.data(), bytes);
  if (omega && nz) memcpy(omega, h.omega.data(), bytes);
  return LZQ_OK;
}

int lzq_aov_batch(const lzq_point* pt_in, const lzq_aov_params* aov, const double* d_y, int64_t n, int32_t nz,
                  double z_max, double* d_out, void* stream) {
  if ((!pt_in && !aov) || n < 0 || (n > 0 && (!d_y || !d_out))) return fail(LZQ_EINVAL, "lzq_aov_batch: bad arguments");
  if (n == 0) return LZQ_OK;
  // aov_kernel reads only the A/V kernel's fields of its point (quad_setup's pref0 / c)
  lzq_point own;
  if (pt_in) own = *pt_in;
  else memset(&own, 0, sizeof(own));
  if (aov) {
    own.I_p = aov->I_p;
    own.beta_over_H = aov->beta_over_H;
    own.T_p_GeV = aov->T_p_GeV;
    own.v_w = aov->v_w;
    own.g_star = aov->g_star;
  }
  const lzq_point* pt = &own;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  int64_t nb = blocks_for(n, lzq::kBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_aov_batch: n too large");
  if (g_exp_variant == lzq::kExpTable)
    hipLaunchKernelGGL(lzq::aov_kernel<lzq::kExpTable>, dim3((unsigned)nb), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, *pt, d_y, n, g.zt, g.nzp, exp_table(dev), d_out);
  else
    hipLaunchKernelGGL(lzq::aov_kernel<lzq::kExpPoly11>, dim3((unsigned)nb), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, *pt, d_y, n, g.zt, g.nzp, exp_table(dev), d_out);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int lzq_jchi_batch(const lzq_point* pt, const double* d_T, int64_t n, double* d_out, void* stream) {
  if (!pt || n < 0 || (n > 0 && (!d_T || !d_out))) return fail(LZQ_EINVAL, "lzq_jchi_batch: bad arguments");
  if (n == 0) return LZQ_OK;
  int64_t nb = blocks_for(n, lzq::kBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_jchi_batch: n too large");
  hipLaunchKernelGGL(lzq::jchi_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream, *pt, d_T, n,
                     d_out);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int lzq_yields_batch(const lzq_point* d_points, int64_t n, int32_t n_y, int32_t nz, double z_max,
                     const double* d_T_lo, const double* d_T_hi, const double* d_P, const lzq_aov_params* d_aov,
                     lzq_yield* d_out, void* stream) {
  if (n < 0 || (n > 0 && (!d_points || !d_out))) return fail(LZQ_EINVAL, "lzq_yields_batch: bad arguments");
  if ((d_T_lo == nullptr) != (d_T_hi == nullptr))
    return fail(LZQ_EINVAL, "lzq_yields_batch: T_lo and T_hi must both be given or both be NULL");
  if (n == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  int64_t nb = blocks_for(n, lzq::kWavesPerBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_yields_batch: n too large");
  const int trunc = g.monotone ? g_truncate : 0;
  const hipStream_t s = (hipStream_t)stream;
  if (d_aov)  // the A/V kernel's own parameters (lzq_aov.hip)
    return lzq::launch_yields_points_aov(g_exp_variant, g.is_default, d_points, d_aov, n, n_y, d_T_lo, d_T_hi, d_P,
                                         g.zt, g.nzp, exp_table(dev), d_out, trunc, s);
#define LZQ_POINTS(EXPV, NZ)                                                                                        \
  hipLaunchKernelGGL((lzq::yields_points_kernel<lzq::kYB, EXPV, NZ>), dim3((unsigned)nb), dim3(lzq::kBlock), 0, s, \
                     d_points, n, n_y, d_T_lo, d_T_hi, d_P, g.zt, g.nzp, exp_table(dev), d_out, trunc)
  if (g_exp_variant == lzq::kExpTable) {
    if (g.is_default) LZQ_POINTS(lzq::kExpTable, lzq::kNZ);
    else LZQ_POINTS(lzq::kExpTable, 0);
  } else {
    if (g.is_default) LZQ_POINTS(lzq::kExpPoly11, lzq::kNZ);
    else LZQ_POINTS(lzq::kExpPoly11, 0);
  }
#undef LZQ_POINTS
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

namespace {
// lzq_sweep_grid's argument checks and GridSpec (shared with lzq_sweep_grid_reuse)
int make_grid(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start, int64_t count,
              const lzq_yield* d_out, const char* who, lzq::GridSpec& g) {
  if (!base || n_axes < 0 || n_axes > LZQ_MAX_AXES || (n_axes > 0 && !axes) || start < 0 || count < 0 ||
      (count > 0 && !d_out))
    return fail(LZQ_EINVAL, "%s: bad arguments", who);
  memset(&g, 0, sizeof(g));
  g.n_axes = n_axes;
  int64_t total = 1;
  bool mix = false, dpr = false;
  for (int a = n_axes - 1; a >= 0; --a) {
    const int32_t f = axes[a].field;
    if (!((f >= 0 && f <= 14) || f == LZQ_F_DELTA_LZ || f == LZQ_F_M_MIX || f == LZQ_F_DPRIME))
      return fail(LZQ_EINVAL, "%s: axis %d has unknown field %d", who, a, f);
    if (axes[a].n <= 0 || !axes[a].values) return fail(LZQ_EINVAL, "%s: axis %d is empty", who, a);
    mix |= f == LZQ_F_M_MIX;
    dpr |= f == LZQ_F_DPRIME;
    g.field[a] = f;
    g.n[a] = axes[a].n;
    g.values[a] = axes[a].values;
    g.stride[a] = total;
    if (total > INT64_MAX / axes[a].n) return fail(LZQ_EINVAL, "%s: grid too large", who);
    total *= axes[a].n;
  }
  if (mix != dpr) return fail(LZQ_EINVAL, "%s: LZQ_F_M_MIX and LZQ_F_DPRIME must be swept together", who);
  if (start > total || count > total - start)
    return fail(LZQ_EINVAL, "%s: range [%lld, %lld) outside grid of %lld points", who, (long long)start,
                (long long)(start + count), (long long)total);
  if (base->regime != LZQ_THERMAL && base->regime != LZQ_NONTHERMAL)
    return fail(LZQ_EUNSUPPORTED, "%s: regime must be thermal or nonthermal (fpy:376-384)", who);
  return LZQ_OK;
}

// the fields quad_setup's y-grid and c depend on (lzq_sweep_grid_reuse's table axes)
bool ztable_field(int32_t f) {
  return f == LZQ_F_I_P || f == LZQ_F_BETA_OVER_H || f == LZQ_F_T_P || f == LZQ_F_T_MIN_OVER_TP ||
         f == LZQ_F_T_MAX_OVER_TP;
}

int64_t ztable_count(const lzq::GridSpec& g) {
  int64_t n = 1;
  for (int a = 0; a < g.n_axes; ++a)
    if (ztable_field(g.field[a])) n *= g.n[a];
  return n;
}
}  // namespace

int lzq_sweep_grid(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start, int64_t count,
                   int32_t n_y, int32_t nz, double z_max, const double* d_P, lzq_yield* d_out, void* stream) {
  lzq::GridSpec gs;
  int rc = make_grid(base, axes, n_axes, start, count, d_out, "lzq_sweep_grid", gs);
  if (rc) return rc;
  if (count == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  int64_t nb = blocks_for(count, lzq::kWavesPerBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_sweep_grid: count too large for one launch");
  const int trunc = g.monotone ? g_truncate : 0;
  const hipStream_t s = (hipStream_t)stream;
#define LZQ_GRID(EXPV, NZ)                                                                                         \
  hipLaunchKernelGGL((lzq::yields_grid_kernel<lzq::kYB, EXPV, NZ>), dim3((unsigned)nb), dim3(lzq::kBlock), 0, s,  \
                     *base, gs, start, count, n_y, d_P, g.zt, g.nzp, exp_table(dev), d_out, trunc)
  if (g_exp_variant == lzq::kExpTable) {
    if (g.is_default) LZQ_GRID(lzq::kExpTable, lzq::kNZ);
    else LZQ_GRID(lzq::kExpTable, 0);
  } else {
    if (g.is_default) LZQ_GRID(lzq::kExpPoly11, lzq::kNZ);
    else LZQ_GRID(lzq::kExpPoly11, 0);
  }
#undef LZQ_GRID
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int lzq_yields_batch_reuse(const lzq_point* d_points, int64_t n, int32_t n_y, int32_t nz, double z_max,
                           const double* d_P, const int64_t* d_rep, const int32_t* d_table_index, int64_t n_tables,
                           double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream) {
  if (n < 0 || n_tables < 0 || (n > 0 && (!d_points || !d_out || !d_rep || !d_table_index || n_tables == 0)))
    return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: bad arguments");
  const int64_t stride = (n_y > LZQ_NY_MIN ? n_y : LZQ_NY_MIN) + lzq::kTabHdr;
  if (n_tables > INT64_MAX / stride) return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: too many tables");
  if (n > 0 && (!d_work || work_doubles < n_tables * stride))
    return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: workspace of %lld doubles < %lld needed", (long long)work_doubles,
                (long long)(n_tables * stride));
  if (n == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  int rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  const int64_t nbt = blocks_for(n_tables, lzq::kWavesPerBlock), nb = blocks_for(n, lzq::kWavesPerBlock);
  if (nbt > kMaxGrid || nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_yields_batch_reuse: too large for one launch");
  const int trunc = g.monotone ? 1 : 0;  // bit-identical to the dense sums either way
  if (g_exp_variant == lzq::kExpTable)
    hipLaunchKernelGGL((lzq::points_ztable_kernel<lzq::kExpTable>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, d_points, d_rep, n_tables, n_y, stride, g.zt, g.nzp, g.key,
                       exp_table(dev), d_work, trunc);
  else
    hipLaunchKernelGGL((lzq::points_ztable_kernel<lzq::kExpPoly11>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                       (hipStream_t)stream, d_points, d_rep, n_tables, n_y, stride, g.zt, g.nzp, g.key,
                       exp_table(dev), d_work, trunc);
  LZQ_HIP(hipGetLastError());
  hipLaunchKernelGGL(lzq::points_reuse_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream, d_points,
                     n, n_y, d_P, g.key, d_table_index, d_work, stride, d_out);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

int64_t lzq_sweep_grid_reuse_workspace(const lzq_axis* axes, int32_t n_axes, int32_t n_y) {
  if (n_axes < 0 || n_axes > LZQ_MAX_AXES || (n_axes > 0 && !axes)) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: bad arguments");
  int64_t n = 1;
  for (int a = 0; a < n_axes; ++a) {
    if (axes[a].n <= 0) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: axis %d is empty", a);
    if (ztable_field(axes[a].field)) {
      if (n > INT64_MAX / 16 / axes[a].n) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: too many tables");
      n *= axes[a].n;
    }
  }
  const int64_t ny = n_y > LZQ_NY_MIN ? n_y : LZQ_NY_MIN;
  if (n > INT64_MAX / (ny + lzq::kTabHdr)) return fail(LZQ_EINVAL, "lzq_sweep_grid_reuse_workspace: too many tables");
  return n * (ny + lzq::kTabHdr);
}

// lzq_sweep_grid_reuse in its two halves: build every z-sum table of the grid (parts & 1) and
// integrate [start, start + count) from them (parts & 2).
static int sweep_grid_reuse_parts(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start,
                                  int64_t count, int32_t n_y, int32_t nz, double z_max, const double* d_P,
                                  double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream, int parts,
                                  const char* fn) {
  lzq::GridSpec gs;
  int rc = make_grid(base, axes, n_axes, start, count, d_out, fn, gs);
  if (rc) return rc;
  const int64_t need = lzq_sweep_grid_reuse_workspace(axes, n_axes, n_y);
  if (need < 0) return (int)need;
  const bool work = (parts & 1) || count > 0;
  if (work && (!d_work || work_doubles < need))
    return fail(LZQ_EINVAL, "%s: workspace of %lld doubles < %lld needed", fn, (long long)work_doubles,
                (long long)need);
  if (!(parts & 1) && count == 0) return LZQ_OK;
  int dev;
  DevZGrid g;
  rc = zgrid_for(nz, z_max, g, &dev);
  if (rc) return rc;
  const int64_t n_tab = ztable_count(gs);
  int64_t ts = 1;
  for (int a = gs.n_axes - 1; a >= 0; --a)
    if (ztable_field(gs.field[a])) {
      gs.tstride[a] = ts;
      ts *= gs.n[a];
    }
  const int64_t stride = (n_y > LZQ_NY_MIN ? n_y : LZQ_NY_MIN) + lzq::kTabHdr;
  const int64_t nbt = blocks_for(n_tab, lzq::kWavesPerBlock), nb = blocks_for(count, lzq::kWavesPerBlock);
  if (nbt > kMaxGrid || nb > kMaxGrid) return fail(LZQ_EINVAL, "%s: too large for one launch", fn);
  if (parts & 1) {
    // the tables use the exact-underflow truncation: bit-identical to the dense sums
    const int trunc = g.monotone ? 1 : 0;
    if (g_exp_variant == lzq::kExpTable)
      hipLaunchKernelGGL((lzq::grid_ztable_kernel<lzq::kExpTable>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                         (hipStream_t)stream, *base, gs, n_tab, n_y, stride, g.zt, g.nzp, g.key, exp_table(dev), d_work,
                         trunc);
    else
      hipLaunchKernelGGL((lzq::grid_ztable_kernel<lzq::kExpPoly11>), dim3((unsigned)nbt), dim3(lzq::kBlock), 0,
                         (hipStream_t)stream, *base, gs, n_tab, n_y, stride, g.zt, g.nzp, g.key, exp_table(dev), d_work,
                         trunc);
    LZQ_HIP(hipGetLastError());
  }
  if ((parts & 2) && count > 0) {
    hipLaunchKernelGGL(lzq::grid_reuse_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream, *base, gs,
                       start, count, n_y, d_P, g.key, d_work, stride, d_out);
    LZQ_HIP(hipGetLastError());
  }
  return LZQ_OK;
}

int lzq_sweep_grid_reuse(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start, int64_t count,
                         int32_t n_y, int32_t nz, double z_max, const double* d_P, double* d_work, int64_t work_doubles,
                         lzq_yield* d_out, void* stream) {
  if (count == 0) {  // nothing to integrate: validate only (tables need not be built)
    lzq::GridSpec g;
    return make_grid(base, axes, n_axes, start, count, d_out, "lzq_sweep_grid_reuse", g);
  }
  return sweep_grid_reuse_parts(base, axes, n_axes, start, count, n_y, nz, z_max, d_P, d_work, work_doubles, d_out,
                                stream, 3, "lzq_sweep_grid_reuse");
}

int lzq_sweep_grid_ztables(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int32_t n_y, int32_t nz,
                           double z_max, double* d_work, int64_t work_doubles, void* stream) {
  return sweep_grid_reuse_parts(base, axes, n_axes, 0, 0, n_y, nz, z_max, nullptr, d_work, work_doubles, nullptr,
                                stream, 1, "lzq_sweep_grid_ztables");
}

int lzq_sweep_grid_from_ztables(const lzq_point* base, const lzq_axis* axes, int32_t n_axes, int64_t start,
                                int64_t count, int32_t n_y, int32_t nz, double z_max, const double* d_P,
                                const double* d_work, int64_t work_doubles, lzq_yield* d_out, void* stream) {
  return sweep_grid_reuse_parts(base, axes, n_axes, start, count, n_y, nz, z_max, d_P, const_cast<double*>(d_work),
                                work_doubles, d_out, stream, 2, "lzq_sweep_grid_from_ztables");
}

int lzq_p_closed_form(const double* d_lambda, int64_t n, double* d_P, void* stream) {
  if (n < 0 || (n > 0 && (!d_lambda || !d_P))) return fail(LZQ_EINVAL, "lzq_p_closed_form: bad arguments");
  if (n == 0) return LZQ_OK;
  int64_t nb = blocks_for(n, lzq::kBlock);
  if (nb > kMaxGrid) return fail(LZQ_EINVAL, "lzq_p_closed_form: n too large");
  hipLaunchKernelGGL(lzq::p_closed_form_kernel, dim3((unsigned)nb), dim3(lzq::kBlock), 0, (hipStream_t)stream,
                     d_lambda, n, d_P);
  LZQ_HIP(hipGetLastError());
  return LZQ_OK;
}

}  // extern "C"
