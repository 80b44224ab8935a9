// lzq_aov.hip -- the quadrature kernels for a BoltzmannSystem whose A/V kernel has parameters of
// its own (fpy = /root/reference/first_principles_yields.py).
//
// The reference composes two objects: the outer integrand of integrate_YB_by_quadrature reads
// self.cfg (y-grid, T(y), H, s, J, window: fpy:234-262) while A/V is self.aov.A_over_V_y
// (fpy:261), an AoverVKernel built from its own (I_p, beta_over_H, T_p, v_w, g_star)
// (fpy:141-151).  main() builds it from cfg (fpy:197), but bs.aov is a public attribute: a caller
// that replaces it integrates cfg's integrand against another kernel's A/V.  build_tables does
// the same (y(T) from cfg, A/V from self.aov: fpy:211), and so does S_B_T (fpy:226-228).
//
// The kernels here are the headline ones (lzq_quad.h: same setup, same z-sum, same y-loop, same
// epilogue) with the A/V constants of fpy:162-163, pref0 = (I_p/2)(beta/v_w) and c = -I_p/6,
// taken from a per-point lzq_aov_params block instead of the point.  They live in their own
// translation unit so the headline code object (lzq_kernels.hip, whose rocprof PMC profile the
// bench's roofline is tied to by hash) is unchanged by them.
#include <hip/hip_runtime.h>

#define LZQ_QUAD_CONST_LINKAGE static
#include "lzq_quad.h"
#include "lzq_internal.h"

namespace lzq {

// fpy:146-151 + fpy:162-163: the A/V kernel's constants, in the reference's rounding order
// (quad_setup forms the same two values from the point)
__device__ __forceinline__ void aov_override(QuadSetup& s, const lzq_aov_params& a) {
  const double v_w = pymax(a.v_w, 1e-12);           // fpy:146
  const double H_p = H_std(a.T_p_GeV, a.g_star);    // fpy:150
  const double beta = a.beta_over_H * H_p;          // fpy:151
  s.pref0 = uniform((a.I_p / 2.0) * (beta / v_w));  // fpy:162
  s.cneg = uniform(-(a.I_p / 6.0));                 // fpy:163
}

// lzq_yields_batch with d_aov: yields_points_kernel (lzq_kernels.hip) with the A/V constants of aov[idx]
template <int YB, int EXPV, int NZ>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void yields_points_aov_kernel(
    const lzq_point* __restrict__ pts, const lzq_aov_params* __restrict__ aov, int64_t n, int32_t n_y,
    const double* __restrict__ T_lo, const double* __restrict__ T_hi, const double* __restrict__ Pov,
    const ZNode* __restrict__ zt, int32_t nzp, const double* __restrict__ gtab, lzq_yield* __restrict__ out,
    int truncate) {
  __shared__ double lds_tab[kTabN];
  const double* tab = stage_table<EXPV>(gtab, lds_tab);
  __shared__ WaveSlot slots[kWavesPerBlock];
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t idx = (int64_t)blockIdx.x * kWavesPerBlock + w;
  if (idx >= n) return;  // wave-uniform
  {
    const lzq_point pt = pts[idx];
    const double P = Pov ? Pov[idx] : pt.P_chi_to_B;
    const double tlo = T_lo ? T_lo[idx] : pt.T_min_over_Tp * pt.T_p_GeV;  // fpy:369
    const double thi = T_hi ? T_hi[idx] : pt.T_max_over_Tp * pt.T_p_GeV;  // fpy:368
    QuadSetup s = quad_setup(pt, P, tlo, thi, n_y);                       // cfg: fpy:234-262
    aov_override(s, aov[idx]);                                            // self.aov: fpy:261
    park(slots[w], s, epilogue_pre(pt, P), lane);
  }
  point_yields<YB, EXPV, NZ>(slots, w, zt, nzp, tab, lane, truncate, out + idx);
}

// lzq_ode_tables with d_aov: build_tables (fpy:207-212) with y(T) from the point (cfg) and A/V
// from aov[idx] (self.aov); ode_aov_table_kernel (lzq_kernels.hip) otherwise
template <int EXPV>
__global__ __launch_bounds__(kBlock, LZQ_MIN_WAVES) void ode_aov_table_aov_kernel(
    const lzq_point* __restrict__ pts, const lzq_aov_params* __restrict__ aov, int64_t n, int32_t nt,
    const ZNode* __restrict__ zt, int32_t nzp, const double* __restrict__ gtab, const double* __restrict__ Tlo,
    const double* __restrict__ Thi, double* __restrict__ ws, int truncate,
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
  const double Tp = uniform(pt.T_p_GeV), B = uniform(pt.beta_over_H);  // fpy:211 y_of_T(T, cfg.T_p, cfg.beta/H)
  const double T_lo = uniform(Tlo ? Tlo[idx] : pt.T_min_over_Tp * Tp);
  const double T_hi = uniform(Thi ? Thi[idx] : pt.T_max_over_Tp * Tp);
  const double stepT = uniform((T_hi - T_lo) / (double)(nt - 1));
  QuadSetup s;
  aov_override(s, aov[idx]);
  const double pref0 = s.pref0, cneg = s.cneg;
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

}  // namespace lzq

int lzq::launch_yields_points_aov(int exp_variant, bool default_grid, const lzq_point* d_points,
                                  const lzq_aov_params* d_aov, int64_t n, int32_t n_y, const double* d_T_lo,
                                  const double* d_T_hi, const double* d_P, const ZNode* zt, int32_t nzp,
                                  const double* gtab, lzq_yield* d_out, int truncate, hipStream_t s) {
  const int64_t nb = (n + kWavesPerBlock - 1) / kWavesPerBlock;
#define LZQ_POINTS_AOV(EXPV, NZ)                                                                                   \
  hipLaunchKernelGGL((yields_points_aov_kernel<kYB, EXPV, NZ>), dim3((unsigned)nb), dim3(kBlock), 0, s, d_points, \
                     d_aov, n, n_y, d_T_lo, d_T_hi, d_P, zt, nzp, gtab, d_out, truncate)
  if (exp_variant == kExpTable) {
    if (default_grid) LZQ_POINTS_AOV(kExpTable, kNZ);
    else LZQ_POINTS_AOV(kExpTable, 0);
  } else {
    if (default_grid) LZQ_POINTS_AOV(kExpPoly11, kNZ);
    else LZQ_POINTS_AOV(kExpPoly11, 0);
  }
#undef LZQ_POINTS_AOV
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LZQ_OK : lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
}

int lzq::launch_ode_aov_tables_aov(int exp_variant, const lzq_point* d_points, const lzq_aov_params* d_aov,
                                   int64_t n, int32_t nt, const ZNode* zt, int32_t nzp, const double* gtab,
                                   const double* d_T_lo, const double* d_T_hi, double* d_work, int truncate,
                                   hipStream_t s, int chunks) {
  const int64_t nb = (n * chunks + kWavesPerBlock - 1) / kWavesPerBlock;
  if (exp_variant == kExpTable)
    hipLaunchKernelGGL(ode_aov_table_aov_kernel<kExpTable>, dim3((unsigned)nb), dim3(kBlock), 0, s, d_points, d_aov,
                       n, nt, zt, nzp, gtab, d_T_lo, d_T_hi, d_work, truncate, chunks);
  else
    hipLaunchKernelGGL(ode_aov_table_aov_kernel<kExpPoly11>, dim3((unsigned)nb), dim3(kBlock), 0, s, d_points, d_aov,
                       n, nt, zt, nzp, gtab, d_T_lo, d_T_hi, d_work, truncate, chunks);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LZQ_OK : lzq_set_error(LZQ_EHIP, hipGetErrorString(e));
}
