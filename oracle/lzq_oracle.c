/*
 * lzq_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY:
 * the parity checker for the HIP path and the CPU baseline timed by bench.py.  Nothing in
 * the product (include/lzq.h, the HIP library, the package's host code) links or calls it.
 *
 * Reference: /root/reference/first_principles_yields.py ("fpy").  Each function cites the
 * lines it restates.  Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 * Pinned by tests/test_oracle_golden.py against the JSON files in tests/golden, which
 * tests/golden/make_golden.py produced by executing fpy itself.
 *
 * Numerics notes: the reference's numpy uses AVX-512 exp/pow, which differ
 * from libm by <= 1 ulp; np.trapezoid reduces with numpy's pairwise summation, which is
 * reproduced here exactly (oracle_pairwise_sum).  Expected agreement with the golden
 * vectors is ~1e-13 relative, limited by those ulp differences.
 */
#include "lzq_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* fpy:33-39 */
static const double ZETA3 = 1.202056903159594;
static const double PI = 3.141592653589793;
static const double MPL_GEV = 1.220890e19;
static const double S0_M3 = 2891.0 * 1e6;
static const double GEV_TO_KG = 1.78266192e-27;
static const double M_PROTON_KG = 1.67262192369e-27;

/* fpy:142 defaults of AoverVKernel(z_max=30.0, nz=1200), used unchanged at fpy:197. */
#define ORACLE_NZ 1200
static const double ORACLE_ZMAX = 30.0;

static double pymax(double a, double b) { return (b > a) ? b : a; } /* Python max(a, b) */
static double pymin(double a, double b) { return (b < a) ? b : a; } /* Python min(a, b) */

/* numpy/_core/src/umath/loops_utils.h.src pairwise_sum for contiguous doubles. */
static double pairwise(const double* a, int64_t n) {
  if (n < 8) {
    double res = 0.0;
    for (int64_t i = 0; i < n; i++) res += a[i];
    return res;
  } else if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int64_t i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; j++) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += a[i];
    return res;
  } else {
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise(a, n2) + pairwise(a + n2, n - n2);
  }
}

/* np.add.reduce over a 1-D contiguous array (numpy 2.x): the iterator feeds the inner loop
 * in buffers of 8192 elements; each buffer is one pairwise pass added to the accumulator
 * (seeded with the identity).  Bit-exact vs numpy 2.2.6 (tests/test_oracle_golden.py). */
double oracle_pairwise_sum(const double* a, int64_t n) {
  double res = 0.0;
  for (int64_t s = 0; s < n; s += 8192) res += pairwise(a + s, (n - s) < 8192 ? (n - s) : 8192);
  return res;
}

/* numpy.linspace (numpy/_core/function_base.py): y = arange(num)*step + start; y[-1] = stop. */
void oracle_linspace(double start, double stop, int64_t num, double* out) {
  int64_t div = num - 1;
  double delta = stop - start;
  if (div > 0) {
    double step = delta / (double)div;
    if (step == 0.0) {
      for (int64_t i = 0; i < num; i++) out[i] = ((double)i / (double)div) * delta + start;
    } else {
      for (int64_t i = 0; i < num; i++) out[i] = (double)i * step + start;
    }
    out[num - 1] = stop;
  } else if (num == 1) {
    out[0] = 0.0 * delta + start;
  }
}

/* np.trapezoid(f, x) = add.reduce(diff(x) * (f[1:] + f[:-1]) / 2.0) */
static double trapezoid(const double* f, const double* x, int64_t n, double* scratch) {
  for (int64_t i = 0; i + 1 < n; i++) scratch[i] = ((x[i + 1] - x[i]) * (f[i + 1] + f[i])) / 2.0;
  return oracle_pairwise_sum(scratch, n - 1);
}

/* fpy:84-85 */
static double H_std(double T, double g_star) { return 1.66 * sqrt(g_star) * T * T / MPL_GEV; }
/* fpy:87-88 ; `PI**2` is pow(pi, 2) == pi*pi (correctly rounded), `T**3` pow */
static double s_entropy(double T, double g_star_s) {
  return (2.0 * (PI * PI) / 45.0) * g_star_s * pow(T, 3.0);
}
/* fpy:90-107 n_chi_eq (scalar form; strict T > m/3 branch) */
static double n_chi_eq(double T, double m, double g, int stats) {
  if (T > (m / 3.0)) {
    double c_rel = (stats == 0) ? g * (3.0 * ZETA3 / (4.0 * (PI * PI))) : g * (ZETA3 / (PI * PI));
    return c_rel * pow(T, 3.0);
  }
  double coeff = g * pow(m / (2.0 * PI), 1.5);
  return coeff * pow(T, 1.5) * exp(-m / pymax(T, 1e-30));
}
/* fpy:109-120 vbar_chi */
static double vbar_chi(double T, double m) {
  if (T > (m / 3.0)) return 1.0;
  double val = 8.0 * T / (PI * pymax(m, 1e-20));
  return sqrt(pymax(val, 0.0));
}
/* fpy:126-128 y_of_T ; `x**2` on a Python float is pow(x, 2) == x*x */
static double y_of_T(double T, double T_p, double B) {
  double q = T_p / pymax(T, 1e-30);
  return 0.5 * B * (q * q - 1.0);
}

/* fpy:141-156: z = linspace(0, z_max, nz); g4 = 6 - e^{-z}(z^3 + 3 z^2 + 6 z + 6) (verbatim).
 * One table per AoverVKernel z grid; the default (1200, 30) one is built once and shared. */
typedef struct {
  int64_t nz;
  double *z, *w, *g4;
} ztab_t;
static ztab_t g_ztab;
static int g_ztab_ready = 0;

static void ztab_build(ztab_t* t, int64_t nz, double z_max) {
  t->nz = nz;
  size_t n = (size_t)(nz > 0 ? nz : 1);
  t->z = (double*)malloc(sizeof(double) * n);
  t->w = (double*)malloc(sizeof(double) * n);
  t->g4 = (double*)malloc(sizeof(double) * n);
  oracle_linspace(0.0, z_max, nz, t->z);
  for (int64_t k = 0; k < nz; k++) {
    double z = t->z[k];
    double ez = exp(-z);
    double zz = z * z; /* numpy z**2 is square() */
    t->g4[k] = 6.0 - ez * (((pow(z, 3.0) + 3.0 * zz) + 6.0 * z) + 6.0);
    t->w[k] = zz * ez; /* z**2 * exp(-z) */
  }
}

static void ztab_free(ztab_t* t) {
  free(t->z);
  free(t->w);
  free(t->g4);
}

/* Double-checked initialisation with acquire/release on the flag: a thread that sees it set
 * also sees the table's pointers and contents (oracle_points_batch calls this from OpenMP). */
static void ztab_init(void) {
  if (__atomic_load_n(&g_ztab_ready, __ATOMIC_ACQUIRE)) return;
#pragma omp critical(lzq_oracle_ztab)
  {
    if (!__atomic_load_n(&g_ztab_ready, __ATOMIC_ACQUIRE)) {
      ztab_build(&g_ztab, ORACLE_NZ, ORACLE_ZMAX);
      __atomic_store_n(&g_ztab_ready, 1, __ATOMIC_RELEASE);
    }
  }
}

/* The table of grid (nz, z_max): the shared default, or a new one the caller frees (ztab_put). */
static const ztab_t* ztab_get(int64_t nz, double z_max, ztab_t* scratch) {
  if (nz == ORACLE_NZ && z_max == ORACLE_ZMAX) {
    ztab_init();
    return &g_ztab;
  }
  ztab_build(scratch, nz, z_max);
  return scratch;
}

static void ztab_put(const ztab_t* t) {
  if (t != &g_ztab) ztab_free((ztab_t*)t);
}

/* fpy:158-165 A_over_V_y, kernel constants from fpy:143-151. */
typedef struct { double I_p, beta, v_w; } aov_t;

static aov_t aov_make(double I_p, double B, double T_p, double v_w, double g_star) {
  aov_t a;
  a.I_p = I_p;
  a.v_w = pymax(v_w, 1e-12);
  double H_p = H_std(T_p, g_star);
  a.beta = B * H_p;
  return a;
}

/* The kernel of BoltzmannSystem.aov: its own parameters if given (bs.aov replaced, fpy:141-151),
 * else the one fpy:197 builds from the point (cfg). */
static aov_t aov_of(const oracle_point* p, const oracle_aov_params* av) {
  if (av) return aov_make(av->I_p, av->beta_over_H, av->T_p_GeV, av->v_w, av->g_star);
  return aov_make(p->I_p, p->beta_over_H, p->T_p_GeV, p->v_w, p->g_star);
}

/* f, scratch: >= max(nz, 1) doubles.  np.trapezoid of fewer than 2 nodes is 0.0. */
static double aov_eval(const aov_t* a, const ztab_t* zt, double y, double* f, double* scratch) {
  if (y > 50.0) return 0.0;
  double expy = exp(pymax(pymin(y, 50.0), -50.0));
  double pref = (a->I_p / 2.0) * (a->beta / a->v_w) * expy;
  double c = -(a->I_p / 6.0) * expy;
  for (int64_t k = 0; k < zt->nz; k++) f[k] = zt->w[k] * exp(c * zt->g4[k]);
  double F = zt->nz >= 2 ? trapezoid(f, zt->z, zt->nz, scratch) : 0.0;
  return pref * F;
}

double oracle_aov_z(double I_p, double B, double T_p, double v_w, double g_star, double y, int64_t nz,
                    double z_max) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  size_t n = (size_t)(nz > 1 ? nz : 1);
  double* f = (double*)malloc(sizeof(double) * n);
  double* s = (double*)malloc(sizeof(double) * n);
  aov_t a = aov_make(I_p, B, T_p, v_w, g_star);
  double r = aov_eval(&a, zt, y, f, s);
  free(f);
  free(s);
  ztab_put(zt);
  return r;
}

double oracle_aov(double I_p, double B, double T_p, double v_w, double g_star, double y) {
  return oracle_aov_z(I_p, B, T_p, v_w, g_star, y, ORACLE_NZ, ORACLE_ZMAX);
}

/* fpy:231-267 integrate_YB_by_quadrature, A/V on the grid zt */
static double yb_quadrature(const oracle_point* p, const oracle_aov_params* av, const ztab_t* zt, double T_lo, double T_hi,
                            int32_t n_y) {
  double B = p->beta_over_H, Tp = p->T_p_GeV, m = p->m_chi_GeV;
  double y_lo_raw = y_of_T(T_hi, Tp, B);
  double y_hi_raw = y_of_T(T_lo, Tp, B);
  double y_lo = pymax(y_lo_raw, -80.0);
  double y_hi = pymin(y_hi_raw, +50.0);
  if (y_hi <= y_lo) return 0.0;
  int64_t n = n_y > 2000 ? n_y : 2000;

  double* ys = (double*)malloc(sizeof(double) * (size_t)n);
  double* integ = (double*)malloc(sizeof(double) * (size_t)n);
  double* scratch = (double*)malloc(sizeof(double) * (size_t)(n > zt->nz ? n : zt->nz));
  double* f = (double*)malloc(sizeof(double) * (size_t)(zt->nz > 1 ? zt->nz : 1));
  oracle_linspace(y_lo, y_hi, n, ys);

  aov_t a = aov_of(p, av); /* fpy:261: self.aov; everything else from self.cfg (fpy:250-262) */
  double Bc = pymax(B, 1e-30);
  double sig = pymax(p->source_shape_sigma_y, 1e-6);
  double sqrtg = sqrt(p->g_star);
  for (int64_t j = 0; j < n; j++) {
    double y = ys[j];
    double denom = 1.0 + 2.0 * y / Bc;
    denom = pymax(denom, 1e-12);
    double T = Tp / sqrt(denom);
    double dTdy = -(Tp / Bc) * pow(denom, -1.5);
    double H = 1.66 * sqrtg * T * T / MPL_GEV;
    double s = (2.0 * (PI * PI) / 45.0) * p->g_star_s * pow(T, 3.0);
    double J = p->incident_flux_scale * 0.25 * n_chi_eq(T, m, p->g_chi, p->stats) * vbar_chi(T, m);
    double Av = aov_eval(&a, zt, y, f, scratch);
    double q = y / sig;
    double window = exp(-0.5 * (q * q));
    double SB = p->P_chi_to_B * J * Av * window;
    integ[j] = SB / (s * H * T) * fabs(dTdy);
  }
  double r = trapezoid(integ, ys, n, scratch);
  free(ys);
  free(integ);
  free(scratch);
  free(f);
  return r;
}

double oracle_yb_quadrature_z(const oracle_point* p, double T_lo, double T_hi, int32_t n_y, int64_t nz,
                              double z_max) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  double r = yb_quadrature(p, NULL, zt, T_lo, T_hi, n_y);
  ztab_put(zt);
  return r;
}

double oracle_yb_quadrature_a(const oracle_point* p, const oracle_aov_params* av, double T_lo, double T_hi, int32_t n_y,
                              int64_t nz, double z_max) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  double r = yb_quadrature(p, av, zt, T_lo, T_hi, n_y);
  ztab_put(zt);
  return r;
}

double oracle_yb_quadrature(const oracle_point* p, double T_lo, double T_hi, int32_t n_y) {
  return oracle_yb_quadrature_z(p, T_lo, T_hi, n_y, ORACLE_NZ, ORACLE_ZMAX);
}

/* fpy:361-417 (fast path only: the callers gate on fpy:372). */
static int point_yields(const oracle_point* p, const oracle_aov_params* av, const ztab_t* zt, oracle_yield* o) {
  double T_p = p->T_p_GeV;
  double T_hi = p->T_max_over_Tp * T_p;
  double T_lo = p->T_min_over_Tp * T_p;
  double YB = yb_quadrature(p, av, zt, T_lo, T_hi, 8000);
  double Ychi;
  if (p->regime == 0) {
    Ychi = n_chi_eq(T_hi, p->m_chi_GeV, p->g_chi, p->stats) / s_entropy(T_hi, p->g_star_s);
  } else if (p->regime == 1) {
    if (p->has_Y_chi_init) Ychi = p->Y_chi_init;
    else if (p->has_n_chi_at_Tp) Ychi = p->n_chi_at_Tp_GeV3 / pymax(s_entropy(T_p, p->g_star_s), 1e-300);
    else Ychi = 1.0e-12;
  } else {
    return -1; /* fpy:376-384 has no else: UnboundLocalError */
  }
  double nB0 = YB * S0_M3, nDM0 = Ychi * S0_M3;
  double rhoB = nB0 * M_PROTON_KG;
  double rhoDM = nDM0 * (p->m_chi_GeV * GEV_TO_KG);
  o->Y_B = YB;
  o->Y_chi = Ychi;
  o->rho_B_kg_m3 = rhoB;
  o->rho_DM_kg_m3 = rhoDM;
  o->DM_over_B = rhoDM / pymax(rhoB, 1e-300);
  o->P_used = p->P_chi_to_B;
  return 0;
}

int oracle_point_yields_z(const oracle_point* p, int64_t nz, double z_max, oracle_yield* o) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  int r = point_yields(p, NULL, zt, o);
  ztab_put(zt);
  return r;
}

int oracle_point_yields_a(const oracle_point* p, const oracle_aov_params* av, int64_t nz, double z_max, oracle_yield* o) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  int r = point_yields(p, av, zt, o);
  ztab_put(zt);
  return r;
}

int oracle_point_yields(const oracle_point* p, oracle_yield* o) {
  return oracle_point_yields_z(p, ORACLE_NZ, ORACLE_ZMAX, o);
}

int64_t oracle_points_batch_z(const oracle_point* p, int64_t n, int64_t nz, double z_max, oracle_yield* out,
                              int32_t nthreads) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  int64_t bad = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : bad)
  for (int64_t i = 0; i < n; i++) {
    if (point_yields(&p[i], NULL, zt, &out[i]) != 0) {
      bad++;
      memset(&out[i], 0xff, sizeof(oracle_yield)); /* NaN pattern */
    }
  }
  ztab_put(zt);
  return bad;
}

int64_t oracle_points_batch(const oracle_point* p, int64_t n, oracle_yield* out, int32_t nthreads) {
  return oracle_points_batch_z(p, n, ORACLE_NZ, ORACLE_ZMAX, out, nthreads);
}

/* fpy:183-184 */
double oracle_p_closed_form(double lam) {
  double P = 1.0 - exp(-2.0 * PI * pymax(lam, 0.0));
  return pymax(pymin(P, 1.0), 0.0);
}

/* fpy:222-223 J_chi = flux * J_chi_flux(T) with fpy:122-123 J_chi_flux = 0.25 n v */
double oracle_j_chi(const oracle_point* p, double T) {
  return p->incident_flux_scale * (0.25 * n_chi_eq(T, p->m_chi_GeV, p->g_chi, p->stats) * vbar_chi(T, p->m_chi_GeV));
}

/* =======================================================================================
 * ODE fallback (fpy:200-219 build_tables / A_over_V_T, fpy:270-286 rhs, fpy:385-410 main).
 * The reference integrates with scipy's adaptive Radau (rtol 1e-8, atol 1e-12, max_step of
 * fpy:404).  Restated here as the same Radau IIA (3 stages, order 5) on uniform steps of
 * h = (x1 - x0)/ceil(|x1 - x0|/max_step) <= max_step, each stage system solved by Newton with
 * the rhs' analytic (diagonal) Jacobian to full precision.  tests/golden/golden_ode.json
 * shows the reference's shipped solution within ~1e-14 of its own converged one, so the
 * restatement is pinned against the shipped outputs at that level.
 * ======================================================================================= */
#define ODE_NT 800

/* scipy.interpolate.CubicSpline(x, y, bc_type='not-a-knot') for n = ODE_NT points
 * (scipy/interpolate/_cubic.py: banded system for the knot slopes s, then the PPoly
 * coefficients of CubicHermiteSpline).  The tridiagonal solve is Thomas elimination
 * (scipy: LAPACK gbsv with partial pivoting; the two agree to rounding).  coef[4k+0..3] =
 * c[0..3][k], the PPoly coefficients of interval k (value c0 s^3 + c1 s^2 + c2 s + c3). */
static void spline_notaknot(const double* x, const double* y, int n, double* coef) {
  double* buf = (double*)malloc(sizeof(double) * 5 * (size_t)n);
  double *dx = buf, *slope = buf + n, *cp = buf + 2 * n, *dp = buf + 3 * n, *s = buf + 4 * n;
  for (int k = 0; k + 1 < n; k++) {
    dx[k] = x[k + 1] - x[k];
    slope[k] = (y[k + 1] - y[k]) / dx[k];
  }
  /* row 0 (not-a-knot): dx1 s0 + (x2 - x0) s1 = ((dx0 + 2d) dx1 slope0 + dx0^2 slope1)/d */
  {
    double d = x[2] - x[0];
    double b = dx[1], c = d;
    double r = ((dx[0] + 2.0 * d) * dx[1] * slope[0] + (dx[0] * dx[0]) * slope[1]) / d;
    cp[0] = c / b;
    dp[0] = r / b;
  }
  for (int k = 1; k < n - 1; k++) {
    double a = dx[k], b = 2.0 * (dx[k - 1] + dx[k]), c = dx[k - 1];
    double r = 3.0 * (dx[k] * slope[k - 1] + dx[k - 1] * slope[k]);
    double den = b - a * cp[k - 1];
    cp[k] = c / den;
    dp[k] = (r - a * dp[k - 1]) / den;
  }
  {
    double d = x[n - 1] - x[n - 3];
    double a = d, b = dx[n - 3];
    double r = ((dx[n - 2] * dx[n - 2]) * slope[n - 3] + (2.0 * d + dx[n - 2]) * dx[n - 3] * slope[n - 2]) / d;
    s[n - 1] = (r - a * dp[n - 2]) / (b - a * cp[n - 2]);
  }
  for (int k = n - 2; k >= 0; k--) s[k] = dp[k] - cp[k] * s[k + 1];
  for (int k = 0; k + 1 < n; k++) {
    double t = (s[k] + s[k + 1] - 2.0 * slope[k]) / dx[k];
    coef[4 * k + 0] = t / dx[k];
    coef[4 * k + 1] = (slope[k] - s[k]) / dx[k] - t;
    coef[4 * k + 2] = s[k];
    coef[4 * k + 3] = y[k];
  }
  free(buf);
}

/* build_tables(T_lo, T_hi, n=nt) with self.aov on the grid zt. */
static int ode_tables(const oracle_point* p, const oracle_aov_params* av, const ztab_t* zt, double T_lo, double T_hi, int nt,
                      double* coef) {
  size_t nzb = (size_t)(zt->nz > 1 ? zt->nz : 1);
  double* Ts = (double*)malloc(sizeof(double) * 2 * (size_t)nt);
  double* Av = Ts + nt;
  double* f = (double*)malloc(sizeof(double) * 2 * nzb);
  double* scratch = f + nzb;
  int rc = 0;
  oracle_linspace(T_lo, T_hi, nt, Ts);
  for (int k = 0; k + 1 < nt; k++)
    if (!(Ts[k + 1] > Ts[k])) rc = -1; /* CubicSpline: `x` must be strictly increasing */
  if (rc == 0) {
    aov_t a = aov_of(p, av); /* fpy:211: A/V from self.aov, y(T) from self.cfg */
    for (int k = 0; k < nt; k++) {
      double y = y_of_T(Ts[k], p->T_p_GeV, p->beta_over_H);
      Av[k] = pymax(aov_eval(&a, zt, y, f, scratch), 0.0); /* np.maximum(Av, 0.0) */
    }
    spline_notaknot(Ts, Av, nt, coef);
  }
  free(Ts);
  free(f);
  return rc;
}

int oracle_ode_tables_z(const oracle_point* p, double T_lo, double T_hi, int32_t nt, int64_t nz, double z_max,
                        double* coef) {
  if (nt < 4) return -2;
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  int rc = ode_tables(p, NULL, zt, T_lo, T_hi, nt, coef);
  ztab_put(zt);
  return rc;
}

int oracle_ode_tables_a(const oracle_point* p, const oracle_aov_params* av, double T_lo, double T_hi, int32_t nt, int64_t nz,
                        double z_max, double* coef) {
  if (nt < 4) return -2;
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  int rc = ode_tables(p, av, zt, T_lo, T_hi, nt, coef);
  ztab_put(zt);
  return rc;
}

int oracle_ode_tables(const oracle_point* p, double T_lo, double T_hi, double* coef) {
  return oracle_ode_tables_z(p, T_lo, T_hi, ODE_NT, ORACLE_NZ, ORACLE_ZMAX, coef);
}

/* fpy:214-218 A_over_V_T: clamp T into [T_lo, T_hi], evaluate the PPoly (scipy _ppoly:
 * interval k with x[k] <= T < x[k+1], T == x[-1] in the last one; value accumulated as
 * c3 + c2 s + c1 s^2 + c0 s^3, powers by repeated multiplication). */
static double ode_aov_T(const double* coef, int nt, double T_lo, double T_hi, double T) {
  double stackbuf[ODE_NT]; /* main()'s tables (the integrator's rhs) need no allocation */
  double* Ts = nt <= ODE_NT ? stackbuf : (double*)malloc(sizeof(double) * (size_t)nt);
  oracle_linspace(T_lo, T_hi, nt, Ts);
  double Tq = pymin(pymax(T, T_lo), T_hi);
  int lo = 0, hi = nt - 1; /* largest k <= n-2 with Ts[k] <= Tq */
  while (hi - lo > 1) {
    int mid = (lo + hi) / 2;
    if (Ts[mid] <= Tq) lo = mid;
    else hi = mid;
  }
  const double* c = coef + 4 * lo;
  double s = Tq - Ts[lo];
  if (Ts != stackbuf) free(Ts);
  double z = s, res = c[3];
  res = res + c[2] * z;
  z = z * s;
  res = res + c[1] * z;
  z = z * s;
  res = res + c[0] * z;
  return res;
}

double oracle_ode_aov_T_n(const double* coef, int32_t nt, double T_lo, double T_hi, double T) {
  return ode_aov_T(coef, nt, T_lo, T_hi, T);
}

double oracle_ode_aov_T(const double* coef, double T_lo, double T_hi, double T) {
  return ode_aov_T(coef, ODE_NT, T_lo, T_hi, T);
}

typedef struct {
  const oracle_point* p;
  const oracle_ode* o;
  const double* coef;
  double T_lo, T_hi;
  int nt;
} ode_ctx;

/* fpy:270-286 rhs(x, Y), plus the diagonal of its Jacobian (the two equations decouple). */
static void ode_rhs(const ode_ctx* c, double x, const double Y[2], double dY[2], double J[2]) {
  const oracle_point* p = c->p;
  double m = p->m_chi_GeV;
  double T = m / pymax(x, 1e-30);
  double H = pymax(H_std(T, p->g_star), 1e-300);
  double s = pymax(s_entropy(T, p->g_star_s), 1e-300);
  double y = y_of_T(T, p->T_p_GeV, p->beta_over_H);
  double q = y / pymax(p->source_shape_sigma_y, 1e-6);
  double window = exp(-0.5 * (q * q));
  double J_chi = p->incident_flux_scale * (0.25 * n_chi_eq(T, m, p->g_chi, p->stats) * vbar_chi(T, m));
  double SB = p->P_chi_to_B * J_chi * ode_aov_T(c->coef, c->nt, c->T_lo, c->T_hi, T) * window;
  double sigmav = pymax(c->o->sigma_v_chi_GeV_m2, 0.0);
  double Yeq = n_chi_eq(T, m, p->g_chi, p->stats) / s;
  double SB_term = c->o->deplete_DM_from_source ? (SB / s) : 0.0;
  double Hx = H * x;
  dY[0] = (-sigmav * s * (Y[0] * Y[0] - Yeq * Yeq) - SB_term) / Hx;
  double gamma_w = pymax(c->o->Gamma_wash_over_H, 0.0);
  dY[1] = (+SB / s - gamma_w * H * Y[1]) / Hx;
  J[0] = (-sigmav * s * (2.0 * Y[0])) / Hx;
  J[1] = (-gamma_w * H) / Hx;
}

void oracle_ode_rhs_n(const oracle_point* p, const oracle_ode* o, const double* coef, int32_t nt, double T_lo,
                      double T_hi, double x, const double* Y, double* dY) {
  ode_ctx c = {p, o, coef, T_lo, T_hi, nt};
  double J[2];
  ode_rhs(&c, x, Y, dY, J);
}

void oracle_ode_rhs(const oracle_point* p, const oracle_ode* o, const double* coef, double T_lo, double T_hi,
                    double x, const double* Y, double* dY) {
  oracle_ode_rhs_n(p, o, coef, ODE_NT, T_lo, T_hi, x, Y, dY);
}

/* 3x3 solve with partial pivoting (M is overwritten). */
static void solve3(double M[3][3], double b[3]) {
  for (int c = 0; c < 3; c++) {
    int piv = c;
    for (int r = c + 1; r < 3; r++)
      if (fabs(M[r][c]) > fabs(M[piv][c])) piv = r;
    if (piv != c) {
      for (int k = 0; k < 3; k++) {
        double t = M[c][k];
        M[c][k] = M[piv][k];
        M[piv][k] = t;
      }
      double t = b[c];
      b[c] = b[piv];
      b[piv] = t;
    }
    for (int r = c + 1; r < 3; r++) {
      double f = M[r][c] / M[c][c];
      for (int k = c; k < 3; k++) M[r][k] -= f * M[c][k];
      b[r] -= f * b[c];
    }
  }
  for (int c = 2; c >= 0; c--) {
    double acc = b[c];
    for (int k = c + 1; k < 3; k++) acc -= M[c][k] * b[k];
    b[c] = acc / M[c][c];
  }
}

/* Radau IIA tableau (scipy/integrate/_ivp/radau.py uses the same method). */
static void radau_tableau(double C[3], double A[3][3]) {
  double s6 = sqrt(6.0);
  C[0] = (4.0 - s6) / 10.0;
  C[1] = (4.0 + s6) / 10.0;
  C[2] = 1.0;
  A[0][0] = (88.0 - 7.0 * s6) / 360.0;
  A[0][1] = (296.0 - 169.0 * s6) / 1800.0;
  A[0][2] = (-2.0 + 3.0 * s6) / 225.0;
  A[1][0] = (296.0 + 169.0 * s6) / 1800.0;
  A[1][1] = (88.0 + 7.0 * s6) / 360.0;
  A[1][2] = (-2.0 - 3.0 * s6) / 225.0;
  A[2][0] = (16.0 - s6) / 36.0;
  A[2][1] = (16.0 + s6) / 36.0;
  A[2][2] = 1.0 / 9.0;
}

/* One Radau IIA step of size h from (x, Y).  Returns 0, or 4 when Newton does not converge. */
static int radau_step(const ode_ctx* c, const double C[3], const double A[3][3], double x, double h, double Y[2]) {
  double Z[3][2], F[3][2], J[3][2];
  for (int i = 0; i < 3; i++) Z[i][0] = Y[0], Z[i][1] = Y[1];
  for (int it = 0; it < 40; it++) {
    for (int i = 0; i < 3; i++) ode_rhs(c, x + C[i] * h, Z[i], F[i], J[i]);
    double dmax = 0.0, zmax = 0.0;
    for (int comp = 0; comp < 2; comp++) {
      double M[3][3], g[3];
      for (int i = 0; i < 3; i++) {
        double acc = Z[i][comp] - Y[comp];
        for (int j = 0; j < 3; j++) {
          acc -= h * A[i][j] * F[j][comp];
          M[i][j] = (i == j ? 1.0 : 0.0) - h * A[i][j] * J[j][comp];
        }
        g[i] = -acc;
      }
      solve3(M, g);
      for (int i = 0; i < 3; i++) {
        Z[i][comp] += g[i];
        dmax = pymax(dmax, fabs(g[i]));
        zmax = pymax(zmax, fabs(Z[i][comp]));
      }
    }
    if (!(dmax > 1e-15 * zmax)) {
      Y[0] = Z[2][0];
      Y[1] = Z[2][1];
      return 0;
    }
  }
  return 4;
}

/* fpy:361-417 for a point on the ODE path; status 0 ok, 1 bad T grid (CubicSpline raises),
 * 2 max_step <= 0 (solve_ivp raises), 3 more than max_steps steps, 4 Newton failure. */
static int ode_point(const oracle_point* p, const oracle_ode* o, const oracle_aov_params* av, const ztab_t* zt,
                     int64_t max_steps, oracle_yield* out, int64_t* n_steps) {
  double T_p = p->T_p_GeV, m = p->m_chi_GeV;
  double T_hi = p->T_max_over_Tp * T_p, T_lo = p->T_min_over_Tp * T_p;
  double* coef = (double*)malloc(sizeof(double) * 4 * ODE_NT);
  int st = 0;
  *n_steps = 0;
  memset(out, 0xff, sizeof(*out)); /* NaN unless filled */
  if (ode_tables(p, av, zt, T_lo, T_hi, ODE_NT, coef) != 0) {
    free(coef);
    return 1;
  }
  double x0 = m / T_hi, x1 = m / pymax(T_lo, 1e-30);
  double Ychi0;
  if (p->regime == 1) {
    if (p->has_Y_chi_init) Ychi0 = p->Y_chi_init;
    else if (p->has_n_chi_at_Tp) Ychi0 = p->n_chi_at_Tp_GeV3 / pymax(s_entropy(T_p, p->g_star_s), 1e-300);
    else Ychi0 = 1.0e-12;
  } else { /* thermal, and the else-branch of fpy:398-399 */
    Ychi0 = n_chi_eq(T_hi, m, p->g_chi, p->stats) / s_entropy(T_hi, p->g_star_s);
  }
  double x_p = m / pymax(T_p, 1e-30);
  double max_step = pymin(pymin(fabs(x1 - x0) / 20000.0, x_p / 1000.0), 5e-4);
  if (!(max_step > 0.0)) {
    free(coef);
    return 2;
  }
  double steps = ceil(fabs(x1 - x0) / max_step);
  if (!(steps <= (double)max_steps)) {
    free(coef);
    return 3;
  }
  int64_t N = (int64_t)steps;
  double h = (x1 - x0) / (double)N;
  double C[3], A[3][3];
  radau_tableau(C, A);
  ode_ctx c = {p, o, coef, T_lo, T_hi, ODE_NT};
  double Y[2] = {Ychi0, 0.0};
  /* n_chi_eq / vbar_chi switch formula at the strict T > m/3 (fpy:100, 111): the rhs jumps at
   * the first x whose T = m/max(x, 1e-30) is not > m/3.  A step that straddles that point is
   * split there (ending one ulp before it), so no Radau stage sees both branches: the fixed
   * step then stays 5th order across the jump (tests/golden/golden_ode_stiff.json). */
  double xb = INFINITY;
  {
    const double m3 = m / 3.0;
    double xg = 3.0;
    if (m / xg > m3) {
      while (m / xg > m3) xg = nextafter(xg, INFINITY);
    } else {
      while (m / nextafter(xg, -INFINITY) <= m3) xg = nextafter(xg, -INFINITY);
    }
    if (x0 < xg && xg < x1) xb = xg;
  }
  for (int64_t k = 0; k < N && st == 0; k++) {
    const double xk = x0 + (double)k * h;
    if (xk < xb && xb <= xk + h) { /* the step's last stage (x = xk + h) would see the other branch */
      const double xa = nextafter(xb, -INFINITY);
      if (xa > xk) st = radau_step(&c, C, A, xk, xa - xk, Y);
      if (st == 0 && xk + h > xb) st = radau_step(&c, C, A, xb, (xk + h) - xb, Y);
    } else {
      st = radau_step(&c, C, A, xk, h, Y);
    }
  }
  free(coef);
  *n_steps = N;
  if (st != 0 && st != 4) return st;
  /* status 4 (Newton failure): the state at the start of the failed step, as the reference
   * reports sol.y[:, -1] after a failed solve_ivp (fpy:408-410) */
  double YB = Y[1], Ychi = Y[0];
  double rhoB = YB * S0_M3 * M_PROTON_KG;
  double rhoDM = Ychi * S0_M3 * (m * GEV_TO_KG);
  out->Y_B = YB;
  out->Y_chi = Ychi;
  out->rho_B_kg_m3 = rhoB;
  out->rho_DM_kg_m3 = rhoDM;
  out->DM_over_B = rhoDM / pymax(rhoB, 1e-300);
  out->P_used = p->P_chi_to_B;
  return st;
}

int oracle_ode_point_z(const oracle_point* p, const oracle_ode* o, int64_t nz, double z_max, int64_t max_steps,
                       oracle_yield* out, int64_t* n_steps) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  int r = ode_point(p, o, NULL, zt, max_steps, out, n_steps);
  ztab_put(zt);
  return r;
}

int oracle_ode_point_a(const oracle_point* p, const oracle_ode* o, const oracle_aov_params* av, int64_t nz, double z_max,
                       int64_t max_steps, oracle_yield* out, int64_t* n_steps) {
  ztab_t own;
  const ztab_t* zt = ztab_get(nz, z_max, &own);
  int r = ode_point(p, o, av, zt, max_steps, out, n_steps);
  ztab_put(zt);
  return r;
}

int oracle_ode_point(const oracle_point* p, const oracle_ode* o, int64_t max_steps, oracle_yield* out,
                     int64_t* n_steps) {
  return oracle_ode_point_z(p, o, ORACLE_NZ, ORACLE_ZMAX, max_steps, out, n_steps);
}

int64_t oracle_ode_batch(const oracle_point* p, const oracle_ode* o, int64_t n, int64_t max_steps, oracle_yield* out,
                         int32_t* status, int32_t nthreads) {
  ztab_init();
  int64_t bad = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : bad)
  for (int64_t i = 0; i < n; i++) {
    int64_t ns;
    int st = oracle_ode_point(&p[i], &o[i], max_steps, &out[i], &ns);
    if (status) status[i] = st;
    bad += st != 0;
  }
  return bad;
}
