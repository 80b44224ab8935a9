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

/* fpy:141-156: z = linspace(0, z_max, nz); g4 = 6 - e^{-z}(z^3 + 3 z^2 + 6 z + 6) (verbatim). */
typedef struct { double z[ORACLE_NZ], w[ORACLE_NZ], g4[ORACLE_NZ]; } ztab_t;
static ztab_t g_ztab;
static int g_ztab_ready = 0;

static void ztab_init(void) {
  if (g_ztab_ready) return;
  oracle_linspace(0.0, ORACLE_ZMAX, ORACLE_NZ, g_ztab.z);
  for (int k = 0; k < ORACLE_NZ; k++) {
    double z = g_ztab.z[k];
    double ez = exp(-z);
    double zz = z * z; /* numpy z**2 is square() */
    g_ztab.g4[k] = 6.0 - ez * (((pow(z, 3.0) + 3.0 * zz) + 6.0 * z) + 6.0);
    g_ztab.w[k] = zz * ez; /* z**2 * exp(-z) */
  }
  g_ztab_ready = 1;
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

static double aov_eval(const aov_t* a, double y, double* f, double* scratch) {
  if (y > 50.0) return 0.0;
  double expy = exp(pymax(pymin(y, 50.0), -50.0));
  double pref = (a->I_p / 2.0) * (a->beta / a->v_w) * expy;
  double c = -(a->I_p / 6.0) * expy;
  for (int k = 0; k < ORACLE_NZ; k++) f[k] = g_ztab.w[k] * exp(c * g_ztab.g4[k]);
  double F = trapezoid(f, g_ztab.z, ORACLE_NZ, scratch);
  return pref * F;
}

double oracle_aov(double I_p, double B, double T_p, double v_w, double g_star, double y) {
  ztab_init();
  double f[ORACLE_NZ], s[ORACLE_NZ];
  aov_t a = aov_make(I_p, B, T_p, v_w, g_star);
  return aov_eval(&a, y, f, s);
}

/* fpy:231-267 integrate_YB_by_quadrature */
double oracle_yb_quadrature(const oracle_point* p, double T_lo, double T_hi, int32_t n_y) {
  ztab_init();
  double B = p->beta_over_H, Tp = p->T_p_GeV, m = p->m_chi_GeV;
  double y_lo_raw = y_of_T(T_hi, Tp, B);
  double y_hi_raw = y_of_T(T_lo, Tp, B);
  double y_lo = pymax(y_lo_raw, -80.0);
  double y_hi = pymin(y_hi_raw, +50.0);
  if (y_hi <= y_lo) return 0.0;
  int64_t n = n_y > 2000 ? n_y : 2000;

  double* ys = (double*)malloc(sizeof(double) * (size_t)n);
  double* integ = (double*)malloc(sizeof(double) * (size_t)n);
  double* scratch = (double*)malloc(sizeof(double) * (size_t)(n > ORACLE_NZ ? n : ORACLE_NZ));
  double f[ORACLE_NZ];
  oracle_linspace(y_lo, y_hi, n, ys);

  aov_t a = aov_make(p->I_p, B, Tp, p->v_w, p->g_star);
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
    double Av = aov_eval(&a, y, f, scratch);
    double q = y / sig;
    double window = exp(-0.5 * (q * q));
    double SB = p->P_chi_to_B * J * Av * window;
    integ[j] = SB / (s * H * T) * fabs(dTdy);
  }
  double r = trapezoid(integ, ys, n, scratch);
  free(ys);
  free(integ);
  free(scratch);
  return r;
}

/* fpy:361-417 (fast path only: the callers gate on fpy:372). */
int oracle_point_yields(const oracle_point* p, oracle_yield* o) {
  double T_p = p->T_p_GeV;
  double T_hi = p->T_max_over_Tp * T_p;
  double T_lo = p->T_min_over_Tp * T_p;
  double YB = oracle_yb_quadrature(p, T_lo, T_hi, 8000);
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

int64_t oracle_points_batch(const oracle_point* p, int64_t n, oracle_yield* out, int32_t nthreads) {
  ztab_init();
  int64_t bad = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : bad)
  for (int64_t i = 0; i < n; i++) {
    if (oracle_point_yields(&p[i], &out[i]) != 0) {
      bad++;
      memset(&out[i], 0xff, sizeof(oracle_yield)); /* NaN pattern */
    }
  }
  return bad;
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
