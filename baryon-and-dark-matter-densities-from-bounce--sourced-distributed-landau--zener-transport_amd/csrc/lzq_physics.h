// lzq_physics.h -- per-node thermo / cosmology ingredients of the quadrature, restated from
// /root/reference/first_principles_yields.py (fpy) in the reference's operation order.
// The library is compiled with -ffp-contract=off, so every expression below rounds exactly
// where numpy's elementwise ops do; pow/exp/sqrt are the device libm (<= 1-2 ulp apart from
// numpy's SIMD versions).
#pragma once
#include <math.h>
#include <stdint.h>

#include "lzq_exp2.h"

namespace lzq {

// fpy:33-39
constexpr double kZeta3 = 1.202056903159594;
constexpr double kPi = 3.141592653589793;
constexpr double kMplGeV = 1.220890e19;
constexpr double kS0M3 = 2891.0 * 1e6;
constexpr double kGeVToKg = 1.78266192e-27;
constexpr double kMProtonKg = 1.67262192369e-27;

LZQ_HD double pymax(double a, double b) { return (b > a) ? b : a; }  // Python max(a, b)
LZQ_HD double pymin(double a, double b) { return (b < a) ? b : a; }  // Python min(a, b)

// fpy:84-85  H = 1.66 sqrt(g*) T^2 / M_Pl  (left-to-right as written)
LZQ_HD double H_std(double T, double g_star) { return 1.66 * sqrt(g_star) * T * T / kMplGeV; }

// fpy:87-88  s = (2 pi^2 / 45) g*s T^3 ; PI**2 == pi*pi (correctly rounded pow)
LZQ_HD double s_entropy(double T, double g_star_s) {
  return (2.0 * (kPi * kPi) / 45.0) * g_star_s * pow(T, 3.0);
}

// fpy:90-107 n_chi_eq, strict relativistic test T > m/3
LZQ_HD double n_chi_eq(double T, double m, double g, int32_t stats) {
  if (T > (m / 3.0)) {
    double c_rel = (stats == 0) ? g * (3.0 * kZeta3 / (4.0 * (kPi * kPi))) : g * (kZeta3 / (kPi * kPi));
    return c_rel * pow(T, 3.0);
  }
  double coeff = g * pow(m / (2.0 * kPi), 1.5);
  return coeff * pow(T, 1.5) * exp(-m / pymax(T, 1e-30));
}

// fpy:109-120 vbar_chi
LZQ_HD double vbar_chi(double T, double m) {
  if (T > (m / 3.0)) return 1.0;
  double val = 8.0 * T / (kPi * pymax(m, 1e-20));
  return sqrt(pymax(val, 0.0));
}

// fpy:126-128 y_of_T ; (x)**2 on a Python float is pow(x, 2) == x*x
LZQ_HD double y_of_T(double T, double T_p, double B) {
  double q = T_p / pymax(T, 1e-30);
  return 0.5 * B * (q * q - 1.0);
}

// numpy.linspace element i of linspace(start, stop, n) (numpy/_core/function_base.py):
// arange(n)*step + start with two roundings; the last element is stop itself.
LZQ_HD double linspace_at(double start, double stop, double step, int64_t i, int64_t n) {
  if (i == n - 1) return stop;
  return (double)i * step + start;
}

// fpy:183-184 closed-form LZ conversion probability with the naive 1 - exp (not expm1).
LZQ_HD double p_closed_form(double lam) {
  double P = 1.0 - exp(-2.0 * kPi * pymax(lam, 0.0));
  return pymax(pymin(P, 1.0), 0.0);
}

}  // namespace lzq
