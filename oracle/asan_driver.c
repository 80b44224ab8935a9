/* Host sanitizer run of the CPU oracle (TEST INFRASTRUCTURE; SURVEY §5 "race detection /
 * sanitizers"): built with -fsanitize=address,undefined by `make -C oracle asan-check` and run
 * by tests/test_oracle_golden.py::test_oracle_under_asan_ubsan.  Exercises the quadrature
 * (shipped config, non-relativistic branch, boson, empty window, the y clamps), the closed form,
 * the ODE tables / rhs / Radau integrator (wash-out, annihilation across T = m/3, a rejected
 * window) and the OpenMP batch; prints one line and exits 0 when every result is finite where
 * it should be.  Any sanitizer report aborts with a non-zero status. */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "lzq_oracle.h"

static oracle_point base(void) {
  oracle_point p;
  memset(&p, 0, sizeof p);
  p.m_chi_GeV = 0.95; p.g_chi = 2; p.T_p_GeV = 100; p.beta_over_H = 100; p.v_w = 0.3; p.I_p = 0.34;
  p.g_star = 106.75; p.g_star_s = 106.75; p.P_chi_to_B = 0.14925839040304145; p.source_shape_sigma_y = 9;
  p.incident_flux_scale = 1.07e-9; p.T_max_over_Tp = 5; p.T_min_over_Tp = 0.001;
  p.Y_chi_init = 4.9e-10; p.has_Y_chi_init = 1; p.regime = 1; p.stats = 0;
  return p;
}

int main(void) {
  int bad = 0;
  oracle_point pts[6];
  for (int i = 0; i < 6; i++) pts[i] = base();
  pts[1].m_chi_GeV = 300; pts[1].regime = 0;              /* thermal, non-relativistic branch */
  pts[2].stats = 1; pts[2].beta_over_H = 1000;            /* boson, y_lo clamp at -80 */
  pts[3].T_min_over_Tp = 6;                               /* empty window -> 0 */
  pts[4].source_shape_sigma_y = 0; pts[4].v_w = 0;        /* the 1e-6 / 1e-12 clamps */
  pts[5].has_Y_chi_init = 0; pts[5].has_n_chi_at_Tp = 1; pts[5].n_chi_at_Tp_GeV3 = 2.5e-2;
  oracle_yield out[6];
  bad += oracle_points_batch(pts, 6, out, 4) != 0;
  for (int i = 0; i < 6; i++) bad += !isfinite(out[i].Y_B) || !isfinite(out[i].DM_over_B);
  bad += out[3].Y_B != 0.0;
  bad += fabs(out[0].Y_B / 8.720885362714675e-11 - 1) > 1e-12;
  bad += !(oracle_p_closed_form(-1.0) == 0.0) || !(oracle_p_closed_form(1e3) == 1.0);

  oracle_point q = base();
  q.T_max_over_Tp = 1.6; q.T_min_over_Tp = 0.6;
  oracle_ode o = {0.0, 1.0, 0, 0};
  oracle_yield y;
  int64_t ns = 0;
  bad += oracle_ode_point(&q, &o, 1 << 26, &y, &ns) != 0 || !isfinite(y.Y_B);
  oracle_point s = q;                                      /* sigma_v across the T = m/3 jump */
  s.m_chi_GeV = 300; s.regime = 0; s.T_max_over_Tp = 1.3; s.T_min_over_Tp = 0.2;
  oracle_ode os = {1e-9, 0.0, 0, 0};
  bad += oracle_ode_point(&s, &os, 1 << 26, &y, &ns) != 0 || !isfinite(y.Y_chi);
  oracle_point r = q;                                      /* inverted window: rejected */
  r.T_max_over_Tp = 0.5; r.T_min_over_Tp = 0.9;
  bad += oracle_ode_point(&r, &o, 1 << 26, &y, &ns) != 1;
  printf("asan/ubsan oracle run: %s (%d failures)\n", bad ? "FAIL" : "ok", bad);
  return bad ? 1 : 0;
}
