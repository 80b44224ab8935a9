#!/usr/bin/env python3
"""Golden fixtures for the A/V kernel's z grid, made by running the REFERENCE itself.

The reference operator is `AoverVKernel(I_p, beta_over_H, T_p, v_w, g_star, z_max=30.0,
nz=1200)` (fpy:141-156); main() always builds it with the defaults (fpy:197), but the operator
takes any grid, and Y_B is not converged in it (+26% / +74% at nz = 2400 / 12000).
This script builds `BoltzmannSystem(cfg, P)` (fpy:192-201), replaces its kernel with
`bs.aov = AoverVKernel(..., z_max=z_max, nz=nz)` and records, per grid:

* Y_B = bs.integrate_YB_by_quadrature(T_lo, T_hi, n_y=8000) on main()'s window (fpy:367-374)
  for the shipped config and seeded random points (the same generator as make_golden.py);
* bs.aov.A_over_V_y(y) (fpy:158-165) at a y sweep;
* bs.build_tables(T_lo, T_hi, n) (fpy:207-212) for several n, then bs.A_over_V_T(T) (fpy:214-218)
  and bs.rhs(x, Y) (fpy:270-286) at sample points;
* main()'s ODE fallback (fpy:385-410, the reference's own solve_ivp call on bs.rhs) for two
  narrow-window wash-out points on non-default grids.

Runs only in the build container (the reference never travels to the GPU box).

    python tests/golden/make_golden_zgrid.py     # ~1-2 min on 8 cores
"""
from __future__ import annotations

import json
import math
import multiprocessing as mp
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _base_cfg, _fpy, random_points  # noqa: E402

GRIDS = [(600, 30.0), (2400, 30.0), (12000, 30.0), (1200, 20.0), (1200, 60.0), (2400, 60.0), (37, 7.5),
         (1, 30.0), (0, 30.0), (5, 0.0)]
N_RANDOM = 6
Y_SWEEP = [-60.0, -45.0, -30.0, -20.0, -10.0, -5.0, -2.0, 0.0, 1.5, 3.0, 6.0, 10.0, 15.975, 25.0, 40.0, 50.0, 50.5]
TABLE_NT = [50, 200, 1600]


def _cfg_obj(fpy, c):
    d = fpy.default_config()
    d.update(c)
    return fpy.Config(**d)


def _window(cfg):
    return cfg.T_min_over_Tp * cfg.T_p_GeV, cfg.T_max_over_Tp * cfg.T_p_GeV


def _system(fpy, c, nz, z_max):
    cfg = _cfg_obj(fpy, c)
    bs = fpy.BoltzmannSystem(cfg, float(cfg.P_chi_to_B))
    bs.aov = fpy.AoverVKernel(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star, z_max=z_max, nz=nz)
    return cfg, bs


def yb_job(args):
    c, nz, z_max = args
    fpy = _fpy()
    cfg, bs = _system(fpy, c, nz, z_max)
    T_lo, T_hi = _window(cfg)
    return {"config": c, "nz": nz, "z_max": z_max, "Y_B": bs.integrate_YB_by_quadrature(T_lo, T_hi, n_y=8000)}


def aov_job(args):
    c, nz, z_max = args
    fpy = _fpy()
    cfg, bs = _system(fpy, c, nz, z_max)
    return {"config": c, "nz": nz, "z_max": z_max, "y": Y_SWEEP, "Av": [bs.aov.A_over_V_y(y) for y in Y_SWEEP]}


def table_job(args):
    c, nz, z_max, nt = args
    import numpy as np
    fpy = _fpy()
    cfg, bs = _system(fpy, c, nz, z_max)
    T_lo, T_hi = _window(cfg)
    bs.build_tables(T_lo, T_hi, n=nt)
    Ts = list(np.linspace(T_lo, T_hi, 23)) + [T_lo * 0.5, T_hi * 2.0, 0.5 * (T_lo + T_hi) + 1e-3]
    xs = [cfg.m_chi_GeV / T for T in np.geomspace(T_lo * 1.01, T_hi * 0.99, 9)]
    Ys = [[4.9e-10, 1e-11], [1e-9, 0.0], [3e-12, 2e-10]]
    rhs = [[float(v) for v in bs.rhs(x, np.array(Y, float))] for x in xs for Y in Ys]
    return {"config": c, "nz": nz, "z_max": z_max, "nt": nt, "T": [float(T) for T in Ts],
            "Av": [float(bs.A_over_V_T(float(T))) for T in Ts], "x": xs, "Y": Ys, "rhs": rhs}


def ode_job(args):
    """main()'s ODE fallback (fpy:385-410) with bs.aov on the given grid."""
    c, nz, z_max = args
    import numpy as np
    from scipy.integrate import solve_ivp
    fpy = _fpy()
    cfg, bs = _system(fpy, c, nz, z_max)
    T_lo, T_hi = _window(cfg)
    T_p = cfg.T_p_GeV
    bs.build_tables(T_lo, T_hi, n=800)
    x0 = cfg.m_chi_GeV / T_hi
    x1 = cfg.m_chi_GeV / max(T_lo, 1e-30)
    Ychi0 = float(cfg.Y_chi_init)
    x_p = cfg.m_chi_GeV / max(T_p, 1e-30)
    max_step = min(abs(x1 - x0) / 20000.0, x_p / 1000.0, 5e-4)
    sol = solve_ivp(lambda x, y: bs.rhs(x, y), (x0, x1), np.array([Ychi0, 0.0], float), method="Radau", rtol=1e-8,
                    atol=1e-12, max_step=max_step)
    return {"config": c, "nz": nz, "z_max": z_max, "success": bool(sol.success), "Y_chi": float(sol.y[0, -1]),
            "Y_B": float(sol.y[1, -1])}


def main():
    import numpy as np
    base = _base_cfg()
    pts = [base] + random_points(N_RANDOM, seed=11) + [dict(base, m_chi_GeV=300.0), dict(base, T_min_over_Tp=0.9)]
    yb_args = [(c, nz, zm) for nz, zm in GRIDS for c in (pts if nz >= 600 else pts[:2])]
    aov_args = [(c, nz, zm) for nz, zm in GRIDS for c in (base, pts[1])]
    tab_args = [(base, 1200, 30.0, nt) for nt in TABLE_NT] + [(pts[2], 2400, 20.0, 200), (base, 600, 60.0, 800)]
    ode_cfg = dict(base, Gamma_wash_over_H=0.5, T_max_over_Tp=1.6, T_min_over_Tp=0.6)
    ode_args = [(ode_cfg, 2400, 30.0), (dict(ode_cfg, deplete_DM_from_source=True, I_p=0.6), 1200, 20.0)]
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        yb = pool.map(yb_job, yb_args, chunksize=1)
        av = pool.map(aov_job, aov_args)
        tabs = pool.map(table_job, tab_args)
        odes = pool.map(ode_job, ode_args)
    out = {"generator": "tests/golden/make_golden_zgrid.py (reference fpy:141-156, 192-286, 385-410)",
           "numpy": np.__version__, "grids": GRIDS, "yields": yb, "aov": av, "tables": tabs, "ode": odes}
    path = os.path.join(HERE, "golden_zgrid.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, len(yb), "Y_B,", len(av), "A/V sweeps,", len(tabs), "tables,", len(odes), "ODE runs")
    for r in [r for r in yb if r["config"] == base]:
        print(r["nz"], r["z_max"], r["Y_B"])
    assert all(math.isfinite(r["Y_B"]) for r in yb)


if __name__ == "__main__":
    main()
