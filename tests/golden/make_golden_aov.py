#!/usr/bin/env python3
"""Golden fixtures for a BoltzmannSystem whose A/V kernel is NOT the one built from its config,
made by running the REFERENCE itself.

BoltzmannSystem.__init__ builds `self.aov = AoverVKernel(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV,
cfg.v_w, cfg.g_star)` (fpy:197), but `aov` is an independent public object with its own
parameters (fpy:141-151): integrate_YB_by_quadrature takes A/V from it (fpy:261) while the
y-grid, T(y), H, s, J and window come from self.cfg (fpy:234-262); build_tables (fpy:211) and
S_B_T (fpy:228) do the same.  This script replaces `bs.aov` with
`AoverVKernel(I_p', beta_over_H', T_p', v_w', g_star', z_max, nz)`, the primed values differing
from cfg's (one field at a time, then all of them), and records:

* Y_B = bs.integrate_YB_by_quadrature(T_lo, T_hi, n_y=8000) on main()'s window (fpy:367-374);
* bs.aov.A_over_V_y(y) (fpy:158-165) at a y sweep and bs.S_B_T(T) (fpy:225-228) at a T sweep;
* bs.build_tables(T_lo, T_hi, n=800) (fpy:207-212), then bs.A_over_V_T(T) (fpy:214-218) and
  bs.rhs(x, Y) (fpy:270-286) at sample points;
* main()'s ODE fallback (fpy:385-410: build_tables + the reference's own solve_ivp on bs.rhs) on
  narrow-window wash-out points.

Runs only in the build container (the reference never travels to the GPU box).

    python tests/golden/make_golden_aov.py     # ~1 min on 8 cores
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

AOV_FIELDS = ("I_p", "beta_over_H", "T_p", "v_w", "g_star")
Y_SWEEP = [-60.0, -30.0, -10.0, -2.0, 0.0, 1.5, 6.0, 15.975, 30.0, 45.0, 50.0, 50.5]


def _cfg_obj(fpy, c):
    d = fpy.default_config()
    d.update(c)
    return fpy.Config(**d)


def _window(cfg):
    return cfg.T_min_over_Tp * cfg.T_p_GeV, cfg.T_max_over_Tp * cfg.T_p_GeV


def _own_aov(c) -> dict:
    """The kernel main() builds from config c (fpy:197)."""
    return {"I_p": c["I_p"], "beta_over_H": c["beta_over_H"], "T_p": c["T_p_GeV"], "v_w": c["v_w"],
            "g_star": c["g_star"]}


def _system(fpy, c, aov, nz=1200, z_max=30.0):
    cfg = _cfg_obj(fpy, c)
    bs = fpy.BoltzmannSystem(cfg, float(cfg.P_chi_to_B))
    bs.aov = fpy.AoverVKernel(aov["I_p"], aov["beta_over_H"], aov["T_p"], aov["v_w"], aov["g_star"], z_max=z_max,
                              nz=nz)
    return cfg, bs


def cases():
    """(config, aov, nz, z_max) with aov != the config's own kernel."""
    import numpy as np
    rng = np.random.default_rng(29)
    base = _base_cfg()
    out = []
    # one field of the kernel changed at a time, on the shipped config
    for f, v in (("I_p", 0.51), ("I_p", 0.12), ("beta_over_H", 250.0), ("beta_over_H", 40.0), ("T_p", 140.0),
                 ("T_p", 60.0), ("v_w", 0.7), ("v_w", 0.05), ("g_star", 60.0), ("v_w", 0.0)):
        out.append((base, dict(_own_aov(base), **{f: v}), 1200, 30.0))
    # every field changed, on random configs (the make_golden.py generator, its own seed)
    for c in [base] + random_points(11, seed=41):
        a = _own_aov(c)
        a = {"I_p": float(a["I_p"] * 10 ** rng.uniform(-0.5, 0.4)),
             "beta_over_H": float(a["beta_over_H"] * 10 ** rng.uniform(-0.6, 0.6)),
             "T_p": float(a["T_p"] * 10 ** rng.uniform(-0.3, 0.3)),
             "v_w": float(rng.uniform(0.05, 0.95)), "g_star": float(rng.uniform(10.0, 110.0))}
        out.append((c, a, 1200, 30.0))
    # the same with a non-default z grid (AoverVKernel(..., z_max, nz), fpy:141-142)
    out.append((base, dict(_own_aov(base), I_p=0.6, v_w=0.45), 2400, 45.0))
    out.append((out[12][0], out[12][1], 600, 20.0))
    return out


def yb_job(args):
    c, a, nz, z_max = args
    fpy = _fpy()
    cfg, bs = _system(fpy, c, a, nz, z_max)
    T_lo, T_hi = _window(cfg)
    Ts = [cfg.T_p_GeV * r for r in (0.3, 0.7, 0.95, 1.0, 1.08, 1.5, 3.0)]
    return {"config": c, "aov": a, "nz": nz, "z_max": z_max,
            "Y_B": bs.integrate_YB_by_quadrature(T_lo, T_hi, n_y=8000),
            "y": Y_SWEEP, "Av": [bs.aov.A_over_V_y(y) for y in Y_SWEEP],
            "T_SB": Ts, "S_B": [bs.S_B_T(T) for T in Ts]}


def table_job(args):
    c, a, nz, z_max = args
    import numpy as np
    fpy = _fpy()
    cfg, bs = _system(fpy, c, a, nz, z_max)
    T_lo, T_hi = _window(cfg)
    bs.build_tables(T_lo, T_hi, n=800)
    Ts = list(np.linspace(T_lo, T_hi, 23)) + [T_lo * 0.5, T_hi * 2.0, 0.5 * (T_lo + T_hi) + 1e-3]
    xs = [cfg.m_chi_GeV / T for T in np.geomspace(T_lo * 1.01, T_hi * 0.99, 9)]
    Ys = [[4.9e-10, 1e-11], [1e-9, 0.0], [3e-12, 2e-10]]
    rhs = [[float(v) for v in bs.rhs(x, np.array(Y, float))] for x in xs for Y in Ys]
    return {"config": c, "aov": a, "nz": nz, "z_max": z_max, "nt": 800, "T": [float(T) for T in Ts],
            "Av": [float(bs.A_over_V_T(float(T))) for T in Ts], "x": xs, "Y": Ys, "rhs": rhs}


def ode_job(args):
    """main()'s ODE fallback (fpy:385-410) with the replaced bs.aov."""
    c, a, nz, z_max = args
    import numpy as np
    from scipy.integrate import solve_ivp
    fpy = _fpy()
    cfg, bs = _system(fpy, c, a, nz, z_max)
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
    return {"config": c, "aov": a, "nz": nz, "z_max": z_max, "success": bool(sol.success),
            "Y_chi": float(sol.y[0, -1]), "Y_B": float(sol.y[1, -1])}


def main():
    import numpy as np
    cs = cases()
    base = _base_cfg()
    ode_cfg = dict(base, Gamma_wash_over_H=0.5, T_max_over_Tp=1.6, T_min_over_Tp=0.6)
    ode_args = [(ode_cfg, dict(_own_aov(ode_cfg), I_p=0.55, beta_over_H=160.0), 1200, 30.0),
                (dict(ode_cfg, deplete_DM_from_source=True), dict(_own_aov(ode_cfg), v_w=0.6, T_p=115.0), 1200, 30.0)]
    tab_args = [cs[0], cs[4], cs[11], cs[14], ode_args[0]]
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        yb = pool.map(yb_job, cs, chunksize=1)
        tabs = pool.map(table_job, tab_args)
        odes = pool.map(ode_job, ode_args)
    out = {"generator": "tests/golden/make_golden_aov.py (reference fpy:141-165, 192-286, 385-410 with bs.aov "
                        "replaced by an AoverVKernel of other parameters)",
           "numpy": np.__version__, "aov_fields": AOV_FIELDS, "yields": yb, "tables": tabs, "ode": odes}
    path = os.path.join(HERE, "golden_aov_params.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, len(yb), "systems,", len(tabs), "tables,", len(odes), "ODE runs")
    for r in yb[:3]:
        print(r["aov"], r["Y_B"])
    for r in odes:
        print(r["success"], r["Y_B"], r["Y_chi"])
    assert all(math.isfinite(r["Y_B"]) for r in yb)


if __name__ == "__main__":
    main()
