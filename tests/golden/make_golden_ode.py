#!/usr/bin/env python3
"""Golden fixtures of the reference's ODE fallback path (fpy:385-410), made by running the
REFERENCE itself: its own `main()` (build_tables + scipy solve_ivp Radau, rtol=1e-8,
atol=1e-12, its own max_step).  Build-container only, like make_golden.py; the reference
never travels to the GPU box, only golden_ode.json does.

Per case it records:
  * `final` / `P_used`: yields_out.json of main() (the shipped path);
  * `tight`: the same ODE re-solved with the reference's own BoltzmannSystem.rhs and
    build_tables at rtol=1e-12, atol=1e-30 (same max_step) -- how far the shipped tolerance
    sits from the converged solution of the reference's equations;
  * `rhs`: BoltzmannSystem.rhs(x, Y) and A_over_V_T(T) at a few x / T after build_tables,
    pinning the ingredients of the equations independently of any integrator.
A case whose reference run raises records the exception type and message instead.

The fallback takes >= 20000 Radau steps per point (max_step <= |x1-x0|/20000, fpy:404), so
most cases use narrow integration windows; one case keeps the shipped window (~1e6 steps,
several minutes).

    python tests/golden/make_golden_ode.py             # ~25 min on 8 cores (one shipped-window case)
    python tests/golden/make_golden_ode.py --cli-only  # golden_cli_ode.json, ~20 s
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (shared reference loader / runner)


def ode_cases() -> list[dict]:
    E = []

    def mk(**kw):
        c = MG._base_cfg()
        c.update(kw)
        E.append(c)

    narrow = dict(T_max_over_Tp=1.6, T_min_over_Tp=0.6)
    # wash-out only (Y_chi stays at Y_chi_init)
    mk(Gamma_wash_over_H=0.5, **narrow)
    mk(Gamma_wash_over_H=5.0, **narrow)
    mk(Gamma_wash_over_H=50.0, **narrow)
    # depletion of chi by the source term
    mk(deplete_DM_from_source=True, **narrow)
    mk(deplete_DM_from_source=True, incident_flux_scale=1e-3, **narrow)
    # annihilation (Riccati in Y_chi): weak and stiff, relativistic and non-relativistic chi
    mk(sigma_v_chi_GeV_m2=1e-20, **narrow)
    mk(sigma_v_chi_GeV_m2=1e-12, **narrow)
    mk(sigma_v_chi_GeV_m2=1e-9, regime="thermal", m_chi_GeV=300.0, **narrow)
    mk(sigma_v_chi_GeV_m2=1e-9, regime="thermal", m_chi_GeV=300.0, T_max_over_Tp=1.3, T_min_over_Tp=0.2)
    mk(sigma_v_chi_GeV_m2=1e-14, m_chi_GeV=150.0, chi_stats="boson", **narrow)
    # everything at once
    mk(sigma_v_chi_GeV_m2=1e-16, Gamma_wash_over_H=2.0, deplete_DM_from_source=True, **narrow)
    mk(sigma_v_chi_GeV_m2=1e-16, Gamma_wash_over_H=2.0, deplete_DM_from_source=True,
       regime="thermal", chi_stats="boson", m_chi_GeV=40.0, **narrow)
    # other initial abundances (fpy:391-399), including the regime with no fast-path branch
    mk(Gamma_wash_over_H=1.0, Y_chi_init=None, n_chi_at_Tp_GeV3=2.5e-2, **narrow)
    mk(Gamma_wash_over_H=1.0, Y_chi_init=None, n_chi_at_Tp_GeV3=None, **narrow)
    mk(Gamma_wash_over_H=1.0, regime="auto", **narrow)
    # other kernels / windows / clamps
    mk(Gamma_wash_over_H=1.0, beta_over_H=30.0, I_p=0.6, v_w=0.6, T_max_over_Tp=2.0, T_min_over_Tp=0.4)
    mk(Gamma_wash_over_H=1.0, T_p_GeV=10.0, source_shape_sigma_y=4.0, **narrow)
    mk(Gamma_wash_over_H=0.3, T_max_over_Tp=1.05, T_min_over_Tp=0.95)
    mk(Gamma_wash_over_H=-1.0, sigma_v_chi_GeV_m2=-1e-12, deplete_DM_from_source=True, **narrow)  # max(., 0)
    # error behaviour: zero-width and inverted windows (CubicSpline rejects the T grid)
    mk(Gamma_wash_over_H=1.0, T_max_over_Tp=1.0, T_min_over_Tp=1.0)
    mk(Gamma_wash_over_H=1.0, T_max_over_Tp=0.5, T_min_over_Tp=0.9)
    # the shipped window (x from m/500 to m/0.1: ~1e6 Radau steps)
    mk(Gamma_wash_over_H=1.0)
    return E


def _setup(cfg: dict, P_used: float):
    fpy = MG._fpy()
    c = fpy.Config(**{**fpy.default_config(), **cfg})
    bs = fpy.BoltzmannSystem(c, P_used)
    T_p = c.T_p_GeV
    T_hi, T_lo = c.T_max_over_Tp * T_p, c.T_min_over_Tp * T_p
    bs.build_tables(T_lo, T_hi, n=800)
    return fpy, c, bs, T_lo, T_hi


def _tight(cfg: dict, P_used: float) -> dict:
    """Same ODE, same tables (reference code), converged integration."""
    import numpy as np
    from scipy.integrate import solve_ivp
    fpy, c, bs, T_lo, T_hi = _setup(cfg, P_used)
    T_p = c.T_p_GeV
    x0, x1 = c.m_chi_GeV / T_hi, c.m_chi_GeV / max(T_lo, 1e-30)
    r = c.regime.lower()
    if r.startswith("therm"):
        Y0 = fpy.n_chi_eq(T_hi, c.m_chi_GeV, c.g_chi, c.chi_stats) / fpy.s_entropy(T_hi, c.g_star_s)
    elif r.startswith("non"):
        if c.Y_chi_init is not None:
            Y0 = float(c.Y_chi_init)
        elif c.n_chi_at_Tp_GeV3 is not None:
            Y0 = float(c.n_chi_at_Tp_GeV3) / max(fpy.s_entropy(T_p, c.g_star_s), 1e-300)
        else:
            Y0 = 1.0e-12
    else:
        Y0 = fpy.n_chi_eq(T_hi, c.m_chi_GeV, c.g_chi, c.chi_stats) / fpy.s_entropy(T_hi, c.g_star_s)
    x_p = c.m_chi_GeV / max(T_p, 1e-30)
    max_step = min(abs(x1 - x0) / 20000.0, x_p / 1000.0, 5e-4)
    sol = solve_ivp(bs.rhs, (x0, x1), np.array([Y0, 0.0], float), method="Radau", rtol=1e-12, atol=1e-30,
                    max_step=max_step)
    return {"Y_chi": float(sol.y[0, -1]), "Y_B": float(sol.y[1, -1]), "nfev": int(sol.nfev),
            "n_steps": int(sol.t.size - 1), "success": bool(sol.success)}


def _rhs_samples(cfg: dict, P_used: float) -> dict:
    import numpy as np
    fpy, c, bs, T_lo, T_hi = _setup(cfg, P_used)
    m = c.m_chi_GeV
    x0, x1 = m / T_hi, m / max(T_lo, 1e-30)
    xs = [float(v) for v in np.linspace(x0, x1, 9)] + [x0 * 0.5, x1 * 1.5]   # incl. the clamp outside [T_lo, T_hi]
    Ys = [[4.9e-10, 0.0], [1e-3, 3e-11], [2.5e-12, 1.5e-10]]
    rows = []
    for x in xs:
        for Y in Ys:
            d = bs.rhs(x, np.array(Y, float))
            rows.append({"x": x, "Y": Y, "dY": [float(d[0]), float(d[1])]})
    Ts = [float(v) for v in np.linspace(T_lo, T_hi, 13)] + [T_lo * 0.5, T_hi * 2.0]
    return {"rhs": rows, "A_over_V_T": {"T": Ts, "Av": [float(bs.A_over_V_T(T)) for T in Ts]}}


def _worker(cfg: dict) -> dict:
    row = {"config": cfg}
    with tempfile.TemporaryDirectory() as d:
        try:
            out = MG._run_main_in(cfg, d)
        except Exception as e:
            row["error"] = {"type": type(e).__name__, "message": str(e)}
            return row
    row["final"], row["P_used"] = out["final"], out["inputs"]["P_used"]
    row["tight"] = _tight(cfg, row["P_used"])
    row.update(_rhs_samples(cfg, row["P_used"]))
    return row


def cli_ode_cases() -> list[dict]:
    """Byte-exact stdout + yields_out.json of the reference CLI on ODE-path configs."""
    import subprocess
    out = []
    for name, over in (("ode_wash", {"Gamma_wash_over_H": 0.5, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}),
                       ("ode_deplete_annihilate", {"deplete_DM_from_source": True, "sigma_v_chi_GeV_m2": 1e-16,
                                                   "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6})):
        with tempfile.TemporaryDirectory() as d:
            c = MG._base_cfg()
            c.update(over)
            cfg_text = json.dumps(c, indent=2)
            with open(os.path.join(d, "cfg.json"), "w") as f:
                f.write(cfg_text)
            r = subprocess.run([sys.executable, "-B", os.path.join(MG.REF_DIR, "first_principles_yields.py"),
                                "--config", "cfg.json"], cwd=d, capture_output=True, text=True)
            with open(os.path.join(d, "yields_out.json")) as f:
                yo = f.read()
            out.append({"name": name, "flags": [], "config_text": cfg_text, "returncode": r.returncode,
                        "stdout": r.stdout, "yields_out_json": yo})
    return out


def main():
    if "--cli-only" in sys.argv:
        with open(os.path.join(HERE, "golden_cli_ode.json"), "w") as f:
            json.dump(cli_ode_cases(), f, indent=1)
        return
    cases = ode_cases()
    order = sorted(range(len(cases)), key=lambda i: -("T_max_over_Tp" not in cases[i] or cases[i]["T_max_over_Tp"] == 5.0))
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(_worker, [cases[i] for i in order], chunksize=1)
    rows = [None] * len(cases)
    for i, r in zip(order, res):
        rows[i] = r
    with open(os.path.join(HERE, "golden_ode.json"), "w") as f:
        json.dump({"points": rows}, f, indent=1)
    print("wrote", len(rows), "ODE points")


if __name__ == "__main__":
    main()
