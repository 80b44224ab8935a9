#!/usr/bin/env python3
"""Converged solutions of the reference's ODE for the two stiff cases where its own Radau gives
up (golden_ode.json: m_chi = 300 GeV, sigma_v = 1e-9, thermal; `tight` has success = False),
made with the REFERENCE's own equations (BoltzmannSystem.rhs + build_tables, fpy:207-212,
270-286) in this build container only.

Why the reference stops: n_chi_eq switches formula at the strict T > m/3 branch (fpy:100-105),
so Y_eq -- and with sigma_v = 1e-9 the Y_chi that tracks it -- jumps at x* = m/T = 3, and an
adaptive step controller cannot cross a jump in the forcing.  Solved here in two pieces,
[x0, x*] and [x*, x1], each by scipy Radau at rtol = 1e-12, atol = 1e-30 with the reference's
max_step (fpy:404), with the state carried across x* (the ODE's solution is continuous there;
only its right-hand side jumps).  Also recorded: a LSODA solve of the same split, as a check
that the split solution is converged (the two agree to ~1e-12).

    python tests/golden/make_golden_ode_stiff.py             # ~1 min; -> golden_ode_stiff.json
    python tests/golden/make_golden_ode_stiff.py --cli-only  # the reference CLI's bytes on the two
                                                             # cases -> golden_cli_ode_stiff.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden_ode as MGO  # noqa: E402


def split_solve(cfg: dict, P_used: float, method: str) -> dict:
    import numpy as np
    from scipy.integrate import solve_ivp
    fpy, c, bs, T_lo, T_hi = MGO._setup(cfg, P_used)
    T_p, m = c.T_p_GeV, c.m_chi_GeV
    x0, x1 = m / T_hi, m / max(T_lo, 1e-30)
    assert c.regime.lower().startswith("therm")
    Y = np.array([fpy.n_chi_eq(T_hi, m, c.g_chi, c.chi_stats) / fpy.s_entropy(T_hi, c.g_star_s), 0.0])
    max_step = min(abs(x1 - x0) / 20000.0, m / max(T_p, 1e-30) / 1000.0, 5e-4)
    # the branch point in floating point: the first x whose T = m/max(x, 1e-30) (fpy:272) is no
    # longer > m/3 (fpy:100); the first piece ends one ulp before it
    xs = 3.0
    while m / xs > m / 3.0:
        xs = np.nextafter(xs, np.inf)
    while m / np.nextafter(xs, -np.inf) <= m / 3.0:
        xs = np.nextafter(xs, -np.inf)
    xa = np.nextafter(xs, -np.inf)
    assert m / xa > m / 3.0 >= m / xs and x0 < xa < xs < x1
    pieces = []
    for a, b in ((x0, xa), (xs, x1)):
        kw = {"max_step": max_step} if method == "Radau" else {}
        sol = solve_ivp(bs.rhs, (a, b), Y, method=method, rtol=1e-12, atol=1e-30, **kw)
        assert sol.success, (method, a, b, sol.message)
        Y = sol.y[:, -1].copy()
        pieces.append({"x": [a, b], "n_steps": int(sol.t.size - 1), "nfev": int(sol.nfev)})
    return {"Y_chi": float(Y[0]), "Y_B": float(Y[1]), "pieces": pieces, "method": method}


def cli_stiff_cases() -> list[dict]:
    """Byte-exact stdout + yields_out.json of the reference CLI (fpy:346-438) on the two stiff cases:
    its Radau gives up at the T = m/3 jump, main() prints the [warn] line (fpy:408-409) and reports
    the state where the solver stopped (fpy:410)."""
    import subprocess
    import tempfile
    gold = json.load(open(os.path.join(HERE, "golden_ode.json")))
    out = []
    for i, r in enumerate(gold["points"]):
        if "error" in r or r["tight"]["success"]:
            continue
        with tempfile.TemporaryDirectory() as d:
            cfg_text = json.dumps(r["config"], indent=2)
            with open(os.path.join(d, "cfg.json"), "w") as f:
                f.write(cfg_text)
            res = subprocess.run([sys.executable, "-B", os.path.join(MGO.MG.REF_DIR, "first_principles_yields.py"),
                                  "--config", "cfg.json"], cwd=d, capture_output=True, text=True)
            with open(os.path.join(d, "yields_out.json")) as f:
                yo = f.read()
        out.append({"name": f"ode_stiff_{i}", "index": i, "flags": [], "config_text": cfg_text,
                    "returncode": res.returncode, "stdout": res.stdout, "yields_out_json": yo})
        print(i, res.stdout.splitlines()[:2])
    return out


def main():
    if "--cli-only" in sys.argv:
        with open(os.path.join(HERE, "golden_cli_ode_stiff.json"), "w") as f:
            json.dump(cli_stiff_cases(), f, indent=1)
        return
    gold = json.load(open(os.path.join(HERE, "golden_ode.json")))
    out = []
    for i, r in enumerate(gold["points"]):
        if "error" in r or r["tight"]["success"]:
            continue
        res = {"index": i, "config": r["config"], "P_used": r["P_used"], "reference_final": r["final"],
               "split_radau": split_solve(r["config"], r["P_used"], "Radau"),
               "split_lsoda": split_solve(r["config"], r["P_used"], "LSODA")}
        a, b = res["split_radau"], res["split_lsoda"]
        print(i, a["Y_chi"], a["Y_B"], "lsoda rel diff", abs(a["Y_B"] - b["Y_B"]) / abs(a["Y_B"]),
              abs(a["Y_chi"] - b["Y_chi"]) / abs(a["Y_chi"]))
        out.append(res)
    with open(os.path.join(HERE, "golden_ode_stiff.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_ode_stiff.py", "cases": out}, f, indent=1)


if __name__ == "__main__":
    main()
