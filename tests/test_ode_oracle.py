"""The CPU restatement of the ODE fallback (oracle/lzq_oracle.c, fpy:200-219, 270-286, 385-417)
against scipy's CubicSpline and against the reference's own outputs (tests/golden/golden_ode.json,
made by tests/golden/make_golden_ode.py running the reference)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, full_cfg, golden, rel_err
from oracle import oracle as O

GOLDEN_ODE = os.path.join(GOLDEN, "golden_ode.json")
needs_golden = pytest.mark.skipif(not os.path.exists(GOLDEN_ODE), reason="golden_ode.json not generated")

NARROW = {"Gamma_wash_over_H": 0.5, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}


def base(**kw):
    from conftest import BASE_CFG
    return full_cfg({**BASE_CFG, **kw})


def test_spline_matches_scipy_cubicspline():
    """build_tables = CubicSpline(Ts, max(A/V, 0)) with scipy's default not-a-knot ends."""
    from scipy.interpolate import CubicSpline
    for over in (NARROW, {"T_max_over_Tp": 5.0, "T_min_over_Tp": 1e-3}, {"T_max_over_Tp": 2.0, "T_min_over_Tp": 0.4,
                                                                           "beta_over_H": 30.0, "I_p": 0.6}):
        cfg = base(**over)
        T_p = cfg["T_p_GeV"]
        Ts = np.linspace(cfg["T_min_over_Tp"] * T_p, cfg["T_max_over_Tp"] * T_p, 800)
        Av = np.array([O.aov(cfg["I_p"], cfg["beta_over_H"], T_p, cfg["v_w"], cfg["g_star"],
                             0.5 * cfg["beta_over_H"] * ((T_p / max(T, 1e-30)) ** 2 - 1.0)) for T in Ts])
        ref = CubicSpline(Ts, np.maximum(Av, 0.0), extrapolate=True).c.T   # (799, 4)
        got = O.ode_tables(cfg)
        scale = np.max(np.abs(ref), axis=0)
        assert np.max(np.abs(got - ref) / scale) < 1e-11
        for T in (Ts[0], Ts[1] * 0.5 + Ts[2] * 0.5, Ts[400], Ts[-1], Ts[0] - 1.0, Ts[-1] + 3.0):
            s = CubicSpline(Ts, np.maximum(Av, 0.0), extrapolate=True)(min(max(T, Ts[0]), Ts[-1]))
            assert abs(O.ode_aov_T(cfg, T) - s) <= 1e-11 * np.max(Av)


def test_bad_windows_status():
    assert O.ode_point(base(Gamma_wash_over_H=1.0, T_max_over_Tp=1.0, T_min_over_Tp=1.0))["status"] == 1
    assert O.ode_point(base(Gamma_wash_over_H=1.0, T_max_over_Tp=0.5, T_min_over_Tp=0.9))["status"] == 1
    assert O.ode_point(base(Gamma_wash_over_H=1.0), max_steps=1000)["status"] == 3


@needs_golden
def test_oracle_vs_reference_ode_outputs():
    pts = golden("golden_ode.json")["points"]
    worst = 0.0
    for r in pts:
        cfg = full_cfg(r["config"])
        got = O.ode_point(cfg)
        if "error" in r:
            assert got["status"] == 1 and r["error"]["type"] == "ValueError", (r["error"], got["status"])
            continue
        assert got["status"] == 0
        if not r["tight"]["success"]:
            continue   # the reference's Radau gives up: test_oracle_stiff_cases_vs_converged_split
        # the reference's shipped Radau (rtol 1e-8, atol 1e-12) vs its own converged solve
        ref_acc = max(rel_err(r["final"]["Y_B"], r["tight"]["Y_B"]), rel_err(r["final"]["Y_chi"], r["tight"]["Y_chi"]))
        for k in ("Y_B", "Y_chi", "rho_B_kg_m3", "rho_DM_kg_m3", "DM_over_B"):
            e = rel_err(got[k], r["final"][k])
            assert e < 1e-8 + 10 * ref_acc, (k, got[k], r["final"][k], r["config"])
            worst = max(worst, e)
    print(f"ODE oracle vs reference: worst rel err {worst:.3e}")


STIFF_TOL = 1e-10   # per case: converged split solve (Radau vs LSODA agree to ~1e-11)


def stiff_cases():
    return golden("golden_ode_stiff.json")["cases"]


@needs_golden
def test_oracle_stiff_cases_vs_converged_split():
    """The two cases where the reference's adaptive Radau gives up (Y_eq jumps at the strict
    T > m/3 branch, fpy:100-105; its main() prints the warning and reports the state where it
    stopped, 68x below the converged Y_B): the fixed-step restatement, which splits the step at
    the branch point, against the reference's equations solved in two pieces around that point
    (tests/golden/make_golden_ode_stiff.py)."""
    for c in stiff_cases():
        got = O.ode_point(full_cfg(c["config"]))
        ref = c["split_radau"]
        assert got["status"] == 0
        e_b, e_c = rel_err(got["Y_B"], ref["Y_B"]), rel_err(got["Y_chi"], ref["Y_chi"])
        lsoda = rel_err(c["split_lsoda"]["Y_B"], ref["Y_B"])
        print(f"stiff case {c['index']}: oracle vs converged split Y_B {e_b:.2e}  Y_chi {e_c:.2e}  "
              f"(split Radau vs LSODA {lsoda:.1e}; tol {STIFF_TOL:g}; the reference's own Y_B is "
              f"{rel_err(c['reference_final']['Y_B'], ref['Y_B']):.2f} off)")
        assert e_b < STIFF_TOL and e_c < STIFF_TOL, (c["index"], got, ref)


@needs_golden
def test_oracle_rhs_and_aov_T_vs_reference():
    for r in golden("golden_ode.json")["points"]:
        if "error" in r:
            continue
        cfg = full_cfg(r["config"])
        scale = np.max(np.abs([s["dY"] for s in r["rhs"]]), axis=0)
        for s in r["rhs"]:
            got = O.ode_rhs(cfg, s["x"], s["Y"])
            for g, e, sc in zip(got, s["dY"], scale):
                assert abs(g - e) <= 1e-10 * abs(e) + 1e-12 * sc, (s, got)
        for T, e in zip(r["A_over_V_T"]["T"], r["A_over_V_T"]["Av"]):
            assert abs(O.ode_aov_T(cfg, T) - e) <= 1e-11 * max(abs(e), 1e-300) + 1e-14 * max(r["A_over_V_T"]["Av"])
