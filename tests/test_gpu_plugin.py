"""The LZ plug-in path end to end on the GPU (fpy:170-187, 317-328):

- lzq's driver with the reference's own stub-module cases (golden_cli_profile.json, made by
  running the reference CLI with those stubs on PYTHONPATH): stdout byte-identical,
  yields_out.json finals within 1e-11;
- the shipped plug-in module plugins/transport_from_profile.py picked up by the hook in the
  fpy:173 order: a one-crossing CSV reproduces P = 1 - exp(-2 pi delta) (eq.(9)) to 1e-8, a
  multi-crossing list gives the propagator's coherent P, a sampled profile (xi, Delta, m_mix)
  is reduced to its spline crossings (estimator = linear) or propagated through (default), the
  paper's phi/Phi bounce format (eqs.(5)-(8)) reproduces a tanh wall's closed-form delta_LZ,
  the module's own command line (PAPER App. A) runs, and the CLI prints the reference's
  `[info] Using P_chi_to_B from profile: ...` line byte-exactly for that P;
- plugins/lzq_binding.py (the reference-side ctypes binding, no torch): the quadrature
  operator on a stand-in with the reference BoltzmannSystem's attributes (self.cfg, self.P,
  fpy:193-196) against the oracle, and its closed form against golden_lz.json.
"""
import importlib
import json
import math
import os
import sys
import types

import numpy as np
import pytest

from conftest import BASE_CFG, ROOT, full_cfg, golden, pkg, rel_err
from oracle import oracle as O
from test_cli import run_cli

pytestmark = pytest.mark.gpu
PLUGINS = os.path.join(ROOT, "plugins")
V_W = 0.30


@pytest.fixture
def plugin_path(monkeypatch):
    monkeypatch.syspath_prepend(PLUGINS)
    for m in ("transport_from_profile", "extended_LZ_lambda", "lambda_local_LZ_from_profile"):
        monkeypatch.delitem(sys.modules, m, raising=False)
    yield PLUGINS
    for m in ("transport_from_profile", "extended_LZ_lambda", "lambda_local_LZ_from_profile"):
        sys.modules.pop(m, None)


def equal_mass_cfg(tmp_path):
    txt = next(c for c in golden("golden_cli.json") if c["name"] == "equal_mass")["config_text"]
    (tmp_path / "cfg.json").write_text(txt)
    return "cfg.json"


@pytest.mark.parametrize("case", golden("golden_cli_profile.json"), ids=lambda c: c["name"])
def test_cli_profile_stubs_match_reference(case, tmp_path, monkeypatch, gpu_engine):
    plug = tmp_path / "plug"
    plug.mkdir()
    for mod, src in zip(case["modules"], case["module_sources"]):
        (plug / (mod + ".py")).write_text(src)
        monkeypatch.delitem(sys.modules, mod, raising=False)
    monkeypatch.syspath_prepend(str(plug))
    importlib.invalidate_caches()
    (tmp_path / "bounce.csv").write_text("xi,m_mix,dprime\n0.0,0.1,1.0\n")
    out = run_cli(["--config", equal_mass_cfg(tmp_path)] + case["flags"], tmp_path)
    for mod in case["modules"]:
        sys.modules.pop(mod, None)
    assert out == case["stdout"]
    ref = json.loads(case["yields_out_json"])
    ours = json.loads((tmp_path / "yields_out.json").read_text())
    assert ours["inputs"] == ref["inputs"]
    for k, v in ref["final"].items():
        assert rel_err(ours["final"][k], v) < 1e-11, (k, ours["final"][k], v)


def test_shipped_module_single_crossing_closed_form(tmp_path, plugin_path, gpu_engine):
    tfp = importlib.import_module("transport_from_profile")
    assert tfp.__file__.startswith(PLUGINS)
    worst = 0.0
    for m, d in [(0.1, 1.0), (0.03, 0.01), (0.3, 0.5), (1e-3, 1e-3), (0.5, 10.0), (0.2, 0.05)]:
        p = tmp_path / "one.csv"
        p.write_text(f"# one crossing\nxi,m_mix,dprime\n1.5,{m!r},{-d!r}\n")
        delta = m * m / (2 * V_W * d)
        P9 = 1.0 - math.exp(-2.0 * math.pi * delta)           # fpy:183-184 / PAPER eq.(9)
        P = tfp.compute_prob_from_profile(str(p), V_W)
        worst = max(worst, abs(P - P9) / P9)
        assert abs(P - P9) <= 1e-8 * P9, (m, d, P, P9)
        (tmp_path / "lam.csv").write_text(f"# v_w = {V_W!r}\nxi,m_mix,dprime\n0.0,{m!r},{d!r}\n")
        assert tfp.compute_lambda_eff_from_profile(str(tmp_path / "lam.csv")) == delta   # eq.(8) exactly
    print(f"one-crossing CSV vs eq.(9): worst rel err {worst:.2e}")


def test_shipped_module_multi_crossing_and_profile(tmp_path, plugin_path, gpu_engine):
    from lz_ref import propagate
    tfp = importlib.import_module("transport_from_profile")
    m, d, x = [0.05, 0.08, 0.04], [0.5, 0.3, 0.7], [0.0, 60.0, 110.0]
    (tmp_path / "list.csv").write_text("xi,m_mix,dprime\n" + "".join(f"{a!r},{b!r},{c!r}\n" for a, b, c in zip(x, m, d)))
    P = tfp.compute_prob_from_profile(str(tmp_path / "list.csv"), V_W)
    eng = gpu_engine.lz_propagate([m], [d], [x], V_W, 20.0, 1000).cpu().numpy()[0]
    assert P == eng                                               # same kernel, same arrays
    assert abs(P - propagate(m, d, x, V_W, 20.0, 1000)) <= 1e-10
    # a sampled bounce profile with the same three crossings: Delta piecewise linear through
    # them (slopes +0.5, -0.3, +0.7), m_mix constant per crossing neighbourhood
    xs = np.linspace(-40.0, 150.0, 3801)
    D = np.where(xs < 22.5, 0.5 * (xs - 0.0), np.where(xs < 95.0, -0.3 * (xs - 60.0), 0.7 * (xs - 110.0)))
    # Delta is continuous at the joins, which are the model's turning points
    assert abs(0.5 * 22.5 - (-0.3) * (22.5 - 60.0)) < 1e-12 and abs(-0.3 * (95.0 - 60.0) - 0.7 * (95.0 - 110.0)) < 1e-12
    mm = np.where(xs < 22.5, 0.05, np.where(xs < 95.0, 0.08, 0.04))
    body = "xi,Delta,m_mix\n" + "".join(f"{float(a)!r},{float(b)!r},{float(c)!r}\n" for a, b, c in zip(xs, D, mm))
    (tmp_path / "prof.csv").write_text(body)
    (tmp_path / "prof_lin.csv").write_text("# estimator = linear\n" + body)
    xc, mc, dc, _ = tfp.read_profile(str(tmp_path / "prof.csv"))
    assert np.allclose(xc, x, atol=1e-9) and np.allclose(mc, m) and np.allclose(dc, d, rtol=1e-9)
    # estimator = linear: the crossings (spline roots) through lzq_lz_propagate's model
    P2 = tfp.compute_prob_from_profile(str(tmp_path / "prof_lin.csv"), V_W)
    assert abs(P2 - P) <= 1e-9
    # default (several crossings): time-ordered through the profile itself, as the engine does it
    P3 = tfp.compute_prob_from_profile(str(tmp_path / "prof.csv"), V_W)
    sh = gpu_engine.profile_shapes(xs, mm, -D)
    assert P3 == gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(0.0, 1.0, 1.0, V_W, 0)).cpu().item()
    assert 0.0 < P3 < 1.0


def test_sampled_levels_format_spline_crossings(tmp_path, plugin_path, gpu_engine):
    """xi,Delta,m_mix samples through the GPU splines: linear samples are reproduced exactly
    (crossing at xi = 1, |Delta'| = 1, m_mix = 0.2); a zero sample that is a sign change is a
    crossing on the knot, and a later root of the cubic is found as the numpy restatement finds
    it."""
    import profile_ref as R
    tfp = importlib.import_module("transport_from_profile")
    rows = "".join(f"{x!r},{x - 1.0!r},{0.1 + 0.1 * x!r}\n" for x in (0.0, 0.5, 0.75, 1.25, 2.0))
    (tmp_path / "b.csv").write_text("xi,Delta,m_mix\n" + rows)
    xs, ms, ds, _ = tfp.read_profile(str(tmp_path / "b.csv"))
    assert len(xs) == 1 and abs(xs[0] - 1.0) < 1e-15 and abs(ds[0] - 1.0) < 1e-14 and abs(ms[0] - 0.2) < 1e-15
    x, D, m = [-1.0, 0.0, 1.0, 2.0], [-1.0, 0.0, 1.0, -1.0], [0.1, 0.1, 0.1, 0.3]
    (tmp_path / "c.csv").write_text("xi,Delta,m_mix\n" + "".join(f"{a},{b},{c}\n" for a, b, c in zip(x, D, m)))
    xs, ms, ds, _ = tfp.read_profile(str(tmp_path / "c.csv"))
    ref = R.crossings(x, R.spline_coefs(x, m), R.spline_coefs(x, [-d for d in D]), 0.0, 1.0, 1.0, 1.0)
    assert len(xs) == 2 == len(ref) and xs[0] == 0.0
    for (a, b, c), (rx, rd, rm, _) in zip(zip(xs, ms, ds), ref):
        assert abs(a - rx) < 1e-14 and abs(b - rm) < 1e-14 and abs(c - abs(rd)) < 1e-14


def _tanh_csv(path, yB, ychi, lam, extra="", header="xi,phi,Phi", shift=0.0, n=8001, span=4.0):
    xs = np.linspace(-span, span, n)
    phi, Phi = 0.5 * (1.0 - np.tanh(xs)), 0.65 * (1.0 + np.tanh(xs))
    lines = [f"# y_B = {yB!r}", f"# y_chi = {ychi!r}", f"# lambda_tr_eff = {lam!r}"] + ([extra] if extra else [])
    lines.append(header)
    lines += [f"{float(a + shift)!r},{float(b)!r},{float(c)!r}" for a, b, c in zip(xs, phi, Phi)]
    path.write_text("\n".join(lines) + "\n")


def test_shipped_module_bounce_fields(tmp_path, plugin_path, gpu_engine):
    """The paper's profile format (PAPER p.3 eqs.(5)-(8)): phi, Phi samples + y_B, y_chi,
    lambda_tr_eff.  A tanh wall (v = 1, V = 1.3) has its crossing in closed form; lambda_eff is
    delta_LZ of eq.(8) to <= 1e-10, P the minimal estimator eq.(9); r = xi + R0 with `# R0`
    gives the same; a missing coupling is an error (parity unpinned against the absent
    upstream module, PAPER-pinned)."""
    tfp = importlib.import_module("transport_from_profile")
    yB, ychi, lam = 1.3, 0.8, 0.1
    t = (yB - ychi * 1.3) / (yB + ychi * 1.3)
    dp = (yB + ychi * 1.3) * (1.0 - t * t) / 2.0
    m = lam * 0.5 * (1.0 - t)
    delta = m * m / (2 * V_W * dp)
    _tanh_csv(tmp_path / "wall.csv", yB, ychi, lam, f"# v_w = {V_W!r}")
    lam_eff = tfp.compute_lambda_eff_from_profile(str(tmp_path / "wall.csv"))
    assert abs(lam_eff - delta) <= 1e-10 * delta, (lam_eff, delta)
    P = tfp.compute_prob_from_profile(str(tmp_path / "wall.csv"), V_W)
    assert P == 1.0 - math.exp(-2.0 * math.pi * lam_eff)            # fpy:183-184 on the GPU
    _tanh_csv(tmp_path / "wall_r.csv", yB, ychi, lam, "# R0 = 7.25", header="r,phi,Phi", shift=7.25)
    (x_r,), _, _, _ = tfp.read_profile(str(tmp_path / "wall_r.csv"))
    assert abs(x_r - math.atanh(t)) <= 1e-10
    # the whole-profile propagation of the same wall (estimator = propagate) is a different,
    # finite-wall quantity; for this wide, smooth wall it is close to eq.(9)
    _tanh_csv(tmp_path / "wall_p.csv", yB, ychi, lam, "# estimator = propagate", n=401, span=12.0)
    Pp = tfp.compute_prob_from_profile(str(tmp_path / "wall_p.csv"), V_W)
    assert abs(Pp - P) <= 0.05 * P, (Pp, P)
    (tmp_path / "nocoupling.csv").write_text("# y_B = 1.0\nxi,phi,Phi\n0,1,0\n1,1,1\n2,1,2\n3,1,3\n")
    with pytest.raises(ValueError):
        tfp.compute_prob_from_profile(str(tmp_path / "nocoupling.csv"), V_W)


def test_transport_from_profile_command_line(tmp_path, plugin_path, gpu_engine, capsys):
    """PAPER App. A: python transport_from_profile.py --params transport_params.json."""
    tfp = importlib.import_module("transport_from_profile")
    _tanh_csv(tmp_path / "wall.csv", 1.0, 1.0, 0.2, n=401)
    (tmp_path / "transport_params.json").write_text(json.dumps({"profile_csv": "wall.csv", "v_w": V_W}))
    assert tfp.main(["--params", str(tmp_path / "transport_params.json"), "--out", str(tmp_path / "P.json")]) == 0
    out = capsys.readouterr().out
    res = json.loads((tmp_path / "P.json").read_text())
    assert out.splitlines()[-1] == f"P_chi_to_B = {res['P_chi_to_B']!r}"
    assert len(res["crossings"]) == 1
    assert res["P_chi_to_B"] == tfp.compute_prob_from_profile(str(tmp_path / "wall.csv"), V_W)


def test_cli_bounce_fields_info_line(tmp_path, plugin_path, gpu_engine):
    """lzq's driver with --maybe-compute-P-from-profile on a phi/Phi profile: the reference's
    `[info] Using P_chi_to_B from profile: {P:.6g}` line (fpy:322) and P_used."""
    tfp = importlib.import_module("transport_from_profile")
    _tanh_csv(tmp_path / "bounce.csv", 1.0, 1.0, 0.2, n=401)
    P = tfp.compute_prob_from_profile(str(tmp_path / "bounce.csv"), 0.30)
    out = run_cli(["--config", equal_mass_cfg(tmp_path), "--maybe-compute-P-from-profile", "bounce.csv"], tmp_path)
    assert out.splitlines()[0] == f"[info] Using P_chi_to_B from profile: {P:.6g}"
    assert json.loads((tmp_path / "yields_out.json").read_text())["inputs"]["P_used"] == P


def test_cli_picks_up_shipped_module(tmp_path, plugin_path, gpu_engine):
    """fpy:173 order with the shipped module: transport_from_profile is found on sys.path,
    its P drives the run, and the info line is the reference's format (fpy:322)."""
    m, d = 0.1, 1.0
    (tmp_path / "bounce.csv").write_text(f"xi,m_mix,dprime\n0.0,{m!r},{d!r}\n")
    tfp = importlib.import_module("transport_from_profile")
    P = tfp.compute_prob_from_profile(str(tmp_path / "bounce.csv"), V_W)
    out = run_cli(["--config", equal_mass_cfg(tmp_path), "--maybe-compute-P-from-profile", "bounce.csv"], tmp_path)
    assert out.splitlines()[0] == f"[info] Using P_chi_to_B from profile: {P:.6g}"
    yo = json.loads((tmp_path / "yields_out.json").read_text())
    assert yo["inputs"]["P_used"] == P
    ref = O.point_yields(full_cfg({**BASE_CFG, "P_chi_to_B": P}))
    assert rel_err(yo["final"]["Y_B"], ref["Y_B"]) < 1e-11
    # an earlier module in the search order wins over the shipped one
    stub = types.ModuleType("extended_LZ_lambda")
    stub.compute_prob_from_profile = lambda path, v_w: 0.125
    sys.modules["extended_LZ_lambda"] = stub
    try:
        assert pkg("lz").try_compute_P_from_profile(str(tmp_path / "bounce.csv"), V_W) == 0.125
    finally:
        del sys.modules["extended_LZ_lambda"]


def test_reference_side_binding(plugin_path, gpu_engine):
    B = importlib.import_module("lzq_binding")
    cfgm = pkg("config")

    import numpy as np

    class KernelStandIn:  # the attributes of the reference's AoverVKernel the binding reads (fpy:141-156)
        def __init__(self, I_p, beta_over_H, T_p, v_w, g_star, z_max=30.0, nz=1200):
            self.I_p, self.beta_over_H, self.T_p, self.v_w, self.g_star = I_p, beta_over_H, T_p, max(v_w, 1e-12), g_star
            self.z = np.linspace(0.0, z_max, nz)

    class StandIn:  # the attributes of the reference's BoltzmannSystem that the binding reads (fpy:193-197)
        def __init__(self, cfg, P):
            self.cfg, self.P = cfg, float(P)
            self.aov = KernelStandIn(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star)

    ns = types.SimpleNamespace(BoltzmannSystem=StandIn, AoverVKernel=KernelStandIn)
    B.install(ns)
    cfg = cfgm.Config(**full_cfg(BASE_CFG))
    bs = ns.BoltzmannSystem(cfg, cfg.P_chi_to_B)
    p = O.point_from_config(full_cfg(BASE_CFG))
    import ctypes
    for (tlo, thi, ny) in ((0.1, 500.0, 8000), (60.0, 150.0, 2000), (90.0, 110.0, 6000)):
        got = bs.integrate_YB_by_quadrature(tlo, thi, n_y=ny)
        ref = O.lib().oracle_yb_quadrature(ctypes.byref(p), tlo, thi, ny)
        assert rel_err(got, ref) < 1e-11, (tlo, thi, ny, got, ref)
    # the operator on another z grid (bs.aov = AoverVKernel(..., z_max, nz), fpy:141-142)
    bs.aov = ns.AoverVKernel(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star, z_max=45.0, nz=2400)
    got = bs.integrate_YB_by_quadrature(0.1, 500.0, n_y=8000)
    ref = O.yb_quadrature(full_cfg(BASE_CFG), 0.1, 500.0, 8000, 2400, 45.0)
    assert rel_err(got, ref) < 1e-11, (got, ref)
    for y in (-20.0, 0.0, 15.975, 49.0, 51.0):
        g, r = bs.aov.A_over_V_y(y), O.aov(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star, y, 2400, 45.0)
        assert (g == r == 0.0) or rel_err(g, r) < 1e-11, (y, g, r)
    y = B.yields(cfg, cfg.P_chi_to_B)
    assert f"{y['Y_B']:.10e}" == "8.7208853627e-11"
    d = golden("golden_lz.json")
    lam = [float(s) for s in d["lambda"]]
    for l, g, r in zip(lam, B.p_closed_form(lam), d["P"]):
        assert abs(g - r) <= 1e-8 * abs(r) + 4.5e-16, (l, g, r)


def test_reference_side_binding_ode(plugin_path, gpu_engine):
    """plugins/lzq_binding.ode_yields (fpy:385-417 for one config, torch-free): the reference's own
    ODE outputs (golden_ode.json) within the tolerance test_gpu_ode.py applies, the Engine's
    sequential integration within 1e-13 (time-parallel) and bit for bit (time_parallel=False), a
    refused window with the reference's status, and bs.aov's own parameters."""
    B = importlib.import_module("lzq_binding")
    cfgm = pkg("config")
    pts = golden("golden_ode.json")["points"]
    for r in pts[::3] + [pts[-1]]:
        c = full_cfg(r["config"])
        cfg = cfgm.Config(**c)
        P = r.get("P_used", c["P_chi_to_B"])
        got = B.ode_yields(cfg, P)
        seq = B.ode_yields(cfg, P, time_parallel=False)
        t, st = gpu_engine.ode(cfgm.to_point(dict(c, P_chi_to_B=P)), cfgm.to_ode_params(c), time_parallel=False)
        row = t.cpu().numpy()[0]
        if "error" in r:
            assert got["status"] == seq["status"] == "bad_grid" and int(st[0]) == 1
            continue
        assert got["status"] == seq["status"] == "ok", (got, r["config"])
        assert seq["Y_B"] == row[0] and seq["Y_chi"] == row[1]
        assert got["Y_B"] == row[0] and got["Y_chi"] == row[1]   # time-parallel: the same bits
        if r["tight"]["success"]:
            ref_acc = max(rel_err(r["final"]["Y_B"], r["tight"]["Y_B"]), rel_err(r["final"]["Y_chi"], r["tight"]["Y_chi"]))
            assert rel_err(got["Y_B"], r["final"]["Y_B"]) < 1e-8 + 10 * ref_acc, (got, r["final"])
    # bs.aov replaced: the A/V kernel's own parameters and z grid behind build_tables

    class KernelStandIn:  # the attributes of the reference's AoverVKernel the binding reads (fpy:141-156)
        def __init__(self, I_p, beta_over_H, T_p, v_w, g_star, z_max=30.0, nz=1200):
            self.I_p, self.beta_over_H, self.T_p, self.v_w, self.g_star = I_p, beta_over_H, T_p, v_w, g_star
            self.z = np.linspace(0.0, z_max, nz)

    c = full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, "sigma_v_chi_GeV_m2": 1e-12, "T_max_over_Tp": 1.6,
                  "T_min_over_Tp": 0.6})
    cfg = cfgm.Config(**c)
    kern = KernelStandIn(0.5, 60.0, cfg.T_p_GeV, 0.45, cfg.g_star, z_max=40.0, nz=1600)
    got = B.ode_yields(cfg, cfg.P_chi_to_B, aov=kern)
    aov = {"I_p": 0.5, "beta_over_H": 60.0, "T_p_GeV": cfg.T_p_GeV, "v_w": 0.45, "g_star": cfg.g_star}
    t, st = gpu_engine.ode(cfgm.to_point(c), cfgm.to_ode_params(c), aov=aov, nz=1600, z_max=40.0, time_parallel=False)
    assert got["status"] == "ok" and int(st[0]) == 0
    assert rel_err(got["Y_B"], float(t[0, 0])) < 1e-13 and rel_err(got["Y_chi"], float(t[0, 1])) < 1e-13
