"""bs.aov's own parameters through the C ABI (include/lzq.h lzq_aov_params): a BoltzmannSystem
whose A/V kernel is an AoverVKernel(I_p', beta_over_H', T_p', v_w', g_star', z_max, nz) other than
the one fpy:197 builds from cfg.  Needs an MI355X.

The reference takes A/V from self.aov (fpy:211, 228, 261) and every other ingredient of the
integrand from self.cfg (fpy:234-262).  Pinned to tests/golden/golden_aov_params.json, which
tests/golden/make_golden_aov.py made by running the reference with bs.aov replaced (24 systems:
each kernel field changed alone, then all of them on random configs, two z grids; build_tables +
A_over_V_T + rhs; two ODE runs), through every layer a user reaches it by:

- the package's reference-shaped facade (boltzmann.BoltzmannSystem with bs.aov replaced);
- the reference-side ctypes binding plugins/lzq_binding.py (installed on a stand-in with the
  reference's attributes: self.cfg, self.P, self.aov with I_p, beta_over_H, T_p, v_w, g_star, z);
- the engine (Engine.yields / ode_tables / ode with aov=...), batched.

Tolerances: north_star's 1e-8 gate and the golden tests' 1e-11 guard band on Y_B; A/V, tables and
rhs as the oracle's own pins (tests/test_oracle_golden.py); the ODE at the 1e-10 of
tests/test_gpu_zgrid.py's fixed-step-vs-adaptive comparison.
"""
import importlib
import types

import numpy as np
import pytest
import torch

from conftest import BASE_CFG, full_cfg, golden, pkg, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GATE = 1e-8
GUARD = 1e-11


def _d():
    return golden("golden_aov_params.json")


def _window(cfg):
    T_p = cfg["T_p_GeV"]
    return cfg["T_min_over_Tp"] * T_p, cfg["T_max_over_Tp"] * T_p


def _facade(r):
    """boltzmann.BoltzmannSystem with bs.aov replaced, as make_golden_aov.py did on the reference."""
    B = pkg("boltzmann")
    cfg = pkg("config").Config(**full_cfg(r["config"]))
    bs = B.BoltzmannSystem(cfg, cfg.P_chi_to_B)
    a = r["aov"]
    bs.aov = B.AoverVKernel(a["I_p"], a["beta_over_H"], a["T_p"], a["v_w"], a["g_star"], z_max=r["z_max"], nz=r["nz"])
    return cfg, bs


def test_facade_matches_reference(gpu_engine):
    """integrate_YB_by_quadrature, A_over_V_y and S_B_T of the facade with bs.aov replaced."""
    worst = 0.0
    for r in _d()["yields"]:
        cfg, bs = _facade(r)
        got = bs.integrate_YB_by_quadrature(*_window(cfg.__dict__), n_y=8000)
        e = rel_err(got, r["Y_B"])
        assert e < GATE, (r["aov"], got, r["Y_B"])
        worst = max(worst, e)
        tol = 1e-11 * max(1.0, r["nz"] / 1200)
        for y, ref, g in zip(r["y"], r["Av"], bs.aov.A_over_V_ys(r["y"])):
            assert (g == ref == 0.0) or rel_err(g, ref) < tol, (r["aov"], y, g, ref)
        for T, ref in zip(r["T_SB"], r["S_B"]):
            g = bs.S_B_T(T)
            assert (g == ref == 0.0) or rel_err(g, ref) < tol, (r["aov"], T, g, ref)
    print(f"bs.aov replaced, facade vs reference: worst Y_B rel err {worst:.3e}")
    assert worst < GUARD


def test_engine_batch_matches_reference_and_oracle(gpu_engine):
    """All fixture systems of one z grid in one lzq_yields_batch launch with per-point
    lzq_aov_params: Y_B against the reference, every field against the oracle with the same kernel;
    and the same batch without the blocks reproduces the points' own kernels (the headline path)."""
    cfgm = pkg("config")
    rows = [r for r in _d()["yields"] if (r["nz"], r["z_max"]) == (1200, 30.0)]
    cfgs = [full_cfg(r["config"]) for r in rows]
    pts = np.concatenate([cfgm.to_point(c) for c in cfgs])
    aov = np.concatenate([cfgm.to_aov(r["aov"]) for r in rows])
    t = gpu_engine.yields(pts, aov=aov).cpu().numpy()
    own = gpu_engine.yields(pts).cpu().numpy()
    for row, o, r, c in zip(t, own, rows, cfgs):
        assert rel_err(row[0], r["Y_B"]) < GUARD, (r["aov"], row[0], r["Y_B"])
        ref = O.point_yields(c, aov=r["aov"])
        for k, v in zip(pkg("_native").YIELD_FIELDS, row):
            assert rel_err(v, ref[k]) < GUARD, (k, v, ref[k])
        assert rel_err(o[0], O.point_yields(c)["Y_B"]) < GUARD
        assert o[0] != row[0]


def test_own_kernel_block_is_bit_identical_to_headline(gpu_engine):
    """A block equal to the point's own kernel (what fpy:197 builds) gives the headline kernels'
    bits: the lzq_aov.hip kernels are the same quadrature with the same operations."""
    cfgm = pkg("config")
    rng = np.random.default_rng(5)
    cfgs = []
    for _ in range(40):
        c = full_cfg(BASE_CFG)
        c.update(I_p=float(rng.uniform(0.05, 1.0)), beta_over_H=float(10 ** rng.uniform(1, 3)),
                 v_w=float(rng.uniform(0.0, 0.95)), T_p_GeV=float(10 ** rng.uniform(0, 3)),
                 g_star=float(rng.uniform(10, 110)), m_chi_GeV=float(10 ** rng.uniform(-1, 3)))
        cfgs.append(c)
    pts = np.concatenate([cfgm.to_point(c) for c in cfgs])
    aov = np.concatenate([cfgm.to_aov(c) for c in cfgs])
    a = gpu_engine.yields(pts, aov=aov)
    b = gpu_engine.yields(pts)
    assert torch.equal(a, b)
    for nz, zm in ((2400, 45.0), (37, 7.5)):
        assert torch.equal(gpu_engine.yields(pts, aov=aov, nz=nz, z_max=zm), gpu_engine.yields(pts, nz=nz, z_max=zm))


def test_tables_rhs_and_ode_match_reference(gpu_engine):
    """build_tables + A_over_V_T + rhs of the facade with bs.aov replaced, and main()'s ODE
    fallback (Engine.ode with the kernel's block) against the reference's own solve_ivp."""
    d = _d()
    for t in d["tables"]:
        cfg, bs = _facade(t)
        bs.build_tables(*_window(cfg.__dict__), n=t["nt"])
        scale = max(abs(v) for v in t["Av"])
        for T, ref, g in zip(t["T"], t["Av"], bs.A_over_V_Ts(t["T"])):
            assert abs(g - ref) <= 1e-11 * abs(ref) + 1e-13 * scale, (T, g, ref)
        Ys = [Y for _ in t["x"] for Y in t["Y"]]
        xs = [x for x in t["x"] for _ in t["Y"]]
        # tests/test_gpu_ode.py's rhs tolerance: relative 1e-10 plus 1e-12 of the component's largest
        # magnitude (a value deep in the source window's tail carries the exponent's argument rounding)
        sc = np.max(np.abs(t["rhs"]), axis=0)
        for got, ref in zip(bs.rhs_batch(xs, Ys), t["rhs"]):
            for g, r, c in zip(got, ref, sc):
                assert abs(g - r) <= 1e-10 * abs(r) + 1e-12 * c, (got, ref)
    cfgm = pkg("config")
    for r in d["ode"]:
        c = full_cfg(r["config"])
        tab, st = gpu_engine.ode(cfgm.to_point(c), cfgm.to_ode_params(c), nz=r["nz"], z_max=r["z_max"], aov=r["aov"])
        o = tab.cpu().numpy()[0]
        assert int(st[0].item()) == 0
        assert rel_err(o[0], r["Y_B"]) < 1e-10, (o[0], r["Y_B"])
        assert rel_err(o[1], r["Y_chi"]) < 1e-10, (o[1], r["Y_chi"])
        ref = O.ode_point(c, nz=r["nz"], z_max=r["z_max"], aov=r["aov"])
        assert rel_err(o[0], ref["Y_B"]) < 1e-11 and rel_err(o[1], ref["Y_chi"]) < 1e-11


def test_ode_batch_with_blocks_in_launch_order(gpu_engine):
    """Engine.ode with per-point blocks over a batch big enough to be regrouped into cooperative
    wavefronts (wave_order): each point's result equals its own single-point run (the blocks follow
    their points through the permutation)."""
    cfgm = pkg("config")
    base = dict(full_cfg(BASE_CFG), Gamma_wash_over_H=0.5, T_max_over_Tp=1.6, T_min_over_Tp=0.6)
    rng = np.random.default_rng(3)
    cfgs, kern = [], []
    for i in range(160):
        c = dict(base, P_chi_to_B=float(rng.uniform(0.05, 0.9)), m_chi_GeV=[0.95, 2.0][i % 2])
        cfgs.append(c)
        kern.append({"I_p": float(rng.uniform(0.1, 0.9)), "beta_over_H": 100.0, "T_p": 100.0,
                     "v_w": float(rng.uniform(0.1, 0.9)), "g_star": 106.75})
    pts = np.concatenate([cfgm.to_point(c) for c in cfgs])
    ods = np.concatenate([cfgm.to_ode_params(c) for c in cfgs])
    aov = np.concatenate([cfgm.to_aov(k) for k in kern])
    tab, st = gpu_engine.ode(pts, ods, aov=aov)
    tab = tab.cpu().numpy()
    assert (st.cpu().numpy() == 0).all()
    for i in (0, 1, 57, 158, 159):
        one, s1 = gpu_engine.ode(pts[i:i + 1], ods[i:i + 1], aov=aov[i:i + 1], time_parallel=False)
        assert int(s1[0].item()) == 0
        assert np.array_equal(one.cpu().numpy()[0], tab[i]), i


def test_reference_side_binding(gpu_engine, monkeypatch):
    """plugins/lzq_binding.py installed on stand-ins with the reference's attributes: the
    quadrature operator, A_over_V_y and the batched build_tables replacement read bs.aov's own
    parameters and z grid."""
    import os
    from conftest import ROOT
    monkeypatch.syspath_prepend(os.path.join(ROOT, "plugins"))
    Bnd = importlib.import_module("lzq_binding")

    class KernelStandIn:  # fpy:141-156's attributes
        def __init__(self, I_p, beta_over_H, T_p, v_w, g_star, z_max=30.0, nz=1200):
            self.I_p, self.beta_over_H, self.T_p, self.v_w, self.g_star = I_p, beta_over_H, T_p, max(v_w, 1e-12), g_star
            self.z = np.linspace(0.0, z_max, nz)

    class SystemStandIn:  # fpy:193-201's attributes
        def __init__(self, cfg, P):
            self.cfg, self.P = cfg, float(P)
            self.aov = KernelStandIn(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star)

    from scipy.interpolate import CubicSpline

    def y_of_T(T, T_p, B):  # fpy:126-128
        return 0.5 * B * ((T_p / max(T, 1e-30)) ** 2 - 1.0)

    ns = types.SimpleNamespace(BoltzmannSystem=SystemStandIn, AoverVKernel=KernelStandIn, np=np,
                               CubicSpline=CubicSpline, y_of_T=y_of_T)
    Bnd.install(ns)
    d = _d()
    for r in d["yields"][::3]:
        cfg = pkg("config").Config(**full_cfg(r["config"]))
        bs = ns.BoltzmannSystem(cfg, cfg.P_chi_to_B)
        a = r["aov"]
        bs.aov = ns.AoverVKernel(a["I_p"], a["beta_over_H"], a["T_p"], a["v_w"], a["g_star"], z_max=r["z_max"],
                                 nz=r["nz"])
        got = bs.integrate_YB_by_quadrature(*_window(cfg.__dict__), n_y=8000)
        assert rel_err(got, r["Y_B"]) < GUARD, (a, got, r["Y_B"])
        tol = 1e-11 * max(1.0, r["nz"] / 1200)
        for y, ref in zip(r["y"], r["Av"]):
            g = bs.aov.A_over_V_y(y)
            assert (g == ref == 0.0) or rel_err(g, ref) < tol, (a, y, g, ref)
    t = d["tables"][0]
    cfg = pkg("config").Config(**full_cfg(t["config"]))
    bs = ns.BoltzmannSystem(cfg, cfg.P_chi_to_B)
    a = t["aov"]
    bs.aov = ns.AoverVKernel(a["I_p"], a["beta_over_H"], a["T_p"], a["v_w"], a["g_star"], z_max=t["z_max"], nz=t["nz"])
    bs.build_tables(*_window(cfg.__dict__), n=t["nt"])
    scale = max(abs(v) for v in t["Av"])
    T_lo, T_hi = _window(cfg.__dict__)
    for T, ref in zip(t["T"], t["Av"]):
        g = float(bs._A_spline(min(max(T, T_lo), T_hi)))   # fpy:214-217
        assert abs(g - ref) <= 1e-11 * abs(ref) + 1e-13 * scale, (T, g, ref)
