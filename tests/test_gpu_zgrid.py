"""The A/V kernel's z grid through the C ABI: AoverVKernel(I_p, beta_over_H, T_p, v_w, g_star,
z_max, nz) (fpy:141-156) for any (nz, z_max), on the GPU.  Needs an MI355X.

Pinned to tests/golden/golden_zgrid.json, which tests/golden/make_golden_zgrid.py made by running
the reference with `bs.aov = AoverVKernel(..., z_max=z_max, nz=nz)` (10 grids: nz = 0, 1, 5, 37,
600, 1200, 2400, 12000; z_max = 0, 7.5, 20, 30, 60), and to the CPU oracle on fresh points.
Tolerances: north_star's 1e-8 gate and the 1e-11 guard band of the golden tests on Y_B; A/V and
tables as the oracle's own pins (tests/test_oracle_golden.py), whose error against numpy grows with
nz through the cancelling gamma4 (fpy:156).
"""
import numpy as np
import pytest
import torch

from conftest import BASE_CFG, full_cfg, golden, pkg, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GATE = 1e-8
GUARD = 1e-11


def recs(cfgs):
    cfgm = pkg("config")
    return np.concatenate([cfgm.to_point(c) for c in cfgs])


def by_grid(rows):
    out = {}
    for r in rows:
        out.setdefault((r["nz"], r["z_max"]), []).append(r)
    return out


def test_zgrid_yields_vs_reference(gpu_engine):
    """Y_B on 10 grids, main()'s window, against the reference run with bs.aov replaced."""
    worst = 0.0
    for (nz, zmax), rows in by_grid(golden("golden_zgrid.json")["yields"]).items():
        cfgs = [full_cfg(r["config"]) for r in rows]
        t = gpu_engine.yields(recs(cfgs), nz=nz, z_max=zmax).cpu().numpy()
        for row, r in zip(t, rows):
            if r["Y_B"] == 0.0:
                assert row[0] == 0.0, (nz, zmax, row[0])
                continue
            e = rel_err(row[0], r["Y_B"])
            assert e < GATE, (nz, zmax, row[0], r["Y_B"])
            worst = max(worst, e)
    print(f"z grids vs reference: worst rel err {worst:.3e}")
    assert worst < GUARD


def test_zgrid_vs_oracle_fresh_points(gpu_engine):
    """Seeded points the fixtures do not hold, every output field, against the C oracle on the
    same grid (both use libm tables: agreement far inside the guard band)."""
    rng = np.random.default_rng(77)
    cfgs = []
    for _ in range(24):
        c = full_cfg(BASE_CFG)
        c.update(m_chi_GeV=float(10 ** rng.uniform(-1, 3.5)), I_p=float(rng.uniform(0.05, 1.0)),
                 beta_over_H=float(10 ** rng.uniform(1, 3)), v_w=float(rng.uniform(0.05, 0.95)),
                 P_chi_to_B=float(rng.uniform(0, 1)), regime=str(rng.choice(["thermal", "nonthermal"])))
        cfgs.append(c)
    for nz, zmax in ((600, 30.0), (2400, 60.0), (4801, 25.0), (13, 3.0)):
        t = gpu_engine.yields(recs(cfgs), nz=nz, z_max=zmax).cpu().numpy()
        ref = O.points_batch(cfgs, nthreads=16, nz=nz, z_max=zmax)
        worst = max(rel_err(a, b) for row, rr in zip(t, ref) for a, b in zip(row, rr))
        print(f"grid ({nz}, {zmax}): worst rel err vs oracle {worst:.3e}")
        assert worst < 1e-12, (nz, zmax, worst)


def test_default_grid_unchanged(gpu_engine):
    """(1200, 30.0) is main()'s grid and runs the compile-time kernels: same bits as the default
    call, and the shipped config's published Y_B."""
    r = recs([full_cfg(BASE_CFG)])
    a = gpu_engine.yields(r).cpu().numpy()
    b = gpu_engine.yields(r, nz=1200, z_max=30.0).cpu().numpy()
    assert np.array_equal(a, b)
    assert f"{a[0, 0]:.10e}" == "8.7208853627e-11"


def test_zgrid_aov_vs_reference(gpu_engine):
    for case in golden("golden_zgrid.json")["aov"]:
        cfg = full_cfg(case["config"])
        got = gpu_engine.aov(cfg, case["y"], nz=case["nz"], z_max=case["z_max"]).cpu().numpy()
        tol = 1e-10 * max(1.0, case["nz"] / 1200)
        for y, g, r in zip(case["y"], got, case["Av"]):
            if r == 0.0:
                assert g == 0.0, (case["nz"], y, g)
            else:
                assert rel_err(g, r) < tol, (case["nz"], case["z_max"], y, g, r)


def test_operator_mirror_zgrid(gpu_engine):
    """The reference-shaped operator API: bs.aov = AoverVKernel(..., z_max, nz), then
    integrate_YB_by_quadrature / A_over_V_y / z / g4, as the fixture generator drove fpy."""
    bz = pkg("boltzmann")
    cfgm = pkg("config")
    d = golden("golden_zgrid.json")
    for r in [r for r in d["yields"] if r["nz"] in (600, 12000, 37, 0)][:8]:
        c = full_cfg(r["config"])
        cfg = cfgm.Config(**c)
        bs = bz.BoltzmannSystem(cfg, cfg.P_chi_to_B)
        bs.aov = bz.AoverVKernel(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star, z_max=r["z_max"],
                                 nz=r["nz"])
        T_p = cfg.T_p_GeV
        got = bs.integrate_YB_by_quadrature(cfg.T_min_over_Tp * T_p, cfg.T_max_over_Tp * T_p, n_y=8000)
        assert (got == 0.0) if r["Y_B"] == 0.0 else rel_err(got, r["Y_B"]) < GUARD, (r["nz"], got, r["Y_B"])
        assert np.array_equal(bs.aov.z, np.linspace(0.0, r["z_max"], r["nz"]))
    with pytest.raises(ValueError):
        bz.AoverVKernel(0.34, 100.0, 100.0, 0.3, 106.75, nz=-2)
    with pytest.raises(TypeError):
        bz.AoverVKernel(0.34, 100.0, 100.0, 0.3, 106.75, nz=1200.0)


def test_zgrid_build_tables_vs_reference(gpu_engine):
    """build_tables(T_lo, T_hi, n) for n = 50 / 200 / 800 / 1600 on three grids, A_over_V_T and rhs,
    through the operator mirror (lzq_ode_tables / lzq_ode_aov_T / lzq_ode_rhs with nt, nz, z_max)."""
    bz = pkg("boltzmann")
    cfgm = pkg("config")
    for t in golden("golden_zgrid.json")["tables"]:
        c = full_cfg(t["config"])
        cfg = cfgm.Config(**c)
        bs = bz.BoltzmannSystem(cfg, cfg.P_chi_to_B)
        bs.aov = bz.AoverVKernel(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star, z_max=t["z_max"],
                                 nz=t["nz"])
        T_p = cfg.T_p_GeV
        bs.build_tables(cfg.T_min_over_Tp * T_p, cfg.T_max_over_Tp * T_p, n=t["nt"])
        got = bs.A_over_V_Ts(t["T"])
        scale = max(abs(v) for v in t["Av"])
        for T, g, r in zip(t["T"], got, t["Av"]):
            assert abs(g - r) <= 1e-10 * abs(r) + 1e-13 * scale, (t["nt"], T, g, r)
        xs = [x for x in t["x"] for _ in t["Y"]]
        Ys = [Y for _ in t["x"] for Y in t["Y"]]
        dY = bs.rhs_batch(xs, Ys)
        for g, r in zip(dY, t["rhs"]):
            for a, b in zip(g, r):
                assert abs(a - b) <= 1e-10 * abs(b) + 1e-300, (t["nt"], a, b)
    with pytest.raises(ValueError):
        bs.build_tables(1.0, 2.0, n=3)


def test_zgrid_ode_vs_reference(gpu_engine):
    """main()'s ODE fallback with bs.aov on (2400, 30) / (1200, 20): Engine.ode(nz, z_max) against
    the reference's adaptive Radau (narrow wash-out windows, ~1e-13 from converged)."""
    cfgm = pkg("config")
    for r in golden("golden_zgrid.json")["ode"]:
        c = full_cfg(r["config"])
        tab, st = gpu_engine.ode(cfgm.to_point(c), cfgm.to_ode_params(c), nz=r["nz"], z_max=r["z_max"])
        o = tab.cpu().numpy()[0]
        assert int(st[0].item()) == 0
        assert rel_err(o[0], r["Y_B"]) < 1e-10, (o[0], r["Y_B"])
        assert rel_err(o[1], r["Y_chi"]) < 1e-10, (o[1], r["Y_chi"])


def test_zgrid_sweep_and_reuse(gpu_engine):
    """A sweep on a runtime grid (Engine.sweep nz / z_max): the dense grid kernel matches the oracle,
    the z-sum reuse mode is bit-identical to it, and a reuse table of another grid is refused
    (its header records (nz, z_max): NaN yields, never another grid's values)."""
    sw = pkg("sweep")
    spec = sw.builtin_specs()["C3"]
    n = 2048
    nz, zmax = 2400, 45.0
    dense = gpu_engine.sweep(spec.base, spec.axes, 1_000_000, n, nz=nz, z_max=zmax).cpu().numpy()
    reuse = gpu_engine.sweep(spec.base, spec.axes, 1_000_000, n, nz=nz, z_max=zmax, reuse=True).cpu().numpy()
    assert gpu_engine.last_reuse == "tables"
    assert np.array_equal(dense, reuse, equal_nan=True)
    idx = np.random.default_rng(3).choice(n, 24, replace=False)
    pts, _ = sw.grid_records(spec, 1_000_000, n, gpu_engine)
    cfgs = []
    cfgm = pkg("config")
    for i in idx:
        c = dict(full_cfg(spec.base))
        for f in ("m_chi_GeV", "I_p", "P_chi_to_B"):
            c[f] = float(pts[f][i])
        cfgs.append(c)
    ref = O.points_batch(cfgs, nthreads=16, nz=nz, z_max=zmax)
    for i, rr in zip(idx, ref):
        for a, b in zip(dense[i], rr):
            assert rel_err(a, b) < 1e-12, (i, a, b)
    # tables built for the default grid, read with the runtime grid's key: NaN rows
    nat = pkg("_native")
    import ctypes
    eng = gpu_engine
    base = cfgm.to_ctypes_point(cfgm.to_point(spec.base))
    vals = [torch.as_tensor(np.asarray(v, dtype=np.float64), device=eng.device) for _, v in spec.axes]
    arr = (nat.LzqAxis * len(spec.axes))()
    for a, ((name, _), t) in enumerate(zip(spec.axes, vals)):
        arr[a].field, arr[a].n, arr[a].values = nat.FIELD[name], t.numel(), t.data_ptr()
    need = eng.lib.lzq_sweep_grid_reuse_workspace(arr, len(spec.axes), 8000)
    work = torch.empty(need, dtype=torch.float64, device=eng.device)
    out = torch.empty((64, 6), dtype=torch.float64, device=eng.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(eng.device).cuda_stream)
    nat.check(eng.lib.lzq_sweep_grid_ztables(ctypes.byref(base), arr, len(spec.axes), 8000, 1200, 30.0,
                                             ctypes.c_void_p(work.data_ptr()), need, s), eng.lib)
    nat.check(eng.lib.lzq_sweep_grid_from_ztables(ctypes.byref(base), arr, len(spec.axes), 0, 64, 8000, nz, zmax, None,
                                                  ctypes.c_void_p(work.data_ptr()), need,
                                                  ctypes.c_void_p(out.data_ptr()), s), eng.lib)
    o = out.cpu().numpy()
    assert np.all(np.isnan(o[:, 0])) and np.all(np.isfinite(o[:, 1]))


def test_zgrid_refused_on_device_entry(gpu_engine):
    """A grid the library refuses (gamma4 < 0) fails the call with LZQ_EINVAL before any launch."""
    nat = pkg("_native")
    with pytest.raises(nat.LzqError, match="gamma4"):
        gpu_engine.yields(recs([full_cfg(BASE_CFG)]), nz=2_000_000, z_max=30.0)
