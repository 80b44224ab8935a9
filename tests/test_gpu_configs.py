"""BASELINE.json configs C1-C5 through the production grid path (lzq_sweep_grid: points
generated on device from the flat index), each named by its own test id.

- C1: the shipped config (yields_config_equal_mass.json) as a 0-axis grid, vs the reference's
  own output (golden_points.json point 0, made by running fpy:346-438).
- C2, C3, C4: >= 256 flat indices drawn with numpy default_rng(0) over the WHOLE builtin grid
  (sweep.builtin_specs()), plus every axis's first and last value, each evaluated
  by the grid kernel and compared with the C oracle (oracle/lzq_oracle.c, pinned to the
  reference by tests/test_oracle_golden.py) built from the host-side decode of the same index.
  Gate: the north_star 1e-8; asserted: the 1e-11 guard band.  No golden point of the
  reference's fixtures lies on these grids except the shipped config (C1), which is checked
  against the reference output directly.
- C4 at full size: one contiguous 1e6-point block (one beta/H value, 10 I_p values, the other axes in
  full) checked through size-independent properties: finite, Y_B linear in P
  along delta, Y_B v_w constant along v_w, the epilogue identities (fpy:413-417), and a
  random subsample against the oracle.
- C5: the multi-crossing spec (tests/test_gpu_sweep.py::test_c5_multicrossing_pipeline and
  tests/test_gpu_propagator.py hold the propagator-level checks); here: the sweep driver's
  C5 path against the propagator restatement + the C1 quadrature on sampled indices.
"""
import numpy as np
import pytest

from conftest import BASE_CFG, full_cfg, golden, pkg, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GATE = 1e-8
GUARD = 1e-11
S0_M3, GEV_TO_KG, M_PROTON_KG = 2891.0 * 1e6, 1.78266192e-27, 1.67262192369e-27  # fpy:33-39


def sample_indices(spec, n=256, seed=0):
    """n uniform flat indices (default_rng(seed)) + the first/last value of every axis."""
    rng = np.random.default_rng(seed)
    idx = set(int(i) for i in rng.integers(0, spec.total, n))
    sizes = [len(v) for _, v in spec.axes]
    strides = np.cumprod([1] + sizes[::-1])[:-1][::-1]
    for a, sz in enumerate(sizes):
        for j in (0, sz - 1):
            base = rng.integers(0, spec.total)
            digits = [(base // strides[b]) % sizes[b] for b in range(len(sizes))]
            digits[a] = j
            idx.add(int(sum(d * s for d, s in zip(digits, strides))))
    idx.update((0, spec.total - 1))
    return sorted(idx)


def oracle_cfg(spec, idx):
    """Host decode of one flat grid index -> reference Config (fpy:44-79) for the oracle."""
    prm = spec.point_params(idx)
    cfg = full_cfg(dict(spec.base))
    lz = {k: prm.pop(k) for k in ("delta_LZ", "m_mix", "dprime") if k in prm}
    cfg.update(prm)
    if "delta_LZ" in lz:
        cfg["P_chi_to_B"] = O.p_closed_form(lz["delta_LZ"])
    elif lz:
        cfg["P_chi_to_B"] = O.p_closed_form(lz["m_mix"] ** 2 / (2.0 * max(cfg["v_w"], 1e-12) * abs(lz["dprime"])))
    return cfg


def grid_rows(engine, spec, idxs):
    import torch
    out = torch.empty((len(idxs), 6), dtype=torch.float64, device=engine.device)
    for i, g in enumerate(idxs):
        engine.sweep(spec.base, spec.axes, g, 1, n_y=spec.n_y, out=out[i:i + 1])
    return out.cpu().numpy()


def check_vs_oracle(got, cfgs, label):
    ref = O.points_batch(cfgs, nthreads=16)
    worst, where = 0.0, None
    for i, (row, rr) in enumerate(zip(got, ref)):
        for k, a, b in zip(O.YIELD_FIELDS, row, rr):
            e = rel_err(a, b)
            assert e < GATE, (label, i, k, a, b, cfgs[i])
            if e > worst:
                worst, where = e, (i, k)
    print(f"{label}: {len(cfgs)} grid points vs oracle, worst rel err {worst:.3e} at {where}")
    assert worst < GUARD
    return ref


def test_config_C1_shipped(gpu_engine):
    """C1 through the grid kernel (0 axes, 1 point) == the reference's own main() output."""
    t = gpu_engine.sweep(full_cfg(BASE_CFG), [], 0, 1).cpu().numpy()[0]
    ref = golden("golden_points.json")["points"][0]
    assert ref["config"]["P_chi_to_B"] == BASE_CFG["P_chi_to_B"]
    for k, v in zip(O.YIELD_FIELDS, t):
        if k in ref["final"]:
            assert rel_err(v, ref["final"][k]) < GUARD, (k, v, ref["final"][k])
    assert f"{t[0]:.10e}" == "8.7208853627e-11" and f"{t[4]:.10f}" == "5.6889263349"  # PAPER eqs.(19),(21)


@pytest.mark.parametrize("name", ["C2", "C3", "C4"])
def test_config_grid_vs_oracle(gpu_engine, name):
    spec = pkg("sweep").builtin_specs()[name]
    idxs = sample_indices(spec)
    assert len(idxs) >= 256
    got = grid_rows(gpu_engine, spec, idxs)
    cfgs = [oracle_cfg(spec, g) for g in idxs]
    check_vs_oracle(got, cfgs, name)
    if name == "C3":
        # the sample must straddle the strict T > m/3 branch of n_chi_eq / vbar_chi (fpy:90-120)
        # inside the integration window [T_min, T_max] = [0.1, 500] GeV
        m = np.array([c["m_chi_GeV"] for c in cfgs])
        assert np.any(m / 3 > 0.1) and np.any(m / 3 < 500.0) and np.any((m / 3 > 0.1) & (m / 3 < 500.0))
    if name == "C4":
        # every axis of C4 (beta/H, I_p, v_w, sigma_y, m_chi, delta) takes >= 5 distinct values
        for a, (field, vals) in enumerate(spec.axes):
            seen = {spec.point_params(g)[field] for g in idxs}
            assert len(seen) >= 5, field


@pytest.mark.parametrize("name,start", [("C2", 123_456), ("C3", 50 * 100_000 + 20_000)])
def test_config_full_occupancy_launch(gpu_engine, name, start):
    """One lzq_sweep_grid launch over a contiguous 65,536-index slice (1024 blocks of 16
    wavefronts: the multi-wave, many-block geometry of the production sweeps, which the one-point
    launches of test_config_grid_vs_oracle do not exercise), 256 default_rng(0)-sampled rows vs the
    oracle at the guard band.  The C3 slice (m_chi index 50, m_chi = 59 GeV) has its T = m/3
    branch inside the integration window."""
    spec = pkg("sweep").builtin_specs()[name]
    n = 65_536
    t = gpu_engine.sweep(spec.base, spec.axes, start, n).cpu().numpy()
    assert np.isfinite(t).all()
    sub = np.sort(np.random.default_rng(0).choice(n, 256, replace=False))
    cfgs = [oracle_cfg(spec, start + int(i)) for i in sub]
    if name == "C3":
        m = {c["m_chi_GeV"] for c in cfgs}
        assert all(0.1 < mm / 3 < 500.0 for mm in m), m
    check_vs_oracle(t[sub], cfgs, f"{name} 65536-point launch")
    # the same rows from one-point launches: bit-identical (geometry-independent results)
    assert np.array_equal(grid_rows(gpu_engine, spec, [start + int(i) for i in sub[:16]]), t[sub[:16]])


def test_config_C4_full_block_properties(gpu_engine):
    """One contiguous 1e6-point block of the 1e8-point C4 grid (beta/H index 3, I_p indices
    40..49, every other axis in full): size-independent properties of the reference's formulas."""
    spec = pkg("sweep").builtin_specs()["C4"]
    names = [n for n, _ in spec.axes]
    assert names == ["beta_over_H", "I_p", "v_w", "source_shape_sigma_y", "m_chi_GeV", "delta_LZ"]
    block = 1_000_000
    per_ip = spec.total // (len(spec.axes[0][1]) * len(spec.axes[1][1]))   # 1e5 points per (beta/H, I_p)
    assert per_ip * 10 == block
    start = 3 * (spec.total // 10) + 40 * per_ip
    t = gpu_engine.sweep(spec.base, spec.axes, start, block).cpu().numpy()
    assert np.isfinite(t).all()
    YB, Ych, rB, rD, ratio, P = (t[:, j] for j in range(6))
    shp = [10] + [len(v) for _, v in spec.axes[2:]]    # (I_p, v_w, sigma_y, m_chi, delta)
    # P_used = eq.(9) of the delta axis (fpy:183-184, naive 1 - exp)
    dl = np.broadcast_to(spec.axes[5][1], shp).ravel()
    assert np.allclose(P, 1.0 - np.exp(-2.0 * np.pi * dl), rtol=1e-13, atol=5e-16)
    # Y_B linear in P along delta (fpy:264): Y_B / P constant to rounding
    r = (YB / P).reshape(shp)
    assert np.max(np.abs(r / r[..., :1] - 1.0)) < 1e-14
    # Y_B proportional to 1/v_w along the v_w axis (A/V prefactor beta/v_w, fpy:162)
    w = (YB.reshape(shp) * np.asarray(spec.axes[2][1])[None, :, None, None, None])
    assert np.max(np.abs(w / w[:, :1] - 1.0)) < 1e-13
    # Y_B > 0 everywhere in this block (the window is never empty)
    assert np.all(YB > 0)
    # epilogue (fpy:376-384, 413-417): nonthermal Y_chi = Y_chi_init; densities and ratio
    assert np.all(Ych == spec.base["Y_chi_init"])
    mchi = np.broadcast_to(np.asarray(spec.axes[4][1])[None, None, None, :, None], shp).ravel()
    assert np.array_equal(rB, (YB * S0_M3) * M_PROTON_KG)
    assert np.allclose(rD, (Ych * S0_M3) * (mchi * GEV_TO_KG), rtol=4.5e-16, atol=0)
    assert np.allclose(ratio, rD / np.maximum(rB, 1e-300), rtol=4.5e-16, atol=0)
    # 64 random points of the block against the oracle
    sub = np.sort(np.random.default_rng(1).choice(block, 64, replace=False))
    check_vs_oracle(t[sub], [oracle_cfg(spec, start + int(i)) for i in sub], "C4 block")


def test_config_C5_sweep_driver(gpu_engine):
    """C5 (N = 8 coherent crossings per point) through sweep.make_compute at 32 sampled
    indices: P_used = the propagator restatement (tests/lz_ref.py, which
    tests/test_propagator_exact.py pins to the exact Weber solution), Y_B = P_used x the C1
    quadrature per unit P."""
    import torch
    from lz_ref import propagate
    sw = pkg("sweep")
    spec = sw.builtin_specs()["C5"]
    comp = sw.make_compute(spec, gpu_engine)
    rng = np.random.default_rng(0)
    YB1 = 8.720885362714675e-11 / 0.14925839040304145
    for g in sorted(int(i) for i in rng.integers(0, spec.total, 32)):
        out = torch.empty((1, 6), dtype=torch.float64, device=gpu_engine.device)
        comp(g, 1, out)
        o = out.cpu().numpy()[0]
        m, dp, xi, v_w = (x.cpu().numpy() if hasattr(x, "cpu") else x for x in spec.crossing_arrays(g, 1, "cpu"))
        ref = propagate(list(m[0]), list(dp[0]), list(xi[0]), float(v_w[0]), spec.crossings.window_lz,
                        spec.crossings.steps)
        assert abs(o[5] - ref) <= 1e-10 * max(ref, 1e-3), (g, o[5], ref)
        if o[5] > 1e-8:
            assert rel_err(o[0] / o[5], YB1) < 1e-11, (g, o)
