"""Edge cases of the HIP path through the C ABI: empty and ragged batches, grid ends, the
n_y floor of fpy:247, and the propagator's limits.  Needs an MI355X.

* empty batches return OK and empty outputs (no launch);
* ragged batch sizes (not multiples of the 16 waves of a block) give the same bits as the
  same points inside a larger batch (one wavefront per point, fixed-order reduction);
* a sweep slice at the very end of the grid equals the explicit points;
* n_y below 2000 is raised to 2000 exactly like ys = linspace(.., max(n_y, 2000)) (fpy:247);
* propagator: no coupling -> P = 0; one adiabatic crossing (delta > 16, closed-form cell)
  -> eq.(9) (fpy:183-184); ragged n.
"""
import math

import numpy as np
import pytest

from conftest import BASE_CFG, full_cfg, golden, pkg

pytestmark = pytest.mark.gpu
V_W = 0.3


def recs(cfgs):
    cfgm = pkg("config")
    return np.concatenate([cfgm.to_point(c) for c in cfgs])


def test_empty_batches(gpu_engine):
    empty = np.zeros(0, dtype=pkg("_native").POINT_DTYPE)
    assert tuple(gpu_engine.yields(empty).shape) == (0, 6)
    axes = [("m_mix", np.logspace(-3, 0, 4)), ("dprime", np.logspace(-3, 1, 4))]
    assert tuple(gpu_engine.sweep(BASE_CFG, axes, 0, 0).shape) == (0, 6)
    assert gpu_engine.p_closed_form(np.zeros(0)).numel() == 0
    assert gpu_engine.aov(full_cfg(BASE_CFG), np.zeros(0)).numel() == 0
    z = np.zeros((0, 3))
    assert gpu_engine.lz_propagate(z, z, z, V_W, 20.0, 100).numel() == 0


def test_ragged_batches_bit_identical(gpu_engine):
    pts = golden("golden_points.json")["points"][:40]
    r = recs([full_cfg(p["config"]) for p in pts])
    full = gpu_engine.yields(r).cpu().numpy()
    for k in (1, 15, 16, 17, 33):
        part = gpu_engine.yields(r[:k]).cpu().numpy()
        assert np.array_equal(part, full[:k], equal_nan=True), k
        tail = gpu_engine.yields(r[-k:]).cpu().numpy()
        assert np.array_equal(tail, full[-k:], equal_nan=True), k


def test_sweep_slice_at_grid_end(gpu_engine):
    m = np.logspace(-3, 0, 7)
    d = np.logspace(-3, 1, 9)
    axes = [("m_mix", m), ("dprime", d)]
    n = len(m) * len(d)
    got = gpu_engine.sweep(BASE_CFG, axes, n - 5, 5).cpu().numpy()
    idx = np.arange(n - 5, n)
    mi, di = m[idx // len(d)], d[idx % len(d)]
    v_w = full_cfg(BASE_CFG)["v_w"]
    P = gpu_engine.p_closed_form(mi * mi / (2.0 * v_w * di)).cpu().numpy()   # PAPER eq.(8)-(9)
    cfgs = [dict(full_cfg(BASE_CFG), P_chi_to_B=float(p)) for p in P]
    ref = gpu_engine.yields(recs(cfgs)).cpu().numpy()
    assert np.array_equal(got, ref)


def test_n_y_floor_matches_fpy247(gpu_engine):
    """Window T in [90, 110] GeV, where the y-grid resolution shows (Y_B moves 1.8e-8 between
    n_y = 2000 and 8000): n_y = 100 must give the n_y = 2000 bits."""
    import ctypes
    from oracle import oracle as O
    r = recs([full_cfg(BASE_CFG)])
    tl, th = np.array([90.0]), np.array([110.0])
    a, b, c = (gpu_engine.yields(r, n_y=ny, T_lo=tl, T_hi=th).cpu().numpy()[0, 0] for ny in (100, 2000, 8000))
    assert a == b
    p = O.point_from_config(full_cfg(BASE_CFG))
    for got, ny in ((b, 2000), (c, 8000)):
        ref = O.lib().oracle_yb_quadrature(ctypes.byref(p), 90.0, 110.0, ny)
        assert abs(got - ref) <= 1e-11 * abs(ref), (ny, got, ref)
    assert abs(b - c) > 1e-9 * abs(c)


def test_propagator_limits(gpu_engine):
    # no coupling: the state never leaves chi
    P0 = gpu_engine.lz_propagate([0.0], [1.0], [0.0], V_W, 10.0, 200).cpu().numpy()[0]
    assert P0 < 1e-24
    # one adiabatic crossing (delta = 33 > 16): the closed-form dressed cell alone
    m, d = 2.0, 0.2
    delta = m * m / (2 * V_W * d)
    P = gpu_engine.lz_propagate([m], [d], [0.0], V_W, 20.0, 100).cpu().numpy()[0]
    assert abs(P - (1.0 - math.exp(-2 * math.pi * delta))) < 1e-12
    # ragged n: each point's P independent of its batch
    rng = np.random.default_rng(3)
    mm = 10 ** rng.uniform(-3, 0, (257, 2))
    dd = 10 ** rng.uniform(-3, 1, (257, 2))
    xx = np.cumsum(np.full((257, 2), 60.0), axis=1) * np.sqrt(V_W / dd.min(axis=1, keepdims=True))
    full = gpu_engine.lz_propagate(mm, dd, xx, V_W, 20.0, 300).cpu().numpy()
    for k in (1, 255, 256):
        part = gpu_engine.lz_propagate(mm[:k], dd[:k], xx[:k], V_W, 20.0, 300).cpu().numpy()
        assert np.array_equal(part, full[:k]), k
    assert np.all((full >= -1e-12) & (full <= 1.0 + 1e-12))


def test_propagator_bounded_steps_and_bad_input(gpu_engine):
    """Round 2: a cell's Magnus steps are bounded by its core whatever the crossing spacing
    (round 1 computed max(S, 3 Phi_cell) with no bound: crossings 1e7 LZ lengths apart
    overflowed int); non-finite input gives NaN, not a hang; out-of-range arguments are
    rejected on the host."""
    import time
    import torch
    m, d = [0.1, 0.12, 0.6], [1.0, 0.8, 0.2]
    for gap in (60.0, 1e4, 1e7):
        x = [0.0, gap, 2 * gap]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        P = gpu_engine.lz_propagate([m], [d], [x], V_W, 20.0, 1000).cpu().numpy()[0]
        dt = time.perf_counter() - t0
        assert np.isfinite(P) and -1e-12 <= P <= 1.0 + 1e-12, (gap, P)
        assert dt < 2.0, (gap, dt)
    P = gpu_engine.lz_propagate([[float("nan"), 0.1]], [[1.0, 1.0]], [[0.0, 50.0]], V_W, 20.0, 100).cpu().numpy()[0]
    assert np.isnan(P)
    with pytest.raises(pkg("_native").LzqError, match="window_lz <= 200"):
        gpu_engine.lz_propagate([0.1], [1.0], [0.0], V_W, 500.0, 1000)
