"""The C-ABI library loads, exports exactly what include/lzq.h declares, and validates
arguments on the host (these calls return before any GPU work, so they run on CPU)."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT, pkg


def header_symbols():
    with open(os.path.join(ROOT, "include", "lzq.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lzq_[A-Za-z0-9_]+)\s*\(", src)))


def test_library_builds_and_exports_header_symbols():
    path = pkg("build").build()
    assert os.path.exists(path)
    L = ctypes.CDLL(path)
    syms = header_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(pkg("_native").EXPORTS) == syms


def test_abi_version_and_struct_layout():
    n = pkg("_native")
    L = n.load()
    assert L.lzq_abi_version() == pkg("_native").ABI_VERSION == 3
    assert ctypes.sizeof(n.LzqPoint) == 136 and ctypes.sizeof(n.LzqYield) == 48


def test_ztables_match_reference_grid():
    """fpy:154-156: z = linspace(0,30,1200), g4 verbatim; omega sums to int z^2 e^-z = 2."""
    z, g4, om = pkg("_native").ztables()
    assert np.array_equal(z, np.linspace(0.0, 30.0, 1200))
    ez = np.exp(-z)
    g4_np = 6.0 - ez * (z ** 3 + 3.0 * z ** 2 + 6.0 * z + 6.0)
    # numpy's AVX-512 exp differs from libm by 1 ulp on a few nodes
    assert np.max(np.abs(g4 - g4_np)) < 8 * np.finfo(float).eps
    assert np.all(g4 >= 0.0)
    assert abs(om.sum() - 2.0) < 1e-8


ZGRIDS = [(600, 30.0), (2400, 30.0), (12000, 30.0), (1200, 20.0), (1200, 60.0), (2400, 60.0), (37, 7.5)]


def test_ztables_runtime_grids():
    """AoverVKernel(..., z_max, nz) (fpy:141-156) for any grid: the library's host tables are
    numpy's linspace bit for bit, gamma4 the cancelling form to a few eps, and the weights
    integrate z^2 e^-z over [0, z_max] to the trapezoid's accuracy."""
    nat = pkg("_native")
    for nz, zmax in ZGRIDS:
        z, g4, om = nat.ztables(nz, zmax)
        assert np.array_equal(z, np.linspace(0.0, zmax, nz)), (nz, zmax)
        ez = np.exp(-z)
        g4_np = 6.0 - ez * (z ** 3 + 3.0 * z ** 2 + 6.0 * z + 6.0)
        assert np.max(np.abs(g4 - g4_np)) <= 16 * np.finfo(float).eps, (nz, zmax)   # 2 ulp(6)
        f = z * z * ez
        assert abs(om.sum() - np.trapezoid(f, z)) <= 1e-13, (nz, zmax)
    # numpy's degenerate grids: no node / one node / zero width -> A/V = 0 (empty trapezoid)
    for nz, zmax in ((0, 30.0), (1, 30.0), (5, 0.0)):
        z, g4, om = nat.ztables(nz, zmax)
        assert np.array_equal(z, np.linspace(0.0, zmax, nz)) and not np.any(om), (nz, zmax)


def test_ztables_refuse_bad_grids():
    """nz < 0 is numpy's ValueError; non-finite / negative z_max and grids so fine that the
    cancelling gamma4 of fpy:156 rounds below 0, or stops being non-decreasing (the exact-underflow
    lane test of zsum_dispatch reads gamma4_1 as the smallest node), are refused (LZQ_EINVAL) before
    any GPU work."""
    import pytest
    nat = pkg("_native")
    L = nat.load()
    for nz, zmax, msg in ((-1, 30.0, b"non-negative"), (1200, float("nan"), b"finite"), (1200, -1.0, b"finite"),
                          (1200, float("inf"), b"finite"), (nat.LZQ_NZ_MAX + 1, 30.0, b"LZQ_NZ_MAX"),
                          (2_000_000, 30.0, b"gamma4"), (20000, 1.0, b"non-decreasing"), (100000, 10.0, b"non-decreasing")):
        assert L.lzq_ztables(nz, zmax, None, None, None) == -1, (nz, zmax)
        assert msg in L.lzq_last_error(), (nz, zmax, L.lzq_last_error())
    with pytest.raises(ValueError, match="non-negative"):
        nat.zgrid(-3, 30.0)
    with pytest.raises(TypeError):
        nat.zgrid(1200.0, 30.0)   # numpy.linspace: 'float' object cannot be interpreted as an integer
    assert nat.zgrid(np.int64(600), 20) == (600, 20.0)


def test_host_side_argument_validation():
    n = pkg("_native")
    L = n.load()
    rc = L.lzq_yields_batch(None, -1, 8000, 1200, 30.0, None, None, None, None, None, None)
    assert rc == -1 and b"bad arguments" in L.lzq_last_error()
    rc = L.lzq_aov_batch(None, None, None, 1, 1200, 30.0, None, None)   # neither point nor block
    assert rc == -1 and b"bad arguments" in L.lzq_last_error()
    assert L.lzq_ode_tables(8, 1, None, None, 3, 1200, 30.0, None, 8, 12, None, None) == -1   # nt < 4
    assert b"nt = 3" in L.lzq_last_error()
    assert L.lzq_ode_tables(8, 2, None, None, 100, 1200, 30.0, None, 8, 799, None, None) == -1  # < 2 x 4 nt
    assert b"workspace" in L.lzq_last_error()
    assert L.lzq_ode_aov_T(None, 1.0, 2.0, 800, None, None, 1, None, None) == -1
    rc = L.lzq_p_closed_form(None, 0, None, None)  # n == 0 is a no-op
    assert rc == 0
    rc = L.lzq_lz_propagate(None, None, None, 4, 0, 0.3, 1.0, 10, None, None)
    assert rc == -1
    # bounded windows / steps (a cell's step count is bounded by its core)
    for K, S in ((300.0, 1000), (20.0, 2_000_000), (float("nan"), 1000)):
        rc = L.lzq_lz_propagate(8, 8, 8, 1, 1, 0.3, K, S, 8, None)
        assert rc == -1 and b"window_lz <= 200" in L.lzq_last_error(), (K, S)
    rc = L.lzq_ode_quadrature(8, 8, 4, 8, 0, 8, 1 << 20, 100, 8, None, None)   # shared index but no tables
    assert rc == -1
    rc = L.lzq_ode_integrate_shared(8, 8, 4, 8, 1, 8, 100, 1, 8, None, None)  # workspace < 1 table
    assert rc == -1 and b"workspace" in L.lzq_last_error()
    cfgm = pkg("config")
    base = cfgm.to_ctypes_point(cfgm.to_point({**cfgm.default_config(), "P_chi_to_B": 0.1}))
    ax = (n.LzqAxis * 1)()
    ax[0].field, ax[0].n, ax[0].values = 99, 3, 8
    rc = L.lzq_sweep_grid(ctypes.byref(base), ax, 1, 0, 1, 8000, 1200, 30.0, None, 8, None)
    assert rc == -1 and b"unknown field" in L.lzq_last_error()
    ax[0].field = n.FIELD["m_mix"]
    rc = L.lzq_sweep_grid(ctypes.byref(base), ax, 1, 0, 1, 8000, 1200, 30.0, None, 8, None)
    assert rc == -1 and b"swept together" in L.lzq_last_error()
    ax[0].field = n.FIELD["I_p"]
    rc = L.lzq_sweep_grid(ctypes.byref(base), ax, 1, 2, 5, 8000, 1200, 30.0, None, 8, None)
    assert rc == -1 and b"outside grid" in L.lzq_last_error()
    base.regime = n.REGIME_OTHER
    rc = L.lzq_sweep_grid(ctypes.byref(base), ax, 1, 0, 1, 8000, 1200, 30.0, None, 8, None)
    assert rc == -3


def test_engine_refuses_without_gpu():
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pkg("engine").Engine()


def test_ode_table_groups_host_logic():
    """Engine.ode's table sharing bookkeeping (engine.table_groups, device-agnostic torch):
    groups = bitwise-equal ODE_TABLE_KEY fields; other fields never split a group."""
    import torch
    n_ = pkg("_native")
    table_groups = pkg("engine").table_groups
    rng = np.random.default_rng(0)
    p = np.zeros(1000, dtype=n_.POINT_DTYPE)
    for f in n_.ODE_TABLE_KEY:
        p[f] = 1.25
    p["P_chi_to_B"] = rng.uniform(size=p.size)
    p["m_chi_GeV"] = rng.uniform(size=p.size)
    t = torch.from_numpy(p.view(np.uint8).copy())
    first, inv = table_groups(t, p.size)
    assert first.tolist() == [0] and int(inv.max()) == 0
    kinds = rng.integers(0, 7, p.size)
    p["I_p"] = 0.1 * kinds
    p["T_max_over_Tp"] = np.where(kinds == 3, 2.0, 1.6)
    first, inv = table_groups(torch.from_numpy(p.view(np.uint8).copy()), p.size)
    assert first.numel() == 7
    key = np.stack([p[f] for f in n_.ODE_TABLE_KEY], axis=1)
    assert np.array_equal(key[first.numpy()][inv.numpy()], key)
    assert all(int(f) == int(np.argmax(kinds == kinds[int(f)])) for f in first)   # first occurrence
    p["I_p"] = rng.uniform(size=p.size)                                           # all distinct: no sharing
    assert table_groups(torch.from_numpy(p.view(np.uint8).copy()), p.size) is None


def test_tune_ode_coop_knob():
    """lzq_tune(LZQ_TUNE_ODE_COOP): on by default, 0/1 only, returns the previous value."""
    n = pkg("_native")
    L = n.load()
    assert L.lzq_tune(n.TUNE_ODE_COOP, 0) == 1
    assert L.lzq_tune(n.TUNE_ODE_COOP, 1) == 0
    assert L.lzq_tune(n.TUNE_ODE_COOP, 2) < 0 and b"ode_coop" in L.lzq_last_error()


def test_tune_ode_tp_interval_knob():
    """lzq_tune(LZQ_TUNE_ODE_TP_INTERVAL): 64 steps by default, multiples of 64 in [64, 2^20] only
    (whole predictor blocks), returns the previous."""
    n = pkg("_native")
    L = n.load()
    assert L.lzq_tune(n.TUNE_ODE_TP_INTERVAL, 128) == 64
    assert L.lzq_tune(n.TUNE_ODE_TP_INTERVAL, 64) == 128
    for bad in (7, 16, 96, (1 << 20) + 64, -64):
        assert L.lzq_tune(n.TUNE_ODE_TP_INTERVAL, bad) < 0 and b"ode_tp_interval" in L.lzq_last_error()
    assert L.lzq_tune(n.TUNE_ODE_TP_INTERVAL, 64) == 64


def test_ode_integrate_tp_argument_checks():
    """lzq_ode_integrate_tp refuses bad arguments before any launch (no GPU needed)."""
    n = pkg("_native")
    L = n.load()
    assert L.lzq_ode_integrate_tp(8, 8, -1, None, 0, 8, 1 << 20, 100, 8, None, None, None) < 0
    assert L.lzq_ode_integrate_tp(8, 8, 4, 8, 0, 8, 1 << 20, 100, 8, None, None, None) < 0   # index, no tables
    assert L.lzq_ode_integrate_tp(8, 8, 4, None, 0, 8, 100, 100, 8, None, None, None) < 0    # workspace < 4 tables
    assert L.lzq_ode_integrate_tp(8, 8, 4, None, 0, 8, 1 << 20, -1, 8, None, None, None) < 0  # max_steps < 0
    assert L.lzq_ode_integrate_tp(None, None, 0, None, 0, None, 0, 0, None, None, None, None) == 0


def test_sweep_grid_reuse_workspace_and_validation():
    """lzq_sweep_grid_reuse_workspace: one table of max(n_y, 2000) + 6 doubles per combination of
    the grid's I_p / beta_over_H / T_p / T_min / T_max values; lzq_sweep_grid_reuse refuses a
    smaller workspace (no GPU work is launched on these paths)."""
    n = pkg("_native")
    L = n.load()
    sw = pkg("sweep")
    cfgm = pkg("config")
    vals = {}
    def axes_of(spec):
        arr = (n.LzqAxis * len(spec.axes))()
        for a, (name, v) in enumerate(spec.axes):
            buf = (ctypes.c_double * len(v))(*[float(x) for x in v])
            vals[(spec.name, a)] = buf
            arr[a].field, arr[a].n, arr[a].values = n.FIELD[name], len(v), ctypes.cast(buf, ctypes.c_void_p).value
        return arr
    specs = sw.builtin_specs()
    for name, tables in (("C2", 1), ("C3", 100), ("C4", 1000)):
        spec = specs[name]
        assert L.lzq_sweep_grid_reuse_workspace(axes_of(spec), len(spec.axes), 8000) == tables * 8006, name
        assert L.lzq_sweep_grid_reuse_workspace(axes_of(spec), len(spec.axes), 100) == tables * 2006, name
    spec = specs["C3"]
    base = cfgm.to_ctypes_point(cfgm.to_point({**cfgm.default_config(), "P_chi_to_B": 0.1}))
    rc = L.lzq_sweep_grid_reuse(ctypes.byref(base), axes_of(spec), len(spec.axes), 0, 10, 8000, 1200, 30.0, None, 8,
                                100 * 8006 - 1, 8, None)
    assert rc < 0 and b"workspace" in L.lzq_last_error()
    rc = L.lzq_sweep_grid_reuse(ctypes.byref(base), axes_of(spec), len(spec.axes), 0, 0, 8000, 1200, 30.0, None, None, 0,
                                None, None)
    assert rc == 0   # empty range: nothing to do


def test_new_entry_points_validate_arguments():
    """lzq_lz_propagate_v and lzq_yields_batch_reuse refuse bad arguments on the host (no GPU
    work is launched on these paths); empty batches are no-ops."""
    n = pkg("_native")
    L = n.load()
    rc = L.lzq_lz_propagate_v(8, 8, 8, None, 4, 1, 20.0, 1000, 8, None)        # no v_w array
    assert rc < 0 and b"lzq_lz_propagate_v" in L.lzq_last_error()
    rc = L.lzq_lz_propagate_v(8, 8, 8, 8, 4, 1, 300.0, 1000, 8, None)          # window too wide
    assert rc < 0 and b"window_lz <= 200" in L.lzq_last_error()
    assert L.lzq_lz_propagate_v(None, None, None, None, 0, 1, 20.0, 1000, None, None) == 0
    rc = L.lzq_yields_batch_reuse(8, 4, 8000, 1200, 30.0, None, None, 8, 1, 8, 10 ** 6, 8, None)   # no rep array
    assert rc < 0 and b"lzq_yields_batch_reuse" in L.lzq_last_error()
    rc = L.lzq_yields_batch_reuse(8, 4, 8000, 1200, 30.0, None, 8, 8, 2, 8, 2 * 8006 - 1, 8, None)  # workspace short
    assert rc < 0 and b"workspace" in L.lzq_last_error()
    assert L.lzq_yields_batch_reuse(None, 0, 8000, 1200, 30.0, None, None, None, 0, None, 0, None, None) == 0
