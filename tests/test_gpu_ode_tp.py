"""lzq_ode_integrate_tp: the ODE fallback integrated parallel in time (multiple shooting with
Newton on the interval boundaries, then the exact chains stitched through candidate starts) --
the latency path for the CLI's single point.  Its result is the sequential integration's
(lzq_ode_integrate, the reference's fixed-step Radau) bit for bit: checked on the reference's own
ODE cases, the stiff split-step cases, a seeded batch and other interval lengths, with the points
it stitched counted (Newton updates > 0); points it does not take (bad windows, step caps,
batches of more than 64) come back from the sequential integration.  Needs an MI355X."""
import os

import numpy as np
import pytest
import torch

from conftest import BASE_CFG, GOLDEN, full_cfg, golden, pkg, rel_err
from test_gpu_ode import NARROW, recs, seeded_cfgs

pytestmark = pytest.mark.gpu


def both(eng, cfgs, **kw):
    p, o = recs(cfgs)
    a, sa = eng.ode(p, o, time_parallel=False, **kw)
    b, sb = eng.ode(p, o, time_parallel=True, **kw)
    it = eng.last_ode_tp_iters.cpu().numpy()
    return a.cpu().numpy(), sa.cpu().numpy(), b.cpu().numpy(), sb.cpu().numpy(), it


def close(a, b):
    """bit for bit (NaN rows of refused points included)"""
    assert np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True), (a, b)
    return 0.0


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLDEN, "golden_ode.json")), reason="golden_ode.json")
def test_tp_reference_cases_one_point_each(gpu_engine):
    """Each of the reference's ODE cases as a single point (Engine.ode's default for n == 1 is
    time-parallel): statuses and yields equal to the sequential integration's bit for bit, and
    the long windows really stitched (Newton updates > 0)."""
    steps = pkg("engine").ode_step_counts
    worst = 0.0
    for r in golden("golden_ode.json")["points"]:
        cfg = full_cfg(r["config"])
        p, o = recs([cfg])
        a, sa = gpu_engine.ode(p, o, time_parallel=False)
        b, sb = gpu_engine.ode(p, o)          # default: time-parallel for one point
        it = int(gpu_engine.last_ode_tp_iters[0])
        assert int(sa[0]) == int(sb[0]), (r["config"], sa, sb)
        if int(sa[0]) == 0:
            worst = max(worst, close(b.cpu().numpy(), a.cpu().numpy()))
            n = steps(p)[0]
            assert (it > 0) == (n > 64), (n, it)   # >= 2 intervals of the default 64 steps
        else:
            assert it == 0 and np.isnan(b.cpu().numpy()[0, :5]).all()
    print("time-parallel vs sequential over the reference's ODE cases: bit-identical")


def test_tp_stiff_split_cases(gpu_engine):
    """The two stiff annihilation cases whose window crosses the T = m/3 branch (the split step lies
    inside an interval; the Riccati Newton iteration runs near its other root), as a batch."""
    from test_ode_oracle import stiff_cases
    cfgs = [full_cfg(c["config"]) for c in stiff_cases()]
    a, sa, b, sb, it = both(gpu_engine, cfgs)
    assert (sa == 0).all() and (sb == 0).all() and (it > 0).all(), (sa, sb, it)
    close(b, a)


def test_tp_seeded_batch_and_fallbacks(gpu_engine):
    """24 seeded configs (thermal/nonthermal, boson/fermion, wash-out, annihilation, depletion) as
    one time-parallel batch, plus points the iteration does not take: a zero-width window
    (LZQ_ODE_BAD_GRID), a reversed one, and a step cap (LZQ_ODE_TOO_MANY_STEPS) -- statuses and
    NaN rows as the sequential integration's, Newton updates 0 for them."""
    cfgs = seeded_cfgs(24, seed=29)
    cfgs += [full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.0, "T_min_over_Tp": 1.0}),
             full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, "T_max_over_Tp": 0.5, "T_min_over_Tp": 0.9})]
    a, sa, b, sb, it = both(gpu_engine, cfgs)
    assert sa.tolist() == sb.tolist()
    assert sa[-2:].tolist() == [1, 1] and it[-2:].tolist() == [0, 0]
    assert (it[:24][sa[:24] == 0] > 0).all()
    close(b, a)
    # the step cap: not iterated, the sequential status
    p, o = recs([full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0})])
    t, st = gpu_engine.ode(p, o, max_steps=100_000, time_parallel=True)
    assert int(st[0]) == 3 and int(gpu_engine.last_ode_tp_iters[0]) == 0 and np.isnan(t.cpu().numpy()[0, :5]).all()


def test_tp_large_batch_is_sequential(gpu_engine):
    """More than 64 points: lzq_ode_integrate_tp is lzq_ode_integrate, bit for bit."""
    cfgs = [dict(c, **NARROW) for c in seeded_cfgs(70, seed=4)]
    a, sa, b, sb, it = both(gpu_engine, cfgs)
    assert (it == 0).all() and np.array_equal(sa, sb) and np.array_equal(a, b, equal_nan=True)


def test_tp_shipped_window_riccati_and_intervals(gpu_engine):
    """The CLI's slow case, one sigma_v != 0 point over the shipped window (~1e6 Radau steps): within
    the sequential result at the default interval (64 steps) and at 128 and 256
    (LZQ_TUNE_ODE_TP_INTERVAL), bit for bit; the per-table and the shared-table entries agree; and
    the A/V kernel's own parameters (per-point tables) go through too."""
    nat = pkg("_native")
    cfg = full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, "sigma_v_chi_GeV_m2": 1e-12})
    p, o = recs([cfg])
    a, sa = gpu_engine.ode(p, o, time_parallel=False)
    a = a.cpu().numpy()
    assert int(sa[0]) == 0
    for L in (64, 128, 256):
        prev = gpu_engine.lib.lzq_tune(nat.TUNE_ODE_TP_INTERVAL, L)
        try:
            for share in (True, False):
                b, sb = gpu_engine.ode(p, o, time_parallel=True, share_tables=share)
                it = int(gpu_engine.last_ode_tp_iters[0])
                assert int(sb[0]) == 0 and it > 0, (L, share, it)
                close(b.cpu().numpy(), a)
                print(f"interval {L} share {share}: {it} Newton updates, bit-identical")
        finally:
            gpu_engine.lib.lzq_tune(nat.TUNE_ODE_TP_INTERVAL, prev)
    assert gpu_engine.lib.lzq_tune(nat.TUNE_ODE_TP_INTERVAL, 64) == 64
    # bs.aov replaced (the A/V parameter block): per-point tables
    aov = {"I_p": 0.4, "beta_over_H": 60.0, "T_p_GeV": cfg["T_p_GeV"], "v_w": 0.5, "g_star": cfg["g_star"]}
    a2, sa2 = gpu_engine.ode(p, o, time_parallel=False, aov=aov)
    b2, sb2 = gpu_engine.ode(p, o, time_parallel=True, aov=aov)
    assert int(sa2[0]) == int(sb2[0]) == 0 and int(gpu_engine.last_ode_tp_iters[0]) > 0
    close(b2.cpu().numpy(), a2.cpu().numpy())
    assert rel_err(float(b2[0, 0]), float(a[0, 0])) > 1e-6   # another kernel, another Y_B


def test_tp_is_stream_ordered_and_deterministic(gpu_engine):
    """No host synchronisation inside the call: two runs on a side stream give the same bits."""
    cfgs = [full_cfg({**BASE_CFG, "sigma_v_chi_GeV_m2": 1e-9}), full_cfg({**BASE_CFG, **NARROW,
                                                                         "sigma_v_chi_GeV_m2": 1e-12})]
    p, o = recs(cfgs)
    s = torch.cuda.Stream(gpu_engine.device)
    with torch.cuda.stream(s):
        x, sx = gpu_engine.ode(p, o, time_parallel=True)
        y, sy = gpu_engine.ode(p, o, time_parallel=True)
    s.synchronize()
    assert torch.equal(sx, sy) and torch.equal(x, y) and bool((sx == 0).all())


def test_tp_raw_abi_large_step_cap(gpu_engine):
    """The C ABI with a step cap far above the window's need (max_steps only sizes the node arrays:
    the point takes intervals of its own length) and with d_iters / d_status NULL."""
    import ctypes
    cfg = full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, "sigma_v_chi_GeV_m2": 1e-12})
    p, o = recs([cfg])
    ref, sr = gpu_engine.ode(p, o, time_parallel=False)
    d_p = gpu_engine.points_to_device(p)
    d_o = torch.from_numpy(np.ascontiguousarray(o).view(np.uint8).copy()).to(gpu_engine.device)
    work, st = gpu_engine.ode_tables(d_p)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    for cap, with_iters in ((1 << 40, True), (1 << 22, False)):
        out = torch.empty((1, 6), dtype=torch.float64, device=gpu_engine.device)
        its = torch.zeros(1, dtype=torch.int32, device=gpu_engine.device)
        rc = gpu_engine.lib.lzq_ode_integrate_tp(vp(d_p), vp(d_o), 1, None, 0, vp(work), work.numel(), cap, vp(out),
                                                 None, vp(its) if with_iters else None, None)
        assert rc == 0
        torch.cuda.synchronize()
        if with_iters:
            assert int(its[0]) > 0
        close(out.cpu().numpy(), ref.cpu().numpy())


def test_wide_tables_bit_identical(gpu_engine):
    """LZQ_TUNE_ODE_TABLE_WIDE (round 6): few tables built a wavefront wide -- the spline's per-knot
    work spread over the lanes around its two recurrences (ode_spline_wave_kernel), the A/V knots
    over 64-knot wavefronts -- give the one-lane / one-wave tables bit for bit: main()'s 800 knots,
    knot counts around the 64-lane chunk edges and the smallest, own windows, the A/V kernel's own
    parameters, and a batch above the wide path's 4096-table limit (which takes the narrow kernels)."""
    rng = np.random.default_rng(11)
    cfgs = seeded_cfgs(7, seed=11)
    p, _ = recs(cfgs)
    n = len(cfgs)
    Tp = np.array([c["T_p_GeV"] for c in cfgs])
    T_lo = torch.tensor(Tp * rng.uniform(0.05, 0.6, n), dtype=torch.float64, device=gpu_engine.device)
    T_hi = torch.tensor(Tp * rng.uniform(1.1, 4.0, n), dtype=torch.float64, device=gpu_engine.device)
    aov = {"I_p": 0.27, "beta_over_H": 63.0, "T_p_GeV": 81.0, "v_w": 0.41, "g_star": 100.5}
    try:
        for kw in ({}, {"T_lo": T_lo, "T_hi": T_hi}, {"aov": aov}):
            for nt in (800, 4, 5, 63, 64, 65, 127, 129, 1000):
                tabs = []
                for wide in (False, True):
                    gpu_engine.tune_ode_table_wide(wide)
                    # a zeroed workspace: a table leaves two spare doubles of its last knot unwritten
                    work = torch.zeros(n * 4 * nt, dtype=torch.float64, device=gpu_engine.device)
                    w, st = gpu_engine.ode_tables(p, nt=nt, work=work, **kw)
                    tabs.append((w.cpu().numpy(), st.cpu().numpy()))
                assert np.array_equal(tabs[0][1], tabs[1][1]), (kw.keys(), nt)
                assert np.array_equal(tabs[0][0], tabs[1][0], equal_nan=True), (list(kw), nt)
        # one point (the CLI's case) and a batch past the wide limit
        for cf in ([cfgs[0]], [cfgs[k % n] for k in range(4100)]):
            pp, _ = recs(cf)
            tabs = []
            for wide in (False, True):
                gpu_engine.tune_ode_table_wide(wide)
                work = torch.zeros(len(cf) * 4 * 800, dtype=torch.float64, device=gpu_engine.device)
                w, st = gpu_engine.ode_tables(pp, work=work)
                tabs.append(w.cpu().numpy())
            assert np.array_equal(tabs[0], tabs[1], equal_nan=True)
    finally:
        gpu_engine.tune_ode_table_wide(True)
