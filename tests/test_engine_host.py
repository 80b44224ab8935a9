"""Host-side logic of engine.py that needs no GPU: the ODE launch order (wave_order), which
puts points with equal stage keys next to each other so that whole wavefronts qualify for the
integrator's cooperative mode."""
import os
import numpy as np
import torch

from conftest import BASE_CFG, full_cfg, pkg


def _recs(cfgs):
    cfgm = pkg("config")
    return (np.concatenate([cfgm.to_point(c) for c in cfgs]), np.concatenate([cfgm.to_ode_params(c) for c in cfgs]))


def _order(p, o):
    """engine.wave_order on CPU byte tensors of the records, as a numpy permutation (or None)."""
    tp = torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).copy())
    to = torch.from_numpy(np.ascontiguousarray(o).view(np.uint8).copy())
    r = pkg("engine").wave_order(tp, to, p.size)
    return None if r is None else r.numpy()


def _cfgs(m_values, reps, rng):
    out = []
    for m in m_values:
        for _ in range(reps):
            c = full_cfg(BASE_CFG)
            c.update(m_chi_GeV=float(m), P_chi_to_B=float(rng.uniform(0.1, 1.0)),
                     sigma_v_chi_GeV_m2=float(rng.choice([0.0, 1e-16])), Gamma_wash_over_H=1.0)
            out.append(c)
    return out


def test_wave_order_groups_interleaved_points():
    rng = np.random.default_rng(3)
    grouped = _cfgs([0.95, 40.0, 300.0], 100, rng)
    p, o = _recs(grouped)
    assert _order(p, o) is None                      # already contiguous
    perm = rng.permutation(len(grouped))
    order = _order(p[perm], o[perm])
    assert order is not None and sorted(order.tolist()) == list(range(len(grouped)))
    m = p[perm]["m_chi_GeV"][order]
    assert int(np.count_nonzero(m[1:] != m[:-1])) == 2  # three contiguous groups
    # stable within a group: the original relative order is kept
    for val in (0.95, 40.0, 300.0):
        idx = order[m == val]
        assert np.all(np.diff(idx) > 0)


def test_wave_order_no_repeats_or_small():
    rng = np.random.default_rng(4)
    distinct = _cfgs(np.linspace(1.0, 2.0, 200), 1, rng)
    p, o = _recs(distinct)
    assert _order(p, o) is None                      # nothing to group
    small = _cfgs([0.95, 40.0], 20, rng)
    p, o = _recs(small)
    assert _order(p[::-1], o[::-1]) is None          # <= 64 points: one wavefront anyway
    # the deplete flag is part of the key (it selects the Y_chi-only stage function)
    cfgs = _cfgs([0.95], 200, rng)
    for i, c in enumerate(cfgs):
        c["deplete_DM_from_source"] = bool(i % 2)
    p, o = _recs(cfgs)
    order = _order(p, o)
    d = o["deplete_DM_from_source"][order]
    assert int(np.count_nonzero(d[1:] != d[:-1])) == 1


def test_wave_order_groups_across_tables():
    """Points that differ only in the A/V kernel (I_p, v_w: their own spline tables) share a
    cooperative key (_native.ODE_COOP_KEY) and are grouped together; within a group, points of
    one table are contiguous (ODE_STAGE_KEY runs)."""
    rng = np.random.default_rng(8)
    cfgs = []
    for i in range(400):
        c = full_cfg(BASE_CFG)
        c.update(m_chi_GeV=(0.95, 40.0)[i % 2], I_p=(0.2, 0.5, 0.8, 0.3)[(i // 2) % 4], Gamma_wash_over_H=1.0,
                 P_chi_to_B=float(rng.uniform(0.1, 1.0)))
        cfgs.append(c)
    p, o = _recs(cfgs)
    order = _order(p, o)
    assert order is not None and sorted(order.tolist()) == list(range(len(cfgs)))
    m, ip = p["m_chi_GeV"][order], p["I_p"][order]
    assert int(np.count_nonzero(m[1:] != m[:-1])) == 1          # two cooperative groups
    runs = int(np.count_nonzero((ip[1:] != ip[:-1]) | (m[1:] != m[:-1])))
    assert runs == 7                                             # 2 groups x 4 tables, each contiguous
    assert set(pkg("_native").ODE_COOP_KEY) == set(pkg("_native").ODE_STAGE_KEY) - {"I_p", "v_w"}


def test_wave_order_groups_gamma_wash():
    """Gamma_wash is part of the order's key (round 6): a wave with one Gamma_wash shares Y_B's step
    maps and runs the Riccati kernel.  A Gamma_wash x sigma_v sweep with Gamma_wash fastest -- one
    cooperative group in the stage key alone, so the old key left it as given -- comes out in
    contiguous Gamma_wash runs, each in its original relative order."""
    rng = np.random.default_rng(12)
    cfgs = []
    for i in range(512):
        c = full_cfg(BASE_CFG)
        c.update(Gamma_wash_over_H=(0.1, 0.5, 2.0, 8.0)[i % 4], sigma_v_chi_GeV_m2=10.0 ** (-20 + (i // 4) % 16),
                 P_chi_to_B=float(rng.uniform(0.1, 1.0)))
        cfgs.append(c)
    p, o = _recs(cfgs)
    order = _order(p, o)
    assert order is not None and sorted(order.tolist()) == list(range(len(cfgs)))
    g = o["Gamma_wash_over_H"][order]
    assert int(np.count_nonzero(g[1:] != g[:-1])) == 3          # four contiguous Gamma_wash runs
    for val in (0.1, 0.5, 2.0, 8.0):
        assert np.all(np.diff(order[g == val]) > 0)
    assert _order(p[order], o[order]) is None                  # grouped input is left as it is


def test_ode_step_counts_device_equals_host():
    """Engine.ode sizes its continuation launches from ode_step_counts_device (torch ops on the
    device records); it must give the numpy ode_step_counts' values exactly, edge cases included
    (T_min = 0, m = 0, NaN T_p).  Run here on CPU tensors."""
    import numpy as np
    import torch
    eng, nat = pkg("engine"), pkg("_native")
    rng = np.random.default_rng(1)
    n = 20000
    pts = np.zeros(n, dtype=nat.POINT_DTYPE)
    pts["m_chi_GeV"] = 10 ** rng.uniform(-1, 3.5, n)
    pts["T_p_GeV"] = 10 ** rng.uniform(0, 3, n)
    pts["T_max_over_Tp"] = rng.uniform(0.5, 3, n)
    pts["T_min_over_Tp"] = rng.uniform(0, 1.5, n)
    pts["T_min_over_Tp"][:10] = 0.0
    pts["m_chi_GeV"][10:20] = 0.0
    pts["T_p_GeV"][20:25] = np.nan
    host = eng.ode_step_counts(pts)
    dev = eng.ode_step_counts_device(torch.from_numpy(pts.view(np.uint8).copy()), n).numpy()
    assert np.array_equal(host, dev, equal_nan=True)


def test_build_inputs_cover_every_include():
    """Every #include "..." of the HIP sources and headers is one of build._inputs(), so the build
    stamp (a content hash of those inputs) changes with any file the library is compiled from."""
    import re
    b = pkg("build")
    inputs = {os.path.normpath(f) for f in b._inputs()}
    for f in list(inputs):
        if not f.endswith((".hip", ".h")):
            continue
        for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', open(f).read(), flags=re.M):
            path = os.path.normpath(os.path.join(os.path.dirname(f), inc))
            assert path in inputs, (f, inc)
    assert "lzq_superadiabatic.h" in b.HEADERS


def test_build_stamp_tracks_content():
    """inputs_hash() is a content hash: it changes with a header's bytes (not its mtime), and the
    stamp written by build() is what up_to_date() compares."""
    import shutil
    import tempfile
    b = pkg("build")
    h0 = b.inputs_hash()
    assert h0 == b.inputs_hash() and h0 != b.inputs_hash({"LZQ_X": 1})
    hdr = os.path.join(b.CSRC, "lzq_superadiabatic.h")
    tmp = tempfile.mktemp()
    shutil.copy2(hdr, tmp)
    try:
        with open(hdr, "a") as f:
            f.write("\n")
        assert b.inputs_hash() != h0
    finally:
        shutil.copy2(tmp, hdr)
        os.remove(tmp)
    assert b.inputs_hash() == h0


def test_library_id_is_a_real_digest():
    """sweep.spec_key's library id: the shipped library's device code objects, never the digest of
    empty input; a library without a matching bundle entry is hashed whole."""
    import hashlib
    import tempfile
    nat = pkg("_native")
    lid = nat.library_id(nat.LIB_PATH)
    assert lid is not None and lid != hashlib.sha256(b"").hexdigest()[:16]
    with tempfile.NamedTemporaryFile(suffix=".so", delete=False) as f:
        f.write(b"not a fat binary")
    try:
        other = nat.library_id(f.name)
        assert other not in (None, lid, hashlib.sha256(b"").hexdigest()[:16])
    finally:
        os.remove(f.name)


def test_bounce_csv_reader_is_the_plugins(tmp_path):
    """sweep ProfileSpec(csv=...) reads the plug-in's xi,phi,Phi format through the plug-in's own
    parser (one reader of the format): options, comments, r + R0 positions."""
    B = pkg("bounce")
    (tmp_path / "p.csv").write_text("# y_B = 1.0\n# R0 = 2.5\nr,phi,Phi\n2.5,0.1,0.3\n3.0,0.2,0.25\n"
                                    "# a comment\n3.5,0.3,0.2\n4.0,0.4,0.1\n")
    xi, a, b, opts = B.read_bounce_csv(str(tmp_path / "p.csv"))
    assert np.array_equal(xi, [0.0, 0.5, 1.0, 1.5]) and np.array_equal(a, [0.1, 0.2, 0.3, 0.4])
    assert np.array_equal(b, [0.3, 0.25, 0.2, 0.1]) and opts["y_B"] == 1.0 and opts["R0"] == 2.5
    (tmp_path / "q.csv").write_text("xi,Delta,m\n0,1,2\n")
    import pytest
    with pytest.raises(ValueError):
        B.read_bounce_csv(str(tmp_path / "q.csv"))


def _runs(p, o, idx, **kw):
    tp = torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).copy())
    to = torch.from_numpy(np.ascontiguousarray(o).view(np.uint8).copy())
    return pkg("engine").ode_runs(tp, to, torch.as_tensor(idx, dtype=torch.int32), p.size, **kw)


def test_ode_runs_linear_stretches():
    """engine.ode_runs (the shared step-row tables of lzq_ode_integrate_rows): maximal stretches of
    linear, non-depleting points equal in the cooperative key, Gamma_wash and table, of >= 64
    points; each run's rows are its first point's step count (ode_step_counts); the rest -1."""
    rng = np.random.default_rng(11)
    cfgs = []
    for blk, (m, gw, sv, dep, cnt) in enumerate([(0.95, 1.0, 0.0, False, 130), (0.95, 2.0, 0.0, False, 70),
                                                 (0.95, 2.0, 1e-16, False, 100), (40.0, 1.0, 0.0, True, 80),
                                                 (40.0, 1.0, 0.0, False, 30), (40.0, 0.5, 0.0, False, 64)]):
        for _ in range(cnt):
            c = full_cfg(BASE_CFG)
            c.update(m_chi_GeV=m, Gamma_wash_over_H=gw, sigma_v_chi_GeV_m2=sv, deplete_DM_from_source=dep,
                     P_chi_to_B=float(rng.uniform(0.1, 1.0)), T_max_over_Tp=1.6, T_min_over_Tp=0.6)
            cfgs.append(c)
    p, o = _recs(cfgs)
    n = p.size
    run_of, rep, off, max_rows, total = _runs(p, o, np.zeros(n))
    run_of, rep, off = run_of.numpy(), rep.numpy(), off.numpy()
    steps = pkg("engine").ode_step_counts(p)
    assert rep.tolist() == [0, 130, 410]                       # blocks 0, 1 and 5 (>= 64 linear, no depletion)
    assert run_of[:130].tolist() == [0] * 130 and run_of[130:200].tolist() == [1] * 70
    assert (run_of[200:410] == -1).all() and run_of[410:].tolist() == [2] * 64
    assert off.tolist() == [0, int(steps[0]), int(steps[0] + steps[130]), int(steps[0] + steps[130] + steps[410])]
    assert max_rows == int(steps.max()) and total == off[-1]
    # a different table index splits a run; under the byte cap only the longest runs stay
    idx = np.zeros(n)
    idx[70:130] = 1                                # 60 points: too short
    run_of2 = _runs(p, o, idx)[0].numpy()
    assert run_of2[:70].tolist() == [0] * 70 and (run_of2[70:130] == -1).all()
    r3 = _runs(p, o, np.zeros(n), max_bytes=int(16 * steps[0]))
    assert r3[1].tolist() == [0] and r3[0].numpy()[130:].max() == -1
    assert _runs(p[:63], o[:63], np.zeros(63)) is None


def test_ode_runs_single_run_fast_path():
    """A chunk that is one linear run (the common wash-out sweep) comes back from the one-transfer
    path: every point in run 0, represented by point 0, with point 0's step count of rows; one
    depleting point among them sends the chunk through the general grouping instead."""
    rng = np.random.default_rng(12)
    cfgs = []
    for _ in range(100):
        c = full_cfg(BASE_CFG)
        c.update(m_chi_GeV=0.95, Gamma_wash_over_H=1.0, sigma_v_chi_GeV_m2=0.0, deplete_DM_from_source=False,
                 P_chi_to_B=float(rng.uniform(0.1, 1.0)), T_max_over_Tp=1.6, T_min_over_Tp=0.6)
        cfgs.append(c)
    p, o = _recs(cfgs)
    steps = pkg("engine").ode_step_counts(p)
    run_of, rep, off, max_rows, total = _runs(p, o, np.zeros(100))
    assert run_of.tolist() == [0] * 100 and rep.tolist() == [0] and off.tolist() == [0, int(steps[0])]
    assert max_rows == total == int(steps[0])
    assert _runs(p, o, np.zeros(100), max_bytes=int(16 * steps[0]) - 1) is None
    o2 = o.copy()
    o2["deplete_DM_from_source"][99] = 1
    run_of2, rep2, off2 = _runs(p, o2, np.zeros(100))[:3]
    assert run_of2.tolist() == [0] * 99 + [-1] and rep2.tolist() == [0] and off2.tolist() == [0, int(steps[0])]
