"""ODE fallback on the GPU (lzq_ode_*): against the reference's own outputs
(tests/golden/golden_ode.json) and against the CPU restatement (oracle), plus its operator API
(build_tables / A_over_V_T / rhs) and error behaviour.  Needs an MI355X."""
import os

import numpy as np
import pytest
import torch

from conftest import BASE_CFG, GOLDEN, full_cfg, golden, pkg, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN_ODE = os.path.join(GOLDEN, "golden_ode.json")
needs_golden = pytest.mark.skipif(not os.path.exists(GOLDEN_ODE), reason="golden_ode.json not generated")
NARROW = {"T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}


def recs(cfgs):
    cfgm = pkg("config")
    return (np.concatenate([cfgm.to_point(c) for c in cfgs]), np.concatenate([cfgm.to_ode_params(c) for c in cfgs]))


def seeded_cfgs(n, seed=11):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        c = full_cfg(BASE_CFG)
        c.update(m_chi_GeV=float(10 ** rng.uniform(-1, 2.7)), I_p=float(rng.uniform(0.05, 1.0)),
                 beta_over_H=float(10 ** rng.uniform(1.3, 2.5)), v_w=float(rng.uniform(0.1, 0.9)),
                 source_shape_sigma_y=float(rng.uniform(3, 20)), P_chi_to_B=float(rng.uniform(0, 1)),
                 chi_stats=str(rng.choice(["fermion", "boson"])), regime=str(rng.choice(["thermal", "nonthermal"])),
                 T_max_over_Tp=float(rng.uniform(1.1, 2.5)), T_min_over_Tp=float(rng.uniform(0.3, 0.9)),
                 Gamma_wash_over_H=float(rng.choice([0.0, 10 ** rng.uniform(-1, 1.5)])),
                 sigma_v_chi_GeV_m2=float(rng.choice([0.0, 10 ** rng.uniform(-20, -10)])),
                 deplete_DM_from_source=bool(rng.uniform() < 0.3))
        if c["Gamma_wash_over_H"] == 0.0 and c["sigma_v_chi_GeV_m2"] == 0.0:
            c["deplete_DM_from_source"] = True
        out.append(c)
    return out


@needs_golden
def test_ode_vs_reference_outputs(gpu_engine):
    pts = golden("golden_ode.json")["points"]
    cfgs = [full_cfg(r["config"]) for r in pts]
    t, st = gpu_engine.ode(*recs(cfgs))
    t, st = t.cpu().numpy(), st.cpu().numpy()
    names = pkg("_native").YIELD_FIELDS
    worst = 0.0
    for row, s, r in zip(t, st, pts):
        if "error" in r:
            assert s == 1 and r["error"]["type"] == "ValueError" and np.isnan(row[0]), (r["error"], s)
            continue
        assert s == 0, (s, r["config"])
        if not r["tight"]["success"]:  # the reference's Radau gives up: test_ode_stiff_cases_vs_converged_split
            continue
        ref_acc = max(rel_err(r["final"]["Y_B"], r["tight"]["Y_B"]), rel_err(r["final"]["Y_chi"], r["tight"]["Y_chi"]))
        tol = 1e-8 + 10 * ref_acc
        case = 0.0
        for k, v in zip(names, row):
            if k in r["final"]:
                e = rel_err(v, r["final"][k])
                assert e < tol, (k, v, r["final"][k], r["config"])
                case = max(case, e)
        worst = max(worst, case)
        c = r["config"]
        print(f"  case m={c['m_chi_GeV']:g} sv={c['sigma_v_chi_GeV_m2']:g} Gw={c['Gamma_wash_over_H']:g} "
              f"T/Tp=[{c['T_min_over_Tp']:g},{c['T_max_over_Tp']:g}]: GPU vs reference {case:.2e}, "
              f"reference vs its converged solve {ref_acc:.2e}, tol {tol:.2e}, "
              f"GPU vs converged {rel_err(row[0], r['tight']['Y_B']):.2e}")
        assert row[5] == r["P_used"]
    print(f"ODE GPU vs reference: worst rel err {worst:.3e}")


@needs_golden
def test_ode_stiff_cases_vs_converged_split(gpu_engine):
    """Per case: the two stiff annihilation cases where the reference's Radau gives up at the
    T = m/3 jump of Y_eq, against the reference's equations solved converged in two pieces
    (golden_ode_stiff.json; split Radau vs LSODA agree to ~1e-11), tolerance 1e-10."""
    from test_ode_oracle import STIFF_TOL, stiff_cases
    cases = stiff_cases()
    t, st = gpu_engine.ode(*recs([full_cfg(c["config"]) for c in cases]))
    t, st = t.cpu().numpy(), st.cpu().numpy()
    for c, row, s in zip(cases, t, st):
        ref = c["split_radau"]
        e_b, e_c = rel_err(row[0], ref["Y_B"]), rel_err(row[1], ref["Y_chi"])
        print(f"stiff case {c['index']}: GPU vs converged split Y_B {e_b:.2e}  Y_chi {e_c:.2e}  (tol {STIFF_TOL:g}; "
              f"the reference's own Y_B is {rel_err(c['reference_final']['Y_B'], ref['Y_B']):.2f} off)")
        assert s == 0 and e_b < STIFF_TOL and e_c < STIFF_TOL, (c["index"], row, ref)


def test_ode_vs_oracle_seeded(gpu_engine):
    cfgs = seeded_cfgs(24)
    t, st = gpu_engine.ode(*recs(cfgs))
    t, st = t.cpu().numpy(), st.cpu().numpy()
    ref, rst = O.ode_batch(cfgs, nthreads=16)
    assert np.array_equal(st, rst)
    for a, b in zip(t.ravel(), ref.ravel()):
        assert rel_err(a, b) < 1e-11, (a, b)


@needs_golden
def test_ode_operator_api_vs_reference(gpu_engine):
    """build_tables / A_over_V_T / rhs of BoltzmannSystem (fpy:207-218, 270-286)."""
    B = pkg("boltzmann")
    cfgm = pkg("config")
    for r in golden("golden_ode.json")["points"][:8]:
        if "error" in r:
            continue
        cfg = cfgm.Config(**full_cfg(r["config"]))
        bs = B.BoltzmannSystem(cfg, r["P_used"])
        T_p = cfg.T_p_GeV
        bs.build_tables(cfg.T_min_over_Tp * T_p, cfg.T_max_over_Tp * T_p, n=800)
        got = bs.A_over_V_Ts(r["A_over_V_T"]["T"])
        amax = max(r["A_over_V_T"]["Av"])
        for g, e in zip(got, r["A_over_V_T"]["Av"]):
            assert abs(g - e) <= 1e-11 * abs(e) + 1e-14 * amax
        xs = [s["x"] for s in r["rhs"]]
        Ys = [s["Y"] for s in r["rhs"]]
        dY = bs.rhs_batch(xs, Ys)
        # per component: relative 1e-10, plus 1e-12 of the component's largest magnitude (the
        # spline's absolute accuracy is relative to max A/V, not to a value deep in its tail)
        scale = np.max(np.abs([s["dY"] for s in r["rhs"]]), axis=0)
        for g, s in zip(dY, r["rhs"]):
            for a, e, sc in zip(g, s["dY"], scale):
                assert abs(a - e) <= 1e-10 * abs(e) + 1e-12 * sc, (s, g)
        assert bs.rhs(xs[3], np.array(Ys[3])).tolist() == list(dY[3])


def test_ode_status_and_step_cap(gpu_engine):
    cfgs = [full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, **NARROW}),
            full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.0, "T_min_over_Tp": 1.0}),
            full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, "T_max_over_Tp": 0.5, "T_min_over_Tp": 0.9}),
            full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0})]                  # ~1e6 steps
    t, st = gpu_engine.ode(*recs(cfgs), max_steps=100_000)
    assert st.cpu().numpy().tolist() == [0, 1, 1, 3]
    t = t.cpu().numpy()
    assert np.isfinite(t[0]).all() and np.isnan(t[1:, :5]).all()


def test_ode_table_of_another_knot_count_is_refused(gpu_engine):
    """lzq_ode_tables builds any nt (build_tables(n=nt)), the integrators read LZQ_ODE_NT-knot tables:
    tables of another nt are refused per point (LZQ_ODE_BAD_TABLE, NaN yields) by the knot count each
    table records, in every integrator kernel; main()'s tables still integrate."""
    import ctypes
    nat = pkg("_native")
    cfgs = [full_cfg({**BASE_CFG, "Gamma_wash_over_H": 1.0, **NARROW}),
            full_cfg({**BASE_CFG, "sigma_v_chi_GeV_m2": 1e-12, **NARROW})]
    p, o = recs(cfgs)
    d_p = gpu_engine.points_to_device(p)
    d_o = torch.from_numpy(np.ascontiguousarray(o).view(np.uint8).copy()).to(gpu_engine.device)
    for nt, want in ((1600, nat.ODE_BAD_TABLE), (nat.ODE_NT, nat.ODE_OK)):
        work, st = gpu_engine.ode_tables(d_p, nt=nt)
        assert (st.cpu().numpy() == 0).all()
        out = torch.empty((2, 6), dtype=torch.float64, device=gpu_engine.device)
        status = torch.full((2,), -1, dtype=torch.int32, device=gpu_engine.device)
        vp = lambda t: ctypes.c_void_p(t.data_ptr())
        for fn in ("lzq_ode_integrate", "lzq_ode_quadrature"):
            if fn == "lzq_ode_integrate":
                rc = gpu_engine.lib.lzq_ode_integrate(vp(d_p), vp(d_o), 2, vp(work), work.numel(), 10**6, vp(out),
                                                      vp(status), None)
            else:
                rc = gpu_engine.lib.lzq_ode_quadrature(vp(d_p), vp(d_o), 2, None, 0, vp(work), work.numel(), 10**6,
                                                       vp(out), vp(status), None)
            assert rc == 0
            torch.cuda.synchronize()
            assert status.cpu().numpy().tolist() == [want, want], (nt, fn, status)
            assert np.isnan(out.cpu().numpy()[:, 0]).all() == (want != nat.ODE_OK), (nt, fn)


def test_ode_deterministic_and_batch_independent(gpu_engine):
    cfgs = seeded_cfgs(20, seed=3)
    p, o = recs(cfgs)
    a = gpu_engine.ode(p, o)[0].cpu().numpy()
    b = gpu_engine.ode(p[::-1], o[::-1])[0].cpu().numpy()[::-1]
    c = np.concatenate([gpu_engine.ode(p[i:i + 7], o[i:i + 7], chunk=3)[0].cpu().numpy() for i in range(0, 20, 7)])
    assert np.array_equal(a, b) and np.array_equal(a, c)
    try:  # the A/V tables' z-sums under exact-underflow truncation: bit-identical
        gpu_engine.tune_truncate(True)
        d = gpu_engine.ode(p, o)[0].cpu().numpy()
    finally:
        gpu_engine.tune_truncate(False)
    assert np.array_equal(a, d)


def test_ode_reduces_to_quadrature_without_sinks(gpu_engine):
    """Depletion alone leaves dY_B/dx = S_B/(s H x): Y_B(ODE) equals the fast path's
    quadrature of the same integrand up to the spline's interpolation of A/V."""
    cfg = full_cfg({**BASE_CFG, "deplete_DM_from_source": True, "T_max_over_Tp": 1.3, "T_min_over_Tp": 0.7})
    t, st = gpu_engine.ode(*recs([cfg]))
    q = gpu_engine.yields(pkg("config").to_point(cfg)).cpu().numpy()[0, 0]
    assert st.item() == 0 and rel_err(t.cpu().numpy()[0, 0], q) < 1e-2


def test_ode_sweep_routes_per_point(gpu_engine, tmp_path):
    """A sweep over Gamma_wash (0 -> fast path, > 0 -> ODE fallback, fpy:372) through the sweep
    driver matches the oracle point by point."""
    sw = pkg("sweep")
    spec = sw.spec_from_json({"name": "ode", "base": {**NARROW},
                              "axes": [{"field": "Gamma_wash_over_H", "values": [0.0, 0.5, 5.0]},
                                       {"field": "delta_LZ", "values": [1e-3, 0.1]}]})
    assert sw.is_ode_spec(spec)
    import torch
    out = torch.empty((6, 6), dtype=torch.float64, device=gpu_engine.device)
    sw.make_compute(spec, gpu_engine)(0, 6, out)
    t = out.cpu().numpy()
    for i in range(6):
        prm = spec.point_params(i)
        cfg = full_cfg({**spec.base, "Gamma_wash_over_H": prm["Gamma_wash_over_H"],
                        "P_chi_to_B": O.p_closed_form(prm["delta_LZ"])})
        ref = O.ode_point(cfg) if prm["Gamma_wash_over_H"] else O.point_yields(cfg)
        for j, k in enumerate(pkg("_native").YIELD_FIELDS):
            assert rel_err(t[i, j], ref[k]) < 1e-11, (i, k, t[i, j], ref[k])


def test_ode_shared_tables_bit_identical(gpu_engine):
    """lzq_ode_integrate_shared: points equal in the A/V kernel + window share one spline table;
    the yields are bit-identical to per-point tables (Engine.ode share_tables=False)."""
    base = seeded_cfgs(6, seed=5)
    cfgs = []
    rng = np.random.default_rng(9)
    for c in base:                     # 6 kernels x 7 points differing only in P / flux / sinks
        for _ in range(7):
            d = dict(c, P_chi_to_B=float(rng.uniform(0.05, 1.0)), incident_flux_scale=float(10 ** rng.uniform(-10, -8)),
                     Gamma_wash_over_H=float(rng.choice([0.5, 2.0])), sigma_v_chi_GeV_m2=float(rng.choice([0.0, 1e-16])))
            cfgs.append(d)
    p, o = recs(cfgs)
    perm = rng.permutation(len(cfgs))
    a, sa = gpu_engine.ode(p[perm], o[perm], share_tables=True)
    b, sb = gpu_engine.ode(p[perm], o[perm], share_tables=False)
    assert torch_equal(a, b) and torch_equal(sa, sb)
    c, _ = gpu_engine.ode(p[perm], o[perm], share_tables=True, chunk=10)   # sharing within chunks
    assert torch_equal(a, c)


def torch_equal(a, b):
    import torch
    return bool(torch.equal(a, b)) or bool(np.array_equal(a.cpu().numpy(), b.cpu().numpy(), equal_nan=True))


@needs_golden
def test_ode_quadrature_vs_converged_reference(gpu_engine):
    """lzq_ode_quadrature (opt-in): Y_B by the exact integrating-factor quadrature for every
    sigma_v, Y_chi too when sigma_v = 0, else Y_chi's Riccati equation stepped alone.  Per case
    against the reference's own rtol-1e-12 re-solve (golden "tight"), and for the two cases where
    that gives up, against the converged split solve (golden_ode_stiff.json)."""
    from test_ode_oracle import stiff_cases
    pts = [r for r in golden("golden_ode.json")["points"] if "error" not in r]
    cfgs = [full_cfg(r["config"]) for r in pts]
    p, o = recs(cfgs)
    q, sq = gpu_engine.ode(p, o, method="quadrature")
    q, sq = q.cpu().numpy(), sq.cpu().numpy()
    split = {c["index"]: c["split_radau"] for c in stiff_cases()}
    gold_idx = [i for i, r in enumerate(golden("golden_ode.json")["points"]) if "error" not in r]
    worst = 0.0
    n_riccati = 0
    for gi, r, c, rq, s in zip(gold_idx, pts, cfgs, q, sq):
        assert s == 0, (c, s)
        conv = r["tight"] if r["tight"]["success"] else split[gi]
        e_b, e_c = rel_err(rq[0], conv["Y_B"]), rel_err(rq[1], conv["Y_chi"])
        riccati = max(c["sigma_v_chi_GeV_m2"], 0.0) != 0.0
        n_riccati += riccati
        print(f"  quadrature sv={c['sigma_v_chi_GeV_m2']:g} Gw={c['Gamma_wash_over_H']:g} "
              f"T/Tp=[{c['T_min_over_Tp']:g},{c['T_max_over_Tp']:g}] deplete={c['deplete_DM_from_source']}: "
              f"vs converged Y_B {e_b:.1e} Y_chi {e_c:.1e} ({'Y_chi stepped' if riccati else 'both by quadrature'}); "
              f"the reference's rtol-1e-8 Y_B is {rel_err(r['final']['Y_B'], conv['Y_B']):.1e} from it")
        assert e_b < 1e-10 and e_c < 1e-10, (c, rq, conv)
        worst = max(worst, e_b, e_c)
    assert n_riccati >= 6
    print(f"ODE quadrature vs converged reference: worst {worst:.2e}")


def test_ode_quadrature_sweep_shared_and_deterministic(gpu_engine):
    """The quadrature form through the sweep driver ("ode_method": "quadrature") equals
    Engine.ode(method="quadrature"); shared vs per-point tables bit-identical; batch order and
    splits do not change a result; agrees with the Radau path to the Radau path's own accuracy
    on narrow windows (~1e-13)."""
    import torch
    sw = pkg("sweep")
    spec = sw.spec_from_json({"name": "q", "base": {**NARROW}, "ode_method": "quadrature",
                              "axes": [{"field": "Gamma_wash_over_H", "values": [0.0, 0.5, 5.0]},
                                       {"field": "I_p", "values": [0.2, 0.6]},
                                       {"field": "delta_LZ", "values": [1e-3, 0.1]}]})
    out = torch.empty((12, 6), dtype=torch.float64, device=gpu_engine.device)
    sw.make_compute(spec, gpu_engine)(0, 12, out)
    t = out.cpu().numpy()
    pts, ods = sw.grid_records(spec, 0, 12, gpu_engine)
    ode = ods["Gamma_wash_over_H"] != 0
    q, sq = gpu_engine.ode(pts[ode], ods[ode], method="quadrature")
    assert np.array_equal(t[ode], q.cpu().numpy()) and bool((sq == 0).all())
    q2, _ = gpu_engine.ode(pts[ode], ods[ode], method="quadrature", share_tables=False)
    assert np.array_equal(q.cpu().numpy(), q2.cpu().numpy())
    perm = np.random.default_rng(0).permutation(int(ode.sum()))
    q3, _ = gpu_engine.ode(pts[ode][perm], ods[ode][perm], method="quadrature", chunk=3)
    assert np.array_equal(q3.cpu().numpy(), q.cpu().numpy()[perm])
    r, _ = gpu_engine.ode(pts[ode], ods[ode])
    rr = r.cpu().numpy()
    assert np.max(np.abs(q.cpu().numpy()[:, :2] - rr[:, :2]) / np.abs(rr[:, :2])) < 1e-11


def test_ode_linear_waves_bit_identical(gpu_engine):
    """The linear-wave fast path (lzq_ode.hip LZQ_ODE_LINFAST: sigma_v = 0 on every lane of a
    cooperative wave with one Gamma_wash per segment; a regular step is Y_B's shared affine map,
    plus Y_chi's three depletion fmas) gives the per-lane mode's bits: wash-out with and without
    depletion, thermal and non-thermal starts, a window crossing T = m/3 (split steps take the
    general path), a group whose Gamma_wash varies within every wave (no fast path), and the same
    batch as continuation launches of 2^12 steps."""
    rng = np.random.default_rng(47)
    cfgs = []
    for m_chi, gw in ((0.95, 0.5), (300.0, 2.0), (3.0, None)):   # 300 GeV: T = m/3 = T_p is inside the window
        for _ in range(128):
            c = full_cfg(BASE_CFG)
            c.update(NARROW, m_chi_GeV=m_chi, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                     incident_flux_scale=float(10 ** rng.uniform(-10, -8)),
                     Gamma_wash_over_H=float(gw if gw is not None else rng.choice([0.5, 1.0, 2.0])),
                     sigma_v_chi_GeV_m2=0.0, deplete_DM_from_source=bool(rng.uniform() < 0.4),
                     regime=str(rng.choice(["thermal", "nonthermal"])))
            cfgs.append(c)
    p, o = recs(cfgs)
    a, sa = gpu_engine.ode(p, o, share_tables=True)
    prev = gpu_engine.tune_ode_coop(False)
    try:
        b, sb = gpu_engine.ode(p, o, share_tables=True)
    finally:
        gpu_engine.tune_ode_coop(prev)
    assert bool((sa == 0).all()) and torch_equal(sa, sb) and torch_equal(a, b)
    prev = gpu_engine.tune_ode_launch_steps(12)
    try:
        c, sc = gpu_engine.ode(p, o, share_tables=True)
    finally:
        gpu_engine.tune_ode_launch_steps(prev)
    assert torch_equal(sa, sc) and torch_equal(a, c)
    ref, sr = O.ode_batch(cfgs[::16], nthreads=16)
    for row, rr in zip(a.cpu().numpy()[::16], ref):
        for v, w in zip(row[:5], rr[:5]):
            assert rel_err(v, w) < 1e-10, (v, w)


def test_ode_row_tables_bit_identical(gpu_engine):
    """Shared step-row tables (lzq_ode_rows + lzq_ode_integrate_rows, engine.ode_runs): linear,
    non-depleting runs of one cooperative key, Gamma_wash and table read Y_B's step maps from one
    table per run instead of filling them per wavefront.  The same bits as without the tables
    (Engine.ode_rows = False) and as the per-lane mode: wash-out runs of 200 and 130 points (waves
    straddling two runs fill their own), a window crossing T = m/3 (split steps), a depleting
    group beside them (no tables), the batch shuffled (wave_order regroups it), and continuation
    launches of 2^11 steps."""
    rng = np.random.default_rng(53)
    cfgs = []
    for m_chi, gw, dep, cnt in ((0.95, 0.5, False, 200), (300.0, 2.0, False, 130), (0.95, 1.0, True, 70),
                                (0.95, 1.0, False, 100)):
        for _ in range(cnt):
            c = full_cfg(BASE_CFG)
            c.update(NARROW, m_chi_GeV=m_chi, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                     incident_flux_scale=float(10 ** rng.uniform(-10, -8)), Gamma_wash_over_H=gw,
                     sigma_v_chi_GeV_m2=0.0, deplete_DM_from_source=dep, regime=str(rng.choice(["thermal", "nonthermal"])))
            cfgs.append(c)
    perm = rng.permutation(len(cfgs))
    p, o = recs([cfgs[i] for i in perm])
    a, sa = gpu_engine.ode(p, o)
    assert gpu_engine.last_ode_tables.get("row_runs", 0) == 3
    gpu_engine.ode_rows = False
    try:
        b, sb = gpu_engine.ode(p, o)
        assert "row_runs" not in gpu_engine.last_ode_tables
        prev = gpu_engine.tune_ode_coop(False)
        try:
            c, sc = gpu_engine.ode(p, o)
        finally:
            gpu_engine.tune_ode_coop(prev)
    finally:
        gpu_engine.ode_rows = True
    assert bool((sa == 0).all()) and torch_equal(sa, sb) and torch_equal(a, b)
    assert torch_equal(sa, sc) and torch_equal(a, c)
    prev = gpu_engine.tune_ode_launch_steps(11)
    try:
        d, sd = gpu_engine.ode(p, o)
    finally:
        gpu_engine.tune_ode_launch_steps(prev)
    assert torch_equal(sa, sd) and torch_equal(a, d)
    # device-resident records (points_to_device / ode_params_to_device): the same bits
    e, se = gpu_engine.ode(gpu_engine.points_to_device(p), gpu_engine.ode_params_to_device(o))
    assert torch_equal(sa, se) and torch_equal(a, e)
    with pytest.raises(ValueError):
        gpu_engine.ode(gpu_engine.points_to_device(p), gpu_engine.ode_params_to_device(o[:-1]))
    # chunks of 128 (tables of chunk c + 1 built on the side stream while chunk c integrates, runs
    # per chunk), from host and from resident records: the same bits
    for args in ((p, o), (gpu_engine.points_to_device(p), gpu_engine.ode_params_to_device(o))):
        f, sf = gpu_engine.ode(*args, chunk=128)
        assert gpu_engine.last_ode_tables["chunks"] == 4 and gpu_engine.last_ode_tables.get("row_runs", 0) >= 3
        assert torch_equal(sa, sf) and torch_equal(a, f)
    sel =[int(np.nonzero(perm == j)[0][0]) for j in (0, 250, 340, 480)]
    ref, _ = O.ode_batch([cfgs[perm[i]] for i in sel], nthreads=4)
    for row, rr in zip(a.cpu().numpy()[sel], ref):
        for v, w in zip(row[:5], rr[:5]):
            assert rel_err(v, w) < 1e-10, (v, w)


def test_ode_row_tables_raw_abi_guards(gpu_engine):
    """lzq_ode_integrate_rows through the C ABI with run tables that must not be read: a row count
    that is not the points' step count, and a representative that differs from its run (another
    Gamma_wash).  Every wavefront then fills its own rows: the bits of lzq_ode_integrate_shared."""
    eng, lib = gpu_engine, gpu_engine.lib
    rng = np.random.default_rng(59)
    cfgs = []
    for _ in range(128):
        c = full_cfg(BASE_CFG)
        c.update(NARROW, m_chi_GeV=0.95, P_chi_to_B=float(rng.uniform(0.05, 1.0)), Gamma_wash_over_H=1.0,
                 sigma_v_chi_GeV_m2=0.0, deplete_DM_from_source=False)
        cfgs.append(c)
    other = dict(cfgs[0], Gamma_wash_over_H=2.0)
    p, o = recs(cfgs + [other])
    n = len(cfgs)
    E = pkg("engine")
    vp = E._vp
    d_pts, d_ode = eng.points_to_device(p), E._to_device_bytes(o, eng.device)
    work = eng.ode_workspace(2)
    idx = torch.zeros(n + 1, dtype=torch.int32, device=eng.device)
    idx[n] = 1
    rep_pts = d_pts.view(n + 1, -1)[[0, n]].contiguous()
    st = torch.zeros(2, dtype=torch.int32, device=eng.device)
    eng._check(lib.lzq_ode_tables(vp(rep_pts), 2, None, None, pkg("_native").ODE_NT, pkg("_native").LZQ_NZ,
                                  pkg("_native").LZQ_Z_MAX, None, vp(work),
                                  work.numel(), vp(st), eng._stream()))
    N = int(E.ode_step_counts(p[:1])[0])
    ms = N + 64
    ref_out = torch.empty((n + 1, 6), dtype=torch.float64, device=eng.device)
    ref_st = torch.zeros(n + 1, dtype=torch.int32, device=eng.device)
    eng._check(lib.lzq_ode_integrate_shared(vp(d_pts), vp(d_ode), n + 1, vp(idx), 2, vp(work), work.numel(), ms,
                                            vp(ref_out), vp(ref_st), eng._stream()))
    run_of = torch.zeros(n + 1, dtype=torch.int32, device=eng.device)
    run_of[n] = -1
    for rep, nrows in ((0, N - 1), (n, N), (0, N)):
        run_rep = torch.tensor([rep], dtype=torch.int64, device=eng.device)
        row_off = torch.tensor([0, nrows], dtype=torch.int64, device=eng.device)
        rows = torch.zeros(2 * N, dtype=torch.float64, device=eng.device)
        eng._check(lib.lzq_ode_rows(vp(d_pts), vp(d_ode), n + 1, vp(idx), 2, vp(work), work.numel(), vp(run_rep),
                                    vp(row_off), 1, nrows, vp(rows), rows.numel(), eng._stream()))
        out = torch.empty((n + 1, 6), dtype=torch.float64, device=eng.device)
        stt = torch.zeros(n + 1, dtype=torch.int32, device=eng.device)
        eng._check(lib.lzq_ode_integrate_rows(vp(d_pts), vp(d_ode), n + 1, vp(idx), 2, vp(work), work.numel(), ms,
                                              vp(run_of), vp(run_rep), vp(row_off), 1, vp(rows), rows.numel(),
                                              vp(out), vp(stt), eng._stream()))
        torch.cuda.synchronize()
        assert torch_equal(stt, ref_st) and torch_equal(out, ref_out), (rep, nrows)
    assert lib.lzq_ode_rows(vp(d_pts), vp(d_ode), -1, None, 0, vp(work), work.numel(), None, None, 0, 0, None, 0,
                            None) < 0


def test_ode_cooperative_waves_bit_identical(gpu_engine):
    """ode_integrate_kernel's cooperative mode (a full wavefront whose points differ only in P,
    flux, sigma_v, Gamma_wash, deplete and the initial state computes each step's stage
    ingredients once, into LDS) gives the same bits as the per-lane mode: the same 2 x 128
    points run grouped (two uniform wavefronts per group) and interleaved (no uniform
    wavefront), with wash-out, depletion, Riccati (sigma_v != 0) and thermal points mixed."""
    rng = np.random.default_rng(31)
    groups = []
    for m_chi in (0.95, 40.0):           # the second crosses T = m/3 inside its window (split step)
        g = []
        for _ in range(128):
            c = full_cfg(BASE_CFG)
            c.update(NARROW, m_chi_GeV=m_chi, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                     incident_flux_scale=float(10 ** rng.uniform(-10, -8)),
                     Gamma_wash_over_H=float(rng.choice([0.0, 0.5, 2.0])),
                     sigma_v_chi_GeV_m2=float(rng.choice([0.0, 1e-16, 1e-12])),
                     deplete_DM_from_source=bool(rng.uniform() < 0.3),
                     regime=str(rng.choice(["thermal", "nonthermal"])))
            if c["Gamma_wash_over_H"] == 0.0 and c["sigma_v_chi_GeV_m2"] == 0.0:
                c["deplete_DM_from_source"] = True
            g.append(c)
        groups.append(g)
    grouped = groups[0] + groups[1]
    inter = [c for pair in zip(groups[0], groups[1]) for c in pair]
    p, o = recs(grouped)
    a, sa = gpu_engine.ode(p, o, share_tables=True)
    p2, o2 = recs(inter)
    b, sb = gpu_engine.ode(p2, o2, share_tables=True, group_waves=False)   # every wave mixed: per-lane
    g2, sg2 = gpu_engine.ode(p2, o2, share_tables=True)   # regrouped for the launch, scattered back
    assert torch_equal(b, g2) and torch_equal(sb, sg2)
    order = np.concatenate([np.arange(0, 256, 2), np.arange(1, 256, 2)])   # interleaved -> grouped order
    b, sb = b[order], sb[order]
    assert torch_equal(sa, sb) and torch_equal(a, b)
    prev = gpu_engine.tune_ode_coop(False)         # the grouped batch again, every wave per-lane
    try:
        c, sc = gpu_engine.ode(p, o, share_tables=True)
    finally:
        gpu_engine.tune_ode_coop(prev)
    assert prev and torch_equal(sa, sc) and torch_equal(a, c)
    # partial wavefronts (here: single points) are filled with clones of their first point, so
    # they run cooperatively too; each must match the batch result bit for bit
    for j in (0, 5, 131, 200):
        one, s1 = gpu_engine.ode(p[j:j + 1], o[j:j + 1], share_tables=True, time_parallel=False)
        assert torch_equal(one[0], a[j]) and torch_equal(s1[0], sa[j])
    # the quadrature method's Riccati stepping of Y_chi (sigma_v != 0) has the same mode
    q1, sq1 = gpu_engine.ode(p, o, share_tables=True, method="quadrature")
    gpu_engine.tune_ode_coop(False)
    try:
        q0, sq0 = gpu_engine.ode(p, o, share_tables=True, method="quadrature")
    finally:
        gpu_engine.tune_ode_coop(True)
    assert torch_equal(sq1, sq0) and torch_equal(q1, q0)
    # and against the C restatement (points both finished normally)
    ref, sr = O.ode_batch(grouped, nthreads=16)
    t, st = a.cpu().numpy(), sa.cpu().numpy()
    assert int((st == 0).sum()) >= 200
    for row, rr, s1, s2 in zip(t, ref, st, sr):
        if s1 == 0 and s2 == 0:
            for v, w in zip(row[:5], rr[:5]):
                assert rel_err(v, w) < 1e-10, (v, w)


def test_ode_continuation_launches_bit_identical(gpu_engine):
    """The fixed-step integration as continuation launches (include/lzq.h
    LZQ_TUNE_ODE_LAUNCH_STEPS): 20000-step windows split into 3 launches of 2^13 steps (and 40
    launches of 2^9) give the same bits as one launch -- cooperative and per-lane waves, split
    steps at T = m/3, Riccati (sigma_v != 0) with its predictor, thermal/nonthermal, and the
    quadrature method's Riccati stepping."""
    rng = np.random.default_rng(41)
    cfgs = []
    for m_chi in (0.95, 40.0):
        for _ in range(70):
            c = full_cfg(BASE_CFG)
            c.update(NARROW, m_chi_GeV=m_chi, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                     Gamma_wash_over_H=float(rng.choice([0.0, 0.5, 2.0])),
                     sigma_v_chi_GeV_m2=float(rng.choice([0.0, 1e-16, 1e-12])),
                     deplete_DM_from_source=bool(rng.uniform() < 0.3),
                     regime=str(rng.choice(["thermal", "nonthermal"])))
            if c["Gamma_wash_over_H"] == 0.0 and c["sigma_v_chi_GeV_m2"] == 0.0:
                c["deplete_DM_from_source"] = True
            cfgs.append(c)
    cfgs += seeded_cfgs(12, seed=8)
    p, o = recs(cfgs)
    steps = pkg("engine").ode_step_counts(p)
    assert steps.max() > 2 ** 13
    one = {m: gpu_engine.ode(p, o, method=m) for m in ("radau", "quadrature")}
    mixed = gpu_engine.ode(p, o, group_waves=False)
    for log2 in (13, 9):
        prev = gpu_engine.tune_ode_launch_steps(log2)
        try:
            for m in ("radau", "quadrature"):
                t, st = gpu_engine.ode(p, o, method=m)
                assert torch_equal(t, one[m][0]) and torch_equal(st, one[m][1]), (log2, m)
            t, st = gpu_engine.ode(p, o, group_waves=False)
            assert torch_equal(t, mixed[0]) and torch_equal(st, mixed[1])
        finally:
            gpu_engine.tune_ode_launch_steps(prev)
    assert bool((one["radau"][1] == 0).all())
    # the cap still applies across launches
    prev = gpu_engine.tune_ode_launch_steps(10)
    try:
        t, st = gpu_engine.ode(p[:2], o[:2], max_steps=5000)
    finally:
        gpu_engine.tune_ode_launch_steps(prev)
    assert st.cpu().tolist() == [3, 3] and bool(torch_isnan(t[:, :5]))


def torch_isnan(t):
    import torch
    return torch.isnan(t).all()


def test_long_window_completes_through_cli(gpu_engine, tmp_path):
    """m_chi = 3500 GeV with sigma_v = 1e-12 over the shipped window needs ~7e7 fixed Radau steps
    (fpy:403-404), beyond round 2's 2^26 cap: the reference integrates it (slowly), and so does
    lzq now, in continuation launches, through the CLI (yields_out.json written, no [warn]).
    Y_B does not depend on sigma_v (its equation is linear, fpy:285), so it is checked against
    the exact quadrature form of the same window at sigma_v = 0."""
    import json
    from test_cli import run_cli
    cfg = dict(full_cfg(BASE_CFG), m_chi_GeV=3500.0, sigma_v_chi_GeV_m2=1e-12)
    p, _ = recs([cfg])
    n = pkg("engine").ode_step_counts(p)[0]
    assert n > 2 ** 26, n
    (tmp_path / "cfg.json").write_text(json.dumps({k: v for k, v in cfg.items()}))
    out = run_cli(["--config", "cfg.json"], tmp_path)
    assert "[warn]" not in out and "Wrote yields_out.json" in out
    fin = json.loads((tmp_path / "yields_out.json").read_text())["final"]
    assert all(np.isfinite(v) for v in fin.values()), fin
    assert 0.0 < fin["Y_chi"] <= cfg["Y_chi_init"]
    q, sq = gpu_engine.ode(*recs([dict(cfg, sigma_v_chi_GeV_m2=0.0)]), method="quadrature")
    yb = float(q.cpu().numpy()[0, 0])
    print(f"m_chi = 3500 GeV, {n:.3g} Radau steps: Y_B {fin['Y_B']!r} vs converged quadrature {yb!r} "
          f"(rel {rel_err(fin['Y_B'], yb):.2e}); Y_chi {fin['Y_chi']!r}")
    assert int(sq[0]) == 0 and rel_err(fin["Y_B"], yb) < 1e-6


def test_ode_quadrature_narrow_window_resolved(gpu_engine):
    """the quadrature form clamped its sub-intervals and could miss a narrow source
    window.  It now integrates only where the window is not exactly 0 in double (|q| <= 40), so
    the sub-interval count no longer grows as sigma_y shrinks: Y_B / sigma_y converges as
    sigma_y -> 0 (the window integrates to sigma sqrt(2 pi)); a scale it still cannot resolve
    (a wash-out rate of 1e9) is reported as LZQ_ODE_UNRESOLVED with NaN yields, never a silent
    answer."""
    rows = []
    for sig in (1e-4, 1e-5, 1e-6):
        cfg = full_cfg({**BASE_CFG, **NARROW, "Gamma_wash_over_H": 0.5, "source_shape_sigma_y": sig})
        q, sq = gpu_engine.ode(*recs([cfg]), method="quadrature")
        assert int(sq[0]) == 0
        rows.append(float(q.cpu().numpy()[0, 0]) / sig)
    print("Y_B / sigma_y:", rows)
    assert rows[2] > 0 and abs(rows[1] / rows[2] - 1.0) < 1e-6 and abs(rows[0] / rows[2] - 1.0) < 1e-4
    cfg = full_cfg({**BASE_CFG, **NARROW, "Gamma_wash_over_H": 1e9})
    q, sq = gpu_engine.ode(*recs([cfg]), method="quadrature")
    assert int(sq[0]) == pkg("_native").ODE_UNRESOLVED and np.isnan(q.cpu().numpy()[0, :5]).all()


def test_sweep_masks_failed_ode_points(gpu_engine, tmp_path):
    """ODE-path points that did not finish normally are NaN rows of a sweep
    table and are counted per status in summary.json (here: the quadrature form's unresolved
    status next to normal points)."""
    import json
    sw = pkg("sweep")
    spec_d = {"name": "fail", "base": {**NARROW}, "ode_method": "quadrature",
              "axes": [{"field": "Gamma_wash_over_H", "values": [0.5, 1e9]},
                       {"field": "delta_LZ", "values": [1e-3, 0.1]}]}
    (tmp_path / "spec.json").write_text(json.dumps(spec_d))
    sw.main(["--spec", str(tmp_path / "spec.json"), "--out", str(tmp_path / "out")])
    tab = np.load(tmp_path / "out" / "table.npy")
    summ = json.loads((tmp_path / "out" / "summary.json").read_text())
    assert np.isfinite(tab[:2]).all() and np.isnan(tab[2:, :5]).all()
    assert summ["ode_status"] == {"ok": 2, "quadrature_unresolved": 2}
    assert summ["final"]["Y_B"]["n_nonfinite"] == 2


def test_ode_cooperative_subgroups_bit_identical(gpu_engine):
    """Cooperative sub-groups: waves whose aligned 32/16/8-lane segments are each uniform in the
    stage key (here 16 and 8 points per m_chi value, in launch order) run cooperatively per
    segment, with segments of different N and step size in one wave; results equal the per-lane
    mode bit for bit, for the Radau path and the quadrature method's Riccati stepping, also as
    continuation launches."""
    rng = np.random.default_rng(77)
    cfgs = []
    for block, n_keys in ((16, 8), (8, 16)):
        for kk in range(n_keys):
            m_chi = float(10 ** rng.uniform(-0.5, 1.8))
            win = dict(T_max_over_Tp=float(rng.uniform(1.3, 1.8)), T_min_over_Tp=float(rng.uniform(0.5, 0.7)))
            for _ in range(block):
                c = full_cfg(BASE_CFG)
                c.update(win, m_chi_GeV=m_chi, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                         Gamma_wash_over_H=float(rng.choice([0.5, 2.0])),
                         sigma_v_chi_GeV_m2=float(rng.choice([0.0, 1e-16, 1e-12])),
                         regime=str(rng.choice(["thermal", "nonthermal"])))
                cfgs.append(c)
    p, o = recs(cfgs)
    for method in ("radau", "quadrature"):
        a, sa = gpu_engine.ode(p, o, method=method, group_waves=False)
        prev = gpu_engine.tune_ode_coop(False)
        try:
            b, sb = gpu_engine.ode(p, o, method=method, group_waves=False)
        finally:
            gpu_engine.tune_ode_coop(prev)
        assert bool((sa == 0).all()) and torch_equal(sa, sb) and torch_equal(a, b), method
        prev = gpu_engine.tune_ode_launch_steps(11)
        try:
            c, sc = gpu_engine.ode(p, o, method=method, group_waves=False)
        finally:
            gpu_engine.tune_ode_launch_steps(prev)
        assert torch_equal(a, c) and torch_equal(sa, sc), method


def test_ode_riccati_segments_bit_identical(gpu_engine):
    """Waves of uniform 16- and 8-lane segments (fewer points per stage key than a wave), each
    segment on one table with one Gamma_wash: ode_riccati_kernel<., false, true> (LZQ_ODE_RICSEG)
    steps them, every segment with its own window, N and step size -- without a T = m/3 split in
    the window (pass 0 alone) and with one (m_chi ~ 40 on the narrow window: the three passes, each
    segment's split at its own step).  The per-lane mode's bits, in one launch and as continuation
    launches, and the C restatement's values."""
    rng = np.random.default_rng(79)
    cfgs = []
    for block, n_keys, split in ((16, 8, False), (8, 16, False), (16, 4, True), (8, 8, True)):
        for kk in range(n_keys):
            if split:
                m_chi = 40.0 + 0.5 * kk
                win = dict(NARROW)
            else:
                m_chi = float(10 ** rng.uniform(-0.5, 0.3))   # T > m/3 over the whole window: no split
                win = dict(T_max_over_Tp=float(rng.uniform(1.3, 1.8)), T_min_over_Tp=float(rng.uniform(0.5, 0.7)))
            gw = float(rng.choice([0.5, 2.0]))
            for _ in range(block):
                c = full_cfg(BASE_CFG)
                c.update(win, m_chi_GeV=m_chi, P_chi_to_B=float(rng.uniform(0.05, 1.0)), Gamma_wash_over_H=gw,
                         sigma_v_chi_GeV_m2=float(rng.choice([1e-16, 1e-12])),
                         deplete_DM_from_source=bool(rng.uniform() < 0.3),
                         regime=str(rng.choice(["thermal", "nonthermal"])))
                cfgs.append(c)
    p, o = recs(cfgs)
    a, sa = gpu_engine.ode(p, o, group_waves=False)
    assert bool((sa == 0).all())
    prev = gpu_engine.tune_ode_coop(False)
    try:
        b, sb = gpu_engine.ode(p, o, group_waves=False)
    finally:
        gpu_engine.tune_ode_coop(prev)
    assert torch_equal(sa, sb) and torch_equal(a, b)
    prev = gpu_engine.tune_ode_launch_steps(11)
    try:
        c, sc = gpu_engine.ode(p, o, group_waves=False)
    finally:
        gpu_engine.tune_ode_launch_steps(prev)
    assert torch_equal(a, c) and torch_equal(sa, sc)
    ref, sr = O.ode_batch(cfgs[::16], nthreads=16)
    for row, rr, s2 in zip(a.cpu().numpy()[::16], ref, sr):
        assert s2 == 0
        for v, w in zip(row[:5], rr[:5]):
            assert rel_err(v, w) < 1e-10, (v, w)


def test_ode_partial_wave_of_segments(gpu_engine):
    """A batch of 40 points in five 8-point stage keys: one partial wavefront whose lanes past the
    batch clone its first point, so it splits into uniform 8-lane segments (the clones one more
    segment of the first key) -- the segment Riccati kernel's wave.  Every point equals the
    per-lane mode's and its own single-point run, bit for bit."""
    rng = np.random.default_rng(83)
    cfgs = []
    for kk in range(5):
        m_chi = float(10 ** rng.uniform(-0.5, 0.3))
        for _ in range(8):
            c = full_cfg(BASE_CFG)
            c.update(NARROW, m_chi_GeV=m_chi, P_chi_to_B=float(rng.uniform(0.05, 1.0)), Gamma_wash_over_H=0.5,
                     sigma_v_chi_GeV_m2=float(rng.choice([1e-16, 1e-12])))
            cfgs.append(c)
    p, o = recs(cfgs)
    a, sa = gpu_engine.ode(p, o, group_waves=False)
    assert bool((sa == 0).all())
    prev = gpu_engine.tune_ode_coop(False)
    try:
        b, sb = gpu_engine.ode(p, o, group_waves=False)
    finally:
        gpu_engine.tune_ode_coop(prev)
    assert torch_equal(sa, sb) and torch_equal(a, b)
    for j in (0, 13, 39):
        one, s1 = gpu_engine.ode(p[j:j + 1], o[j:j + 1], time_parallel=False)
        assert torch_equal(one[0], a[j]) and torch_equal(s1[0], sa[j])


def test_ode_cooperative_table_varying_bit_identical(gpu_engine):
    """Cooperative segments whose points differ in the A/V kernel (I_p, v_w: a spline table each):
    the shared stage rows carry a / Av and the spline location, each lane forms a from its own
    table (ode_integrate_kernel tab_vary).  A table per point (128 distinct kernels, share_tables
    finds nothing to share) and 8 shared tables interleaved (every wavefront spans 8 tables) give
    the per-lane mode's bits, for Radau and the quadrature method, also as continuation launches;
    and the C restatement's values."""
    rng = np.random.default_rng(91)

    def cfg(I_p, v_w):
        c = full_cfg(BASE_CFG)
        c.update(NARROW, m_chi_GeV=40.0, I_p=I_p, v_w=v_w, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                 incident_flux_scale=float(10 ** rng.uniform(-10, -8)),
                 Gamma_wash_over_H=float(rng.choice([0.0, 0.5, 2.0])),
                 sigma_v_chi_GeV_m2=float(rng.choice([0.0, 1e-16, 1e-12])),
                 deplete_DM_from_source=bool(rng.uniform() < 0.3))
        if c["Gamma_wash_over_H"] == 0.0 and c["sigma_v_chi_GeV_m2"] == 0.0:
            c["deplete_DM_from_source"] = True
        return c

    per_point = [cfg(float(rng.uniform(0.1, 1.0)), float(rng.uniform(0.1, 0.9))) for _ in range(128)]
    kern = [(float(rng.uniform(0.1, 1.0)), float(rng.uniform(0.1, 0.9))) for _ in range(8)]
    shared8 = [cfg(*kern[i % 8]) for i in range(128)]
    for cfgs, share in ((per_point, False), (per_point, True), (shared8, True)):
        p, o = recs(cfgs)
        for method in ("radau", "quadrature"):
            a, sa = gpu_engine.ode(p, o, share_tables=share, method=method, group_waves=False)
            prev = gpu_engine.tune_ode_coop(False)
            try:
                b, sb = gpu_engine.ode(p, o, share_tables=share, method=method, group_waves=False)
            finally:
                gpu_engine.tune_ode_coop(prev)
            assert torch_equal(sa, sb) and torch_equal(a, b), (share, method)
            g, sg = gpu_engine.ode(p, o, share_tables=share, method=method)   # regrouped by table
            assert torch_equal(a, g) and torch_equal(sa, sg), (share, method)
            prev = gpu_engine.tune_ode_launch_steps(11)
            try:
                c, sc = gpu_engine.ode(p, o, share_tables=share, method=method, group_waves=False)
            finally:
                gpu_engine.tune_ode_launch_steps(prev)
            assert torch_equal(a, c) and torch_equal(sa, sc), (share, method)
            # chunks of 48 points: the next chunk's tables built on a side stream while one integrates
            d, sd = gpu_engine.ode(p, o, share_tables=share, method=method, group_waves=False, chunk=48)
            assert torch_equal(a, d) and torch_equal(sa, sd), (share, method, "chunked")
            if method == "radau":
                radau = (a.cpu().numpy(), sa.cpu().numpy(), dict(gpu_engine.last_ode_tables))
        if share:
            continue
        t, st, tables = radau
        assert tables["mode"] == "per_point"
        ref, sr = O.ode_batch(cfgs[::8], nthreads=16)
        for row, rr, s1, s2 in zip(t[::8], ref, st[::8], sr):
            assert s1 == 0 and s2 == 0
            for v, w in zip(row[:5], rr[:5]):
                assert rel_err(v, w) < 1e-10, (v, w)


def test_ode_riccati_table_varying_bit_identical(gpu_engine):
    """Whole waves whose points differ in the A/V kernel (I_p, v_w: a spline table each), P, flux,
    sigma_v and deplete, with one Gamma_wash per wave: ode_riccati_kernel<., true> (LZQ_ODE_RICTAB)
    steps them, each lane forming a and Y_B's d from its own table at the rows' shared spline
    location.  The per-lane mode's bits, with a split step (m_chi = 40 crosses T = m/3 inside the
    window: the kernel's three passes) and without (m_chi = 0.95), in one launch and as
    continuation launches; and the C restatement's values."""
    rng = np.random.default_rng(97)
    cfgs = []
    for m_chi in (0.95, 40.0):
        for gw in (0.0, 0.5):
            for _ in range(64):   # one whole wave (group_waves=False keeps the order)
                c = full_cfg(BASE_CFG)
                c.update(NARROW, m_chi_GeV=m_chi, I_p=float(rng.uniform(0.1, 1.0)), v_w=float(rng.uniform(0.1, 0.9)),
                         P_chi_to_B=float(rng.uniform(0.05, 1.0)), incident_flux_scale=float(10 ** rng.uniform(-10, -8)),
                         Gamma_wash_over_H=gw, sigma_v_chi_GeV_m2=float(rng.choice([1e-16, 1e-12])),
                         deplete_DM_from_source=bool(rng.uniform() < 0.3))
                cfgs.append(c)
    p, o = recs(cfgs)
    a, sa = gpu_engine.ode(p, o, group_waves=False)
    assert bool((sa == 0).all())
    prev = gpu_engine.tune_ode_coop(False)     # every wave per lane: the general variant's own stages
    try:
        b, sb = gpu_engine.ode(p, o, group_waves=False)
    finally:
        gpu_engine.tune_ode_coop(prev)
    assert torch_equal(sa, sb) and torch_equal(a, b)
    g, sg = gpu_engine.ode(p, o)               # regrouped for the launch, scattered back
    assert torch_equal(a, g) and torch_equal(sa, sg)
    prev = gpu_engine.tune_ode_launch_steps(11)
    try:
        c, sc = gpu_engine.ode(p, o, group_waves=False)
    finally:
        gpu_engine.tune_ode_launch_steps(prev)
    assert torch_equal(a, c) and torch_equal(sa, sc)
    ref, sr = O.ode_batch(cfgs[::16], nthreads=16)
    for row, rr, s2 in zip(a.cpu().numpy()[::16], ref, sr):
        assert s2 == 0
        for v, w in zip(row[:5], rr[:5]):
            assert rel_err(v, w) < 1e-10, (v, w)


def test_ode_linear_waves_table_varying_bit_identical(gpu_engine):
    """Linear cooperative waves (sigma_v = 0, one Gamma_wash per segment) whose points each have
    their own A/V kernel (I_p): the tight loop forms a_j from each lane's table, reading the lane's
    spline row once per run of steps inside one knot interval (a window with ~60 steps per interval
    takes both branches).  Bits equal the per-lane mode's, also as continuation launches."""
    rng = np.random.default_rng(5)
    cfgs = []
    for _ in range(128):
        c = full_cfg(BASE_CFG)
        c.update(T_max_over_Tp=1.6, T_min_over_Tp=0.3, I_p=float(rng.uniform(0.1, 1.0)), Gamma_wash_over_H=1.0,
                 sigma_v_chi_GeV_m2=0.0, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                 deplete_DM_from_source=bool(rng.uniform() < 0.5))
        cfgs.append(c)
    p, o = recs(cfgs)
    a, sa = gpu_engine.ode(p, o, group_waves=False)
    assert gpu_engine.last_ode_tables["mode"] == "per_point" and bool((sa == 0).all())
    prev = gpu_engine.tune_ode_coop(False)
    try:
        b, sb = gpu_engine.ode(p, o, group_waves=False)
    finally:
        gpu_engine.tune_ode_coop(prev)
    assert torch_equal(a, b) and torch_equal(sa, sb)
    prev = gpu_engine.tune_ode_launch_steps(12)
    try:
        c, sc = gpu_engine.ode(p, o, group_waves=False)
    finally:
        gpu_engine.tune_ode_launch_steps(prev)
    assert torch_equal(a, c) and torch_equal(sa, sc)
    ref, sr = O.ode_batch(cfgs[::32], nthreads=16)
    for row, rr in zip(a.cpu().numpy()[::32], ref):
        for v, w in zip(row[:5], rr[:5]):
            assert rel_err(v, w) < 1e-10, (v, w)


def test_ode_linear_waves_degenerate_step(gpu_engine):
    """A window so narrow that a step is below x's rounding (T_max / T_min - 1 = 2e-12: h ~ 1e-16 x,
    so xk + h == xk on many steps and the general path skips them): the linear integrator
    variant must not step where the general path does not, so it takes every step on the
    general path there (lzq_ode.hip k_split = -1) -- bits equal to the per-lane mode, and to a
    wider window's linear waves run next to it in the same batch."""
    rng = np.random.default_rng(53)
    cfgs = []
    for win in ({"T_max_over_Tp": 1.0 + 2e-12, "T_min_over_Tp": 1.0}, NARROW):
        for _ in range(64):
            c = full_cfg(BASE_CFG)
            c.update(win, m_chi_GeV=3.0, P_chi_to_B=float(rng.uniform(0.05, 1.0)),
                     incident_flux_scale=float(10 ** rng.uniform(-10, -8)), Gamma_wash_over_H=1.0,
                     sigma_v_chi_GeV_m2=0.0, deplete_DM_from_source=bool(rng.uniform() < 0.5))
            cfgs.append(c)
    p, o = recs(cfgs)
    a, sa = gpu_engine.ode(p, o)
    prev = gpu_engine.tune_ode_coop(False)
    try:
        b, sb = gpu_engine.ode(p, o)
    finally:
        gpu_engine.tune_ode_coop(prev)
    assert torch_equal(sa, sb) and torch_equal(a, b)
    assert bool((sa[64:] == 0).all())


def _split_step(m, T_lo, T_hi, T_p):
    """Host restatement of the integrator's first split step (lzq_ode.h branch_x and the linear
    waves' k_split): the step k with x_k < x_b <= x_k + h, x_b the first x whose T = m (1/x) is no
    longer > m/3 (same IEEE operations)."""
    x0, x1 = m / T_hi, m / max(T_lo, 1e-30)
    x_p = m / max(T_p, 1e-30)
    ms = min(min(abs(x1 - x0) / 20000.0, x_p / 1000.0), 5e-4)
    N = int(np.ceil(abs(x1 - x0) / ms))
    h = (x1 - x0) / N
    m3 = m / 3.0
    rel = lambda x: m * (1.0 / max(x, 1e-30)) > m3
    xg = m / m3
    if rel(xg):
        while rel(xg):
            xg = np.nextafter(xg, np.inf)
    else:
        while not rel(np.nextafter(xg, -np.inf)):
            xg = np.nextafter(xg, -np.inf)
    kf = int(np.floor((xg - x0) / h))
    for c in range(max(kf - 3, 0), min(kf + 4, N)):
        xc = x0 + c * h
        if xc < xg <= xc + h:
            return c, N
    return None, N


@pytest.mark.parametrize("offset", [-1, 0])
def test_ode_launch_boundary_at_split_step(gpu_engine, offset):
    """Continuation launches whose boundary falls right after (offset -1: the next launch starts at
    k_split + 1) or right at (offset 0) the T = m/3 split step of a linear cooperative wave: the
    next launch resumes with the single launch's prev_split, so the results are the single
    launch's bits (prev_split was reset at every launch)."""
    L = 6   # 2^6 = 64 steps per launch
    T_p, m = 100.0, 300.0
    for t in np.arange(1.55, 1.75, 1e-4):
        k, N = _split_step(m, 0.6 * T_p, float(t) * T_p, T_p)
        if k is not None and (k - offset) % (1 << L) == 0:
            break
    else:
        pytest.fail("no window puts the split step on a launch boundary")
    rng = np.random.default_rng(5)
    cfgs = []
    for _ in range(64):
        c = full_cfg(BASE_CFG)
        c.update(m_chi_GeV=m, T_max_over_Tp=float(t), T_min_over_Tp=0.6, Gamma_wash_over_H=0.5, sigma_v_chi_GeV_m2=0.0,
                 deplete_DM_from_source=True, P_chi_to_B=float(rng.uniform(0.05, 1.0)))
        cfgs.append(c)
    p, o = recs(cfgs)
    a, sa = gpu_engine.ode(p, o)
    prev = gpu_engine.tune_ode_launch_steps(L)
    try:
        b, sb = gpu_engine.ode(p, o)
    finally:
        gpu_engine.tune_ode_launch_steps(prev)
    assert bool((sa == 0).all()) and torch_equal(sa, sb) and torch_equal(a, b), (k, N, float(t))
