"""Grid sweeps on the GPU: on-device point generation vs explicit points, sharded launches
bit-identical to one launch (the multi-GPU invariant), and the separability identities of
SURVEY §8c at full grid sizes (size-independent properties)."""
import numpy as np
import pytest

from conftest import BASE_CFG, full_cfg, pkg, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def c2_axes(n_mix=1000, n_dp=1000):
    return [("m_mix", np.logspace(-3, 0, n_mix)), ("dprime", np.logspace(-3, 1, n_dp))]


def test_grid_matches_explicit_points(gpu_engine):
    axes = [("m_chi_GeV", np.logspace(0, 3.5, 5)), ("I_p", np.linspace(0.05, 1, 3)),
            ("delta_LZ", np.logspace(-4, 0, 4))]
    t = gpu_engine.sweep(full_cfg(BASE_CFG), axes, 0, 60).cpu().numpy()
    cfgm = pkg("config")
    cfgs = []
    for m in axes[0][1]:
        for ip in axes[1][1]:
            for dl in axes[2][1]:
                P = O.p_closed_form(float(dl))
                cfgs.append(full_cfg({**BASE_CFG, "m_chi_GeV": float(m), "I_p": float(ip), "P_chi_to_B": P}))
    e = gpu_engine.yields(np.concatenate([cfgm.to_point(c) for c in cfgs])).cpu().numpy()
    assert np.array_equal(t, e)
    ref = O.points_batch(cfgs, nthreads=16)
    assert max(rel_err(a, b) for a, b in zip(t.ravel(), ref.ravel())) < 1e-11


def test_shards_bit_identical(gpu_engine):
    axes = c2_axes(16, 16)
    full = gpu_engine.sweep(full_cfg(BASE_CFG), axes, 0, 256).cpu().numpy()
    for W in (2, 4, 8):
        parts = [gpu_engine.sweep(full_cfg(BASE_CFG), axes, r * 256 // W, (r + 1) * 256 // W - r * 256 // W).cpu().numpy()
                 for r in range(W)]
        assert np.array_equal(np.concatenate(parts), full)


def test_c2_full_grid_separability(gpu_engine):
    """Full 1e6-point C2 grid: Y_B / P_used is the same quadrature for every point
    (Y_B is linear in P, PAPER §8), and P_used follows eq.(8)-(9)."""
    axes = c2_axes()
    t = gpu_engine.sweep(full_cfg(BASE_CFG), axes, 0, 1_000_000).cpu().numpy()
    P = t[:, 5]
    ok = P > 1e-6
    ratio = t[ok, 0] / P[ok]
    assert np.max(np.abs(ratio / ratio[0] - 1)) < 1e-14
    m, d = np.meshgrid(axes[0][1], axes[1][1], indexing="ij")
    delta = (m * m / (2.0 * 0.3 * d)).ravel()
    assert np.allclose(P, 1.0 - np.exp(-2.0 * np.pi * delta), rtol=1e-13, atol=5e-16)  # GPU vs numpy exp: 1 ulp of 1.0
    YB1 = 8.720885362714675e-11 / 0.14925839040304145
    assert rel_err(ratio[0], YB1) < 1e-11


def test_known_answer_identities(gpu_engine):
    """SURVEY §8c identities, exact to ~1e-15 in the reference."""
    base = full_cfg(BASE_CFG)
    variants = [base, {**base, "P_chi_to_B": 2 * base["P_chi_to_B"]},
                {**base, "incident_flux_scale": 3 * base["incident_flux_scale"]}, {**base, "v_w": 0.15},
                {**base, "T_p_GeV": 10.0}, {**base, "T_p_GeV": 1000.0}, {**base, "beta_over_H": 50.0},
                {**base, "chi_stats": "boson"}, {**base, "m_chi_GeV": 50.0}, {**base, "T_min_over_Tp": 6.0}]
    cfgm = pkg("config")
    t = gpu_engine.yields(np.concatenate([cfgm.to_point(c) for c in variants])).cpu().numpy()[:, 0]
    y0 = t[0]
    assert rel_err(t[1], 2 * y0) < 1e-14
    assert rel_err(t[2], 3 * y0) < 1e-14
    assert rel_err(t[3], 2 * y0) < 1e-13
    assert rel_err(t[4], y0) < 1e-12 and rel_err(t[5], y0) < 1e-12
    assert rel_err(t[6], y0) < 1e-12
    assert rel_err(t[7], 4.0 / 3.0 * y0) < 1e-14
    assert rel_err(t[8], y0) < 1e-14
    assert t[9] == 0.0


def test_c5_multicrossing_pipeline(gpu_engine):
    """C5: per-point 8-crossing profiles -> coherent P (propagator) -> quadrature.  P_used is
    the propagator's output (checked against the numpy restatement) and Y_B = P_used x the
    C1 quadrature (only P differs between C2-grid points)."""
    from lz_ref import propagate
    sw = pkg("sweep")
    spec = sw.builtin_specs()["C5"]
    start, n = 123_400, 96
    t = gpu_engine.sweep(spec.base, spec.axes, start, n, P_points=None).cpu().numpy()  # closed-form P
    comp = sw.make_compute(spec, gpu_engine)
    import torch
    out = torch.empty((n, 6), dtype=torch.float64, device=gpu_engine.device)
    comp(start, n, out)
    o = out.cpu().numpy()
    m, dp, xi, v_w = (x.cpu().numpy() if hasattr(x, "cpu") else x for x in spec.crossing_arrays(start, n, "cpu"))
    for i in (0, 17, 95):
        ref = propagate(list(m[i]), list(dp[i]), list(xi[i]), float(v_w[i]), spec.crossings.window_lz,
                        spec.crossings.steps)
        assert abs(o[i, 5] - ref) <= 1e-10 * max(ref, 1e-3), (i, o[i, 5], ref)
    YB1 = 8.720885362714675e-11 / 0.14925839040304145
    ok = o[:, 5] > 1e-8
    assert np.all(np.abs(o[ok, 0] / o[ok, 5] / YB1 - 1) < 1e-11)
    assert not np.array_equal(o[:, 5], t[:, 5])  # coherent multi-crossing P differs from eq.(9)


def test_sweep_cli_end_to_end(tmp_path, gpu_engine):
    import json
    sw = pkg("sweep")
    out = tmp_path / "new_subdir"        # main() must create --out itself
    sw.main(["--spec", "C2", "--limit", "2048", "--chunk", "700", "--out", str(out)])
    tab = np.load(out / "table.npy")
    summ = json.loads((out / "summary.json").read_text())
    assert tab.shape == (2048, 6) and summ["n_points"] == 2048
    ref = gpu_engine.sweep(sw.EQUAL_MASS, sw.builtin_specs()["C2"].axes, 0, 2048).cpu().numpy()
    assert np.array_equal(tab, ref)
    sw.main(["--spec", "C2", "--limit", "2048", "--chunk", "700", "--out", str(out), "--resume"])
    assert np.array_equal(np.load(out / "table.npy"), ref)
    # resuming another spec into the same directory is refused, not mixed
    with pytest.raises(RuntimeError, match="another sweep"):
        sw.main(["--spec", "C3", "--limit", "2048", "--chunk", "700", "--out", str(out), "--resume"])


def test_multicrossing_with_ode_fallback(gpu_engine):
    """A multi-crossing sweep (C5-style crossings) over Gamma_wash: every point's P is the
    coherent propagator output, and the points route per fpy:372 -- Gamma_wash = 0 to the
    quadrature, > 0 to the ODE fallback -- bit-identical to calling those directly."""
    import dataclasses

    import torch
    sw = pkg("sweep")
    c5 = sw.builtin_specs()["C5"]
    spec = dataclasses.replace(c5, name="C5_ode", base={**c5.base, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6},
                               axes=[("m_mix", np.logspace(-3, 0, 6)), ("dprime", np.logspace(-3, 1, 5)),
                                     ("Gamma_wash_over_H", np.array([0.0, 0.5]))])
    assert sw.is_ode_spec(spec)
    n = spec.total
    out = torch.empty((n, 6), dtype=torch.float64, device=gpu_engine.device)
    sw.make_compute(spec, gpu_engine)(0, n, out)
    P = sw.coherent_P(spec, 0, n, gpu_engine).cpu().numpy()
    pts, ods = sw.grid_records(spec, 0, n, gpu_engine)
    pts["P_chi_to_B"] = P
    ode = ods["Gamma_wash_over_H"] != 0.0
    want = torch.empty_like(out)
    want[torch.as_tensor(np.nonzero(ode)[0], device=out.device)] = gpu_engine.ode(pts[ode], ods[ode])[0]
    want[torch.as_tensor(np.nonzero(~ode)[0], device=out.device)] = gpu_engine.yields(pts[~ode], n_y=spec.n_y)
    assert torch.equal(out, want)
    t = out.cpu().numpy()
    assert np.isfinite(t).all() and np.array_equal(t[:, 5], P)


@pytest.mark.parametrize("name", ["C2", "C3", "C4"])
def test_reuse_zsums_bit_identical(gpu_engine, name):
    """lzq_sweep_grid_reuse (z-sums shared per y-grid + A/V kernel; not the headline mode) gives
    the same bits as the dense lzq_sweep_grid: 3000-point slices of each config grid at two
    offsets (C3 crosses m_chi's T = m/3 branch, C4 sweeps beta/H, I_p, v_w, sigma_y, m_chi)."""
    import torch
    spec = pkg("sweep").builtin_specs()[name]
    for start in (0, spec.total // 2 - 1500):
        dense = gpu_engine.sweep(spec.base, spec.axes, start, 3000, n_y=spec.n_y)
        reuse = gpu_engine.sweep(spec.base, spec.axes, start, 3000, n_y=spec.n_y, reuse=True)
        assert torch.equal(dense, reuse), (name, start)
        assert bool(torch.isfinite(reuse).all())


def test_reuse_zsums_table_axes_and_overrides(gpu_engine):
    """Every field the z-sums depend on as an axis (I_p, beta/H, T_p, T_min/T_p, T_max/T_p,
    including an empty window), fields they do not (m_chi, v_w, delta) in between, a P override,
    and n_y below the 2000 floor: reuse == dense bit for bit."""
    import torch
    axes = [("T_p_GeV", np.array([10.0, 100.0])), ("m_chi_GeV", np.array([0.95, 40.0])),
            ("T_max_over_Tp", np.array([1.6, 5.0])), ("I_p", np.array([0.1, 0.34, 0.9])),
            ("v_w", np.array([0.2, 0.8])), ("T_min_over_Tp", np.array([0.001, 0.5, 8.0])),
            ("beta_over_H", np.array([30.0, 300.0])), ("delta_LZ", np.array([1e-3, 0.2]))]
    base = {**BASE_CFG, "regime": "thermal"}
    total = int(np.prod([len(v) for _, v in axes]))
    P = torch.rand(total, dtype=torch.float64, device=gpu_engine.device)
    for n_y in (8000, 500):
        dense = gpu_engine.sweep(base, axes, 0, total, n_y=n_y, P_points=P)
        reuse = gpu_engine.sweep(base, axes, 0, total, n_y=n_y, P_points=P, reuse=True)
        assert torch.equal(dense, reuse)
    t = reuse.cpu().numpy()
    assert (t[:, 0] == 0.0).any() and np.isfinite(t[:, 1]).all()   # T_min/T_p = 8: empty window, Y_B = 0
    prev = gpu_engine.tune_exp("poly11")            # the tables follow the exponential variant too
    try:
        dense = gpu_engine.sweep(base, axes, 0, total, P_points=P)
        reuse = gpu_engine.sweep(base, axes, 0, total, P_points=P, reuse=True)
    finally:
        gpu_engine.tune_exp(prev)
    assert torch.equal(dense, reuse)


def test_profile_sweep_P1(gpu_engine):
    """P1: P of every grid point from a bounce profile (PAPER eqs.(5)-(9)) through the sweep
    driver.  P_used equals the engine's profile kernels on the same couplings bit for bit (eq.(9)
    of the crossing's delta for one crossing, the propagation through the profile otherwise),
    Y_B / P_used is the shipped config's quadrature per unit P, and 64 rows match the oracle."""
    import torch
    sw = pkg("sweep")
    spec = sw.builtin_specs()["P1"]
    s, n = 302_000, 4096      # y_B index 30, y_chi 20..61: one and three crossings
    out = torch.empty((n, 6), dtype=torch.float64, device=gpu_engine.device)
    sw.make_compute(spec, gpu_engine)(s, n, out)
    t = out.cpu().numpy()
    assert np.isfinite(t).all()
    vals = {k: v.cpu().numpy() for k, v in spec.axis_values(s, n, "cpu").items()}
    sh = gpu_engine.profile_shapes(*spec.profile.arrays())
    pts = gpu_engine.profile_points(vals["y_B"], vals["y_chi"], vals["lambda_tr_eff"], spec.base["v_w"], 0)
    cr = gpu_engine.profile_crossings(sh, pts, 1)
    cnt = cr["count"].cpu().numpy()
    P9 = gpu_engine.p_closed_form(cr["delta_lz"][:, 0]).cpu().numpy()
    Pp = gpu_engine.lz_propagate_profile(sh, pts).cpu().numpy()
    want = np.where(cnt == 1, P9, Pp)
    assert (cnt == 1).any() and (cnt != 1).any(), np.unique(cnt)
    assert np.array_equal(t[:, 5], want)
    YB1 = 8.720885362714675e-11 / 0.14925839040304145
    pos = t[:, 5] > 1e-6
    assert np.max(np.abs(t[pos, 0] / t[pos, 5] / YB1 - 1.0)) < 1e-11
    sub = np.sort(np.random.default_rng(2).choice(n, 64, replace=False))
    cfgs = [full_cfg({**BASE_CFG, "P_chi_to_B": float(t[i, 5])}) for i in sub]
    ref = O.points_batch(cfgs, nthreads=16)
    assert np.max(np.abs(t[sub] - ref) / np.abs(ref)) < 1e-11


def test_profile_sweep_csv_matches_plugin(gpu_engine, tmp_path, monkeypatch):
    """A profile sweep over y_B from a bounce-profile CSV: its P_used is the plug-in module's
    compute_prob_from_profile for the same couplings (the reference hook's path), bit for bit."""
    import importlib
    import json
    import os
    import torch
    from conftest import ROOT
    sw = pkg("sweep")
    xs = np.linspace(-4.0, 4.0, 2001)
    phi, Phi = 0.5 * (1.0 - np.tanh(xs)), 0.65 * (1.0 + np.tanh(xs))
    body = "xi,phi,Phi\n" + "".join(f"{float(a)!r},{float(b)!r},{float(c)!r}\n" for a, b, c in zip(xs, phi, Phi))
    (tmp_path / "bounce.csv").write_text(body)
    yBs = [0.7, 1.0, 1.3, 1.9]
    spec = sw.spec_from_json({"name": "csv", "profile": {"csv": str(tmp_path / "bounce.csv"), "y_chi": 0.8,
                                                          "lambda_tr_eff": 0.1},
                              "axes": [{"field": "y_B", "values": yBs}]})
    out = torch.empty((4, 6), dtype=torch.float64, device=gpu_engine.device)
    sw.make_compute(spec, gpu_engine)(0, 4, out)
    monkeypatch.syspath_prepend(os.path.join(ROOT, "plugins"))
    tfp = importlib.import_module("transport_from_profile")
    for i, yB in enumerate(yBs):
        (tmp_path / "p.csv").write_text(f"# y_B = {yB!r}\n# y_chi = 0.8\n# lambda_tr_eff = 0.1\n" + body)
        assert out[i, 5].item() == tfp.compute_prob_from_profile(str(tmp_path / "p.csv"), 0.30), yB
