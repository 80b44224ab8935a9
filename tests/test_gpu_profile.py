"""Bounce-profile LZ path on the GPU (lzq_profile_splines / lzq_profile_crossings /
lzq_lz_propagate_profile): PAPER p.3 eqs.(5)-(9), the module the reference's hook imports
(fpy:170-187, fpy:173) and does not ship.

Parity is UNPINNED against that absent upstream module; these tests pin the kernels to the
paper's equations instead:
* splines: scipy CubicSpline (not-a-knot, the interpolant fpy:212 uses), coefficients to
  rounding;
* crossings: an analytic tanh-wall profile whose xi*, Delta'* and m_mix(xi*) are known in closed
  form (delta_LZ of eq.(8) to <= 1e-10), the numpy restatement tests/profile_ref.py on random
  multi-crossing profiles (to rounding), and O(h^4) convergence under coarse sampling;
* propagation: the numpy restatement (same steps, to rounding); lzq_lz_propagate's
  piecewise-linear model written as a profile (<= 1e-10 against lzq_lz_propagate, both
  step-converged); the 53 exact Weber-function solutions of that model (<= 2e-9 at the default
  3 steps per radian); one linear crossing in a wide window -> eq.(9) (<= 1e-8).
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN
import profile_ref as R

pytestmark = pytest.mark.gpu
WEBER = json.load(open(os.path.join(GOLDEN, "golden_weber.json")))


def tanh_wall(n, w=1.0, span=10.0, v=1.0, V=1.3, shift=0.0):
    """phi = v/2 (1 - tanh(xi/w)), Phi = V/2 (1 + tanh((xi - shift)/w)) on n uniform knots."""
    x = np.linspace(-span * w, span * w, n)
    return x, 0.5 * v * (1.0 - np.tanh(x / w)), 0.5 * V * (1.0 + np.tanh((x - shift) / w))


def tanh_wall_exact(yB, ychi, lam, vw, w=1.0, v=1.0, V=1.3):
    """Closed-form crossing of tanh_wall (shift = 0): tanh(xi*/w) = t* solves eq.(5)."""
    t = (yB * v - ychi * V) / (yB * v + ychi * V)
    xi = w * math.atanh(t)
    dp = -(yB * v + ychi * V) * (1.0 - t * t) / (2.0 * w)
    m = lam * 0.5 * v * (1.0 - t)
    return xi, dp, m, m * m / (2.0 * vw * abs(dp))


def wiggly(n, seed, span=6.0):
    """A profile with several crossings: tanh walls plus a smooth bump train."""
    rng = np.random.default_rng(seed)
    x = np.linspace(-span, span, n)
    x[1:-1] += rng.uniform(-0.3, 0.3, n - 2) * (x[1] - x[0])   # non-uniform, spacing >= 0.4 h
    phi = 0.5 * (1.0 - np.tanh(x)) + 0.3
    Phi = 0.5 * (1.0 + np.tanh(x - 0.5)) + 0.6 * np.sin(2.3 * x + rng.uniform(0, 6))
    return x, phi, Phi


def test_splines_match_scipy(gpu_engine):
    for seed, n in ((0, 4), (1, 5), (2, 37), (3, 300)):
        x, phi, Phi = wiggly(n, seed)
        sh = gpu_engine.profile_shapes(x, phi, Phi)
        c = sh.coef.cpu().numpy()[0]
        for f, y in ((0, phi), (1, Phi)):
            ref = R.spline_coefs(x, y)
            got = c[:, 4 * f:4 * f + 4]
            scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-300
            err = (np.abs(got - ref) / scale).max()
            assert err <= 1e-11, (seed, n, f, err)


def test_splines_batch_and_bad_knots(gpu_engine):
    xs, ps, Ps = zip(*(wiggly(40, s) for s in range(6)))
    sh = gpu_engine.profile_shapes(np.stack(xs), np.stack(ps), np.stack(Ps))
    one = gpu_engine.profile_shapes(xs[3], ps[3], Ps[3])
    assert sh.n_shapes == 6 and sh.n_knots == 40
    assert np.array_equal(sh.coef[3].cpu().numpy(), one.coef[0].cpu().numpy())   # bit-identical
    x = np.array(xs[0])
    x[7] = x[6]
    with pytest.raises(ValueError):
        gpu_engine.profile_shapes(x, ps[0], Ps[0])


def test_tanh_wall_closed_form(gpu_engine):
    """delta_LZ of eq.(8) at the analytic crossing to <= 1e-10 (8001 knots over +-4 w; the spline's
    Delta' converges as h^3, measured 3.6e-11 here)."""
    x, phi, Phi = tanh_wall(8001, span=4.0)
    sh = gpu_engine.profile_shapes(x, phi, Phi)
    cases = [(1.0, 1.0, 0.1, 0.3), (2.0, 0.7, 0.05, 0.1), (0.4, 1.9, 0.3, 0.9), (1.0, 0.05, 1e-3, 0.5)]
    pts = gpu_engine.profile_points(*zip(*cases), 0)
    cr = {k: v.cpu().numpy() for k, v in gpu_engine.profile_crossings(sh, pts, 4).items()}
    for i, (yB, ychi, lam, vw) in enumerate(cases):
        xi, dp, m, delta = tanh_wall_exact(yB, ychi, lam, vw)
        assert cr["count"][i] == 1
        assert abs(cr["xi"][i, 0] - xi) <= 1e-10, (i, cr["xi"][i, 0], xi)
        assert abs(cr["dprime"][i, 0] - dp) <= 1e-10 * abs(dp)
        assert abs(cr["m_mix"][i, 0] - m) <= 1e-10 * abs(m)
        assert abs(cr["delta_lz"][i, 0] - delta) <= 1e-10 * delta, (i, cr["delta_lz"][i, 0], delta)
        P9 = -math.expm1(-2 * math.pi * cr["delta_lz"][i, 0])
        assert abs(P9 - -math.expm1(-2 * math.pi * delta)) <= 1e-8 * P9


def test_spline_crossings_converge(gpu_engine):
    """Coarse sampling: with the spline, delta_LZ converges as h^3 (xi* as h^4): 16x finer knots
    cut its error >= 300x (numpy restatement: 970x, to 6e-9 at h = w/128); the linear-
    interpolation / secant estimate of round 2 converges as ~h (18x, still 4e-4 off)."""
    yB, ychi, lam, vw = 1.3, 0.8, 0.1, 0.3
    exact = tanh_wall_exact(yB, ychi, lam, vw)[3]
    errs, lin = [], []
    for n in (161, 2561):
        x, phi, Phi = tanh_wall(n)
        sh = gpu_engine.profile_shapes(x, phi, Phi)
        cr = gpu_engine.profile_crossings(sh, gpu_engine.profile_points(yB, ychi, lam, vw, 0), 2)
        errs.append(abs(cr["delta_lz"].cpu().numpy()[0, 0] / exact - 1.0))
        D = yB * phi - ychi * Phi
        k = int(np.nonzero(D[:-1] * D[1:] < 0)[0][0])
        t = D[k] / (D[k] - D[k + 1])
        m = lam * (phi[k] + t * (phi[k + 1] - phi[k]))
        dp = (D[k + 1] - D[k]) / (x[k + 1] - x[k])
        lin.append(abs(m * m / (2 * vw * abs(dp)) / exact - 1.0))
    assert errs[0] / errs[1] >= 300.0 and errs[1] < 1e-8, errs
    assert lin[0] / lin[1] < 50.0 and lin[1] > 1e4 * errs[1], (errs, lin)


def test_crossings_match_restatement(gpu_engine):
    rng = np.random.default_rng(7)
    shapes = [wiggly(60, s) for s in range(4)]
    sh = gpu_engine.profile_shapes(*(np.stack(a) for a in zip(*shapes)))
    n = 64
    yB, ychi = rng.uniform(0.5, 2.0, n), rng.uniform(0.5, 2.0, n)
    lam, vw, shp = rng.uniform(0.01, 0.5, n), rng.uniform(0.1, 0.9, n), rng.integers(0, 4, n)
    cr = {k: v.cpu().numpy() for k, v in
          gpu_engine.profile_crossings(sh, gpu_engine.profile_points(yB, ychi, lam, vw, shp), 8).items()}
    coef = sh.coef.cpu().numpy()
    total = 0
    for i in range(n):
        x = shapes[shp[i]][0]
        ref = R.crossings(x, coef[shp[i]][:, :4], coef[shp[i]][:, 4:], yB[i], ychi[i], lam[i], vw[i])
        assert cr["count"][i] == len(ref), (i, cr["count"][i], ref)
        total += len(ref)
        for k, (xi, dp, m, d) in enumerate(ref):
            assert abs(cr["xi"][i, k] - xi) <= 1e-13 * max(1.0, abs(xi))
            assert abs(cr["dprime"][i, k] - dp) <= 1e-12 * abs(dp)
            assert abs(cr["m_mix"][i, k] - m) <= 1e-12 * abs(m)
            assert abs(cr["delta_lz"][i, k] - d) <= 1e-11 * d
    assert total >= 2 * n    # several crossings per profile on average
    bad = gpu_engine.profile_points(1.0, 1.0, 0.1, 0.3, [0, 4, -1])
    assert gpu_engine.profile_crossings(sh, bad, 2)["count"].cpu().tolist()[1:] == [-1, -1]


def test_propagation_matches_restatement(gpu_engine):
    shapes = [wiggly(24, s, span=4.0) for s in range(2)]
    sh = gpu_engine.profile_shapes(*(np.stack(a) for a in zip(*shapes)))
    coef = sh.coef.cpu().numpy()
    cases = [(1.0, 1.1, 0.2, 0.3, 0), (0.8, 1.5, 0.05, 0.6, 1), (1.6, 0.9, 0.4, 0.2, 0), (1.2, 1.2, 1.0, 0.9, 1)]
    got = gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(*zip(*cases)), 3.0, 8).cpu().numpy()
    got1 = gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(*zip(*cases))).cpu().numpy()
    for i, (yB, ychi, lam, vw, s) in enumerate(cases):
        ref = R.propagate_profile(shapes[s][0], coef[s][:, :4], coef[s][:, 4:], yB, ychi, lam, vw, spr=3.0, n_min=8)
        assert 0.0 <= got[i] <= 1.0
        assert abs(got[i] - ref) <= 1e-11, (i, got[i], ref)
        ref1 = R.propagate_profile(shapes[s][0], coef[s][:, :4], coef[s][:, 4:], yB, ychi, lam, vw)   # the defaults
        assert abs(got1[i] - ref1) <= 1e-11, (i, got1[i], ref1)
    # the defaults (4 steps per radian, min_steps 1) against the step-converged result (16)
    conv = gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(*zip(*cases)), 16.0).cpu().numpy()
    assert np.max(np.abs(got1 - conv)) <= 2e-9, (got1, conv)


def _linear_shape(engine, c):
    """lzq_lz_propagate's piecewise-linear model as a profile (tests/profile_ref.py
    linear_cells_profile): with y_B = 0, y_chi = -1, lambda = 1, Delta = Phi and m = phi exactly.
    phi is piecewise constant (m jumps at the turning points), which a spline would smooth, so the
    rows are written directly, 4 knot intervals per cell."""
    import torch
    from conftest import pkg
    kn, cD, cM = R.linear_cells_profile(c["m"], c["d"], c["x"], WEBER["v_w"], c["K"])
    xs, rows = [], []
    for j in range(len(kn) - 1):
        for f in (0.0, 0.25, 0.5, 0.75):
            t = f * (kn[j + 1] - kn[j])
            xs.append(kn[j] + t)
            rows.append([cM[j][0], 0.0, 0.0, 0.0, cD[j][0] + cD[j][1] * t, cD[j][1], 0.0, 0.0])
    xs.append(kn[-1])
    k = torch.as_tensor(np.array(xs)[None, :], device=engine.device)
    cf = torch.as_tensor(np.array(rows)[None, :, :], device=engine.device)
    return pkg("engine").ProfileShapes(k, cf)


def _profile_P(engine, c, spr):
    sh = _linear_shape(engine, c)
    return engine.lz_propagate_profile(sh, engine.profile_points(0.0, -1.0, 1.0, WEBER["v_w"], 0), spr)


def test_piecewise_linear_profile_matches_lz_propagate(gpu_engine):
    """Delta exactly piecewise linear and m constant per cell: the profile propagator agrees with
    lzq_lz_propagate (the model's dedicated kernel) to <= 1e-10, both step-converged."""
    cases = [c for c in WEBER["cases"] if c["kind"] in ("multi", "single")][::4]
    cases += [c for c in WEBER["cases"] if c["kind"] == "c5" and len(c["m"]) == 8][:2]
    for c in cases:
        P = float(_profile_P(gpu_engine, c, 8.0).cpu().numpy()[0])
        Q = float(gpu_engine.lz_propagate([c["m"]], [c["d"]], [c["x"]], WEBER["v_w"], c["K"], 16000).cpu().numpy()[0])
        assert abs(P - Q) <= 1e-10, (c["kind"], c["m"], P, Q)


def test_weber_fixtures_default_steps(gpu_engine):
    """All 53 exact Weber-function solutions at 3 steps per radian: <= 2e-9 (measured 9.2e-10;
    lzq_lz_propagate at the C5 default: 7.2e-10); at the default 4: <= 2.5e-10 (measured 1.64e-10;
    4.9e-10 while the step midpoint was a running sum)."""
    worst, worst4 = 0.0, 0.0
    for c in WEBER["cases"]:
        P4 = float(_profile_P(gpu_engine, c, 4.0).cpu().numpy()[0])
        worst4 = max(worst4, abs(P4 - c["P"]))
        P = float(_profile_P(gpu_engine, c, 3.0).cpu().numpy()[0])
        worst = max(worst, abs(P - c["P"]))
        assert abs(P - c["P"]) <= 2e-9, (c["kind"], c["m"], c["d"], P, c["P"])
    print(f"profile propagator vs 53 Weber fixtures: worst {worst:.3g} (3 steps/rad), {worst4:.3g} (4)")
    assert worst4 <= 2.5e-10


def test_single_linear_crossing_is_eq9(gpu_engine):
    """Constant phi and linear Phi through splines (not-a-knot reproduces both exactly): one
    crossing, +-20 LZ lengths -> P = 1 - exp(-2 pi delta) (eq.(9)) to <= 1e-8 relative."""
    vw = 0.3
    for lam, slope in ((0.05, 1.0), (0.3, 0.7), (1.0, 2.0), (0.02, 5.0)):
        delta = lam * lam / (2 * vw * slope)
        L = math.sqrt(vw / slope) * max(1.0, math.sqrt(delta))
        x = np.linspace(-20 * L, 20 * L, 81)
        sh = gpu_engine.profile_shapes(x, np.ones_like(x), slope * x)
        pts = gpu_engine.profile_points(0.0, -1.0, lam, vw, 0)   # Delta = slope xi, m = lam
        assert abs(gpu_engine.profile_crossings(sh, pts, 1)["delta_lz"].cpu().numpy()[0, 0] - delta) <= 1e-13 * delta
        P = float(gpu_engine.lz_propagate_profile(sh, pts).cpu().numpy()[0])
        P9 = -math.expm1(-2 * math.pi * delta)
        assert abs(P - P9) <= 1e-8 * P9, (lam, slope, P, P9)


def test_batch_invariance_and_bad_inputs(gpu_engine):
    """A point's P does not depend on its batch: LDS-staged (the block's shape) and HBM-read
    (another shape in the block) paths are bit-identical; bad wall speed / shape -> NaN."""
    shapes = [wiggly(30, s, span=3.0) for s in range(3)]
    sh = gpu_engine.profile_shapes(*(np.stack(a) for a in zip(*shapes)))
    rng = np.random.default_rng(3)
    n = 600
    args = (rng.uniform(0.8, 1.5, n), rng.uniform(0.8, 1.5, n), rng.uniform(0.05, 0.3, n), rng.uniform(0.2, 0.8, n))
    shp = rng.integers(0, 3, n)
    mixed = gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(*args, shp)).cpu().numpy()
    order = np.argsort(shp, kind="stable")
    grouped = gpu_engine.lz_propagate_profile(
        sh, gpu_engine.profile_points(*(a[order] for a in args), shp[order])).cpu().numpy()
    assert np.array_equal(mixed[order], grouped)
    # >= 16384 points run cost-ordered (profile_cost_kernel + counting sort); < 16384 in index
    # order: the same bits
    n2 = 20_000
    big = (rng.uniform(0.5, 2.0, n2), rng.uniform(0.5, 2.0, n2), 10 ** rng.uniform(-3, 0, n2), rng.uniform(0.1, 0.9, n2))
    shp2 = rng.integers(0, 3, n2)
    whole = gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(*big, shp2)).cpu().numpy()
    parts = np.concatenate([gpu_engine.lz_propagate_profile(
        sh, gpu_engine.profile_points(*(a[k:k + 5000] for a in big), shp2[k:k + 5000])).cpu().numpy()
        for k in range(0, n2, 5000)])
    assert np.array_equal(whole, parts) and np.isfinite(whole).all()
    bad = gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(1.0, 1.0, 0.1, [0.3, 0.0, 0.3, 0.3],
                                                                         [0, 0, 3, -2])).cpu().numpy()
    assert np.isfinite(bad[0]) and np.isnan(bad[1:]).all()
    from conftest import pkg
    with pytest.raises(pkg("_native").LzqError):
        gpu_engine.lz_propagate_profile(sh, gpu_engine.profile_points(1.0, 1.0, 0.1, 0.3, 0), 0.1)


def test_flat_propagation_bit_identical_to_interval_loop(gpu_engine):
    """The flattened propagation (LZQ_TUNE_PROFILE_FLAT, opt-in: the step rule ahead of the
    propagation, one Magnus loop per lane crossing knot intervals on its own) performs each lane's
    interval-loop operations: P bit-identical on mixed shapes, index-ordered and ordered batches
    (>= 16384 points: the flat path's cost bins, the loop's keyed radix order), NaN inputs, and steps
    that do not fit the uint16 step record (huge steps_per_radian on a long interval: recomputed from
    the samples)."""
    shapes = [wiggly(40, s, span=5.0) for s in range(3)]
    sh = gpu_engine.profile_shapes(*(np.stack(a) for a in zip(*shapes)))
    rng = np.random.default_rng(11)
    for n in (700, 20_000):
        args = (rng.uniform(0.5, 2.0, n), rng.uniform(0.5, 2.0, n), 10 ** rng.uniform(-3, 0, n),
                rng.uniform(0.05, 0.9, n))
        shp = rng.integers(0, 3, n)
        pts = gpu_engine.profile_points(*args, shp)
        loop = gpu_engine.lz_propagate_profile(sh, pts).cpu().numpy()
        prev = gpu_engine.tune_profile_flat(True)
        try:
            flat = gpu_engine.lz_propagate_profile(sh, pts).cpu().numpy()
        finally:
            gpu_engine.tune_profile_flat(prev)
        assert prev is False and np.array_equal(flat, loop) and np.isfinite(flat).all(), n
    # > 65534 steps in one interval (the record's overflow path) and bad inputs
    pts = gpu_engine.profile_points(1.0, 1.0, 0.1, [0.3, 0.0, 0.3, 0.0005], [0, 0, 3, 1])
    loop = gpu_engine.lz_propagate_profile(sh, pts, 900.0).cpu().numpy()
    prev = gpu_engine.tune_profile_flat(True)
    try:
        flat = gpu_engine.lz_propagate_profile(sh, pts, 900.0).cpu().numpy()
    finally:
        gpu_engine.tune_profile_flat(prev)
    assert np.array_equal(flat, loop, equal_nan=True) and np.isnan(flat[1:3]).all() and np.isfinite(flat[[0, 3]]).all()
