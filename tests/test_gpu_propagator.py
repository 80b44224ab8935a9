"""LZ propagator kernel (lzq_lz_propagate) on the GPU.

* vs the numpy restatement tests/lz_ref.py (same scheme): agreement to rounding, for one and
  for several crossings (parity UNPINNED w.r.t. the reference, which has no propagator);
* single crossing vs the reference's closed form (fpy:183-184, PAPER eq.(9)) over the C2
  (m_mix, |Delta'|) grid (delta 1.7e-7 .. 1.7e3) at K = 20 LZ lengths, S = 1000: stated
  tolerance 1e-8 relative (north_star's P_LZ gate; the dressed window edges leave ~2e-9);
* vs the EXACT finite-window solution (Weber functions, tests/golden/golden_weber.json):
  stated tolerance 1e-10 at the C5 default S = 64 and step-converged (S = 16000), exact
  adiabatic cells included;
* phase averaging: widely separated crossings averaged over position jitter reproduce the
  incoherent composition (1 - prod(1 - 2 P_c)) / 2.
"""
import math

import numpy as np
import pytest

from conftest import pkg
from lz_ref import propagate

pytestmark = pytest.mark.gpu
V_W = 0.3


def test_matches_numpy_restatement(gpu_engine):
    cases = [([0.1], [1.0], [0.0]),
             ([0.05, 0.08, 0.2], [1.0, 0.5, 2.0], [0.0, 3.0, 7.5]),
             ([0.3, 0.01], [0.2, 0.05], [-1.0, 20.0])]
    for m, d, x in cases:
        got = gpu_engine.lz_propagate([m], [d], [x], V_W, 12.0, 300).cpu().numpy()[0]
        ref = propagate(m, d, x, V_W, 12.0, 300)
        assert abs(got - ref) <= 1e-11 * max(abs(ref), 1e-3), (m, d, x, got, ref)


def test_single_crossing_closed_form(gpu_engine):
    m, d = np.meshgrid(np.logspace(-3, 0, 12), np.logspace(-3, 1, 12), indexing="ij")
    m, d = m.ravel(), d.ravel()
    got = gpu_engine.lz_propagate(m, d, np.zeros_like(m), V_W, 20.0, 1000).cpu().numpy()
    delta = m * m / (2 * V_W * d)
    P = -np.expm1(-2 * np.pi * delta)
    rel = np.abs(got - P) / np.maximum(P, 1e-300)
    assert np.all(rel < 1e-8), rel.max()
    # the reference's own naive 1 - exp (fpy:183) on the same grid, through the C ABI
    P = 1.0 - np.exp(-2 * np.pi * delta)
    lam = gpu_engine.p_closed_form(delta).cpu().numpy()
    assert np.allclose(lam, P, rtol=1e-13, atol=5e-16)


def test_phase_average_is_incoherent_composition(gpu_engine):
    rng = np.random.default_rng(5)
    n, N = 4096, 4
    m = np.full((n, N), 0.1)
    d = np.full((n, N), 1.0)
    base = np.arange(N) * 40.0
    x = base[None, :] + rng.uniform(-2.0, 2.0, (n, N))
    got = gpu_engine.lz_propagate(m, d, x, V_W, 20.0, 2000).cpu().numpy()
    P1 = 1.0 - math.exp(-2 * math.pi * 0.1 ** 2 / (2 * V_W * 1.0))
    inc = pkg("lz").p_incoherent([P1] * N)
    assert abs(got.mean() - inc) < 4 * got.std() / math.sqrt(n) + 1e-3, (got.mean(), inc)
    assert got.std() > 1e-3  # coherent (Stueckelberg) oscillations are present


def test_kernel_vs_exact_weber_solution(gpu_engine):
    """Kernel vs the EXACT finite-window solution of its model (cell-by-cell Weber functions,
    tests/golden/golden_weber.json; tests/test_propagator_exact.py states the tolerances):
    C5 default S = 64 and S = 16000: <= 1e-10 (cores + superadiabatic following; the numpy
    restatement measures 3.4e-11 and 4.2e-11), exact adiabatic cells included."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_weber.json")))
    groups = {}
    for c in g["cases"]:
        groups.setdefault((len(c["m"]), c["K"]), []).append(c)
    n = 0
    for (N, K), cs in groups.items():
        m = np.array([c["m"] for c in cs])
        d = np.array([c["d"] for c in cs])
        x = np.array([c["x"] for c in cs])
        ex = np.array([c["P"] for c in cs])
        for S, tol in ((64, 1e-10), (16000, 1e-10)):
            got = gpu_engine.lz_propagate(m, d, x, g["v_w"], K, S).cpu().numpy()
            assert np.all(np.abs(got - ex) <= tol), (N, K, S, np.abs(got - ex).max())
        n += len(cs)
    assert n == len(g["cases"]) == 53


def test_longest_first_order_is_bit_identical(gpu_engine):
    """Batches of >= 16384 points run in longest-first order (lz_cost_kernel + counting sort,
    lzq_propagator.hip): P must be bit-identical to index order, which smaller batches use.
    A C5 slice of 40000 points (8 jittered crossings) whose step counts span ~1e3..6e4, plus
    NaN and adiabatic-only points mixed in."""
    import torch
    sw = pkg("sweep")
    spec = sw.builtin_specs()["C5"]
    n = 40000
    m, dp, xi, v_w = spec.crossing_arrays((spec.total - n) // 2, n, gpu_engine.device)
    m = m.clone()
    m[7] = float("nan")            # the kernel's NaN exit
    m[12345] *= 100.0              # every cell adiabatic (closed form only)
    args = (float(v_w[0]), spec.crossings.window_lz, spec.crossings.steps)
    whole = gpu_engine.lz_propagate(m, dp, xi, *args)
    parts = torch.cat([gpu_engine.lz_propagate(m[i:i + 10000], dp[i:i + 10000], xi[i:i + 10000], *args)
                       for i in range(0, n, 10000)])   # < 16384: index order
    assert torch.isnan(whole[7]) and torch.isnan(parts[7])
    ok = ~torch.isnan(parts)
    assert int(ok.sum()) == n - 1
    assert torch.equal(whole[ok], parts[ok])


def test_per_point_wall_speed(gpu_engine):
    """lzq_lz_propagate_v (a wall speed per point, for sweeps over v_w with crossings): equal bit
    for bit to lzq_lz_propagate called per v_w value, in both launch orders (>= 16384 points:
    longest-first), and NaN for a non-positive v_w."""
    import torch
    sw = pkg("sweep")
    spec = sw.builtin_specs()["C5"]
    n = 20000
    m, dp, xi, _ = spec.crossing_arrays((spec.total - n) // 2, n, gpu_engine.device)
    speeds = torch.tensor([0.1, 0.3, 0.9], dtype=torch.float64, device=gpu_engine.device)
    vw = speeds[torch.arange(n, device=gpu_engine.device) % 3].clone()
    K, S = spec.crossings.window_lz, spec.crossings.steps
    got = gpu_engine.lz_propagate(m, dp, xi, vw, K, S)
    for k in range(3):
        sel = torch.arange(k, n, 3, device=gpu_engine.device)
        want = gpu_engine.lz_propagate(m[sel], dp[sel], xi[sel], float(speeds[k]), K, S)
        assert torch.equal(got[sel], want)
    small = gpu_engine.lz_propagate(m[:500], dp[:500], xi[:500], vw[:500], K, S)   # index order
    assert torch.equal(small, got[:500])
    vw[3] = 0.0
    bad = gpu_engine.lz_propagate(m[:8], dp[:8], xi[:8], vw[:8], K, S)
    assert torch.isnan(bad[3]) and bool(torch.isfinite(bad[torch.arange(8) != 3]).all())


def test_multicrossing_sweep_over_wall_speed(gpu_engine):
    """A C5-style sweep with a v_w axis (the C4 scan's v_w values) runs through the sweep driver
    (it used to refuse): every point's P is the per-point-v_w propagator output."""
    import dataclasses

    import torch
    sw = pkg("sweep")
    c5 = sw.builtin_specs()["C5"]
    spec = dataclasses.replace(c5, name="C5_vw", axes=[("v_w", np.linspace(0.05, 0.95, 10)),
                                                       ("m_mix", np.logspace(-3, 0, 8)), ("dprime", np.logspace(-3, 1, 8))])
    n = spec.total
    out = torch.empty((n, 6), dtype=torch.float64, device=gpu_engine.device)
    sw.make_compute(spec, gpu_engine)(0, n, out)
    m, dp, xi, vw = spec.crossing_arrays(0, n, gpu_engine.device)
    P = gpu_engine.lz_propagate(m, dp, xi, vw, spec.crossings.window_lz, spec.crossings.steps)
    assert torch.equal(out[:, 5], P) and bool(torch.isfinite(out).all())


def test_follow_slices_bit_identical(gpu_engine):
    """Batches of more than 2^23 (point, cell) pairs run in slices (the follow matrices take 80 B
    per pair, lzq_propagator.hip kFollowMaxPairs): 270,000 points x 32 crossings (two slices) give
    the same P bit for bit as the points run in separate smaller calls."""
    import dataclasses

    import torch
    sw = pkg("sweep")
    spec = sw.builtin_specs()["C5"]
    spec = dataclasses.replace(spec, crossings=dataclasses.replace(spec.crossings, n_cross=32))
    n = 270_000
    m, dp, xi, v_w = spec.crossing_arrays((spec.total - n) // 2, n, gpu_engine.device)
    args = (float(v_w[0]), spec.crossings.window_lz, spec.crossings.steps)
    whole = gpu_engine.lz_propagate(m, dp, xi, *args)
    cut = 100_000
    parts = torch.cat([gpu_engine.lz_propagate(m[:cut], dp[:cut], xi[:cut], *args),
                       gpu_engine.lz_propagate(m[cut:], dp[cut:], xi[cut:], *args)])
    assert bool(torch.isfinite(whole).all())
    assert torch.equal(whole, parts)


def test_edge_couplings_match_restatement(gpu_engine):
    """Cells at the edges of the superadiabatic scheme, kernel vs the numpy restatement: zero
    coupling (P = 0: the frames are the diabatic basis), couplings below the core-width floor
    (m_hat < 0.05), delta just below / above the closed-form threshold 16, a mix of adiabatic and
    Magnus cells in one point, and very unequal slopes (long follow stretches)."""
    cases = [([0.0], [1.0], [0.0]),
             ([0.0, 0.0], [1.0, 2.0], [0.0, 30.0]),
             ([1e-4], [5.0], [0.0]),
             ([1e-3, 2e-4], [10.0, 0.5], [0.0, 25.0]),
             ([math.sqrt(2 * 16 * V_W * 0.5) * 0.999], [0.5], [0.0]),      # delta = 15.97
             ([math.sqrt(2 * 16 * V_W * 0.5) * 1.001], [0.5], [0.0]),      # delta = 16.03 (closed form)
             ([0.3, 2.5, 0.05], [0.25, 0.5, 1.0], [0.0, 120.0, 400.0]),    # Magnus, adiabatic, Magnus
             ([0.1, 0.1], [0.01, 5.0], [0.0, 400.0])]
    for m, d, x in cases:
        got = gpu_engine.lz_propagate([m], [d], [x], V_W, 20.0, 64).cpu().numpy()[0]
        ref = propagate(m, d, x, V_W, 20.0, 64)
        assert abs(got - ref) <= 1e-11 * max(abs(ref), 1e-3), (m, d, x, got, ref)
        if max(m) == 0.0:
            assert abs(got) < 1e-15, got
