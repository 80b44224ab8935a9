"""Bounce-profile batches for the GPU profile path (include/lzq.h lzq_profile_*; PAPER p.3 §3,
eqs.(5)-(9); the reference's hook imports the absent `transport_from_profile` for this, fpy:173).

A batch is a set of profile SHAPES (the bounce's background fields phi(xi), Phi(xi) on knots)
and POINTS (a shape + the couplings y_B, y_chi, lambda_tr_eff and the wall speed v_w).  The
reference ships no bounce solution, so `synthetic_shapes` generates a reproducible family with
the structure of one: phi a kink wall, Phi a wall displaced from it with a bounce-shaped bump
(several Delta = 0 crossings for a range of couplings).  Its only use is as benchmark and test
input; users pass their own solver's samples.
"""
from __future__ import annotations

import numpy as np


def synthetic_shapes(n_shapes: int = 16, n_knots: int = 256, span: float = 12.0, seed: int = 6):
    """(knots, phi, Phi), each [n_shapes, n_knots]: xi in [-span, span] (wall width 1),
    phi = v/2 (1 - tanh(xi)), Phi = V/2 (1 + tanh(xi - s)) + A exp(-((xi - c)/b)^2) sin(k xi),
    with (v, V, s, A, c, b, k) drawn from numpy default_rng(seed)."""
    rng = np.random.default_rng(seed)
    x = np.linspace(-span, span, n_knots)
    X = np.broadcast_to(x, (n_shapes, n_knots)).copy()
    v = rng.uniform(0.8, 1.2, (n_shapes, 1))
    V = rng.uniform(0.8, 1.6, (n_shapes, 1))
    s = rng.uniform(-1.0, 1.0, (n_shapes, 1))
    A = rng.uniform(0.5, 1.5, (n_shapes, 1))
    c = rng.uniform(-2.0, 2.0, (n_shapes, 1))
    b = rng.uniform(1.0, 3.0, (n_shapes, 1))
    k = rng.uniform(1.0, 3.0, (n_shapes, 1))
    phi = 0.5 * v * (1.0 - np.tanh(X))
    Phi = 0.5 * V * (1.0 + np.tanh(X - s)) + A * np.exp(-((X - c) / b) ** 2) * np.sin(k * X)
    return X, phi, Phi


def synthetic_couplings(n_points: int, n_shapes: int, seed: int = 6):
    """Per-point (y_B, y_chi, lambda_tr_eff, v_w, shape), points grouped by shape (the launch order
    the kernel's per-block LDS staging of a shape wants): y_B, y_chi ~ U(0.5, 2),
    lambda_tr_eff log-uniform on [1e-3, 1], v_w ~ U(0.1, 0.9), numpy default_rng(seed + 1)."""
    rng = np.random.default_rng(seed + 1)
    yB = rng.uniform(0.5, 2.0, n_points)
    ychi = rng.uniform(0.5, 2.0, n_points)
    lam = 10.0 ** rng.uniform(-3.0, 0.0, n_points)
    vw = rng.uniform(0.1, 0.9, n_points)
    shape = (np.arange(n_points) * n_shapes) // n_points
    return yB, ychi, lam, vw, shape.astype(np.int32)


def interval_steps(knots, coef, yB, ychi, lam, vw, spr: float = 4.0, n_min: int = 1,
                   hdot_rate: float = 4.0, per_interval: bool = False) -> np.ndarray:
    """Magnus steps per point of lzq_lz_propagate_profile (its per-interval rule, vectorised over
    points; knots [n_knots], coef [n_knots - 1, 8] of ONE shape): the launch's work model.  The
    kernel's rule (tests/profile_ref.py interval_steps restates it exactly): rates at t = (q/4) L,
    q = 0..3, and at the interval's end from the next interval's cubic (the last: its own), E^2 and
    |dH/dt|^2 as quadratic forms in the shape's samples,
    W2 = max(max E^2, hdot_rate^2 v_w sqrt(max |dH/dt|^2)), S = ceil(spr L / v_w sqrt(W2)).  numpy
    has no fused multiply-add, so a count can differ from the kernel's where spr L / v_w sqrt(W2)
    lies within rounding of an integer (reporting only).  per_interval: the [point, interval]
    counts instead of their sum."""
    total = np.zeros(np.broadcast(yB, ychi, lam, vw).shape)
    cols = []
    ivw = 1.0 / np.asarray(vw, dtype=float)
    nI = len(knots) - 1
    A, B, C = yB * yB + lam * lam, (-2.0 * yB) * ychi, ychi * ychi   # the kernel's quadratic forms

    def rates(j, t):
        a = coef[j, 0] + t * (coef[j, 1] + t * (coef[j, 2] + t * coef[j, 3]))
        b = coef[j, 4] + t * (coef[j, 5] + t * (coef[j, 6] + t * coef[j, 7]))
        da = coef[j, 1] + t * (2.0 * coef[j, 2] + t * 3.0 * coef[j, 3])
        db = coef[j, 5] + t * (2.0 * coef[j, 6] + t * 3.0 * coef[j, 7])
        return A * (a * a) + B * (a * b) + C * (b * b), A * (da * da) + B * (da * db) + C * (db * db)

    for j in range(nI):
        L = knots[j + 1] - knots[j]
        e2, h2 = np.zeros_like(total), np.zeros_like(total)
        pts = [(j, (0.25 * q) * L) for q in range(4)] + [(j + 1, 0.0) if j + 1 < nI else (j, L)]
        for jj, t in pts:
            e, h = rates(jj, t)
            e2, h2 = np.maximum(e2, e), np.maximum(h2, h)
        W2 = np.maximum(e2, (hdot_rate * hdot_rate) * (vw * np.sqrt(h2)))
        Sj = np.maximum(n_min, np.ceil((spr * (L * ivw)) * np.sqrt(W2)))
        total += Sj
        if per_interval:
            cols.append(Sj)
    return np.stack(cols, axis=-1) if per_interval else total


def _plugin_reader():
    """plugins/transport_from_profile.py's CSV reader: the one parser of the profile format (the
    plug-in is torch-free and loads its GPU binding lazily, so importing it costs nothing)."""
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plugins",
                        "transport_from_profile.py")
    spec = importlib.util.spec_from_file_location("_lzq_transport_from_profile", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.read_csv


def read_bounce_csv(path: str):
    """The bounce-profile CSV of plugins/transport_from_profile.py (header `xi,phi,Phi`, or
    `r,phi,Phi` with `# R0 = ...`; `# key = value` option lines) -> (xi, phi, Phi, options),
    parsed by the plug-in's own reader."""
    header, rows, opts = _plugin_reader()(path)
    if len(rows) < 4:
        raise ValueError(f"{path}: a bounce profile needs a header and >= 4 rows")
    col = {h: i for i, h in enumerate(header)}
    low = {h.lower(): i for i, h in enumerate(header)}
    if not ("phi" in col and "Phi" in col and ("xi" in low or "r" in low)):
        raise ValueError(f"{path}: header must be 'xi,phi,Phi' or 'r,phi,Phi', got {header}")
    a = np.asarray(rows, dtype=np.float64)
    xi = a[:, low["xi"]] if "xi" in low else a[:, low["r"]] - float(opts.get("R0", 0.0))
    return xi, a[:, col["phi"]], a[:, col["Phi"]], opts
