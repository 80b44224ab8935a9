#!/usr/bin/env python3
"""Golden vectors for the LZ propagator (csrc/lzq_propagator.hip): the EXACT finite-window
conversion probability of the piecewise-linear model, cell by cell in Weber functions
(tests/weber_ref.py, mpmath at 40 digits), for the kernel's own windows, start state and
projection.  The reference has no propagator; these fixtures pin the
model's solution, independently of any time stepping.

    python tests/golden/make_golden_weber.py     # writes tests/golden/golden_weber.json

Cases:
  single  - one crossing, (m_mix, |Delta'|) on a 6 x 6 log grid of the C2 ranges, K = 20;
  multi   - the 2- and 3-crossing cases of tests/test_gpu_propagator.py (K = 12) and the
            adiabatic-cell case of tests/test_propagator_math.py (K = 20);
  c5      - sweep.CrossingSpec's defaults (8 crossings 40 LZ lengths apart, jitter 0.1,
            numpy default_rng(5), K = 20) at 8 (m_mix, |Delta'|) grid points, plus N = 16, 32;
  wide    - crossings hundreds of LZ lengths apart (K = 20): cells far wider than the kernel's
            Magnus cores, so most of each cell is crossed by dressed following (round 2).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from weber_ref import propagate_exact  # noqa: E402

V_W = 0.3


def c5_case(m0, d0, n_cross=8, spacing=40.0, jitter=0.1, seed=5):
    """sweep.CrossingSpec.crossing_arrays for one grid point (same formulas, in numpy)."""
    a, b, dd = np.random.default_rng(seed).uniform(-1.0, 1.0, (3, n_cross))
    delta0 = m0 * m0 / (2.0 * V_W * d0)
    L = np.sqrt(V_W / d0) * max(np.sqrt(delta0), 1.0)
    m = m0 * (1.0 + jitter * a)
    d = d0 * (1.0 + jitter * b)
    x = L * (spacing * np.arange(n_cross) + jitter * dd)
    return [float(v) for v in m], [float(v) for v in d], [float(v) for v in x]


def main():
    out = {"v_w": V_W, "dps": 40, "generator": "tests/golden/make_golden_weber.py", "cases": []}

    def add(kind, m, d, x, K):
        P = propagate_exact(m, d, x, V_W, K)
        out["cases"].append({"kind": kind, "m": m, "d": d, "x": x, "K": K, "P": P})

    for m in np.logspace(-3, 0, 6):
        for d in np.logspace(-3, 1, 6):
            add("single", [float(m)], [float(d)], [0.0], 20.0)
    for m, d, x in [([0.1], [1.0], [0.0]),
                    ([0.05, 0.08, 0.2], [1.0, 0.5, 2.0], [0.0, 3.0, 7.5]),
                    ([0.3, 0.01], [0.2, 0.05], [-1.0, 20.0])]:
        add("multi", m, d, x, 12.0)
    add("multi", [0.3, 1.2], [0.25, 0.1], [0.0, 200.0], 20.0)
    for m0, d0 in [(0.001, 0.001), (0.01, 0.01), (0.05, 0.1), (0.1, 1.0), (0.3, 0.05), (1.0, 10.0),
                   (0.2, 0.01), (1.0, 0.001)]:
        add("c5", *c5_case(m0, d0), 20.0)
    for n in (16, 32):
        add("c5", *c5_case(0.05, 0.1, n_cross=n), 20.0)
    for m, d, x in [([0.1, 0.12], [1.0, 0.8], [0.0, 400.0]),                  # delta 0.017, 0.03
                    ([0.6, 0.5, 0.7], [0.2, 0.25, 0.3], [0.0, 150.0, 260.0]),  # delta 3, 1.7, 2.7
                    ([1.0, 0.9], [0.1, 0.12], [0.0, 300.0])]:                  # delta 16.7 (adiabatic), 11.25
        add("wide", m, d, x, 20.0)
    with open(os.path.join(HERE, "golden_weber.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
