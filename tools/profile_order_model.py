#!/usr/bin/env python3
"""How much of lzq_lz_propagate_profile's interval-loop kernel is idle lanes, per launch order
(host model, no GPU).  The kernel steps a wavefront through knot interval j for the largest step
count S_j of its 64 lanes, so a launch order costs sum over waves and intervals of max_lane S_j
Magnus steps against the useful sum S_j.  The step counts come from the host work model
(bounce.interval_steps, per interval), on tools/bench_profile.py's synthetic workload; the
candidate orders are the kernel's cost bins (4 per octave of the total) and finer keys.

    python tools/profile_order_model.py [n_points] [--json out.json]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def wave_cost(S, order):
    """sum over waves of sum_j max over the wave's lanes of S_j (padded to whole waves)."""
    Sp = S[order]
    n = Sp.shape[0]
    pad = (-n) % 64
    if pad:
        Sp = np.concatenate([Sp, np.zeros((pad, Sp.shape[1]))])
    return 64.0 * float(Sp.reshape(-1, 64, Sp.shape[1]).max(axis=1).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="?", default=131072)
    ap.add_argument("--shapes", type=int, default=16)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    B = importlib.import_module(PKG + ".bounce")
    X, phi, Phi = B.synthetic_shapes(a.shapes, 256)
    yB, ychi, lam, vw, shape = B.synthetic_couplings(a.n, a.shapes)
    from scipy.interpolate import CubicSpline
    S = np.zeros((a.n, X.shape[1] - 1))
    for s in range(a.shapes):
        sel = shape == s
        cp = CubicSpline(X[s], phi[s]).c[::-1].T
        cP = CubicSpline(X[s], Phi[s]).c[::-1].T
        coef = np.concatenate([cp, cP], axis=1)
        S[sel] = B.interval_steps(X[s], coef, yB[sel], ychi[sel], lam[sel], vw[sel], per_interval=True)
    tot = S.sum(axis=1)
    useful = float(S.sum())
    idx = np.arange(a.n)
    cost_bin = np.floor(4.0 * np.log2(1.0 + tot))                    # the kernel's bins (4 per octave)
    peak = S.argmax(axis=1)                                           # the interval with the most steps
    ratio = np.arctan2(ychi, yB)                                      # where Delta = 0 sits
    orders = {
        "input (shape, random)": idx,
        "cost bins (kernel)": np.lexsort((idx, -cost_bin)),
        "cost bins 16/octave": np.lexsort((idx, -np.floor(16.0 * np.log2(1.0 + tot)))),
        "shape, cost bins": np.lexsort((idx, -cost_bin, shape)),
        "cost bins, peak interval": np.lexsort((peak, -cost_bin)),
        "cost bins, y_chi/y_B angle": np.lexsort((ratio, -cost_bin)),
        "shape, cost bins, angle": np.lexsort((ratio, -cost_bin, shape)),
        "shape, angle bins(32), cost": np.lexsort((-tot, np.floor(ratio * 32 / (np.pi / 2)), shape)),
        "shape, v_w bins(16), angle": np.lexsort((ratio, np.floor(vw * 16), shape)),
        "shape, cost 2/oct, angle": np.lexsort((ratio, -np.floor(2.0 * np.log2(1.0 + tot)), shape)),
        "shape, cost 1/oct, angle": np.lexsort((ratio, -np.floor(np.log2(1.0 + tot)), shape)),
        "shape, cost 8/oct, angle": np.lexsort((ratio, -np.floor(8.0 * np.log2(1.0 + tot)), shape)),
        "shape, cost bins, lambda": np.lexsort((lam, -cost_bin, shape)),
        "shape, cost bins, angle bins(8), lambda": np.lexsort((lam, np.floor(ratio * 8 / (np.pi / 2)), -cost_bin, shape)),
    }
    res = {}
    for name, o in orders.items():
        c = wave_cost(S, o)
        res[name] = {"idle_factor": c / useful}
        print(f"{name:34s} wave steps / useful = {c / useful:.3f}")
    rec = {"points": a.n, "shapes": a.shapes, "useful_steps_per_point": useful / a.n, "orders": res}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
