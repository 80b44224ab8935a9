#!/usr/bin/env python3
"""Throughput of the bounce-profile path on one MI355X (include/lzq.h lzq_profile_*):
a batch of synthetic bounce profiles (bounce.synthetic_shapes: 16 shapes x 256 knots) and 1e5
coupling points (bounce.synthetic_couplings), timed with HIP events on the launch stream:

  splines     lzq_profile_splines   (the 32 not-a-knot splines, once per batch)
  crossings   lzq_profile_crossings (eqs.(5)-(8) per point)
  minimal     crossings + lzq_p_closed_form of a one-crossing point (eq.(9))
  propagate   lzq_lz_propagate_profile (sixth-order Magnus through the whole profile)

    python tools/bench_profile.py [n_points] [repeats] [--json out.json]
One JSON line: points/s per stage, Magnus steps per point (the kernel's own rule, host
restatement bounce.interval_steps), crossings per point, and P statistics.
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def timed(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        out = fn()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    return min(ts), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="?", default=100_000)
    ap.add_argument("reps", type=int, nargs="?", default=3)
    ap.add_argument("--shapes", type=int, default=16)
    ap.add_argument("--knots", type=int, default=256)
    ap.add_argument("--spr", type=float, default=4.0)
    ap.add_argument("--min-steps", type=int, default=1)
    ap.add_argument("--only", default=None, help="propagate | crossings: time that stage alone (profiling)")
    ap.add_argument("--sort-vw", action="store_true", help="launch the points ordered by (shape, v_w): the "
                    "cost-ordered launch's upper bound (a lane's step count scales as 1/v_w)")
    ap.add_argument("--ab", action="store_true", help="also time the flattened propagation (same process)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    B = importlib.import_module(PKG + ".bounce")
    eng = importlib.import_module(PKG + ".engine").Engine(0)
    X, phi, Phi = B.synthetic_shapes(a.shapes, a.knots)
    yB, ychi, lam, vw, shape = B.synthetic_couplings(a.n, a.shapes)
    if a.sort_vw:
        o = np.lexsort((vw, shape))
        yB, ychi, lam, vw, shape = yB[o], ychi[o], lam[o], vw[o], shape[o]
    pts = eng.profile_points(yB, ychi, lam, vw, shape)
    rec = {"points": a.n, "shapes": a.shapes, "knots": a.knots, "steps_per_radian": a.spr, "min_steps": a.min_steps,
           "order": "shape, v_w" if a.sort_vw else "shape, random"}
    sh = eng.profile_shapes(X, phi, Phi)
    if a.only in (None, "propagate"):
        t_p, P = timed(lambda: eng.lz_propagate_profile(sh, pts, a.spr, a.min_steps), a.reps)
        P = P.cpu().numpy()
        rec["propagate"] = {"seconds": t_p, "points_per_s": a.n / t_p, "finite": bool(np.isfinite(P).all()),
                            "P_mean": float(P.mean()), "P_min": float(P.min()), "P_max": float(P.max())}
        if a.ab:   # the flattened propagation in the same process (LZQ_TUNE_PROFILE_FLAT = 1)
            prev = eng.tune_profile_flat(True)
            try:
                t_i, Pi = timed(lambda: eng.lz_propagate_profile(sh, pts, a.spr, a.min_steps), a.reps)
            finally:
                eng.tune_profile_flat(prev)
            rec["propagate"]["flat"] = {"seconds": t_i, "points_per_s": a.n / t_i,
                                                 "bit_identical": bool(np.array_equal(Pi.cpu().numpy(), P,
                                                                                      equal_nan=True))}
    if a.only in (None, "crossings"):
        t_c, cr = timed(lambda: eng.profile_crossings(sh, pts, 8), a.reps)
        cnt = cr["count"].cpu().numpy()
        rec["crossings"] = {"seconds": t_c, "points_per_s": a.n / t_c,
                            "per_point": {str(k): int((cnt == k).sum()) for k in np.unique(cnt)}}
    if a.only is None:
        t_s, _ = timed(lambda: eng.profile_shapes(X, phi, Phi), a.reps)
        rec["splines"] = {"seconds": t_s, "shapes_per_s": a.shapes / t_s}
        one = cnt == 1
        t_m, _ = timed(lambda: eng.p_closed_form(cr["delta_lz"][torch.as_tensor(one, device=eng.device), 0]), a.reps)
        rec["minimal"] = {"seconds": t_c + t_m, "points_per_s": a.n / (t_c + t_m),
                          "note": "crossings + eq.(9) of the one-crossing points"}
        coef = sh.coef.cpu().numpy()
        steps = np.concatenate([B.interval_steps(X[s], coef[s], yB[shape == s], ychi[shape == s], lam[shape == s],
                                                 vw[shape == s], a.spr, a.min_steps) for s in range(a.shapes)])
        rec["magnus_steps_per_point"] = {"mean": float(steps.mean()), "min": float(steps.min()),
                                         "max": float(steps.max()), "total": float(steps.sum())}
        if "propagate" in rec:
            rec["propagate"]["steps_per_s"] = float(steps.sum()) / rec["propagate"]["seconds"]
    line = json.dumps(rec)
    print(line)
    if a.json:
        with open(a.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
