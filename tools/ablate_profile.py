#!/usr/bin/env python3
"""Time lzq_lz_propagate_profile of every library variant under <package>/_build/variants/ in
ONE process, interleaved rounds, on the synthetic bounce batch of tools/bench_profile.py
(bounce.synthetic_shapes / synthetic_couplings); reports whether each variant's P equals the
first variant's bit for bit (variants that change the arithmetic, e.g. polynomial degree, are
compared at 1e-12 instead).  One JSON line.

    python tools/build_variants.py LZQ_PROF_PAIR=0 LZQ_PROF_PAIR=1 ... && python tools/ablate_profile.py [n] [rounds]
"""
import glob
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    B = importlib.import_module(PKG + ".bounce")
    E = importlib.import_module(PKG + ".engine").Engine
    paths = sorted(glob.glob(os.path.join(ROOT, PKG, "_build", "variants", "*.so")))
    engs = {os.path.basename(p)[7:-3]: E(0, lib_path=p) for p in paths}
    if not engs:
        print(json.dumps({"note": "no variants under _build/variants (tools/build_variants.py)"}))
        return
    X, phi, Phi = B.synthetic_shapes()
    cols = B.synthetic_couplings(n, X.shape[0])
    e0 = next(iter(engs.values()))
    pts = e0.profile_points(*cols)
    shapes = {k: e.profile_shapes(X, phi, Phi) for k, e in engs.items()}
    best, P = {}, {}
    s = torch.cuda.current_stream()
    for _ in range(rounds):
        for k, e in engs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            P[k] = e.lz_propagate_profile(shapes[k], pts)
            b.record(s)
            torch.cuda.synchronize()
            t = a.elapsed_time(b) / 1e3
            best[k] = min(best.get(k, t), t)
    ref = next(iter(P))
    out = {"points": n, "rounds": rounds, "variants": {}}
    for k in engs:
        same = bool(torch.equal(P[k], P[ref]))
        diff = float((P[k] - P[ref]).abs().max())
        out["variants"][k] = {"seconds": best[k], "points_per_s": n / best[k], "bit_identical_to_first": same,
                              "max_abs_diff_vs_first": diff}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
