#!/usr/bin/env python3
"""Time the LZ propagator (lz_propagate_kernel) of every library variant under
<package>/_build/variants/ in ONE process, interleaved rounds, on the C5 crossing arrays
(sweep.builtin_specs()["C5"]); reports whether every variant returns the same P bit for bit, and the largest |dP|."""
import glob
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sw = importlib.import_module(PKG + ".sweep")
    E = importlib.import_module(PKG + ".engine").Engine
    paths = sorted(glob.glob(os.path.join(ROOT, PKG, "_build", "variants", "*.so")))
    engs = {os.path.basename(p)[7:-3]: E(0, lib_path=p) for p in paths}
    spec = sw.builtin_specs()["C5"]
    start = (spec.total - n) // 2
    dev = next(iter(engs.values())).device
    m, dp, xi, v_w = spec.crossing_arrays(start, n, dev)
    args = (m, dp, xi, float(v_w[0]), spec.crossings.window_lz, spec.crossings.steps)
    ref, same, dmax = None, True, 0.0
    for e in engs.values():
        p = e.lz_propagate(*args)
        ref = p if ref is None else ref
        same = same and bool(torch.equal(p, ref))
        dmax = max(dmax, float((p - ref).abs().max()))
    res = {k: [] for k in engs}
    for _ in range(rounds):
        for k, e in engs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.lz_propagate(*args)
            torch.cuda.synchronize()
            res[k].append(time.perf_counter() - t0)
    print(json.dumps({"points": n, "bit_identical": same, "max_abs_dP": dmax, "seconds_min": {k: min(v) for k, v in res.items()}}, indent=1))


if __name__ == "__main__":
    main()
