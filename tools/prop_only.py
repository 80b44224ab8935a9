#!/usr/bin/env python3
"""Run lz_propagate_kernel alone on a C5 slice (for rocprofv3 PMC / kernel-trace passes):
    python tools/prop_only.py [n_points] [n_cross] [repeats] [library path (default: the in-tree build)]"""
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
    import dataclasses
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
    nc = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    sw = importlib.import_module(PKG + ".sweep")
    lib = sys.argv[4] if len(sys.argv) > 4 else None
    eng = importlib.import_module(PKG + ".engine").Engine(0, lib_path=lib)
    spec = sw.builtin_specs()["C5"]
    spec = dataclasses.replace(spec, crossings=dataclasses.replace(spec.crossings, n_cross=nc))
    start = (spec.total - n) // 2
    m, dp, xi, v_w = spec.crossing_arrays(start, n, eng.device)
    args = (m, dp, xi, float(v_w[0]), spec.crossings.window_lz, spec.crossings.steps)
    eng.lz_propagate(*args)
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        P = eng.lz_propagate(*args)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    print(json.dumps({"points": n, "n_cross": nc, "seconds_min": min(times), "points_per_s": n / min(times),
                      "finite": bool(torch.isfinite(P).all())}))


if __name__ == "__main__":
    main()
