#!/usr/bin/env python3
"""Time every library variant under <package>/_build/variants/ in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24), on the bench workload (C2 grid)."""
import glob
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reuse = len(sys.argv) > 3 and sys.argv[3] == "reuse"   # time lzq_sweep_grid_reuse instead of the dense sweep
    E = importlib.import_module(bench.PKG + ".engine").Engine
    paths = sorted(glob.glob(os.path.join(ROOT, bench.PKG, "_build", "variants", "*.so")))
    engs = {os.path.basename(p)[7:-3]: E(0, lib_path=p) for p in paths}
    axes = bench.grid_axes(1)
    ref = None
    res = {k: [] for k in engs}
    for k, e in engs.items():  # warm-up + cross-variant agreement
        t = e.sweep(bench.BASE, axes, 0, n, reuse=reuse).cpu().numpy()
        if ref is None:
            ref = t
        nz = ref != 0
        assert np.max(np.abs(t[nz] - ref[nz]) / np.abs(ref[nz])) < 1e-13, k
    for _ in range(rounds):
        for k, e in engs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.sweep(bench.BASE, axes, 0, n, reuse=reuse)
            torch.cuda.synchronize()
            res[k].append(n / (time.perf_counter() - t0))
    out = {k: round(float(np.median(v))) for k, v in sorted(res.items(), key=lambda kv: -np.median(kv[1]))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
