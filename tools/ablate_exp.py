#!/usr/bin/env python3
"""A/B of the inner-loop exponential variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Prints per-variant points/s (median, min) and the
max relative difference of the yield tables between variants."""
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

PKG = bench.PKG


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    eng = importlib.import_module(PKG + ".engine").Engine(0)
    axes = bench.grid_axes(1)
    res = {"poly11": [], "table": []}
    tabs = {}
    for v in res:
        eng.tune_exp(v)
        tabs[v] = eng.sweep(bench.BASE, axes, 0, n).clone()  # warm-up + table
    torch.cuda.synchronize()
    for _ in range(rounds):
        for v in res:
            eng.tune_exp(v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.sweep(bench.BASE, axes, 0, n)
            torch.cuda.synchronize()
            res[v].append(n / (time.perf_counter() - t0))
    a, b = tabs["poly11"].cpu().numpy(), tabs["table"].cpu().numpy()
    nz = a != 0
    out = {v: {"median": float(np.median(r)), "min": float(np.min(r))} for v, r in res.items()}
    out["max_rel_diff"] = float(np.max(np.abs(a[nz] - b[nz]) / np.abs(a[nz])))
    out["speedup_table_vs_poly"] = out["table"]["median"] / out["poly11"]["median"]
    eng.tune_exp("table")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
