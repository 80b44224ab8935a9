#!/usr/bin/env python3
"""The headline step (bench.py's C2 sweep of 1e6 dense points) for several liblzq.so builds in ONE
process, interleaved rounds, best of N: tells a box's speed from a library's (box-to-box spread on
the same machine code is ~15%, DESIGN.md's numbers table).  Each library's table is compared bit
for bit with the first one's.

    python tools/headline_ab.py LIB [LIB ...] [--rounds 3]
"""
import argparse
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--points", type=int, default=1_000_000)
    a = ap.parse_args()
    E = importlib.import_module(bench.PKG + ".engine").Engine
    engs = {os.path.basename(p): E(0, lib_path=p) for p in a.libs}
    axes = bench.grid_axes(1)
    outs = {k: torch.empty((a.points, 6), dtype=torch.float64, device=e.device) for k, e in engs.items()}
    best = {}
    for k, e in engs.items():  # warm-up
        e.sweep(bench.BASE, axes, 0, a.points, out=outs[k])
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k, e in engs.items():
            s = torch.cuda.current_stream()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record(s)
            e.sweep(bench.BASE, axes, 0, a.points, out=outs[k])
            t1.record(s)
            torch.cuda.synchronize()
            ms = t0.elapsed_time(t1)
            best[k] = min(best.get(k, ms), ms)
    first = next(iter(outs))
    print(json.dumps({"points": a.points, "rounds": a.rounds,
                      "ms_per_step": best, "points_per_s": {k: a.points / (v / 1e3) for k, v in best.items()},
                      "bit_identical_to_first": {k: bool(torch.equal(v, outs[first])) for k, v in outs.items()}}))


if __name__ == "__main__":
    main()
