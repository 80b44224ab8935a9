#!/usr/bin/env python3
"""lzq_ode_tables with LZQ_TUNE_ODE_TABLE_WIDE 0 / 1 / 2 / 3 on seeded points: which variant's
tables differ from the narrow ones, and where (point, knot, slot)."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402


def main():
    from test_gpu_ode import recs, seeded_cfgs
    eng = importlib.import_module(bench.PKG + ".engine").Engine(0)
    cfgs = seeded_cfgs(7, seed=11)
    p, _ = recs(cfgs)
    for nt in (800, 65):
        tabs = {}
        for v in (0, 1, 2, 3):
            eng.tune_ode_table_wide(v)
            w, st = eng.ode_tables(p, nt=nt)
            tabs[v] = w.cpu().numpy().reshape(len(cfgs), nt, 4)
        for v in (1, 2, 3):
            d = np.argwhere(~((tabs[v] == tabs[0]) | (np.isnan(tabs[v]) & np.isnan(tabs[0]))))
            print(f"nt {nt} mask {v}: {len(d)} entries differ", d[:8].tolist(),
                  [(float(tabs[0][tuple(i)]), float(tabs[v][tuple(i)])) for i in d[:3]])
    eng.tune_ode_table_wide(3)


if __name__ == "__main__":
    main()
