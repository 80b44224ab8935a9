#!/usr/bin/env python3
"""Latency of one ODE point (the CLI's case, fpy:385-417 for a single config) through
Engine.ode: the 20000-step narrow window, and the shipped window (~1e6 steps) with wash-out
(sigma_v = 0: a linear wavefront of clones) and with annihilation (sigma_v = 1e-12: Riccati).
Best of 3 after a warm-up.

    python tools/time_ode_single.py
"""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from bench_ode import cfgs_for  # noqa: E402


def main():
    cfgm = importlib.import_module(bench.PKG + ".config")
    eng = importlib.import_module(bench.PKG + ".engine").Engine(0)
    cases = {"narrow_wash": {"Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6},
             "shipped_window_wash": {"Gamma_wash_over_H": 1.0},
             "shipped_window_riccati": {"Gamma_wash_over_H": 1.0, "sigma_v_chi_GeV_m2": 1e-12}}
    for name, over in cases.items():
        c = cfgs_for(over, 1)
        p, o = cfgm.to_point(c[0]), cfgm.to_ode_params(c[0])
        tab, st = eng.ode(p, o)
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tab, st = eng.ode(p, o)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"config": name, "seconds": min(ts), "status": int(st[0]),
                          "Y_B": float(tab[0, 0])}), flush=True)


if __name__ == "__main__":
    main()
