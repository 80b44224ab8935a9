#!/usr/bin/env python3
"""The workload of the ODE PMC passes (`tools/gpu.sh ode-pmc`): three 262,144-point batches of
the Radau fallback (fpy:385-417), each ONE integrator launch (ode_integrate_kernel<false, kLin, kNoSplit>, every variant) after a
64-point warm-up, in this order:

  narrow_wash      equal-mass config, Gamma_wash/H = 1, T in [0.6, 1.6] T_p (20000 steps/point);
                   points differ in P and flux: whole cooperative wavefronts
  stiff_thermal    sigma_v = 1e-9, thermal, m_chi = 300 GeV, T in [0.2, 1.3] T_p (25385 steps)
  riccati_mchi_sv  VERDICT r2 item 4: m_chi fastest over 4 values x 16 sigma_v values, narrow
                   window (Riccati Y_chi; Engine.ode groups the 4 stage keys)

One JSON line per case with the wall time of the dispatch batch; tools/summarize_ode_pmc.py
joins the PMC and kernel-trace passes with these lines."""
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

N = 262144
CASES = [("narrow_wash", {"Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}, 20000),
         ("stiff_thermal", {"sigma_v_chi_GeV_m2": 1e-9, "regime": "thermal", "m_chi_GeV": 300.0,
                            "T_max_over_Tp": 1.3, "T_min_over_Tp": 0.2}, 25385),
         ("riccati_mchi_sv", {"T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}, 20000)]


def case_points(cfgm, name, over, n=N):
    cfgs = cfgs_for(over, n)
    if name == "riccati_mchi_sv":
        for i, c in enumerate(cfgs):
            c["m_chi_GeV"] = (0.95, 3.0, 10.0, 30.0)[i % 4]
            c["sigma_v_chi_GeV_m2"] = 10.0 ** (-20 + ((i // 4) % 16) * 0.6)
    return (np.concatenate([cfgm.to_point(c) for c in cfgs]),
            np.concatenate([cfgm.to_ode_params(c) for c in cfgs]))


def main():
    cfgm = importlib.import_module(bench.PKG + ".config")
    eng = importlib.import_module(bench.PKG + ".engine").Engine(0)
    for name, over, steps in CASES:
        pts, ods = case_points(cfgm, name, over)
        eng.ode(pts[:64], ods[:64])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tab, st = eng.ode(pts, ods, chunk=N)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"config": name, "points": N, "steps_per_point": steps, "wall_s": dt,
                          "points_per_s": N / dt, "all_ok": bool((st == 0).all())}), flush=True)


if __name__ == "__main__":
    main()
