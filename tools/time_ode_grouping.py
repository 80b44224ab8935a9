#!/usr/bin/env python3
"""Repeated timings of Engine.ode on the narrow wash-out case: all points in one stage group,
and m_chi cycling over 4 values (grouped by Engine.ode or left in input order).  With a
-DLZQ_ODE_COOP_DEBUG variant under _build/variants it also reports how many points ran in
cooperative wavefronts.
    python tools/time_ode_grouping.py [n]"""
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
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from bench_ode import cfgs_for  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    cfgm = importlib.import_module(bench.PKG + ".config")
    E = importlib.import_module(bench.PKG + ".engine").Engine
    eng = E(0)
    base = cfgs_for({"Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}, n)
    mixed = [dict(c, m_chi_GeV=(0.95, 3.0, 10.0, 30.0)[i % 4]) for i, c in enumerate(base)]
    out = {}
    for name, cfgs in (("one_group", base), ("mchi_fastest", mixed)):
        pts = np.concatenate([cfgm.to_point(c) for c in cfgs])
        ods = np.concatenate([cfgm.to_ode_params(c) for c in cfgs])
        for g in (True, False):
            ts = []
            for _ in range(4):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.ode(pts, ods, group_waves=g)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            out[f"{name}_group{int(g)}"] = [round(n / t) for t in ts]
        dbg = sorted(glob.glob(os.path.join(ROOT, bench.PKG, "_build", "variants", "*coop_debug*.so")))
        if dbg:
            e2 = E(0, lib_path=dbg[0])
            for g in (True, False):
                t, _ = e2.ode(pts, ods, group_waves=g)
                out[f"{name}_group{int(g)}_coop_points"] = int((t[:, 5] == 1.0).sum())
    # one point alone (the CLI's case): a wavefront of 1 real lane + 63 clones
    for name, over in (("single_narrow", {"Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}),
                       ("single_full_window", {"Gamma_wash_over_H": 1.0})):
        c = cfgs_for(over, 1)
        pts, ods = cfgm.to_point(c[0]), cfgm.to_ode_params(c[0])
        for coop in (True, False):
            eng.tune_ode_coop(coop)
            eng.ode(pts, ods)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.ode(pts, ods)
            torch.cuda.synchronize()
            out[f"{name}_coop{int(coop)}_seconds"] = round(time.perf_counter() - t0, 4)
        eng.tune_ode_coop(True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
