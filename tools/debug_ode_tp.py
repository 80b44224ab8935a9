#!/usr/bin/env python3
"""Per-iteration trace of lzq_ode_integrate_tp on the reference's ODE cases (tests/golden/
golden_ode.json), one point each: a library built with -DLZQ_ODE_TP_DEBUG prints every Newton
update's largest relative correction.

    python tools/debug_ode_tp.py [--build] [--cases 0 1 2]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402

DBG = os.path.join(ROOT, bench.PKG, "_build", "debug", "liblzq_tpdebug.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true", help="build the debug library (CPU side)")
    ap.add_argument("--cases", type=int, nargs="*", default=None)
    ap.add_argument("--over", type=str, default=None,
                    help="JSON overrides of the shipped config to trace instead of the golden cases")
    a = ap.parse_args()
    if a.build:
        importlib.import_module(bench.PKG + ".build").build(defines={"LZQ_ODE_TP_DEBUG": 1}, out=DBG)
        return
    import torch
    cfgm = importlib.import_module(bench.PKG + ".config")
    from conftest import full_cfg
    eng = importlib.import_module(bench.PKG + ".engine").Engine(0, lib_path=DBG)
    pts = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_ode.json")))["points"]
    if a.over is not None:
        from conftest import BASE_CFG
        pts = [{"config": {**BASE_CFG, **json.loads(a.over)}}]
    for i, r in enumerate(pts):
        if a.cases is not None and i not in a.cases:
            continue
        cfg = full_cfg(r["config"])
        p, o = cfgm.to_point(cfg), cfgm.to_ode_params(cfg)
        x, sx = eng.ode(p, o, time_parallel=False)
        print(f"--- case {i}: {json.dumps(r['config'])}", flush=True)
        y, sy = eng.ode(p, o, time_parallel=True)
        torch.cuda.synchronize()
        it = int(eng.last_ode_tp_iters[0])
        xa, ya = x.cpu().numpy()[0], y.cpu().numpy()[0]
        d = [abs(u - v) / max(abs(v), 1e-300) for u, v in zip(ya[:2], xa[:2])]
        print(f"case {i}: status {int(sx[0])}/{int(sy[0])} updates {it} rel diff Y_B {d[0]:.2e} Y_chi {d[1]:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
