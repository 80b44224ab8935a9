#!/usr/bin/env python3
"""Latency of one ODE point (the CLI's case, fpy:385-417 for a single config) through
Engine.ode: the 20000-step narrow window, and the shipped window (~1e6 steps) with wash-out
(sigma_v = 0: a linear wavefront of clones) and with annihilation (sigma_v = 1e-12: Riccati),
each integrated sequentially (time_parallel=False: one wavefront of clones steps the window)
and parallel in time (time_parallel=True: lzq_ode_integrate_tp, the Engine default for one
point).  Best of 3 after a warm-up; the two results' relative difference and the Newton updates.

    python tools/time_ode_single.py [--interval L ...]
"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from bench_ode import cfgs_for  # noqa: E402


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--interval", type=int, nargs="*", default=[],
                    help="LZQ_TUNE_ODE_TP_INTERVAL values to time as well (default: the library's 64)")
    ap.add_argument("--lib", default=None, help="a liblzq.so variant to time instead of the in-tree build")
    a = ap.parse_args()
    cfgm = importlib.import_module(bench.PKG + ".config")
    nat = importlib.import_module(bench.PKG + "._native")
    eng = importlib.import_module(bench.PKG + ".engine").Engine(0, **({"lib_path": a.lib} if a.lib else {}))
    cases = {"narrow_wash": {"Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6},
             "narrow_riccati": {"Gamma_wash_over_H": 1.0, "sigma_v_chi_GeV_m2": 1e-12, "T_max_over_Tp": 1.6,
                                "T_min_over_Tp": 0.6},
             "shipped_window_wash": {"Gamma_wash_over_H": 1.0},
             "shipped_window_riccati": {"Gamma_wash_over_H": 1.0, "sigma_v_chi_GeV_m2": 1e-12},
             "shipped_window_riccati_strong": {"sigma_v_chi_GeV_m2": 1e-9}}

    def timed(p, o, tp):
        tab, st = eng.ode(p, o, time_parallel=tp)
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tab, st = eng.ode(p, o, time_parallel=tp)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        it = int(eng.last_ode_tp_iters[0]) if tp else 0
        return min(ts), tab.cpu().numpy()[0], int(st[0]), it

    for L in [None] + a.interval:
        prev = eng.lib.lzq_tune(nat.TUNE_ODE_TP_INTERVAL, L) if L else None
        for name, over in cases.items():
            c = cfgs_for(over, 1)
            p, o = cfgm.to_point(c[0]), cfgm.to_ode_params(c[0])
            t_seq, r_seq, s_seq, _ = timed(p, o, False) if L is None else (None, None, None, None)
            t_tp, r_tp, s_tp, it = timed(p, o, True)
            rec = {"config": name, "interval": L or 64, "seconds_tp": t_tp, "newton_updates": it, "status_tp": s_tp,
                   "Y_B": float(r_tp[0]), "Y_chi": float(r_tp[1])}
            if r_seq is not None:
                rec.update(seconds_sequential=t_seq, status_sequential=s_seq, speedup=t_seq / t_tp,
                           rel_diff_Y_B=rel(float(r_tp[0]), float(r_seq[0])),
                           rel_diff_Y_chi=rel(float(r_tp[1]), float(r_seq[1])))
            print(json.dumps(rec), flush=True)
        if L:
            eng.lib.lzq_tune(nat.TUNE_ODE_TP_INTERVAL, prev)


if __name__ == "__main__":
    main()
