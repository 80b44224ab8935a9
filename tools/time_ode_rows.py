#!/usr/bin/env python3
"""Engine.ode on the tools/ode_pmc_run.py cases with and without the shared step-row tables
(Engine.ode_rows; lzq_ode_rows + lzq_ode_integrate_rows), from host records and from
device-resident ones (Engine.ode on points_to_device / ode_params_to_device tensors), best of 5
wall times each, bit equality of all, and a cProfile of one resident call (its host time).

    python tools/time_ode_rows.py [--cases narrow_wash,...] [--points N] [--out FILE]
"""
import argparse
import cProfile
import importlib
import io
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="narrow_wash")
    ap.add_argument("--points", type=int, default=262144)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--only", default=None, help="one mode: rows, no_rows, rows_resident, no_rows_resident "
                    "(for a kernel trace of that mode alone)")
    a = ap.parse_args()
    from ode_pmc_run import CASES, case_points
    cfgm = importlib.import_module(PKG + ".config")
    eng = importlib.import_module(PKG + ".engine").Engine(0)
    recs = []
    for name in a.cases.split(","):
        case = {c[0]: c for c in CASES}[name]
        pts, ods = case_points(cfgm, case[0], case[1], a.points)
        d_in = (eng.points_to_device(pts), eng.ode_params_to_device(ods))
        res, outs = {}, {}
        for key in (("rows", True, False), ("no_rows", False, False), ("rows", True, True),
                    ("no_rows", False, True), ("rows", True, False)):
            tag, rows, resident = key[0] + ("_resident" if key[2] else ""), key[1], key[2]
            if a.only and tag != a.only:
                continue
            eng.ode_rows = rows
            args = d_in if resident else (pts, ods)
            eng.ode(*args)   # warm-up
            best = None
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                tab, st = eng.ode(*args)
                torch.cuda.synchronize()
                d = time.perf_counter() - t0
                best = d if best is None else min(best, d)
            res[tag] = min(best, res.get(tag, best))
            outs[tag] = (tab.clone(), st.clone(), dict(eng.last_ode_tables))
        ref = next(iter(outs.values()))
        same = all(bool(torch.equal(o[0].view(torch.int64), ref[0].view(torch.int64)) and torch.equal(o[1], ref[1]))
                   for o in outs.values())
        rec = {"case": name, "points": a.points, "bit_identical": same,
               "row_runs": max(o[2].get("row_runs", 0) for o in outs.values()), "all_ok": bool((ref[1] == 0).all())}
        for tag, t in res.items():
            rec[tag + "_s"] = t
            rec[tag + "_points_per_s"] = a.points / t
        if "rows_resident" in res and "no_rows_resident" in res:
            rec["rows_speedup_resident"] = res["no_rows_resident"] / res["rows_resident"]
        if a.profile:
            eng.ode_rows = True
            pr = cProfile.Profile()
            torch.cuda.synchronize()
            pr.enable()
            eng.ode(*d_in)
            torch.cuda.synchronize()
            pr.disable()
            s = io.StringIO()
            pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(14)
            rec["host_profile"] = s.getvalue().splitlines()[:40]
        print(json.dumps({k: v for k, v in rec.items() if k != "host_profile"}), flush=True)
        if a.profile:
            print("\n".join(rec["host_profile"]), flush=True)
        recs.append(rec)
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
