#!/usr/bin/env python3
"""Throughput of every BASELINE.json sweep config on one GPU, one JSON line each: the quadrature
sweeps C2-C4 (subsets of the C3/C4 grids; points/s is per-point work, uniform within a config),
C5 with 8/16/32 sequential crossings (propagator + quadrature), P1 (bounce profile -> P ->
quadrature), and the ODE fallback sweeps of tools/ode_pmc_run.py (narrow wash-out, stiff thermal,
the Riccati m_chi x sigma_v sweep: tables + integrator, fpy:385-417).  The dense path (the
headline's) is timed; the quadrature configs also carry the z-sum reuse mode
(lzq_sweep_grid_reuse) and its bit-identity to the dense table as a secondary field.

    python tools/bench_configs.py [--points N] [--only C2,P1,...] [--pmc]

--pmc: the workload of a rocprofv3 --pmc pass (tools/gpu.sh configs): no warm-up and no secondary
legs, so the counters of the run are exactly the timed config's (tools/summarize_configs.py divides
them by the points and joins them with the timed lines into executed-FP64 fractions)."""
import argparse
import dataclasses
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
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"

SWEEPS = ("C2", "C3", "C4", "C5", "C5_N16", "C5_N32", "P1")
ODE = ("O_narrow_wash", "O_stiff_thermal", "O_riccati_mchi_sv")
ALL = SWEEPS + ODE


def sweep_specs(sw):
    specs = sw.builtin_specs()
    for nc in (16, 32):   # BASELINE C5: N >= 8 crossings per point; also 16 and 32
        c5 = specs["C5"]
        specs[f"C5_N{nc}"] = dataclasses.replace(c5, name=f"C5_N{nc}",
                                                 crossings=dataclasses.replace(c5.crossings, n_cross=nc))
    return specs


def sync():
    torch.cuda.synchronize()


def run_sweep(name, spec, sw, eng, n, pmc):
    cnt = min(n, spec.total)
    start = (spec.total - cnt) // 2
    comp = sw.make_compute(spec, eng)
    out = torch.empty((cnt, 6), dtype=torch.float64, device=eng.device)
    if not pmc:
        comp(start, cnt, out)  # warm-up at full size
    sync()
    t0 = time.perf_counter()
    comp(start, cnt, out)
    sync()
    dt = time.perf_counter() - t0
    rec = {"config": name, "points": cnt, "start": start, "points_per_s": cnt / dt, "seconds": dt,
           "finite": bool(torch.isfinite(out).all()), "notes": spec.notes}
    if pmc:
        return rec
    if spec.crossings is not None:
        m, dp, xi, v_w = spec.crossing_arrays(start, cnt, eng.device)
        sync()
        t0 = time.perf_counter()
        eng.lz_propagate(m, dp, xi, float(v_w[0]), spec.crossings.window_lz, spec.crossings.steps)
        sync()
        rec["propagator_seconds"] = time.perf_counter() - t0
        rec["crossings"] = spec.crossings.__dict__
    if spec.profile is None:
        # secondary (not the headline): z-sums shared per y-grid / A/V kernel, bit-identical
        comp_r = sw.make_compute(spec, eng, reuse=True)
        out_r = torch.empty_like(out)
        comp_r(start, min(cnt, 4096), out_r[:min(cnt, 4096)])
        sync()
        t0 = time.perf_counter()
        comp_r(start, cnt, out_r)
        sync()
        dtr = time.perf_counter() - t0
        rec["reuse_zsums"] = {"points_per_s": cnt / dtr, "bit_identical": bool(torch.equal(out, out_r))}
    return rec


def run_ode(name, eng, n, pmc):
    """An ODE case timed from device-resident records (Engine.ode on points_to_device /
    ode_params_to_device tensors: the headline's convention, inputs in HBM before the clock) and,
    beside it, from host records (their ~42 MB per 2.6e5 points of H2D copies inside the clock)."""
    from ode_pmc_run import CASES, case_points
    cfgm = importlib.import_module(PKG + ".config")
    case = {c[0]: c for c in CASES}[name[2:]]
    pts, ods = case_points(cfgm, case[0], case[1], n)
    d_in = (eng.points_to_device(pts), eng.ode_params_to_device(ods))
    reps = 1 if pmc else 3
    best = {}
    for tag, args in (("resident", d_in), ("host", (pts, ods))):
        if not pmc:
            eng.ode(*args, chunk=1 << 18)   # warm-up at full size (workspaces, the launch-order kernels)
        elif tag == "host":
            break
        for _ in range(reps):  # best of 3 (tools/ablate_ode.py's figure of merit)
            sync()
            t0 = time.perf_counter()
            tab, st = eng.ode(*args, chunk=1 << 18)
            sync()
            d = time.perf_counter() - t0
            best[tag] = d if tag not in best else min(best[tag], d)
    dt = best["resident"]
    rec = {"config": name, "points": n, "points_per_s": n / dt, "seconds": dt, "steps_per_point": case[2],
           "all_ok": bool((st == 0).all()), "finite": bool(torch.isfinite(tab).all()),
           "notes": f"ODE fallback (fpy:385-417), tools/ode_pmc_run.py case {case[0]}: spline tables + Radau "
                    f"integrator, {case[2]} fixed steps per point; records resident on the device"}
    if "host" in best:
        rec["host_records"] = {"points_per_s": n / best["host"], "seconds": best["host"]}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=400_000, help="points per quadrature / propagator config")
    ap.add_argument("--ode-points", type=int, default=262_144, help="points per ODE config")
    ap.add_argument("--only", default=",".join(ALL))
    ap.add_argument("--pmc", action="store_true")
    a = ap.parse_args()
    sw = importlib.import_module(PKG + ".sweep")
    eng = importlib.import_module(PKG + ".engine").Engine(0)
    specs = sweep_specs(sw)
    for name in a.only.split(","):
        if name in SWEEPS:
            rec = run_sweep(name, specs[name], sw, eng, a.points, a.pmc)
        elif name in ODE:
            rec = run_ode(name, eng, a.ode_points, a.pmc)
        else:
            raise SystemExit(f"unknown config {name}")
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
