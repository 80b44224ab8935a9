#!/usr/bin/env python3
"""Throughput of the BASELINE.json sweep configs C2-C5 on one GPU (subsets of C3/C4 grids;
points/s is per-point work, which is uniform within a config).  One JSON line per config, with
the dense path (the headline's) and, as a secondary field, the z-sum reuse mode
(lzq_sweep_grid_reuse) and its bit-identity to the dense table."""
import importlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
    sw = importlib.import_module(PKG + ".sweep")
    eng = importlib.import_module(PKG + ".engine").Engine(0)
    import dataclasses
    specs = sw.builtin_specs()
    for nc in (16, 32):   # BASELINE C5: N >= 8 crossings per point; also 16 and 32
        c5 = specs["C5"]
        specs[f"C5_N{nc}"] = dataclasses.replace(c5, name=f"C5_N{nc}",
                                                 crossings=dataclasses.replace(c5.crossings, n_cross=nc))
    for name in ("C2", "C3", "C4", "C5", "C5_N16", "C5_N32"):
        spec = specs[name]
        cnt = min(n, spec.total)
        start = (spec.total - cnt) // 2
        comp = sw.make_compute(spec, eng)
        out = torch.empty((cnt, 6), dtype=torch.float64, device=eng.device)
        comp(start, min(cnt, 4096), out[:min(cnt, 4096)])  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        comp(start, cnt, out)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rec = {"config": name, "points": cnt, "start": start, "points_per_s": cnt / dt, "seconds": dt,
               "finite": bool(torch.isfinite(out).all()), "notes": spec.notes}
        if spec.crossings is not None:
            m, dp, xi, v_w = spec.crossing_arrays(start, cnt, eng.device)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.lz_propagate(m, dp, xi, float(v_w[0]), spec.crossings.window_lz, spec.crossings.steps)
            torch.cuda.synchronize()
            rec["propagator_seconds"] = time.perf_counter() - t0
            rec["crossings"] = spec.crossings.__dict__
        # secondary (not the headline): z-sums shared per y-grid / A/V kernel, bit-identical
        comp_r = sw.make_compute(spec, eng, reuse=True)
        out_r = torch.empty_like(out)
        comp_r(start, min(cnt, 4096), out_r[:min(cnt, 4096)])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        comp_r(start, cnt, out_r)
        torch.cuda.synchronize()
        dtr = time.perf_counter() - t0
        rec["reuse_zsums"] = {"points_per_s": cnt / dtr, "bit_identical": bool(torch.equal(out, out_r))}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
