#!/usr/bin/env python3
"""A/B of the LZ propagator's cell scheme on a C5 slice, in one process: the library under test
(<package>/_build/liblzq.so, default S of sweep.CrossingSpec) against a reference build
(<package>/_build/ref/liblzq_<tag>.so, with its own S), each timed best-of-R with the
follow / cost / sort kernels included, plus the largest |P_new - P_ref| over the slice.

    python tools/ab_prop_scheme.py [n_points] [n_cross] [rounds] [ref_tag] [ref_steps]
"""
import dataclasses
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
    nc = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    tag = sys.argv[4] if len(sys.argv) > 4 else "r3head"
    ref_steps = int(sys.argv[5]) if len(sys.argv) > 5 else 1000
    sw = importlib.import_module(PKG + ".sweep")
    E = importlib.import_module(PKG + ".engine").Engine
    new = E(0)
    old = E(0, lib_path=os.path.join(ROOT, PKG, "_build", "ref", f"liblzq_{tag}.so"))
    spec = sw.builtin_specs()["C5"]
    spec = dataclasses.replace(spec, crossings=dataclasses.replace(spec.crossings, n_cross=nc))
    m, dp, xi, v_w = spec.crossing_arrays((spec.total - n) // 2, n, new.device)
    K = spec.crossings.window_lz
    runs = {"new": (new, spec.crossings.steps), "ref": (old, ref_steps)}
    P, best = {}, {}
    for k, (e, S) in runs.items():
        P[k] = e.lz_propagate(m, dp, xi, float(v_w[0]), K, S)
        best[k] = []
    for _ in range(rounds):
        for k, (e, S) in runs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.lz_propagate(m, dp, xi, float(v_w[0]), K, S)
            torch.cuda.synchronize()
            best[k].append(time.perf_counter() - t0)
    d = (P["new"] - P["ref"]).abs()
    print(json.dumps({"points": n, "n_cross": nc, "steps_new": spec.crossings.steps, "steps_ref": ref_steps,
                      "ref_lib": f"liblzq_{tag}.so", "seconds_new": min(best["new"]), "seconds_ref": min(best["ref"]),
                      "speedup": min(best["ref"]) / min(best["new"]), "max_abs_dP": float(d.max()),
                      "finite": bool(torch.isfinite(P["new"]).all())}), flush=True)


if __name__ == "__main__":
    main()
