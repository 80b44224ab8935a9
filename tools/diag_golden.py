#!/usr/bin/env python3
"""Worst golden-point errors (tests/golden/golden_points.json, the reference's own outputs)
of every library variant under <package>/_build/variants/: the five worst (point, field)
pairs per variant, for accuracy A/B of kernel changes.

    python tools/diag_golden.py
"""
import glob
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def main():
    import test_gpu_parity as T
    E = importlib.import_module(PKG + ".engine").Engine
    nat = importlib.import_module(PKG + "._native")
    pts = T.golden("golden_points.json")["points"]
    cfgs = [T.full_cfg(r["config"]) for r in pts]
    paths = sorted(glob.glob(os.path.join(ROOT, PKG, "_build", "variants", "*.so")))
    out = {}
    for p in paths:
        eng = E(0, lib_path=p)
        t = eng.yields(T.recs(cfgs)).cpu().numpy()
        errs = []
        for i, (row, r) in enumerate(zip(t, pts)):
            for k, v in zip(nat.YIELD_FIELDS, row):
                if k in r["final"]:
                    errs.append((T.rel_err(v, r["final"][k]), i, k))
        errs.sort(reverse=True)
        out[os.path.basename(p)[7:-3]] = [
            {"err": e, "point": i, "field": k,
             "cfg": {c: pts[i]["config"].get(c) for c in ("m_chi_GeV", "beta_over_H", "source_shape_sigma_y", "T_p_GeV",
                                                            "regime", "T_max_over_Tp", "T_min_over_Tp")}}
            for e, i, k in errs[:5]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
