#!/usr/bin/env python3
"""Time the ODE fallback (Engine.ode, one chunk of up to 2^18 points) of every library variant under
<package>/_build/variants/ in ONE process, interleaved rounds, on tools/bench_ode.py's
narrow-window and stiff cases (ABLATE_GENERAL=1: also an I_p x v_w sweep, table-varying
cooperative waves and per-lane waves -- the general variant's).  Variants must agree with the first one to 1e-11.

    python tools/ablate_ode.py [n_points] [rounds] [radau|quadrature]
"""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    method = sys.argv[3] if len(sys.argv) > 3 else "radau"   # or "quadrature" (the opt-in form)
    cfgm = importlib.import_module(bench.PKG + ".config")
    E = importlib.import_module(bench.PKG + ".engine").Engine
    paths = sorted(glob.glob(os.path.join(ROOT, bench.PKG, "_build", "variants", "*.so")))
    engs = {os.path.basename(p)[7:-3]: E(0, lib_path=p) for p in paths}
    cases = {"narrow_wash": {"Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6},
             "stiff_thermal": {"sigma_v_chi_GeV_m2": 1e-9, "regime": "thermal", "m_chi_GeV": 300.0,
                               "T_max_over_Tp": 1.3, "T_min_over_Tp": 0.2},
             "riccati_mchi_sv": {"T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}}
    if os.environ.get("ABLATE_GENERAL"):
        # the general variant's waves: an A/V-parameter sweep (I_p x v_w fastest: a spline table per
        # point, cooperative table-varying waves) and the same points with every wave mixed (per lane)
        cases["riccati_ipvw"] = {"T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6, "sigma_v_chi_GeV_m2": 1e-12}
        cases["riccati_ipvw_perlane"] = dict(cases["riccati_ipvw"])
        # a Gamma_wash x sigma_v sweep (Gamma_wash fastest): grouped by the engine's wave order into
        # one Gamma_wash per wave, and as given (every wave mixes four: the general variant)
        cases["riccati_gw"] = {"T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}
        cases["riccati_gw_perlane"] = dict(cases["riccati_gw"])
        # 16 points per m_chi (16 sigma_v each): 16-lane cooperative segments, the general variant
        cases["riccati_g16"] = {"T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}
        # the stiff thermal window (T = m/3 crossed: a split step per segment) with 16 points per m_chi
        cases["stiff_g16"] = {"regime": "thermal", "T_max_over_Tp": 1.3, "T_min_over_Tp": 0.2}
    out = {}
    for cname, over in cases.items():
        cfgs = cfgs_for(over, n)
        if cname == "riccati_mchi_sv":   # m_chi fastest over 4 values x 16 sigma_v values
            for i, c in enumerate(cfgs):
                c["m_chi_GeV"] = (0.95, 3.0, 10.0, 30.0)[i % 4]
                c["sigma_v_chi_GeV_m2"] = 10.0 ** (-20 + ((i // 4) % 16) * 0.6)
        if cname.startswith("riccati_ipvw"):
            for i, c in enumerate(cfgs):
                c["I_p"] = (0.1, 0.2, 0.4, 0.8)[i % 4]
                c["v_w"] = (0.2, 0.4, 0.6, 0.8)[(i // 4) % 4]
        if cname == "riccati_g16":
            for i, c in enumerate(cfgs):
                c["m_chi_GeV"] = 0.5 + 0.001 * (i // 16)
                c["sigma_v_chi_GeV_m2"] = 10.0 ** (-20 + (i % 16) * 0.6)
        if cname == "stiff_g16":
            for i, c in enumerate(cfgs):
                c["m_chi_GeV"] = 300.0 + 0.01 * (i // 16)
                c["sigma_v_chi_GeV_m2"] = 10.0 ** (-10 + (i % 16) * 0.1)
        if cname.startswith("riccati_gw"):
            for i, c in enumerate(cfgs):
                c["Gamma_wash_over_H"] = (0.1, 0.5, 2.0, 8.0)[i % 4]
                c["sigma_v_chi_GeV_m2"] = 10.0 ** (-20 + ((i // 4) % 16) * 0.6)
        kw = {"group_waves": False} if cname.endswith("_perlane") else {}
        pts = np.concatenate([cfgm.to_point(c) for c in cfgs])
        ods = np.concatenate([cfgm.to_ode_params(c) for c in cfgs])
        ref = None
        for k, e in engs.items():  # warm-up + agreement
            t = e.ode(pts[:256], ods[:256], method=method, **kw)[0].cpu().numpy()
            if ref is None:
                ref = t
            if not os.environ.get("ABLATE_NOCHECK"):  # diagnostic variants that change results
                assert np.max(np.abs(t - ref) / np.maximum(np.abs(ref), 1e-300)) < 1e-11, k
        res = {k: [] for k in engs}
        last = {}
        for _ in range(rounds):
            for k, e in engs.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                last[k] = e.ode(pts, ods, chunk=1 << 18, method=method, **kw)[0]
                torch.cuda.synchronize()
                res[k].append(n / (time.perf_counter() - t0))
        out[cname] = {k: round(max(v)) for k, v in res.items()}
        first = next(iter(last))
        # every variant's full timed table against the first variant's, bit for bit (NaN rows equal)
        out[cname + "_bit_identical_to_" + first] = {
            k: bool(torch.equal(torch.nan_to_num(v, nan=1.5e308), torch.nan_to_num(last[first], nan=1.5e308)))
            for k, v in last.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
