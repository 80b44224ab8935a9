#!/usr/bin/env python3
"""Which mode ode_integrate_kernel's wavefronts ran in, with a -DLZQ_ODE_COOP_DEBUG build under
<package>/_build/variants (the kernel then writes the cooperative segment width G -- 64 = whole
wavefront, 32/16/8 = sub-groups -- or 0 = per-lane into P_used):
    python tools/build_variants.py LZQ_ODE_COOP_DEBUG=1 && python tools/dbg_ode_coop.py"""
import sys, glob, importlib, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'tools')
import bench
from bench_ode import cfgs_for
cfgm = importlib.import_module(bench.PKG + ".config")
E = importlib.import_module(bench.PKG + ".engine").Engine
p = glob.glob(bench.PKG + "/_build/variants/*.so")[0]
e = E(0, lib_path=p)
cfgs = cfgs_for({"Gamma_wash_over_H": 1.0, "T_max_over_Tp": 1.6, "T_min_over_Tp": 0.6}, 1024)
pts = np.concatenate([cfgm.to_point(c) for c in cfgs]); ods = np.concatenate([cfgm.to_ode_params(c) for c in cfgs])
t, st = e.ode(pts, ods)
v = t[:, 5].cpu().numpy()
print("modes:", dict(zip(*np.unique(v, return_counts=True))), "status", dict(zip(*np.unique(st.cpu().numpy(), return_counts=True))))
