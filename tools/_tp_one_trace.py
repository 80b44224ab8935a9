import importlib, os, sys, json, time
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import bench
from bench_ode import cfgs_for
import torch
cfgm = importlib.import_module(bench.PKG + ".config")
eng = importlib.import_module(bench.PKG + ".engine").Engine(0)
c = cfgs_for({"Gamma_wash_over_H": 1.0, "sigma_v_chi_GeV_m2": 1e-12}, 1)[0]
p, o = cfgm.to_point(c), cfgm.to_ode_params(c)
for _ in range(3):
    eng.ode(p, o, time_parallel=True)
torch.cuda.synchronize()
print("ok")
