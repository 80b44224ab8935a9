#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

This script is the only place that touches /root/reference, and it runs only in the
build container (the reference never travels to the GPU box).  It imports
`first_principles_yields` from /root/reference with bytecode writing disabled and
drives its own code paths:

* `main()` (fpy:346-438) per parameter point, in a scratch CWD, reading back the
  `yields_out.json` it writes (fpy:423-427) -> the per-point golden table;
* `AoverVKernel.A_over_V_y` (fpy:158-165) at a set of y values for several kernels;
* `try_compute_P_from_profile` (fpy:170-187) with a stub plug-in module that returns
  a chosen lambda, i.e. the reference's own closed form fpy:183-184;
* the CLI (`run.txt`) as a subprocess for the byte-exact stdout / yields_out.json.

Outputs (all JSON, small): golden_points.json, golden_aov.json, golden_lz.json,
golden_cli.json, plus env.json (numpy version / CPU flags).

    python tests/golden/make_golden.py        # ~1 min on 8 cores
"""
from __future__ import annotations

import contextlib
import io
import json
import math
import multiprocessing as mp
import os
import platform
import subprocess
import sys
import tempfile
import types

REF_DIR = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
N_RANDOM = 512


def _fpy():
    sys.dont_write_bytecode = True
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import first_principles_yields as fpy  # noqa: E402
    return fpy


# --------------------------------------------------------------------------------------
# parameter points
# --------------------------------------------------------------------------------------
def _base_cfg() -> dict:
    with open(os.path.join(REF_DIR, "yields_config_equal_mass.json")) as f:
        return json.load(f)


def random_points(n: int, seed: int = 0) -> list[dict]:
    import numpy as np
    rng = np.random.default_rng(seed)
    pts = []
    for _ in range(n):
        c = _base_cfg()
        c["m_chi_GeV"] = float(10 ** rng.uniform(-1.0, 3.5))
        c["g_chi"] = int(rng.choice([1, 2, 4]))
        c["chi_stats"] = str(rng.choice(["fermion", "boson"]))
        c["regime"] = "thermal" if rng.uniform() < 0.25 else "nonthermal"
        c["T_p_GeV"] = float(10 ** rng.uniform(0.0, 3.0))
        c["beta_over_H"] = float(10 ** rng.uniform(1.0, 3.0))
        c["v_w"] = float(rng.uniform(0.05, 0.95))
        c["I_p"] = float(rng.uniform(0.05, 1.0))
        c["g_star"] = float(rng.uniform(10.0, 110.0))
        c["g_star_s"] = float(c["g_star"] * rng.uniform(0.9, 1.1))
        c["P_chi_to_B"] = float(rng.uniform(0.0, 1.0))
        c["source_shape_sigma_y"] = float(rng.uniform(3.0, 30.0))
        c["incident_flux_scale"] = float(10 ** rng.uniform(-12.0, 0.0))
        c["T_max_over_Tp"] = 5.0 if rng.uniform() < 0.5 else float(rng.uniform(1.2, 10.0))
        c["T_min_over_Tp"] = 1e-3 if rng.uniform() < 0.5 else float(10 ** rng.uniform(-4.0, -0.05))
        u = rng.uniform()
        if u < 0.6:
            c["Y_chi_init"], c["n_chi_at_Tp_GeV3"] = 4.9e-10, None
        elif u < 0.85:
            c["Y_chi_init"], c["n_chi_at_Tp_GeV3"] = None, float(10 ** rng.uniform(-3.0, 3.0))
        else:
            c["Y_chi_init"], c["n_chi_at_Tp_GeV3"] = None, None
        pts.append(c)
    return pts


def edge_points() -> list[dict]:
    """Edge cases SURVEY §7 step 1 / §8(c) names: empty window, T_min cutting the
    support, y_lo < -50 clamp and y_lo < -80 cut, non-relativistic everywhere,
    boson stats, clamps on v_w / sigma_y, P = 0, zero flux, thermal regime."""
    E = []

    def mk(**kw):
        c = _base_cfg()
        c.update(kw)
        E.append(c)

    mk()                                             # C1 itself
    mk(T_min_over_Tp=6.0)                            # empty window -> Y_B = 0.0
    mk(T_min_over_Tp=0.9)                            # T_min cuts the support (y_hi ~ 11.7)
    mk(T_min_over_Tp=0.97)                           # y_hi ~ 3.1
    mk(T_max_over_Tp=100.0, beta_over_H=1000.0)      # y_lo_raw << -80 -> cut at -80, expy clamp
    mk(T_max_over_Tp=1.2)                            # narrow lower window
    mk(m_chi_GeV=3000.0)                             # non-relativistic over the whole window
    mk(m_chi_GeV=300.0)                              # T = m/3 = T_p: branch inside the window
    mk(m_chi_GeV=50.0)                               # relativistic (== 0.95 by separability)
    mk(chi_stats="boson")                            # boson/fermion = 4/3
    mk(v_w=0.0)                                      # v_w clamp 1e-12
    mk(v_w=-0.5)                                     # negative v_w clamp
    mk(source_shape_sigma_y=0.0)                     # sigma clamp 1e-6
    mk(P_chi_to_B=0.0)                               # P = 0 -> Y_B = 0, ratio guard 1e-300
    mk(incident_flux_scale=0.0)
    mk(regime="thermal")
    mk(regime="thermal", chi_stats="boson", m_chi_GeV=2000.0)
    mk(Y_chi_init=None, n_chi_at_Tp_GeV3=1e-3)
    mk(Y_chi_init=None, n_chi_at_Tp_GeV3=None)
    mk(T_p_GeV=10.0)                                 # T_p invariance
    mk(T_p_GeV=1000.0)
    mk(beta_over_H=50.0)                             # beta/H invariance
    mk(beta_over_H=10.0)
    mk(I_p=0.05)
    mk(I_p=1.0)
    mk(I_p=5.0)
    mk(g_star=10.75, g_star_s=10.75)
    mk(P_chi_to_B=1.0)
    mk(P_chi_to_B=2.0 * 0.14925839040304145)
    mk(incident_flux_scale=3.0 * 1.07e-9)
    mk(v_w=0.15)
    mk(g_chi=1)
    mk(T_max_over_Tp=1.0, T_min_over_Tp=1.0)         # zero-width window -> 0
    return E


def _run_main_in(cfg: dict, workdir: str) -> dict:
    """Run the reference main() on one config in workdir; return yields_out.json."""
    fpy = _fpy()
    path = os.path.join(workdir, "cfg.json")
    with open(path, "w") as f:
        json.dump(cfg, f)
    old = os.getcwd()
    argv = sys.argv
    try:
        os.chdir(workdir)
        sys.argv = ["first_principles_yields.py", "--config", path]
        with contextlib.redirect_stdout(io.StringIO()):
            fpy.main()
        with open(os.path.join(workdir, "yields_out.json")) as f:
            return json.load(f)
    finally:
        sys.argv = argv
        os.chdir(old)


def _worker(cfg: dict) -> dict:
    with tempfile.TemporaryDirectory() as d:
        try:
            out = _run_main_in(cfg, d)
            return {"config": cfg, "final": out["final"], "P_used": out["inputs"]["P_used"]}
        except Exception as e:  # regime 'auto' etc.: record the reference's exception type
            return {"config": cfg, "error": type(e).__name__}


# --------------------------------------------------------------------------------------
# A/V kernel, LZ closed form, CLI
# --------------------------------------------------------------------------------------
def aov_cases() -> list[dict]:
    import numpy as np
    fpy = _fpy()
    ys = sorted(set([float(v) for v in np.linspace(-90.0, 60.0, 61)]
                    + [-80.0, -50.0, -49.999, 0.0, 1e-3, 7.435, 15.975, 30.0, 49.99, 50.0, 50.0000001, 150.0]))
    kernels = [
        dict(I_p=0.34, beta_over_H=100.0, T_p=100.0, v_w=0.30, g_star=106.75),
        dict(I_p=0.05, beta_over_H=10.0, T_p=1.0, v_w=0.05, g_star=10.75),
        dict(I_p=1.0, beta_over_H=1000.0, T_p=1000.0, v_w=0.95, g_star=106.75),
        dict(I_p=0.34, beta_over_H=100.0, T_p=100.0, v_w=0.0, g_star=106.75),
    ]
    out = []
    for kw in kernels:
        k = fpy.AoverVKernel(**kw)
        out.append({"kernel": kw, "y": ys, "aov": [k.A_over_V_y(y) for y in ys]})
    return out


def lz_cases() -> dict:
    fpy = _fpy()
    lams = [-10.0, -1e-3, -0.0, 0.0, 1e-300, 1e-200, 1e-20, 1e-16, 1e-12, 1e-10, 3e-9, 1e-8,
            1e-6, 1e-4, 1e-2, 0.025726891712928787, 0.1, 0.5, 1.0, 3.0, 10.0, 120.0, 1e3, 1e300,
            float("inf")]
    P = []
    for lam in lams:
        stub = types.ModuleType("extended_LZ_lambda")
        stub.compute_lambda_eff_from_profile = (lambda _p, _l=lam: _l)
        sys.modules["extended_LZ_lambda"] = stub
        try:
            P.append(fpy.try_compute_P_from_profile("unused.csv", 0.3))
        finally:
            del sys.modules["extended_LZ_lambda"]
    return {"lambda": [repr(v) for v in lams], "P": P}


def cli_cases() -> list[dict]:
    """Byte-exact stdout + yields_out.json of the reference CLI for a few configs."""
    cases = []
    configs = {
        "equal_mass": None,  # the shipped file itself (run.txt)
        "thermal_boson": dict(regime="thermal", chi_stats="boson", m_chi_GeV=400.0),
        "n_chi_at_Tp": dict(Y_chi_init=None, n_chi_at_Tp_GeV3=2.5e-2),
        "empty_window": dict(T_min_over_Tp=6.0),
    }
    for name, over in configs.items():
        with tempfile.TemporaryDirectory() as d:
            if over is None:
                cfgpath = os.path.join(REF_DIR, "yields_config_equal_mass.json")
                with open(cfgpath) as f:
                    cfg_text = f.read()
            else:
                c = _base_cfg(); c.update(over)
                cfg_text = json.dumps(c, indent=2)
                cfgpath = os.path.join(d, "cfg.json")
                with open(cfgpath, "w") as f:
                    f.write(cfg_text)
            for flags in (["--diagnostics"], []):
                r = subprocess.run([sys.executable, "-B", os.path.join(REF_DIR, "first_principles_yields.py"),
                                    "--config", cfgpath] + flags, cwd=d, capture_output=True, text=True)
                with open(os.path.join(d, "yields_out.json")) as f:
                    yo = f.read()
                cases.append({"name": name, "flags": flags, "config_text": cfg_text,
                              "returncode": r.returncode, "stdout": r.stdout, "yields_out_json": yo})
    # error behaviours (fpy:358-359 prints ERROR and exits 0; regime auto -> UnboundLocalError)
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([sys.executable, "-B", os.path.join(REF_DIR, "first_principles_yields.py")],
                           cwd=d, capture_output=True, text=True)
        cases.append({"name": "no_config", "flags": [], "config_text": None, "returncode": r.returncode,
                      "stdout": r.stdout, "yields_out_json": None})
        r = subprocess.run([sys.executable, "-B", os.path.join(REF_DIR, "first_principles_yields.py"),
                            "--write-template", "--config", "tmpl.json"], cwd=d, capture_output=True, text=True)
        with open(os.path.join(d, "tmpl.json")) as f:
            tmpl = f.read()
        cases.append({"name": "write_template", "flags": ["--write-template"], "config_text": None,
                      "returncode": r.returncode, "stdout": r.stdout, "yields_out_json": None,
                      "template_text": tmpl})
        c = _base_cfg(); c["regime"] = "auto"
        with open(os.path.join(d, "auto.json"), "w") as f:
            json.dump(c, f)
        r = subprocess.run([sys.executable, "-B", os.path.join(REF_DIR, "first_principles_yields.py"),
                            "--config", "auto.json"], cwd=d, capture_output=True, text=True)
        cases.append({"name": "regime_auto", "flags": [], "config_text": json.dumps(c), "returncode": r.returncode,
                      "stdout": r.stdout, "stderr_last_line": r.stderr.strip().splitlines()[-1],
                      "yields_out_json": None})
        # profile flag with no plug-in module importable -> [warn] + fallback to config P
        r = subprocess.run([sys.executable, "-B", os.path.join(REF_DIR, "first_principles_yields.py"),
                            "--config", os.path.join(REF_DIR, "yields_config_equal_mass.json"),
                            "--maybe-compute-P-from-profile", "bounce.csv"], cwd=d, capture_output=True, text=True)
        cases.append({"name": "profile_fallback", "flags": ["--maybe-compute-P-from-profile", "bounce.csv"],
                      "config_text": None, "returncode": r.returncode, "stdout": r.stdout, "yields_out_json": None})
    return cases


def main():
    import numpy as np
    pts = edge_points() + random_points(N_RANDOM)
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        rows = pool.map(_worker, pts, chunksize=4)
    with open(os.path.join(HERE, "golden_points.json"), "w") as f:
        json.dump({"n_edge": len(edge_points()), "points": rows}, f, separators=(",", ":"))
    with open(os.path.join(HERE, "golden_aov.json"), "w") as f:
        json.dump(aov_cases(), f, separators=(",", ":"))
    with open(os.path.join(HERE, "golden_lz.json"), "w") as f:
        json.dump(lz_cases(), f, indent=1)
    with open(os.path.join(HERE, "golden_cli.json"), "w") as f:
        json.dump(cli_cases(), f, indent=1)
    flags = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    flags = " ".join(w for w in line.split() if w.startswith("avx"))
                    break
    except OSError:
        pass
    with open(os.path.join(HERE, "env.json"), "w") as f:
        json.dump({"python": platform.python_version(), "numpy": np.__version__,
                   "cpu": platform.processor(), "cpu_avx_flags": flags,
                   "reference": "first_principles_yields.py (fpy) @ /root/reference"}, f, indent=1)
    print("wrote", len(rows), "points")


if __name__ == "__main__":
    main()
