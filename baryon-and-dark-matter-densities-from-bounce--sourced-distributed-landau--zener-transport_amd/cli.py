"""Drop-in driver: the CLI, stdout and yields_out.json of fpy:346-438, computed on the GPU.

    python -m <package>.cli --config yields_config_equal_mass.json --diagnostics

Flags, messages, exit behaviour and output bytes follow the reference (checked against
the reference's own output in tests/golden/golden_cli.json).  Configurations outside the
fast quadrature path (fpy:372) take the ODE fallback (fpy:385-410) on the GPU
(engine.Engine.ode -> lzq_ode_batch), with the reference's error behaviour.
"""
from __future__ import annotations

import argparse
import json
import math

import numpy as np

from . import _native
from .config import fast_path_ok, load_config, to_ode_params, to_point, write_template
from .engine import default_engine
from .lz import maybe_P
from .physics_host import y_of_T

S0_M3 = 2891.0 * 1e6  # fpy:36-37


def main(argv=None):
    ap = argparse.ArgumentParser(description="First-principles DM/Baryon yields from bounce-sourced transport")
    ap.add_argument("--config", required=False, help="Path to yields_config.json")
    ap.add_argument("--write-template", action="store_true", help="Write a template config and exit")
    ap.add_argument("--maybe-compute-P-from-profile", dest="profile_csv", default=None,
                    help="Try to compute P_chi_to_B from local LZ modules using this profile CSV.")
    ap.add_argument("--diagnostics", action="store_true",
                    help="Print a small table of y(T), A/V(T), J_chi(T), S_B(T) around T_p.")
    args = ap.parse_args(argv)

    if args.write_template:
        write_template(args.config or "yields_config.json")
        return
    if not args.config:
        print("ERROR: --config is required (or use --write-template).")
        return

    cfg = load_config(args.config)
    P_used = maybe_P(cfg, args.profile_csv)
    if fast_path_ok(cfg):
        low = cfg.regime.lower()
        if not (low.startswith("therm") or low.startswith("non")):
            # fpy:376-384 has no else-branch on the fast path
            raise UnboundLocalError("local variable 'Ychi_fin' referenced before assignment")
    eng = default_engine()
    if fast_path_ok(cfg):
        table = eng.yields(to_point(cfg, P=P_used), n_y=8000)  # fpy:374 + fpy:376-417 on the GPU
    else:
        # fpy:385-410: build_tables + Radau, then fpy:412-417; one point: Engine.ode integrates it
        # parallel in time (lzq_ode_integrate_tp, the sequential steps' bits)
        table, status = eng.ode(to_point(cfg, P=P_used), to_ode_params(cfg))
        st = int(status[0].item())
        if st in (_native.ODE_BAD_GRID, _native.ODE_BAD_STEP):  # scipy's ValueError (CubicSpline / solve_ivp)
            raise ValueError(_native.ODE_STATUS[st])
        if st == _native.ODE_NEWTON:  # fpy:408-410: warn, then report the state where the solver stopped
            print("[warn] ODE solver reported failure:", _native.ODE_STATUS[st])
        elif st != 0:  # not reachable for a window the reference accepts (Engine.ode sizes max_steps)
            raise RuntimeError(f"lzq ODE fallback: {_native.ODE_STATUS[st]}")
    YB_fin, Ychi_fin, rhoB0, rhoDM0, ratio, _ = (float(v) for v in table[0].cpu().numpy())

    print("\n=== Results (today) ===")
    print(f"rho_B^0   = {rhoB0:.3e} kg/m^3")
    print(f"rho_DM^0  = {rhoDM0:.3e} kg/m^3")
    print(f"DM/B ratio= {ratio:.6g}")
    with open("yields_out.json", "w", encoding="utf-8") as f:
        json.dump({"inputs": {**cfg.__dict__, "P_used": P_used},
                   "final": {"Y_B": YB_fin, "Y_chi": Ychi_fin,
                             "rho_B_kg_m3": rhoB0, "rho_DM_kg_m3": rhoDM0,
                             "DM_over_B": ratio}}, f, indent=2)
    print("Wrote yields_out.json")

    if args.diagnostics:  # fpy:430-438
        print("\n# Diagnostics around percolation")
        Ts = np.geomspace(cfg.T_p_GeV * 0.5, cfg.T_p_GeV * 2.0, 21)
        ys = [y_of_T(T, cfg.T_p_GeV, cfg.beta_over_H) for T in Ts]
        aovs = eng.aov(cfg, ys).cpu().numpy()
        Js = eng.jchi(cfg, Ts).cpu().numpy()
        print(" T/Tp      y(T)        A/V [GeV]         J_chi [GeV^3]      S_B [GeV^3]")
        for T, y, aov, J in zip(Ts, ys, aovs, Js):
            aov, J = float(aov), float(J)
            SB = P_used * J * aov * math.exp(-0.5 * (y / max(cfg.source_shape_sigma_y, 1e-6)) ** 2)
            print(f"{T/cfg.T_p_GeV:7.3f}  {y:9.3f}  {aov:14.6e}  {J:16.6e}  {SB:14.6e}")


if __name__ == "__main__":
    main()
