"""LZ probability plug-in hook (fpy:170-187) and P selection (fpy:317-328).

`try_compute_P_from_profile` searches the same module names in the same order and applies
the same clamps and exception swallowing as the reference; the closed form
P = 1 - exp(-2 pi max(lambda, 0)) (fpy:183-184) is evaluated by the HIP kernel
`lzq_p_closed_form` (naive 1 - exp kept, not expm1: SURVEY §8a a5).
"""
from __future__ import annotations

import importlib
from typing import Optional

PLUGIN_MODULES = ("lambda_local_LZ_from_profile", "extended_LZ_lambda", "transport_from_profile")


def p_closed_form(lam: float) -> float:
    from .engine import default_engine
    return float(default_engine().p_closed_form([float(lam)])[0].item())


def try_compute_P_from_profile(profile_csv_path: str, v_w: float) -> Optional[float]:
    """fpy:170-187: same module order, clamps and swallowing of the PLUG-IN's exceptions.
    The closed form itself runs on the GPU (lzq_p_closed_form) outside the swallowing block:
    a failure of the HIP library raises instead of silently falling back to the config P.
    Plug-in modules are found on sys.path, as in the reference (lzq ships one in plugins/)."""
    try:
        for modname in PLUGIN_MODULES:
            try:
                mod = importlib.import_module(modname)
            except Exception:
                continue
            if hasattr(mod, "compute_prob_from_profile"):
                P = mod.compute_prob_from_profile(profile_csv_path, v_w)
                return float(max(min(P, 1.0), 0.0))
            if hasattr(mod, "compute_lambda_eff_from_profile"):
                lam_eff = float(mod.compute_lambda_eff_from_profile(profile_csv_path))
                break
        else:
            return None
    except Exception:
        return None
    return p_closed_form(lam_eff)


def maybe_P(cfg, profile_csv: Optional[str]) -> float:
    """fpy:317-328 (same messages, same RuntimeError)."""
    P_used = cfg.P_chi_to_B
    if profile_csv:
        P_try = try_compute_P_from_profile(profile_csv, cfg.v_w)
        if P_try is not None:
            print(f"[info] Using P_chi_to_B from profile: {P_try:.6g}")
            P_used = P_try
        else:
            print("[warn] Could not compute P from profile automatically; falling back to config.")
    if P_used is None:
        raise RuntimeError("P_chi_to_B is not set and could not be computed from profile.")
    return float(P_used)


def p_incoherent(P_list) -> float:
    """Phase-averaged composition of sequential independent crossings (two-state Markov
    chain with swap probability P_c per crossing): P_tot = (1 - prod(1 - 2 P_c)) / 2.
    The coherent composition is lzq_lz_propagate ("Multi-crossing")."""
    prod = 1.0
    for P in P_list:
        prod *= (1.0 - 2.0 * float(P))
    return 0.5 * (1.0 - prod)
