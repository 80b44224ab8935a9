"""Config schema of the reference driver, kept byte-compatible (fpy = first_principles_yields.py).

`Config` has the fields, defaults and field ORDER of fpy:44-79 (the order is visible in
yields_out.json, whose "inputs" block dumps `cfg.__dict__`, fpy:424).  `default_config`,
`load_config` and `write_template` keep the semantics of fpy:291-312, including the
differences between the dataclass defaults and `default_config()` (P_chi_to_B None,
source_shape_sigma_y 15.0) and the TypeError raised by an unknown JSON key.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from . import _native


@dataclass
class Config:
    # microphysics / DM
    m_chi_GeV: float = 0.95
    g_chi: int = 2
    chi_stats: str = "fermion"
    regime: str = "nonthermal"
    sigma_v_chi_GeV_m2: float = 0.0
    # transition / percolation
    T_p_GeV: float = 100.0
    beta_over_H: float = 100.0
    v_w: float = 0.30
    I_p: float = 0.34
    # relativistic degrees of freedom
    g_star: float = 106.75
    g_star_s: float = 106.75
    # source normalisation / shape
    P_chi_to_B: Optional[float] = None
    source_shape_sigma_y: float = 15.0
    Gamma_wash_over_H: float = 0.0
    incident_flux_scale: float = 1.0
    deplete_DM_from_source: bool = False
    # integration window
    T_max_over_Tp: float = 5.0
    T_min_over_Tp: float = 1e-3
    # non-thermal initial abundance
    Y_chi_init: Optional[float] = 4.90e-10
    n_chi_at_Tp_GeV3: Optional[float] = None


_DEFAULTS = {
    "m_chi_GeV": 0.95, "g_chi": 2, "chi_stats": "fermion", "regime": "nonthermal",
    "sigma_v_chi_GeV_m2": 0.0,
    "T_p_GeV": 100.0, "beta_over_H": 100.0, "v_w": 0.30, "I_p": 0.34,
    "g_star": 106.75, "g_star_s": 106.75,
    "P_chi_to_B": None, "source_shape_sigma_y": 15.0, "Gamma_wash_over_H": 0.0,
    "incident_flux_scale": 1.0, "deplete_DM_from_source": False,
    "T_max_over_Tp": 5.0, "T_min_over_Tp": 1.0e-3,
    "Y_chi_init": 4.90e-10, "n_chi_at_Tp_GeV3": None,
}


def default_config() -> Dict:
    """fpy:291-301 (a fresh dict in the reference's key order)."""
    return dict(_DEFAULTS)


def load_config(path: str) -> Config:
    """fpy:303-307: defaults overlaid with the JSON file; unknown keys raise TypeError."""
    with open(path, "r", encoding="utf-8") as f:
        raw = json.load(f)
    base = default_config()
    base.update(raw)
    return Config(**base)


def write_template(path: str) -> None:
    """fpy:309-312."""
    with open(path, "w", encoding="utf-8") as f:
        json.dump(default_config(), f, indent=2)
    print(f"Wrote template config to {path}")


def fast_path_ok(cfg: Config) -> bool:
    """fpy:372 gate of the direct-quadrature path (the only path this engine implements)."""
    return (not cfg.deplete_DM_from_source) and (cfg.sigma_v_chi_GeV_m2 == 0.0) and (cfg.Gamma_wash_over_H == 0.0)


def stats_code(stats) -> int:
    return _native.FERMION if str(stats).lower().startswith("ferm") else _native.BOSON  # fpy:96


def regime_code(regime) -> int:
    r = str(regime).lower()  # fpy:376-384
    if r.startswith("therm"):
        return _native.THERMAL
    if r.startswith("non"):
        return _native.NONTHERMAL
    return _native.REGIME_OTHER


def to_point(cfg, P: Optional[float] = None) -> np.ndarray:
    """Config (or fpy-schema dict) -> one lzq_point record (numpy structured scalar array).

    P overrides cfg.P_chi_to_B (maybe_P's result, fpy:362)."""
    c = cfg if isinstance(cfg, dict) else cfg.__dict__
    rec = np.zeros(1, dtype=_native.POINT_DTYPE)
    for n in ("m_chi_GeV", "g_chi", "T_p_GeV", "beta_over_H", "v_w", "I_p", "g_star", "g_star_s",
              "source_shape_sigma_y", "incident_flux_scale", "T_max_over_Tp", "T_min_over_Tp"):
        rec[n] = float(c[n])
    Pv = c["P_chi_to_B"] if P is None else P
    rec["P_chi_to_B"] = float("nan") if Pv is None else float(Pv)
    rec["stats"] = stats_code(c["chi_stats"])
    rec["regime"] = regime_code(c["regime"])
    rec["has_Y_chi_init"] = int(c["Y_chi_init"] is not None)
    rec["Y_chi_init"] = float(c["Y_chi_init"]) if c["Y_chi_init"] is not None else 0.0
    rec["has_n_chi_at_Tp"] = int(c["n_chi_at_Tp_GeV3"] is not None)
    rec["n_chi_at_Tp_GeV3"] = float(c["n_chi_at_Tp_GeV3"]) if c["n_chi_at_Tp_GeV3"] is not None else 0.0
    return rec


def to_ode_params(cfg) -> np.ndarray:
    """The three Config fields of the ODE fallback (fpy:279-284) -> one lzq_ode_params record."""
    c = cfg if isinstance(cfg, dict) else cfg.__dict__
    rec = np.zeros(1, dtype=_native.ODE_DTYPE)
    rec["sigma_v_chi_GeV_m2"] = float(c["sigma_v_chi_GeV_m2"])
    rec["Gamma_wash_over_H"] = float(c["Gamma_wash_over_H"])
    rec["deplete_DM_from_source"] = int(bool(c["deplete_DM_from_source"]))
    return rec


def to_ctypes_ode(rec: np.ndarray) -> "_native.LzqOdeParams":
    o = _native.LzqOdeParams()
    o.sigma_v_chi_GeV_m2 = float(rec["sigma_v_chi_GeV_m2"].item())
    o.Gamma_wash_over_H = float(rec["Gamma_wash_over_H"].item())
    o.deplete_DM_from_source = int(rec["deplete_DM_from_source"].item())
    return o


def to_aov(obj) -> np.ndarray:
    """An A/V kernel's own parameters (fpy:141-151) -> one lzq_aov_params record.  obj: an
    AoverVKernel (reference or boltzmann.AoverVKernel: attributes I_p, beta_over_H, T_p, v_w,
    g_star), a dict with those keys (T_p or T_p_GeV), or a Config / fpy-schema dict (its own
    kernel, fpy:197)."""
    get = (lambda k: obj[k]) if isinstance(obj, dict) else (lambda k: getattr(obj, k))
    def has(k):
        return (k in obj) if isinstance(obj, dict) else hasattr(obj, k)
    rec = np.zeros(1, dtype=_native.AOV_DTYPE)
    for n in ("I_p", "beta_over_H", "v_w", "g_star"):
        rec[n] = float(get(n))
    rec["T_p_GeV"] = float(get("T_p") if has("T_p") else get("T_p_GeV"))
    return rec


def to_ctypes_aov(rec: np.ndarray) -> "_native.LzqAovParams":
    a = _native.LzqAovParams()
    for n in _native.AOV_FIELDS:
        setattr(a, n, float(rec[n].item() if hasattr(rec[n], "item") else rec[n]))
    return a


def to_ctypes_point(rec: np.ndarray) -> "_native.LzqPoint":
    p = _native.LzqPoint()
    for n in _native.POINT_DOUBLE_FIELDS + _native.POINT_INT_FIELDS:
        setattr(p, n, rec[n].item() if hasattr(rec[n], "item") else rec[n])
    return p
