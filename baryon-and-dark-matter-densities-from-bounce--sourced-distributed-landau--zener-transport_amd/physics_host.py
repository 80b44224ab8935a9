"""Host-side scalar helpers for printing and the reference-shaped API only (never on the hot
path): y(T) for the CLI's diagnostics rows (fpy:126-128, fpy:430-438) and the one-line
H(T), s(T) wrappers of BoltzmannSystem (fpy:84-88, 203-204).  Every evaluation on the hot path
runs on the GPU (csrc/lzq_physics.h)."""
from __future__ import annotations

import math


def y_of_T(T: float, T_p: float, beta_over_H: float) -> float:
    """fpy:126-128."""
    B = beta_over_H
    return 0.5 * B * ((T_p / max(T, 1e-30)) ** 2 - 1.0)


M_PL_GEV = 1.220890e19   # fpy:35 MPL_GEV
PI = math.pi             # fpy:34


def H_std(T: float, g_star: float) -> float:
    """fpy:84-85."""
    return 1.66 * math.sqrt(g_star) * T * T / M_PL_GEV


def s_entropy(T: float, g_star_s: float) -> float:
    """fpy:87-88."""
    return (2.0 * PI ** 2 / 45.0) * g_star_s * T ** 3
