"""Host-side scalar helper for printing only (never on the hot path): y(T) for the
diagnostics rows of the CLI (fpy:126-128, fpy:430-438).  Every other physics function runs on
the GPU (csrc/lzq_physics.h)."""
from __future__ import annotations


def y_of_T(T: float, T_p: float, beta_over_H: float) -> float:
    """fpy:126-128."""
    B = beta_over_H
    return 0.5 * B * ((T_p / max(T, 1e-30)) ** 2 - 1.0)
