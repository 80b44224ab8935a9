"""Host-side scalar helpers the driver needs for input preparation and printing only
(never on the hot path): y(T) for the diagnostics rows (fpy:126-128) and the scalar
entropy/number density used nowhere in the timed path."""
from __future__ import annotations


def y_of_T(T: float, T_p: float, beta_over_H: float) -> float:
    """fpy:126-128."""
    B = beta_over_H
    return 0.5 * B * ((T_p / max(T, 1e-30)) ** 2 - 1.0)
