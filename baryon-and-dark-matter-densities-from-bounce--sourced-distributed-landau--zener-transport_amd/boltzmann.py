"""Reference-shaped operator API of the hot path (fpy = first_principles_yields.py).

`AoverVKernel` and `BoltzmannSystem` keep the constructor signatures and method names of
fpy:140-165 and fpy:192-267 so code written against the reference reads the same, but every
evaluation runs on the GPU through the C ABI (engine.Engine).  Only the direct-quadrature
path and the ODE fallback's operators (build_tables / A_over_V_T / rhs, fpy:207-219, 270-286)
run on the GPU; the integration itself is engine.Engine.ode (lzq_ode_batch), used by cli.py.
"""
from __future__ import annotations

import math

import numpy as np

from . import _native
from .config import Config, fast_path_ok, to_ode_params, to_point
from .engine import default_engine
from .physics_host import H_std

LZQ_NZ, LZQ_ZMAX = _native.LZQ_NZ, _native.LZQ_Z_MAX


class AoverVKernel:
    """fpy:140-165 for any z grid: z = linspace(0, z_max, nz) and the cancelling gamma4 are built
    by the library (lzq_ztables) and uploaded once per grid; every A_over_V_y runs on the GPU."""

    def __init__(self, I_p: float, beta_over_H: float, T_p: float, v_w: float, g_star: float,
                 z_max: float = LZQ_ZMAX, nz: int = LZQ_NZ):
        self.nz, self.z_max = _native.zgrid(nz, z_max)  # numpy linspace's TypeError / ValueError
        self.I_p = I_p
        self.beta_over_H = beta_over_H
        self.T_p = T_p
        self.v_w = max(v_w, 1e-12)                      # fpy:146
        self.g_star = g_star
        self.H_p = H_std(T_p, g_star)                   # fpy:150-151
        self.beta = self.beta_over_H * self.H_p
        self._tables = None

    @property
    def z(self) -> np.ndarray:
        """fpy:154 (the library's host copy of the grid it integrates on)."""
        return self._ztables()[0]

    @property
    def g4(self) -> np.ndarray:
        """fpy:155-156, the cancelling form verbatim."""
        return self._ztables()[1]

    def _ztables(self):
        if self._tables is None:
            self._tables = _native.ztables(self.nz, self.z_max)
        return self._tables

    def A_over_V_y(self, y: float) -> float:
        return float(self.A_over_V_ys([y])[0])

    def A_over_V_ys(self, ys) -> np.ndarray:
        """Batched fpy:158-165 (one GPU lane per y), with this kernel's own I_p, beta_over_H, T_p,
        v_w and g_star (lzq_aov_batch's lzq_aov_params block)."""
        return default_engine().aov(self, ys, nz=self.nz, z_max=self.z_max).cpu().numpy()


class BoltzmannSystem:
    """fpy:192-267 direct-quadrature path.

    As in the reference, self.aov is an independent public object (fpy:197): the integrand's
    y-grid, T(y), H, s, J and window come from self.cfg, A/V from self.aov's own parameters and z
    grid (fpy:211, 228, 261).  Replacing bs.aov with another AoverVKernel changes A/V only; every
    operator below passes its parameters through the C ABI (lzq_aov_params)."""

    def __init__(self, cfg: Config, P_chi_to_B: float):
        self.cfg = cfg
        self.P = float(P_chi_to_B)
        self.m = float(cfg.m_chi_GeV)
        self.aov = AoverVKernel(cfg.I_p, cfg.beta_over_H, cfg.T_p_GeV, cfg.v_w, cfg.g_star)

    # Cosmology/thermo wrappers (fpy:203-204; scalar host arithmetic, not on the hot path)
    def H(self, T: float) -> float:
        from .physics_host import H_std
        return H_std(T, self.cfg.g_star)

    def s(self, T: float) -> float:
        from .physics_host import s_entropy
        return s_entropy(T, self.cfg.g_star_s)

    def J_chi(self, T: float) -> float:
        """fpy:222-223."""
        return float(self.J_chi_T([T])[0])

    def J_chi_T(self, Ts) -> np.ndarray:
        return default_engine().jchi(self.cfg, Ts).cpu().numpy()

    def S_B_T(self, T: float) -> float:
        """fpy:225-228."""
        from .physics_host import y_of_T
        y = y_of_T(T, self.cfg.T_p_GeV, self.cfg.beta_over_H)
        window = math.exp(-0.5 * (y / max(self.cfg.source_shape_sigma_y, 1e-6)) ** 2)
        return self.P * self.J_chi(T) * self.aov.A_over_V_y(y) * window

    def integrate_YB_by_quadrature(self, T_lo: float, T_hi: float, n_y: int = 6000) -> float:
        """fpy:231-267 on the GPU (one wavefront)."""
        rec = to_point(self.cfg, P=self.P)
        out = default_engine().yields(rec, n_y=int(n_y), T_lo=[float(T_lo)], T_hi=[float(T_hi)], P=[self.P],
                                      nz=self.aov.nz, z_max=self.aov.z_max, aov=self.aov)
        return float(out[0, 0].item())

    # ---- ODE fallback operators (fpy:207-219, 270-286) --------------------------------------
    def build_tables(self, T_lo: float, T_hi: float, n: int = 800):
        """fpy:207-212 on the GPU: A/V (on self.aov's z grid) at linspace(T_lo, T_hi, n) + the
        not-a-knot cubic spline.  4 <= n <= LZQ_ODE_NT_MAX (scipy's not-a-knot spline needs at
        least 4 knots for the cubic form the library evaluates)."""
        import operator
        n = operator.index(n)
        if not 4 <= n <= _native.ODE_NT_MAX:
            raise ValueError(f"build_tables: n = {n} outside [4, {_native.ODE_NT_MAX}]")
        if not (float(T_hi) > float(T_lo)):
            raise ValueError("`x` must be strictly increasing sequence.")
        eng = default_engine()
        self._T_lo, self._T_hi = float(T_lo), float(T_hi)
        self._nt = int(n)
        self._rec = to_point(self.cfg, P=self.P)
        self._work, status = eng.ode_tables(self._rec, [self._T_lo], [self._T_hi], nt=self._nt, nz=self.aov.nz,
                                            z_max=self.aov.z_max, aov=self.aov)
        if int(status[0].item()) != 0:
            raise ValueError("`x` must be strictly increasing sequence.")

    def _need_tables(self):
        if getattr(self, "_work", None) is None:
            raise RuntimeError("call build_tables(T_lo, T_hi) first (fpy:207)")

    def A_over_V_Ts(self, Ts) -> np.ndarray:
        """Batched fpy:214-218: the spline after build_tables, else A/V(y(T)) directly (fpy:218-219)."""
        if getattr(self, "_work", None) is None:
            from .physics_host import y_of_T
            ys = [y_of_T(float(T), self.cfg.T_p_GeV, self.cfg.beta_over_H) for T in np.atleast_1d(Ts)]
            return self.aov.A_over_V_ys(ys)
        return default_engine().ode_aov_T(self._rec, self._T_lo, self._T_hi, self._work, Ts,
                                          nt=self._nt).cpu().numpy()

    def A_over_V_T(self, T: float) -> float:
        """fpy:214-219."""
        return float(self.A_over_V_Ts([T])[0])

    def rhs_batch(self, xs, Ys) -> np.ndarray:
        """Batched fpy:270-286: (n, 2) array of (dY_chi/dx, dY_B/dx)."""
        self._need_tables()
        return default_engine().ode_rhs(self._rec, to_ode_params(self.cfg), self._T_lo, self._T_hi, self._work, xs,
                                        Ys, nt=self._nt).cpu().numpy()

    def rhs(self, x: float, Y) -> np.ndarray:
        """fpy:270-286."""
        return self.rhs_batch([float(x)], [[float(Y[0]), float(Y[1])]])[0]

    def fast_path_ok(self) -> bool:
        return fast_path_ok(self.cfg)
