"""ctypes front-end of the CPU oracle (oracle/lzq_oracle.c).

TEST INFRASTRUCTURE ONLY.  Importable only from tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, and there only as the checker / the timed CPU baseline.
The product (the HIP library + package host code) never imports this module.

The C code restates /root/reference/first_principles_yields.py (fpy) verbatim; see the
per-function citations in lzq_oracle.c.  Pinned by tests/test_oracle_golden.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liblzq_oracle.so")


class OraclePoint(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "m_chi_GeV", "g_chi", "T_p_GeV", "beta_over_H", "v_w", "I_p", "g_star", "g_star_s",
        "P_chi_to_B", "source_shape_sigma_y", "incident_flux_scale",
        "T_max_over_Tp", "T_min_over_Tp", "Y_chi_init", "n_chi_at_Tp_GeV3")] + [
        (n, ctypes.c_int32) for n in ("stats", "regime", "has_Y_chi_init", "has_n_chi_at_Tp")]


class OracleAov(ctypes.Structure):  # oracle_aov_params: AoverVKernel's own parameters (fpy:141-151)
    _fields_ = [(n, ctypes.c_double) for n in ("I_p", "beta_over_H", "T_p_GeV", "v_w", "g_star")]


def aov_from(a) -> "OracleAov | None":
    """An A/V kernel's parameters (dict with I_p, beta_over_H, T_p (or T_p_GeV), v_w, g_star) ->
    OracleAov; None stays None (the point's own kernel, fpy:197)."""
    if a is None:
        return None
    return OracleAov(float(a["I_p"]), float(a["beta_over_H"]), float(a["T_p"] if "T_p" in a else a["T_p_GeV"]),
                     float(a["v_w"]), float(a["g_star"]))


def _ref(o):
    return None if o is None else ctypes.byref(o)


YIELD_FIELDS = ("Y_B", "Y_chi", "rho_B_kg_m3", "rho_DM_kg_m3", "DM_over_B", "P_used")


class OracleYield(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in YIELD_FIELDS]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        d, i32, i64 = ctypes.c_double, ctypes.c_int32, ctypes.c_int64
        P = ctypes.POINTER
        L.oracle_aov.restype = d
        L.oracle_aov.argtypes = [d, d, d, d, d, d]
        L.oracle_yb_quadrature.restype = d
        L.oracle_yb_quadrature.argtypes = [P(OraclePoint), d, d, i32]
        L.oracle_point_yields.restype = ctypes.c_int
        L.oracle_point_yields.argtypes = [P(OraclePoint), P(OracleYield)]
        L.oracle_points_batch.restype = i64
        L.oracle_points_batch.argtypes = [P(OraclePoint), i64, P(OracleYield), i32]
        L.oracle_p_closed_form.restype = d
        L.oracle_p_closed_form.argtypes = [d]
        L.oracle_j_chi.restype = d
        L.oracle_j_chi.argtypes = [P(OraclePoint), d]
        L.oracle_pairwise_sum.restype = d
        L.oracle_pairwise_sum.argtypes = [P(d), i64]
        L.oracle_linspace.restype = None
        L.oracle_linspace.argtypes = [d, d, i64, P(d)]
        L.oracle_aov_z.restype = d
        L.oracle_aov_z.argtypes = [d, d, d, d, d, d, i64, d]
        L.oracle_yb_quadrature_z.restype = d
        L.oracle_yb_quadrature_z.argtypes = [P(OraclePoint), d, d, i32, i64, d]
        L.oracle_point_yields_z.restype = ctypes.c_int
        L.oracle_point_yields_z.argtypes = [P(OraclePoint), i64, d, P(OracleYield)]
        L.oracle_points_batch_z.restype = i64
        L.oracle_points_batch_z.argtypes = [P(OraclePoint), i64, i64, d, P(OracleYield), i32]
        L.oracle_yb_quadrature_a.restype = d
        L.oracle_yb_quadrature_a.argtypes = [P(OraclePoint), P(OracleAov), d, d, i32, i64, d]
        L.oracle_point_yields_a.restype = ctypes.c_int
        L.oracle_point_yields_a.argtypes = [P(OraclePoint), P(OracleAov), i64, d, P(OracleYield)]
        _lib = L
    return _lib


def point_from_config(cfg: dict) -> OraclePoint:
    """Config dict (fpy schema, defaults already applied) -> OraclePoint."""
    p = OraclePoint()
    for n in ("m_chi_GeV", "g_chi", "T_p_GeV", "beta_over_H", "v_w", "I_p", "g_star", "g_star_s",
              "source_shape_sigma_y", "incident_flux_scale", "T_max_over_Tp", "T_min_over_Tp"):
        setattr(p, n, float(cfg[n]))
    p.P_chi_to_B = float(cfg["P_chi_to_B"])
    p.stats = 0 if str(cfg["chi_stats"]).lower().startswith("ferm") else 1
    r = str(cfg["regime"]).lower()
    p.regime = 0 if r.startswith("therm") else (1 if r.startswith("non") else 2)
    p.has_Y_chi_init = int(cfg["Y_chi_init"] is not None)
    p.Y_chi_init = float(cfg["Y_chi_init"]) if cfg["Y_chi_init"] is not None else 0.0
    p.has_n_chi_at_Tp = int(cfg["n_chi_at_Tp_GeV3"] is not None)
    p.n_chi_at_Tp_GeV3 = float(cfg["n_chi_at_Tp_GeV3"]) if cfg["n_chi_at_Tp_GeV3"] is not None else 0.0
    return p


NZ, Z_MAX = 1200, 30.0   # fpy:142 defaults, main()'s grid (fpy:197)


def point_yields(cfg: dict, nz: int = NZ, z_max: float = Z_MAX, aov: dict | None = None) -> dict:
    """main()'s fast path (fpy:361-417) for one config, A/V on AoverVKernel(..., z_max, nz) with the
    kernel's own parameters `aov` (None: cfg's, fpy:197)."""
    p = point_from_config(cfg)
    o = OracleYield()
    rc = lib().oracle_point_yields_a(ctypes.byref(p), _ref(aov_from(aov)), int(nz), float(z_max), ctypes.byref(o))
    if rc != 0:
        raise UnboundLocalError("local variable 'Ychi_fin' referenced before assignment")
    return {n: getattr(o, n) for n in YIELD_FIELDS}


def points_batch(cfgs: list[dict], nthreads: int = 0, nz: int = NZ, z_max: float = Z_MAX) -> np.ndarray:
    """Returns an (n, 6) float64 array in YIELD_FIELDS order (NaN rows for failed points)."""
    n = len(cfgs)
    arr = (OraclePoint * n)(*[point_from_config(c) for c in cfgs])
    out = (OracleYield * n)()
    lib().oracle_points_batch_z(arr, n, int(nz), float(z_max), out, int(nthreads))
    return np.frombuffer(out, dtype=np.float64).reshape(n, 6).copy()


def yb_quadrature(cfg: dict, T_lo: float, T_hi: float, n_y: int = 8000, nz: int = NZ, z_max: float = Z_MAX,
                  aov: dict | None = None) -> float:
    """BoltzmannSystem.integrate_YB_by_quadrature (fpy:231-267) with bs.aov on (nz, z_max) and, if
    given, its own parameters `aov` (fpy:141-151)."""
    p = point_from_config(cfg)
    return lib().oracle_yb_quadrature_a(ctypes.byref(p), _ref(aov_from(aov)), float(T_lo), float(T_hi), int(n_y),
                                        int(nz), float(z_max))


def aov(I_p, beta_over_H, T_p, v_w, g_star, y, nz: int = NZ, z_max: float = Z_MAX) -> float:
    return lib().oracle_aov_z(I_p, beta_over_H, T_p, v_w, g_star, y, int(nz), float(z_max))


def p_closed_form(lam: float) -> float:
    return lib().oracle_p_closed_form(lam)


def j_chi(cfg: dict, T: float) -> float:
    p = point_from_config(cfg)
    return lib().oracle_j_chi(ctypes.byref(p), T)


def pairwise_sum(a) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().oracle_pairwise_sum(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.size)


def linspace(start, stop, num) -> np.ndarray:
    out = np.empty(num, dtype=np.float64)
    lib().oracle_linspace(start, stop, num, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return out


# ---- ODE fallback (fpy:200-219, 270-286, 385-417) -------------------------------------
class OracleOde(ctypes.Structure):
    _fields_ = [("sigma_v_chi_GeV_m2", ctypes.c_double), ("Gamma_wash_over_H", ctypes.c_double),
                ("deplete_DM_from_source", ctypes.c_int32), ("reserved", ctypes.c_int32)]


ODE_NT = 800
ODE_STATUS = {0: "ok", 1: "T grid not strictly increasing", 2: "max_step <= 0", 3: "too many steps",
              4: "Newton failure"}


def _ode_lib():
    L = lib()
    if not hasattr(L, "_ode_ready"):
        d, i32, i64, P = ctypes.c_double, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER
        L.oracle_ode_tables.restype = ctypes.c_int
        L.oracle_ode_tables.argtypes = [P(OraclePoint), d, d, P(d)]
        L.oracle_ode_aov_T.restype = d
        L.oracle_ode_aov_T.argtypes = [P(d), d, d, d]
        L.oracle_ode_rhs.restype = None
        L.oracle_ode_rhs.argtypes = [P(OraclePoint), P(OracleOde), P(d), d, d, d, P(d), P(d)]
        L.oracle_ode_point.restype = ctypes.c_int
        L.oracle_ode_point.argtypes = [P(OraclePoint), P(OracleOde), i64, P(OracleYield), P(i64)]
        L.oracle_ode_batch.restype = i64
        L.oracle_ode_batch.argtypes = [P(OraclePoint), P(OracleOde), i64, i64, P(OracleYield), P(i32), i32]
        L.oracle_ode_tables_z.restype = ctypes.c_int
        L.oracle_ode_tables_z.argtypes = [P(OraclePoint), d, d, i32, i64, d, P(d)]
        L.oracle_ode_aov_T_n.restype = d
        L.oracle_ode_aov_T_n.argtypes = [P(d), i32, d, d, d]
        L.oracle_ode_rhs_n.restype = None
        L.oracle_ode_rhs_n.argtypes = [P(OraclePoint), P(OracleOde), P(d), i32, d, d, d, P(d), P(d)]
        L.oracle_ode_point_z.restype = ctypes.c_int
        L.oracle_ode_point_z.argtypes = [P(OraclePoint), P(OracleOde), i64, d, i64, P(OracleYield), P(i64)]
        L.oracle_ode_tables_a.restype = ctypes.c_int
        L.oracle_ode_tables_a.argtypes = [P(OraclePoint), P(OracleAov), d, d, i32, i64, d, P(d)]
        L.oracle_ode_point_a.restype = ctypes.c_int
        L.oracle_ode_point_a.argtypes = [P(OraclePoint), P(OracleOde), P(OracleAov), i64, d, i64, P(OracleYield),
                                         P(i64)]
        L._ode_ready = True
    return L


def ode_from_config(cfg: dict) -> OracleOde:
    o = OracleOde()
    o.sigma_v_chi_GeV_m2 = float(cfg["sigma_v_chi_GeV_m2"])
    o.Gamma_wash_over_H = float(cfg["Gamma_wash_over_H"])
    o.deplete_DM_from_source = int(bool(cfg["deplete_DM_from_source"]))
    return o


def _window(cfg):
    T_p = float(cfg["T_p_GeV"])
    return float(cfg["T_min_over_Tp"]) * T_p, float(cfg["T_max_over_Tp"]) * T_p


def ode_tables(cfg: dict) -> np.ndarray:
    """build_tables -> (799, 4) PPoly coefficients (rows = intervals, cols = c0..c3)."""
    p = point_from_config(cfg)
    T_lo, T_hi = _window(cfg)
    coef = np.zeros(4 * ODE_NT)
    rc = _ode_lib().oracle_ode_tables(ctypes.byref(p), T_lo, T_hi, coef.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if rc != 0:
        raise ValueError("`x` must be strictly increasing sequence.")
    return coef[:4 * (ODE_NT - 1)].reshape(ODE_NT - 1, 4).copy()


def ode_rhs(cfg: dict, x: float, Y) -> tuple:
    p, o = point_from_config(cfg), ode_from_config(cfg)
    T_lo, T_hi = _window(cfg)
    coef = np.zeros(4 * ODE_NT)
    dp = ctypes.POINTER(ctypes.c_double)
    L = _ode_lib()
    L.oracle_ode_tables(ctypes.byref(p), T_lo, T_hi, coef.ctypes.data_as(dp))
    Yv = np.asarray(Y, dtype=np.float64)
    dY = np.zeros(2)
    L.oracle_ode_rhs(ctypes.byref(p), ctypes.byref(o), coef.ctypes.data_as(dp), T_lo, T_hi, float(x),
                     Yv.ctypes.data_as(dp), dY.ctypes.data_as(dp))
    return float(dY[0]), float(dY[1])


def ode_aov_T(cfg: dict, T: float) -> float:
    p = point_from_config(cfg)
    T_lo, T_hi = _window(cfg)
    coef = np.zeros(4 * ODE_NT)
    dp = ctypes.POINTER(ctypes.c_double)
    L = _ode_lib()
    L.oracle_ode_tables(ctypes.byref(p), T_lo, T_hi, coef.ctypes.data_as(dp))
    return L.oracle_ode_aov_T(coef.ctypes.data_as(dp), T_lo, T_hi, float(T))


class OdeTables:
    """build_tables(T_lo, T_hi, n=nt) with bs.aov on (nz, z_max) (fpy:207-212), then A_over_V_T
    (fpy:214-218) and rhs (fpy:270-286) on them."""

    def __init__(self, cfg: dict, T_lo: float, T_hi: float, nt: int = ODE_NT, nz: int = NZ, z_max: float = Z_MAX,
                 aov: dict | None = None):
        self.p, self.o = point_from_config(cfg), ode_from_config(cfg)
        self.T_lo, self.T_hi, self.nt = float(T_lo), float(T_hi), int(nt)
        self.coef = np.zeros(4 * self.nt)
        rc = _ode_lib().oracle_ode_tables_a(ctypes.byref(self.p), _ref(aov_from(aov)), self.T_lo, self.T_hi, self.nt,
                                            int(nz), float(z_max), self.coef.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        if rc != 0:
            raise ValueError("`x` must be strictly increasing sequence.")

    def aov_T(self, T: float) -> float:
        return _ode_lib().oracle_ode_aov_T_n(self.coef.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), self.nt,
                                             self.T_lo, self.T_hi, float(T))

    def rhs(self, x: float, Y) -> tuple:
        dp = ctypes.POINTER(ctypes.c_double)
        Yv = np.asarray(Y, dtype=np.float64)
        dY = np.zeros(2)
        _ode_lib().oracle_ode_rhs_n(ctypes.byref(self.p), ctypes.byref(self.o), self.coef.ctypes.data_as(dp), self.nt,
                                    self.T_lo, self.T_hi, float(x), Yv.ctypes.data_as(dp), dY.ctypes.data_as(dp))
        return float(dY[0]), float(dY[1])


def ode_point(cfg: dict, max_steps: int = 1 << 26, nz: int = NZ, z_max: float = Z_MAX, aov: dict | None = None) -> dict:
    p, o, out, ns = point_from_config(cfg), ode_from_config(cfg), OracleYield(), ctypes.c_int64()
    st = _ode_lib().oracle_ode_point_a(ctypes.byref(p), ctypes.byref(o), _ref(aov_from(aov)), int(nz), float(z_max),
                                       int(max_steps), ctypes.byref(out), ctypes.byref(ns))
    r = {n: getattr(out, n) for n in YIELD_FIELDS}
    r["status"], r["n_steps"] = st, ns.value
    return r


def ode_batch(cfgs: list[dict], max_steps: int = 1 << 26, nthreads: int = 0):
    n = len(cfgs)
    pts = (OraclePoint * n)(*[point_from_config(c) for c in cfgs])
    ods = (OracleOde * n)(*[ode_from_config(c) for c in cfgs])
    out = (OracleYield * n)()
    st = np.zeros(n, dtype=np.int32)
    _ode_lib().oracle_ode_batch(pts, ods, n, int(max_steps), out, st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                int(nthreads))
    return np.frombuffer(out, dtype=np.float64).reshape(n, 6).copy(), st
