"""ctypes binding of the lzq C ABI (include/lzq.h) -> `_build/liblzq.so`.

There is no fallback: if the HIP library is missing or fails to load, every entry point
raises.  Structures mirror include/lzq.h field for field (sizes are asserted).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import build as _build

LIB_PATH = _build.LIB_PATH

# ---- struct mirrors of include/lzq.h ---------------------------------------------------
POINT_DOUBLE_FIELDS = (
    "m_chi_GeV", "g_chi", "T_p_GeV", "beta_over_H", "v_w", "I_p", "g_star", "g_star_s",
    "P_chi_to_B", "source_shape_sigma_y", "incident_flux_scale", "T_max_over_Tp",
    "T_min_over_Tp", "Y_chi_init", "n_chi_at_Tp_GeV3")
POINT_INT_FIELDS = ("stats", "regime", "has_Y_chi_init", "has_n_chi_at_Tp")
YIELD_FIELDS = ("Y_B", "Y_chi", "rho_B_kg_m3", "rho_DM_kg_m3", "DM_over_B", "P_used")


class LzqPoint(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in POINT_DOUBLE_FIELDS] + \
               [(n, ctypes.c_int32) for n in POINT_INT_FIELDS]


class LzqYield(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in YIELD_FIELDS]


class LzqAxis(ctypes.Structure):
    _fields_ = [("field", ctypes.c_int32), ("n", ctypes.c_int32), ("values", ctypes.c_void_p)]


AOV_FIELDS = ("I_p", "beta_over_H", "T_p_GeV", "v_w", "g_star")


class LzqAovParams(ctypes.Structure):  # struct lzq_aov_params: AoverVKernel's own fields (fpy:141-151)
    _fields_ = [(n, ctypes.c_double) for n in AOV_FIELDS]


AOV_DTYPE = np.dtype([(n, "<f8") for n in AOV_FIELDS])
assert ctypes.sizeof(LzqAovParams) == 40 == AOV_DTYPE.itemsize


class LzqOdeParams(ctypes.Structure):
    _fields_ = [("sigma_v_chi_GeV_m2", ctypes.c_double), ("Gamma_wash_over_H", ctypes.c_double),
                ("deplete_DM_from_source", ctypes.c_int32), ("reserved", ctypes.c_int32)]


ODE_DTYPE = np.dtype([("sigma_v_chi_GeV_m2", "<f8"), ("Gamma_wash_over_H", "<f8"),
                      ("deplete_DM_from_source", "<i4"), ("reserved", "<i4")])
assert ctypes.sizeof(LzqOdeParams) == 24 == ODE_DTYPE.itemsize
ODE_NT, ODE_WS_PER_POINT = 800, 3200  # LZQ_ODE_NT, LZQ_ODE_WS_PER_POINT
ODE_OK, ODE_BAD_GRID, ODE_BAD_STEP, ODE_TOO_MANY_STEPS, ODE_NEWTON, ODE_NOT_LINEAR, ODE_UNRESOLVED, ODE_BAD_TABLE = \
    range(8)  # enum lzq_ode_status
ODE_STATUS = {0: "ok", 1: "`x` must be strictly increasing sequence.", 2: "`max_step` must be positive.",
              3: "more than max_steps integration steps", 4: "Radau stage Newton iteration did not converge",
              5: "sigma_v != 0: the quadrature form needs a linear Y_chi equation",
              6: "quadrature form: a knot interval needs more than 4096 sub-intervals",
              7: "spline table not built for LZQ_ODE_NT knots"}

# struct lzq_profile_point (40 B): a bounce-profile shape + the couplings of PAPER eqs.(5)-(8)
PROFILE_POINT_DTYPE = np.dtype([("y_B", "<f8"), ("y_chi", "<f8"), ("lambda_tr_eff", "<f8"), ("v_w", "<f8"),
                                ("shape", "<i4"), ("reserved", "<i4")])
assert PROFILE_POINT_DTYPE.itemsize == 40
PROFILE_COEF = 8  # doubles per knot-interval row: (phi c0..c3, Phi c0..c3)

POINT_DTYPE = np.dtype([(n, "<f8") for n in POINT_DOUBLE_FIELDS] + [(n, "<i4") for n in POINT_INT_FIELDS])
assert ctypes.sizeof(LzqPoint) == 136 == POINT_DTYPE.itemsize
assert ctypes.sizeof(LzqYield) == 48

# enum lzq_field
FIELD = {n: i for i, n in enumerate(POINT_DOUBLE_FIELDS)}
FIELD.update({"delta_LZ": 32, "m_mix": 33, "dprime": 34})
FERMION, BOSON = 0, 1
THERMAL, NONTHERMAL, REGIME_OTHER = 0, 1, 2
LZQ_NZ, LZQ_Z_MAX = 1200, 30.0  # fpy:142 AoverVKernel defaults, main()'s grid (fpy:197)
LZQ_NZ_MAX = 1 << 22
ODE_NT_MAX = 1 << 20
REUSE_TABLE_HEADER = 6  # LZQ_REUSE_TABLE_HEADER
(TUNE_EXP, TUNE_TRUNCATE, TUNE_ODE_COOP, TUNE_ODE_LAUNCH_STEPS, TUNE_PROFILE_FLAT, TUNE_ODE_TP_INTERVAL,
 TUNE_ODE_TABLE_WIDE) = 0, 1, 2, 3, 4, 5, 6  # enum lzq_tune_key
ODE_MAX_LAUNCHES = 65536  # lzq_ode_*: max_steps <= 65536 x 2^(launch log2)
# tuning state that changes result bits (the inner-loop exponential, ~1e-14): part of the
# sweep checkpoint key (sweep.spec_key); Engine.tune_exp keeps it current
TUNE_STATE = {"exp": "table"}


_loaded_path = None   # the library load() opened last (what the engines run)


def library_id(path: str | None = None) -> str | None:
    """sha256 (16 hex) of every device code object (build.ARCH) in the library the engine loaded
    (else `path`, else LIB_PATH): changes whenever any kernel's machine code does
    (sweep.spec_key: checkpoints of another build are never mixed in).  A library with no such
    uncompressed bundle entry (another arch, compressed bundles) is hashed whole, never as the
    empty input."""
    import hashlib
    from . import codeobj
    p = path or _loaded_path or LIB_PATH
    if not os.path.exists(p):
        return None
    objs = codeobj.device_objects(p, _build.ARCH)
    h = hashlib.sha256()
    if objs:
        for obj in objs:
            h.update(obj)
    else:
        with open(p, "rb") as f:
            h.update(b"whole-file:" + f.read())
    return h.hexdigest()[:16]
EXP_POLY11, EXP_TABLE = 0, 1  # enum lzq_exp_variant
LZQ_MAX_AXES = 8
ABI_VERSION = 3  # LZQ_ABI_VERSION (tests/test_capi.py checks it against the library)

# Symbols declared in include/lzq.h (checked by tests/test_capi.py against the header).
EXPORTS = ("lzq_abi_version", "lzq_last_error", "lzq_init", "lzq_zgrid_init", "lzq_ztables", "lzq_tune", "lzq_aov_batch",
           "lzq_jchi_batch", "lzq_yields_batch", "lzq_sweep_grid", "lzq_sweep_grid_reuse_workspace",
           "lzq_sweep_grid_reuse", "lzq_sweep_grid_ztables", "lzq_sweep_grid_from_ztables",
           "lzq_yields_batch_reuse", "lzq_p_closed_form",
           "lzq_lz_propagate", "lzq_lz_propagate_v", "lzq_ode_tables", "lzq_ode_integrate", "lzq_ode_integrate_shared", "lzq_ode_rows", "lzq_ode_integrate_rows", "lzq_ode_integrate_tp", "lzq_ode_quadrature", "lzq_ode_batch",
           "lzq_ode_aov_T", "lzq_ode_rhs", "lzq_profile_splines", "lzq_profile_crossings",
           "lzq_lz_propagate_profile")
# the lzq_point fields an ODE spline table depends on (A/V kernel fpy:141-156 + window fpy:368-369)
ODE_TABLE_KEY = ("I_p", "beta_over_H", "T_p_GeV", "v_w", "g_star", "T_min_over_Tp", "T_max_over_Tp")
# the lzq_point fields the quadrature's z-sums depend on (its y-grid and c; lzq_yields_batch_reuse)
ZSUM_KEY = ("I_p", "beta_over_H", "T_p_GeV", "T_min_over_Tp", "T_max_over_Tp")
# every point field the ODE integrator's stage ingredients read besides P, flux and the ODE
# parameters (ode_stage_base / ode_stage_chi_base + the spline table): points equal in these can
# share a cooperative wavefront (include/lzq.h LZQ_TUNE_ODE_COOP)
ODE_STAGE_KEY = ODE_TABLE_KEY + ("m_chi_GeV", "g_chi", "g_star_s", "source_shape_sigma_y", "stats")
# the stage key without the fields that enter only through the spline table: points equal in these
# share a cooperative segment even when their tables differ (round 4: each lane then scales the
# shared rows by its own table's A/V, ode_integrate_kernel tab_vary)
ODE_COOP_KEY = tuple(f for f in ODE_STAGE_KEY if f not in ("I_p", "v_w"))


class LzqError(RuntimeError):
    """A negative status from the C ABI (message from lzq_last_error())."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"lzq error {code}: {msg}")
        self.code = code


_lib = None


def load(path: str | None = None):
    """Load liblzq.so (does not touch the GPU).  Raises if the library is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"lzq HIP library not built ({p}); run __graft_entry__.build() "
                           "or python -m <package>.build")
    L = ctypes.CDLL(p)
    global _loaded_path
    _loaded_path = p
    i32, i64, d, vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
    P = ctypes.POINTER
    L.lzq_abi_version.restype = ctypes.c_int
    L.lzq_last_error.restype = ctypes.c_char_p
    L.lzq_init.argtypes = [ctypes.c_int]
    L.lzq_zgrid_init.argtypes = [ctypes.c_int, i32, d]
    L.lzq_ztables.argtypes = [i32, d, P(d), P(d), P(d)]
    L.lzq_tune.argtypes = [i32, i32]
    L.lzq_aov_batch.argtypes = [P(LzqPoint), P(LzqAovParams), vp, i64, i32, d, vp, vp]
    L.lzq_jchi_batch.argtypes = [P(LzqPoint), vp, i64, vp, vp]
    L.lzq_yields_batch.argtypes = [vp, i64, i32, i32, d, vp, vp, vp, vp, vp, vp]
    L.lzq_sweep_grid.argtypes = [P(LzqPoint), P(LzqAxis), i32, i64, i64, i32, i32, d, vp, vp, vp]
    L.lzq_sweep_grid_reuse_workspace.argtypes = [P(LzqAxis), i32, i32]
    L.lzq_sweep_grid_reuse.argtypes = [P(LzqPoint), P(LzqAxis), i32, i64, i64, i32, i32, d, vp, vp, i64, vp, vp]
    L.lzq_sweep_grid_ztables.argtypes = [P(LzqPoint), P(LzqAxis), i32, i32, i32, d, vp, i64, vp]
    L.lzq_sweep_grid_from_ztables.argtypes = [P(LzqPoint), P(LzqAxis), i32, i64, i64, i32, i32, d, vp, vp, i64, vp,
                                              vp]
    L.lzq_yields_batch_reuse.argtypes = [vp, i64, i32, i32, d, vp, vp, vp, i64, vp, i64, vp, vp]
    L.lzq_p_closed_form.argtypes = [vp, i64, vp, vp]
    L.lzq_lz_propagate.argtypes = [vp, vp, vp, i64, i32, d, d, i32, vp, vp]
    L.lzq_lz_propagate_v.argtypes = [vp, vp, vp, vp, i64, i32, d, i32, vp, vp]
    L.lzq_ode_tables.argtypes = [vp, i64, vp, vp, i32, i32, d, vp, vp, i64, vp, vp]
    L.lzq_ode_integrate.argtypes = [vp, vp, i64, vp, i64, i64, vp, vp, vp]
    L.lzq_ode_integrate_shared.argtypes = [vp, vp, i64, vp, i64, vp, i64, i64, vp, vp, vp]
    L.lzq_ode_rows.argtypes = [vp, vp, i64, vp, i64, vp, i64, vp, vp, i64, i64, vp, i64, vp]
    L.lzq_ode_integrate_rows.argtypes = [vp, vp, i64, vp, i64, vp, i64, i64, vp, vp, vp, i64, vp, i64, vp, vp, vp]
    L.lzq_ode_integrate_tp.argtypes = [vp, vp, i64, vp, i64, vp, i64, i64, vp, vp, vp, vp]
    L.lzq_ode_quadrature.argtypes = [vp, vp, i64, vp, i64, vp, i64, i64, vp, vp, vp]
    L.lzq_ode_batch.argtypes = [vp, vp, i64, i32, d, vp, vp, i64, i64, vp, vp, vp]
    L.lzq_ode_aov_T.argtypes = [P(LzqPoint), d, d, i32, vp, vp, i64, vp, vp]
    L.lzq_ode_rhs.argtypes = [P(LzqPoint), P(LzqOdeParams), d, d, i32, vp, vp, vp, i64, vp, vp]
    L.lzq_profile_splines.argtypes = [vp, vp, vp, i32, i32, vp, vp, vp]
    L.lzq_profile_crossings.argtypes = [vp, vp, i32, i32, vp, i64, i32, vp, vp, vp, vp, vp, vp]
    L.lzq_lz_propagate_profile.argtypes = [vp, vp, i32, i32, vp, i64, d, i32, vp, vp]
    for name in EXPORTS:
        if name not in ("lzq_abi_version", "lzq_last_error"):
            getattr(L, name).restype = ctypes.c_int
    L.lzq_sweep_grid_reuse_workspace.restype = ctypes.c_int64
    if path is None:
        _lib = L
    return L


def check(rc: int, lib=None) -> None:
    if rc != 0:
        msg = (lib or load()).lzq_last_error()
        raise LzqError(rc, msg.decode() if msg else "")


def ztables(nz: int = LZQ_NZ, z_max: float = LZQ_Z_MAX) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Host copies of the z grid, gamma4 and the quadrature weights the library builds for the
    A/V kernel's grid linspace(0, z_max, nz) (fpy:154-156)."""
    n = max(int(nz), 0)
    z, g4, om = (np.empty(n) for _ in range(3))
    dp = ctypes.POINTER(ctypes.c_double)
    check(load().lzq_ztables(int(nz), float(z_max), z.ctypes.data_as(dp), g4.ctypes.data_as(dp),
                             om.ctypes.data_as(dp)))
    return z, g4, om


def zgrid(nz, z_max) -> tuple[int, float]:
    """Validate an AoverVKernel (nz, z_max) the way numpy's linspace takes them (fpy:154): nz an
    integer (operator.index, TypeError otherwise) >= 0 (ValueError), z_max a float."""
    import operator
    n = operator.index(nz)
    if n < 0:
        raise ValueError(f"Number of samples, {n}, must be non-negative.")
    return int(n), float(z_max)
