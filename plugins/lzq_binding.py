"""lzq_binding -- reference-side ctypes binding of the lzq C ABI (include/lzq.h).

This is the file a maintainer of the reference drops next to first_principles_yields.py
("fpy") to run its hot operator on the MI355X.  It needs neither torch nor numpy: device
buffers come from hipMalloc through ctypes, and every number is computed by liblzq.so.

    import lzq_binding
    lzq_binding.install(first_principles_yields)   # BoltzmannSystem.integrate_YB_by_quadrature -> GPU

Entry points (each cites the fpy code it replaces):
  integrate_YB_by_quadrature(self, T_lo, T_hi, n_y=6000)  fpy:231-267 (method replacement; A/V from self.aov:
                                                          its own I_p, beta_over_H, T_p, v_w, g_star and z grid)
  build_tables(self, T_lo, T_hi, n=800)                   fpy:207-212 (method replacement: the n A/V knots in
                                                          one lzq_aov_batch call, the spline by fpy's CubicSpline)
  A_over_V_y(self, y)                                     fpy:158-165 (AoverVKernel method replacement, any z grid)
  aov_batch(aov, ys)                                      fpy:158-165 for many y in one call
  yields(cfg, P, T_lo=None, T_hi=None, n_y=8000, nz=1200, z_max=30.0, aov=None)
                                                          fpy:231-267 + fpy:372-384 + fpy:413-417
  ode_yields(cfg, P, aov=None, nz=1200, z_max=30.0, time_parallel=True)
                                                          fpy:385-417 (build_tables + the Radau solve +
                                                          densities) for one sigma_v / Gamma_wash /
                                                          depletion config
  p_closed_form(lams)                                     fpy:183-184
  lz_propagate(m_mix, dprime, xi, v_w, window_lz, steps)  no fpy counterpart (north_star (1))
  profile_crossings(knots, phi, Phi, y_B, y_chi, lam, v_w)  PAPER eqs.(5)-(8) (the absent modules of fpy:173)
  lz_propagate_profile(knots, phi, Phi, y_B, y_chi, lam, v_w) time-ordered P through a bounce profile
  install(fpy_module)                                     monkey-patches fpy's BoltzmannSystem and AoverVKernel

The library is found at $LZQ_LIB, else at <repo>/<package>/_build/liblzq.so next to this
file's directory.  Failures raise RuntimeError with lzq_last_error(); there is no CPU path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"
DEFAULT_LIB = os.path.join(os.path.dirname(_HERE), _PKG, "_build", "liblzq.so")

_H2D, _D2H = 1, 2  # hipMemcpyHostToDevice, hipMemcpyDeviceToHost


class lzq_point(ctypes.Structure):  # include/lzq.h: struct lzq_point (136 B)
    _fields_ = [(n, ctypes.c_double) for n in (
        "m_chi_GeV", "g_chi", "T_p_GeV", "beta_over_H", "v_w", "I_p", "g_star", "g_star_s",
        "P_chi_to_B", "source_shape_sigma_y", "incident_flux_scale", "T_max_over_Tp",
        "T_min_over_Tp", "Y_chi_init", "n_chi_at_Tp_GeV3")] + \
        [(n, ctypes.c_int32) for n in ("stats", "regime", "has_Y_chi_init", "has_n_chi_at_Tp")]


class lzq_aov_params(ctypes.Structure):  # include/lzq.h: struct lzq_aov_params (40 B)
    _fields_ = [(n, ctypes.c_double) for n in ("I_p", "beta_over_H", "T_p_GeV", "v_w", "g_star")]


class lzq_yield(ctypes.Structure):  # include/lzq.h: struct lzq_yield (48 B)
    _fields_ = [(n, ctypes.c_double) for n in ("Y_B", "Y_chi", "rho_B_kg_m3", "rho_DM_kg_m3", "DM_over_B",
                                                "P_used")]


class lzq_ode_params(ctypes.Structure):  # include/lzq.h: struct lzq_ode_params (24 B)
    _fields_ = [("sigma_v_chi_GeV_m2", ctypes.c_double), ("Gamma_wash_over_H", ctypes.c_double),
                ("deplete_DM_from_source", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class lzq_profile_point(ctypes.Structure):  # include/lzq.h: struct lzq_profile_point (40 B)
    _fields_ = [(n, ctypes.c_double) for n in ("y_B", "y_chi", "lambda_tr_eff", "v_w")] + \
        [(n, ctypes.c_int32) for n in ("shape", "reserved")]


assert ctypes.sizeof(lzq_point) == 136 and ctypes.sizeof(lzq_yield) == 48 and ctypes.sizeof(lzq_profile_point) == 40
assert ctypes.sizeof(lzq_aov_params) == 40 and ctypes.sizeof(lzq_ode_params) == 24
ODE_NT = 800                # LZQ_ODE_NT: main()'s build_tables knots (fpy:387)
ODE_WS_PER_POINT = 3200     # LZQ_ODE_WS_PER_POINT
ODE_STATUS = {0: "ok", 1: "bad_grid", 2: "bad_step", 3: "too_many_steps", 4: "newton", 5: "not_linear", 6: "unresolved",
              7: "bad_table"}  # enum lzq_ode_status
ABI_VERSION = 3  # include/lzq.h LZQ_ABI_VERSION this binding is written against

_hip = None
_lzq = None


def _libs():
    global _hip, _lzq
    if _lzq is None:
        hip = ctypes.CDLL("libamdhip64.so")
        path = os.environ.get("LZQ_LIB", DEFAULT_LIB)
        if not os.path.exists(path):
            raise RuntimeError(f"liblzq.so not found at {path} (build it, or set LZQ_LIB)")
        L = ctypes.CDLL(path)
        vp, i64, i32, d = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
        hip.hipFree.argtypes = [vp]
        hip.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
        hip.hipGetDevice.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.lzq_last_error.restype = ctypes.c_char_p
        L.lzq_abi_version.restype = ctypes.c_int
        L.lzq_init.argtypes = [ctypes.c_int]
        L.lzq_yields_batch.argtypes = [vp, i64, i32, i32, d, vp, vp, vp, vp, vp, vp]
        L.lzq_aov_batch.argtypes = [ctypes.POINTER(lzq_point), ctypes.POINTER(lzq_aov_params), vp, i64, i32, d, vp,
                                    vp]
        L.lzq_p_closed_form.argtypes = [vp, i64, vp, vp]
        L.lzq_ode_tables.argtypes = [vp, i64, vp, vp, i32, i32, d, vp, vp, i64, vp, vp]
        L.lzq_ode_integrate.argtypes = [vp, vp, i64, vp, i64, i64, vp, vp, vp]
        L.lzq_ode_integrate_tp.argtypes = [vp, vp, i64, vp, i64, vp, i64, i64, vp, vp, vp, vp]
        L.lzq_lz_propagate.argtypes = [vp, vp, vp, i64, i32, d, d, i32, vp, vp]
        L.lzq_profile_splines.argtypes = [vp, vp, vp, i32, i32, vp, vp, vp]
        L.lzq_profile_crossings.argtypes = [vp, vp, i32, i32, vp, i64, i32, vp, vp, vp, vp, vp, vp]
        L.lzq_lz_propagate_profile.argtypes = [vp, vp, i32, i32, vp, i64, d, i32, vp, vp]
        _ok(L.lzq_abi_version() == ABI_VERSION,
            f"liblzq.so ABI {L.lzq_abi_version()} != {ABI_VERSION} (rebuild the library or update the binding)")
        dev = ctypes.c_int(0)
        _ok(hip.hipGetDevice(ctypes.byref(dev)) == 0, "hipGetDevice failed (no GPU?)")
        _hip = hip
        _lzq = L
        _check(L.lzq_init(dev.value))
    return _hip, _lzq


def _ok(cond, msg):
    if not cond:
        raise RuntimeError(msg)


def _check(rc):
    if rc != 0:
        msg = _lzq.lzq_last_error() if _lzq is not None else b""
        raise RuntimeError(f"lzq error {rc}: {(msg or b'').decode()}")


class _Dev:
    """A device buffer holding a copy of a host ctypes object (freed on exit)."""

    def __init__(self, nbytes, host=None):
        hip, _ = _libs()
        self.p = ctypes.c_void_p()
        self.n = nbytes
        _ok(hip.hipMalloc(ctypes.byref(self.p), max(1, nbytes)) == 0, "hipMalloc failed")
        if host is not None:
            _ok(hip.hipMemcpy(self.p, ctypes.addressof(host), nbytes, _H2D) == 0, "hipMemcpy H2D failed")

    def read(self, host):
        # the null stream orders this after the launches on it (stream = NULL below)
        _ok(_hip.hipMemcpy(ctypes.addressof(host), self.p, self.n, _D2H) == 0, "hipMemcpy D2H failed")
        return host

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        _hip.hipFree(self.p)


def _doubles(xs):
    xs = [float(x) for x in xs]
    return (ctypes.c_double * len(xs))(*xs)


def point_from_cfg(c, P: float) -> lzq_point:
    """A reference Config (fpy:44-79) + the P it runs with -> lzq_point."""
    reg = str(c.regime).lower()
    return lzq_point(c.m_chi_GeV, c.g_chi, c.T_p_GeV, c.beta_over_H, c.v_w, c.I_p, c.g_star, c.g_star_s,
                     float(P), c.source_shape_sigma_y, c.incident_flux_scale, c.T_max_over_Tp, c.T_min_over_Tp,
                     0.0 if c.Y_chi_init is None else float(c.Y_chi_init),
                     0.0 if c.n_chi_at_Tp_GeV3 is None else float(c.n_chi_at_Tp_GeV3),
                     0 if str(c.chi_stats).lower().startswith("ferm") else 1,
                     0 if reg.startswith("therm") else (1 if reg.startswith("non") else 2),
                     int(c.Y_chi_init is not None), int(c.n_chi_at_Tp_GeV3 is not None))


def aov_params(aov) -> lzq_aov_params:
    """A reference AoverVKernel (fpy:141-151: attributes I_p, beta_over_H, T_p, v_w, g_star) ->
    lzq_aov_params."""
    return lzq_aov_params(float(aov.I_p), float(aov.beta_over_H), float(aov.T_p), float(aov.v_w), float(aov.g_star))


def yields(cfg, P: float, T_lo=None, T_hi=None, n_y: int = 8000, nz: int = 1200, z_max: float = 30.0,
           aov=None) -> dict:
    """fpy:231-267 (Y_B) + fpy:372-384, 413-417 (Y_chi, densities) for one config on the GPU
    (T_lo/T_hi default to main()'s window, fpy:367-369), A/V on the z grid linspace(0, z_max, nz)
    (fpy:141-156) with the A/V kernel's own parameters `aov` (an AoverVKernel; None: cfg's own,
    fpy:197)."""
    _, L = _libs()
    pt = point_from_cfg(cfg, P)
    out = lzq_yield()
    tl, th = ctypes.c_double(T_lo or 0.0), ctypes.c_double(T_hi or 0.0)
    ap = aov_params(aov) if aov is not None else lzq_aov_params()
    with _Dev(136, pt) as d_pt, _Dev(8, tl) as d_tl, _Dev(8, th) as d_th, _Dev(40, ap) as d_aov, _Dev(48) as d_out:
        _check(L.lzq_yields_batch(d_pt.p, 1, int(n_y), int(nz), float(z_max), d_tl.p if T_lo is not None else None,
                                  d_th.p if T_hi is not None else None, None, d_aov.p if aov is not None else None,
                                  d_out.p, None))
        d_out.read(out)
    return {n: getattr(out, n) for n, _ in lzq_yield._fields_}


def zgrid_of(aov) -> tuple:
    """(nz, z_max) of a reference AoverVKernel from its z array (fpy:154: linspace sets
    z[-1] = z_max exactly; with fewer than 2 nodes A/V is 0 whatever z_max is)."""
    z = aov.z
    nz = len(z)
    return nz, (float(z[-1]) if nz >= 2 else 0.0)


def integrate_YB_by_quadrature(self, T_lo: float, T_hi: float, n_y: int = 6000) -> float:
    """Drop-in for BoltzmannSystem.integrate_YB_by_quadrature (fpy:231-267): same arguments,
    same result (north_star tolerance 1e-8; measured ~1e-13), computed by lzq_yields_batch on
    self.aov's z grid (any AoverVKernel(..., z_max, nz))."""
    nz, z_max = zgrid_of(self.aov)
    return yields(self.cfg, self.P, T_lo, T_hi, n_y, nz, z_max, aov=self.aov)["Y_B"]


def aov_batch(aov, ys) -> list:
    """A_over_V_y (fpy:158-165) of the AoverVKernel `aov` (its own parameters and z grid) at every
    y, in one lzq_aov_batch launch."""
    _, L = _libs()
    nz, z_max = zgrid_of(aov)
    h = _doubles(ys)
    n = len(h)
    out = (ctypes.c_double * max(n, 1))()
    ap = aov_params(aov)
    if n == 0:
        return []
    with _Dev(8 * n, h) as d_y, _Dev(8 * n) as d_out:
        _check(L.lzq_aov_batch(None, ctypes.byref(ap), d_y.p, n, nz, z_max, d_out.p, None))
        d_out.read(out)
    return list(out)[:n]


def A_over_V_y(self, y: float) -> float:
    """Drop-in for AoverVKernel.A_over_V_y (fpy:158-165) on the kernel's own z grid
    (lzq_aov_batch).  Reads I_p, beta_over_H, T_p, v_w and g_star from the kernel object.  One
    launch per call: batch callers (build_tables below) use aov_batch."""
    return aov_batch(self, [y])[0]


def make_build_tables(fpy_module):
    """Drop-in for BoltzmannSystem.build_tables (fpy:207-212) of `fpy_module`: the same Ts
    (np.linspace) and y(T) (fpy's y_of_T, from self.cfg), A/V of self.aov at all n knots in one
    lzq_aov_batch launch (instead of n scalar A_over_V_y round trips), and fpy's own
    CubicSpline(Ts, np.maximum(Av, 0.0), extrapolate=True)."""
    def build_tables(self, T_lo: float, T_hi: float, n: int = 800):
        np = fpy_module.np
        self._T_lo, self._T_hi = float(T_lo), float(T_hi)
        Ts = np.linspace(self._T_lo, self._T_hi, n)
        ys = [fpy_module.y_of_T(T, self.cfg.T_p_GeV, self.cfg.beta_over_H) for T in Ts]
        Av = np.array(aov_batch(self.aov, ys), float)
        self._A_spline = fpy_module.CubicSpline(Ts, np.maximum(Av, 0.0), extrapolate=True)

    return build_tables


def ode_steps(cfg) -> int:
    """The fixed Radau step count of fpy:403-404's window for a config: x0 = m/T_hi, x1 = m/T_lo,
    max_step = min(|x1 - x0|/20000, x_p/1000, 5e-4), N = ceil(|x1 - x0| / max_step) -- the integrator's
    own expression (0 when the window is degenerate; the library then reports the status)."""
    import math
    m, Tp = float(cfg.m_chi_GeV), float(cfg.T_p_GeV)
    T_hi, T_lo = float(cfg.T_max_over_Tp) * Tp, float(cfg.T_min_over_Tp) * Tp
    x0, x1 = m / T_hi, m / max(T_lo, 1e-30)
    x_p = m / max(Tp, 1e-30)
    ms = min(min(abs(x1 - x0) / 20000.0, x_p / 1000.0), 5e-4)
    n = abs(x1 - x0) / ms if ms > 0.0 else float("nan")
    return int(math.ceil(n)) if math.isfinite(n) else 0


def ode_yields(cfg, P: float, aov=None, nz: int = 1200, z_max: float = 30.0, time_parallel: bool = True) -> dict:
    """fpy:385-417 for one config on the GPU: build_tables(T_lo, T_hi, n=800) of the A/V kernel
    (`aov`: an AoverVKernel with its own parameters and z grid, None: cfg's own on (nz, z_max)), the
    reference's Radau IIA on its fixed-step window (fpy:403-404), Y_chi(x1), Y_B(x1) and the
    densities; plus "status" (enum lzq_ode_status name).  time_parallel (default): the few-point
    latency path lzq_ode_integrate_tp (the sequential steps' bits; the shipped window's sigma_v != 0
    point in milliseconds instead of ~0.8 s); False: lzq_ode_integrate."""
    _, L = _libs()
    if aov is not None:
        nz, z_max = zgrid_of(aov)
    pt = point_from_cfg(cfg, P)
    od = lzq_ode_params(max(float(cfg.sigma_v_chi_GeV_m2), 0.0), max(float(cfg.Gamma_wash_over_H), 0.0),
                        int(bool(cfg.deplete_DM_from_source)), 0)
    ap = aov_params(aov) if aov is not None else lzq_aov_params()
    out, st = lzq_yield(), ctypes.c_int32(-1)
    max_steps = ode_steps(cfg) + 64
    with _Dev(136, pt) as d_pt, _Dev(24, od) as d_od, _Dev(40, ap) as d_aov, _Dev(8 * ODE_WS_PER_POINT) as d_w, \
            _Dev(48) as d_out, _Dev(4) as d_st:
        _check(L.lzq_ode_tables(d_pt.p, 1, None, None, ODE_NT, int(nz), float(z_max),
                                d_aov.p if aov is not None else None, d_w.p, ODE_WS_PER_POINT, d_st.p, None))
        if time_parallel:
            _check(L.lzq_ode_integrate_tp(d_pt.p, d_od.p, 1, None, 0, d_w.p, ODE_WS_PER_POINT, max_steps, d_out.p,
                                          d_st.p, None, None))
        else:
            _check(L.lzq_ode_integrate(d_pt.p, d_od.p, 1, d_w.p, ODE_WS_PER_POINT, max_steps, d_out.p, d_st.p, None))
        d_out.read(out)
        d_st.read(st)
    res = {n: getattr(out, n) for n, _ in lzq_yield._fields_}
    res["status"] = ODE_STATUS.get(st.value, str(st.value))
    return res


def p_closed_form(lams) -> list:
    """fpy:183-184 on the GPU: clamp(1 - exp(-2 pi max(lambda, 0)), 0, 1) per entry."""
    _, L = _libs()
    h = _doubles(lams)
    n = len(h)
    out = (ctypes.c_double * n)()
    with _Dev(8 * n, h) as d_l, _Dev(8 * n) as d_p:
        _check(L.lzq_p_closed_form(d_l.p, n, d_p.p, None))
        d_p.read(out)
    return list(out)


def lz_propagate(m_mix, dprime, xi, v_w: float, window_lz: float = 20.0, steps: int = 1000) -> float:
    """Coherent conversion probability through the crossings of ONE profile
    (lzq_lz_propagate; xi increasing).  One crossing: 1 - exp(-2 pi delta) to <= 1e-8."""
    _, L = _libs()
    n_cross = len(m_mix)
    _ok(n_cross > 0 and len(dprime) == n_cross and len(xi) == n_cross, "need equal-length crossing lists")
    m, d, x = _doubles(m_mix), _doubles(dprime), _doubles(xi)
    P = ctypes.c_double()
    with _Dev(8 * n_cross, m) as d_m, _Dev(8 * n_cross, d) as d_d, _Dev(8 * n_cross, x) as d_x, _Dev(8) as d_P:
        _check(L.lzq_lz_propagate(d_m.p, d_d.p, d_x.p, 1, n_cross, float(v_w), float(window_lz), int(steps),
                                  d_P.p, None))
        d_P.read(P)
    return P.value


class _Shape:
    """One bounce profile on the device: knots + the not-a-knot splines of phi, Phi."""

    def __init__(self, knots, phi, Phi):
        _, L = _libs()
        n = len(knots)
        _ok(n >= 4 and len(phi) == n and len(Phi) == n, "a profile needs >= 4 knots and equal-length columns")
        self.n = n
        self.x = _Dev(8 * n, _doubles(knots))
        self.coef = _Dev(8 * 8 * (n - 1))
        bad = ctypes.c_int32()
        with _Dev(8 * n, _doubles(phi)) as d_a, _Dev(8 * n, _doubles(Phi)) as d_b, _Dev(4) as d_bad:
            _check(L.lzq_profile_splines(self.x.p, d_a.p, d_b.p, 1, n, self.coef.p, d_bad.p, None))
            d_bad.read(bad)
        if bad.value:
            self.close()
            raise ValueError("profile knots must be strictly increasing (scipy CubicSpline rule)")

    def close(self):
        self.x.__exit__()
        self.coef.__exit__()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def profile_crossings(knots, phi, Phi, y_B, y_chi, lambda_tr_eff, v_w, max_cross: int = 256) -> list:
    """PAPER eqs.(5)-(8) on the GPU: [(xi*, Delta'*, m_mix(xi*), delta_LZ)] of every sign change
    of Delta = y_B phi - y_chi Phi, phi and Phi not-a-knot cubic splines of the samples."""
    _, L = _libs()
    pt = lzq_profile_point(y_B, y_chi, lambda_tr_eff, v_w, 0, 0)
    cnt = ctypes.c_int32()
    with _Shape(knots, phi, Phi) as sh, _Dev(40, pt) as d_pt, _Dev(4) as d_cnt, \
            _Dev(8 * max_cross) as d_x, _Dev(8 * max_cross) as d_d, _Dev(8 * max_cross) as d_m, _Dev(8 * max_cross) as d_l:
        _check(L.lzq_profile_crossings(sh.x.p, sh.coef.p, 1, sh.n, d_pt.p, 1, max_cross, d_x.p, d_d.p, d_m.p, d_l.p,
                                       d_cnt.p, None))
        d_cnt.read(cnt)
        _ok(cnt.value <= max_cross, f"more than {max_cross} crossings")
        cols = []
        for dv in (d_x, d_d, d_m, d_l):
            h = (ctypes.c_double * max_cross)()
            dv.read(h)
            cols.append(list(h)[:cnt.value])
    return list(zip(*cols))


def lz_propagate_profile(knots, phi, Phi, y_B, y_chi, lambda_tr_eff, v_w, steps_per_radian: float = 4.0,
                         min_steps: int = 1) -> float:
    """Time-ordered conversion probability through the whole bounce profile
    (lzq_lz_propagate_profile): H = Delta(xi) sz + m_mix(xi) sx, xi = v_w t."""
    _, L = _libs()
    pt = lzq_profile_point(y_B, y_chi, lambda_tr_eff, v_w, 0, 0)
    P = ctypes.c_double()
    with _Shape(knots, phi, Phi) as sh, _Dev(40, pt) as d_pt, _Dev(8) as d_P:
        _check(L.lzq_lz_propagate_profile(sh.x.p, sh.coef.p, 1, sh.n, d_pt.p, 1, float(steps_per_radian),
                                          int(min_steps), d_P.p, None))
        d_P.read(P)
    return P.value


def install(fpy_module) -> None:
    """Route the reference's quadrature operator, its ODE tables and its A/V kernel through the GPU
    (INTEGRATION.md §2)."""
    fpy_module.BoltzmannSystem.integrate_YB_by_quadrature = integrate_YB_by_quadrature
    fpy_module.BoltzmannSystem.build_tables = make_build_tables(fpy_module)
    fpy_module.AoverVKernel.A_over_V_y = A_over_V_y
