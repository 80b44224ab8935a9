"""Device-side plumbing around the C ABI: torch-ROCm tensors as device buffers, torch's
current HIP stream as the launch stream.  Torch is plumbing only; every number is computed
by the HIP kernels in csrc/.  There is no CPU path: constructing an Engine without a GPU,
or without the built library, raises.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np
import torch

import logging

from . import _native
from .config import to_aov, to_ctypes_aov, to_ctypes_ode, to_ctypes_point, to_point

_log = logging.getLogger("lzq")

YIELD_FIELDS = _native.YIELD_FIELDS


def _vp(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class Engine:
    """One engine per process/device (torch.cuda.current_device() unless given)."""

    def __init__(self, device: Optional[int] = None, lib_path: Optional[str] = None):
        if not torch.cuda.is_available():
            raise RuntimeError("lzq Engine needs a ROCm GPU (torch.cuda.is_available() is False); "
                               "there is no CPU fallback")
        self.lib = _native.load(lib_path)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self._zwork = None  # lzq_sweep_grid_reuse's z-sum tables (grown on demand)
        self._ztab_key = None  # the grid whose tables _zwork holds (Engine.sweep reuse)
        self._exp_variant = "table"
        self.last_reuse = None
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_init(self.device.index))

    def tune_exp(self, variant: str) -> str:
        """Select the inner-loop exponential ('table' default, 'poly11'); returns the previous."""
        v = {"poly11": _native.EXP_POLY11, "table": _native.EXP_TABLE}[variant]
        prev = self.lib.lzq_tune(_native.TUNE_EXP, v)
        if prev < 0:
            self._check(prev)
        self._exp_variant = variant
        _native.TUNE_STATE["exp"] = variant
        return {_native.EXP_POLY11: "poly11", _native.EXP_TABLE: "table"}[prev]

    def tune_ode_coop(self, on: bool) -> bool:
        """Cooperative stage tables in the ODE integrator (include/lzq.h LZQ_TUNE_ODE_COOP; on by
        default, bit-identical results either way).  Returns the previous setting."""
        prev = self.lib.lzq_tune(_native.TUNE_ODE_COOP, 1 if on else 0)
        if prev < 0:
            self._check(prev)
        return bool(prev)

    def tune_ode_table_wide(self, on) -> int:
        """Few ODE tables (<= 4096) built wide (include/lzq.h LZQ_TUNE_ODE_TABLE_WIDE): True / 3 both,
        1 the A/V knots over 64-knot wavefronts, 2 the spline around its two recurrences over a
        wavefront, False / 0 neither; bit-identical tables either way.  Returns the previous mask."""
        v = 3 if on is True else (0 if on is False else int(on))
        prev = self.lib.lzq_tune(_native.TUNE_ODE_TABLE_WIDE, v)
        if prev < 0:
            self._check(prev)
        return prev

    def tune_ode_launch_steps(self, log2: int) -> int:
        """Fixed Radau steps per ODE continuation launch, as a power of two (include/lzq.h
        LZQ_TUNE_ODE_LAUNCH_STEPS, default 24; bit-identical results).  Returns the previous."""
        prev = self.lib.lzq_tune(_native.TUNE_ODE_LAUNCH_STEPS, int(log2))
        if prev < 0:
            self._check(prev)
        self._ode_launch_log2 = int(log2)
        return prev

    def tune_profile_flat(self, on: bool) -> bool:
        """lzq_lz_propagate_profile's flattened propagation (include/lzq.h LZQ_TUNE_PROFILE_FLAT; off by
        default -- the interval loop in keyed launch order is faster, DESIGN §4.5 -- bit-identical P
        either way).  Returns the previous setting."""
        prev = self.lib.lzq_tune(_native.TUNE_PROFILE_FLAT, 1 if on else 0)
        if prev < 0:
            self._check(prev)
        return bool(prev)

    def tune_truncate(self, on: bool) -> bool:
        """Exact-underflow truncation of the z-sums (bit-identical results, fewer nodes
        executed; include/lzq.h LZQ_TUNE_TRUNCATE).  Returns the previous setting."""
        prev = self.lib.lzq_tune(_native.TUNE_TRUNCATE, 1 if on else 0)
        if prev < 0:
            self._check(prev)
        return bool(prev)

    # -- helpers -------------------------------------------------------------------------
    def _check(self, rc: int) -> None:
        _native.check(rc, self.lib)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _f64(self, x) -> torch.Tensor:
        t = torch.as_tensor(np.asarray(x, dtype=np.float64) if not isinstance(x, torch.Tensor) else x,
                            dtype=torch.float64)
        return t.to(self.device).contiguous()

    def points_to_device(self, recs: np.ndarray) -> torch.Tensor:
        """lzq_point records (numpy POINT_DTYPE array) -> device byte tensor."""
        return _to_device_bytes(np.ascontiguousarray(recs, dtype=_native.POINT_DTYPE), self.device)

    def aov_to_device(self, aov, n: int) -> Optional[torch.Tensor]:
        """The A/V kernels of n points (include/lzq.h lzq_aov_params) as a device byte tensor, or
        None.  aov: None (each point's own fields, fpy:197), one kernel for every point (an
        AoverVKernel, a dict or Config, or a 1-record AOV_DTYPE array), or n AOV_DTYPE records."""
        if aov is None:
            return None
        if isinstance(aov, torch.Tensor):
            if aov.numel() != n * _native.AOV_DTYPE.itemsize:
                raise ValueError("aov: need one lzq_aov_params record per point")
            return aov
        rec = aov if isinstance(aov, np.ndarray) and aov.dtype == _native.AOV_DTYPE else to_aov(aov)
        rec = np.ascontiguousarray(rec, dtype=_native.AOV_DTYPE).reshape(-1)
        if rec.size == 1 and n != 1:
            rec = np.repeat(rec, n)
        if rec.size != n:
            raise ValueError(f"aov: {rec.size} records for {n} points")
        return _to_device_bytes(rec, self.device)

    # -- fpy:158-165 -----------------------------------------------------------------------
    def aov(self, kernel, ys, nz: int = _native.LZQ_NZ, z_max: float = _native.LZQ_Z_MAX) -> torch.Tensor:
        """A_over_V_y at every y for the kernel AoverVKernel(I_p, beta_over_H, T_p, v_w, g_star, z_max, nz)
        (fpy:141-165); kernel: an AoverVKernel, or a Config / fpy-schema dict (the kernel main() builds
        from it, fpy:197)."""
        nz, z_max = _native.zgrid(nz, z_max)
        y = self._f64(ys).reshape(-1)
        out = torch.empty_like(y)
        a = to_ctypes_aov(to_aov(kernel))
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_aov_batch(None, ctypes.byref(a), _vp(y), y.numel(), nz, z_max, _vp(out),
                                               self._stream()))
        return out

    # -- fpy:222-223 ------------------------------------------------------------------------
    def jchi(self, cfg, Ts) -> torch.Tensor:
        T = self._f64(Ts).reshape(-1)
        out = torch.empty_like(T)
        p = to_ctypes_point(to_point(cfg, P=0.0))
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_jchi_batch(ctypes.byref(p), _vp(T), T.numel(), _vp(out), self._stream()))
        return out

    # -- fpy:231-267 + epilogue ----------------------------------------------------------------
    def yields(self, points, n_y: int = 8000, T_lo=None, T_hi=None, P=None, reuse: bool = False,
               nz: int = _native.LZQ_NZ, z_max: float = _native.LZQ_Z_MAX, aov=None) -> torch.Tensor:
        """points: POINT_DTYPE numpy array or a device byte tensor from points_to_device.
        Returns (n, 6) float64 device tensor in YIELD_FIELDS order.
        reuse: lzq_yields_batch_reuse -- points equal in _native.ZSUM_KEY share one table of
        z-sums (bit-identical; not the dense headline path).  Used only with main()'s window
        and when points do share; otherwise the dense path.
        nz, z_max: the A/V kernel's z grid (AoverVKernel(..., z_max, nz), fpy:141-156).
        aov: the A/V kernel's own parameters when it is not the points' own (bs.aov replaced,
        fpy:261; see aov_to_device); such batches run the dense kernels (no reuse)."""
        nz, z_max = _native.zgrid(nz, z_max)
        d_pts = points if isinstance(points, torch.Tensor) else self.points_to_device(points)
        n = d_pts.numel() // _native.POINT_DTYPE.itemsize
        d_aov = self.aov_to_device(aov, n)
        out = torch.empty((n, 6), dtype=torch.float64, device=self.device)
        tl = None if T_lo is None else self._f64(T_lo)
        th = None if T_hi is None else self._f64(T_hi)
        Pv = None if P is None else self._f64(P)
        with torch.cuda.device(self.device):
            groups = table_groups(d_pts, n, _ZSUM_WORDS) if reuse and tl is None and th is None and d_aov is None \
                else None
            stride = max(int(n_y), 2000) + _native.REUSE_TABLE_HEADER
            if groups is not None and groups[0].numel() * stride * 8 <= REUSE_MAX_BYTES:
                rep, inv = groups
                need = rep.numel() * stride
                if self._zwork is None or self._zwork.numel() < need:
                    self._zwork = torch.empty(need, dtype=torch.float64, device=self.device)
                self._ztab_key = None   # the grid tables in _zwork are overwritten
                idx = inv.to(torch.int32)
                self._check(self.lib.lzq_yields_batch_reuse(_vp(d_pts), n, int(n_y), nz, z_max, _vp(Pv), _vp(rep),
                                                              _vp(idx), rep.numel(), _vp(self._zwork),
                                                              self._zwork.numel(), _vp(out), self._stream()))
                self._keepalive_reuse = (rep, idx, d_pts)
            else:
                self._check(self.lib.lzq_yields_batch(_vp(d_pts), n, int(n_y), nz, z_max, _vp(tl), _vp(th), _vp(Pv),
                                                        _vp(d_aov), _vp(out), self._stream()))
                self._keepalive_aov = d_aov
        return out

    # -- grid sweep ----------------------------------------------------------------------------
    def sweep(self, base_cfg, axes: Sequence[tuple], start: int, count: int, n_y: int = 8000,
              out: Optional[torch.Tensor] = None, P: Optional[float] = None,
              P_points: Optional[torch.Tensor] = None, reuse: bool = False, nz: int = _native.LZQ_NZ,
              z_max: float = _native.LZQ_Z_MAX) -> torch.Tensor:
        """axes: sequence of (field_name, values) (C order, last fastest); field names are
        the lzq_point double fields or 'delta_LZ' / 'm_mix' / 'dprime'.  P_points: optional
        per-point P override ([count], device), e.g. from lz_propagate (config C5).
        reuse: lzq_sweep_grid_reuse -- the z-sums computed once per combination of the grid's
        I_p / beta_over_H / T_p_GeV / T_min_over_Tp / T_max_over_Tp values and shared by the
        points (bit-identical results; NOT the dense headline path).
        nz, z_max: the A/V kernel's z grid (fpy:141-156; main()'s default 1200, 30)."""
        nz, z_max = _native.zgrid(nz, z_max)
        if len(axes) > _native.LZQ_MAX_AXES:
            raise ValueError(f"at most {_native.LZQ_MAX_AXES} sweep axes")
        dev_vals = [self._f64(v).reshape(-1) for _, v in axes]
        arr = (_native.LzqAxis * max(1, len(axes)))()
        for a, ((name, _), t) in enumerate(zip(axes, dev_vals)):
            if name not in _native.FIELD:
                raise ValueError(f"unknown sweep field {name!r}")
            arr[a].field = _native.FIELD[name]
            arr[a].n = t.numel()
            arr[a].values = t.data_ptr()
        base = to_ctypes_point(to_point(base_cfg, P=P))
        if out is None:
            out = torch.empty((count, 6), dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            Pp = None if P_points is None else self._f64(P_points).reshape(-1)
            if Pp is not None and Pp.numel() != count:
                raise ValueError("P_points must have `count` entries")
            need = self.lib.lzq_sweep_grid_reuse_workspace(arr, len(axes), int(n_y)) if reuse else 0
            if need < 0:
                self._check(int(need))
            n_tables = need // (max(int(n_y), 2000) + _native.REUSE_TABLE_HEADER)
            # the tables of a grid are built once and reused by every later chunk of the same sweep
            # (base, axes, n_y and exponential variant: tkey); every table costs one dense point, so
            # building them pays only with at least as many points to come as tables; and their
            # workspace stays bounded (REUSE_MAX_BYTES): otherwise the dense path, same bits
            tkey = None
            if reuse:
                tkey = (bytes(base), tuple((n, np.asarray(v, dtype=np.float64).tobytes()) for n, v in axes), int(n_y),
                        self._exp_variant, nz, z_max)
                built = tkey == self._ztab_key
                why = None if need * 8 <= REUSE_MAX_BYTES else f"{n_tables} z-sum tables exceed REUSE_MAX_BYTES"
                if why is None and not built and not 0 < n_tables <= count:
                    why = f"{n_tables} z-sum tables for a chunk of {count} points"
                if why:
                    _log.warning("lzq reuse_zsums: dense path (same bits): %s", why)
                    reuse = False
            self.last_reuse = "tables" if reuse else "dense"
            if reuse:
                if not built:
                    if self._zwork is None or self._zwork.numel() < need:
                        self._zwork = torch.empty(max(int(need), 1), dtype=torch.float64, device=self.device)
                    self._check(self.lib.lzq_sweep_grid_ztables(ctypes.byref(base), arr, len(axes), int(n_y), nz,
                                                                z_max, _vp(self._zwork), self._zwork.numel(),
                                                                self._stream()))
                    self._ztab_key = tkey
                self._check(self.lib.lzq_sweep_grid_from_ztables(
                    ctypes.byref(base), arr, len(axes), int(start), int(count), int(n_y), nz, z_max, _vp(Pp),
                    _vp(self._zwork), self._zwork.numel(), _vp(out), self._stream()))
            else:
                self._check(self.lib.lzq_sweep_grid(ctypes.byref(base), arr, len(axes), int(start), int(count),
                                                      int(n_y), nz, z_max, _vp(Pp), _vp(out), self._stream()))
        self._keepalive = dev_vals  # axis buffers must outlive the async launch
        return out

    # -- ODE fallback (fpy:200-219, 270-286, 385-417) ---------------------------------------
    def ode_params_to_device(self, recs: np.ndarray) -> torch.Tensor:
        """lzq_ode_params records (numpy ODE_DTYPE array) -> device byte tensor (Engine.ode's
        device-resident input, with points_to_device)."""
        return _to_device_bytes(np.ascontiguousarray(recs, dtype=_native.ODE_DTYPE), self.device)

    def ode_workspace(self, n: int, nt: int = _native.ODE_NT) -> torch.Tensor:
        return torch.empty(n * 4 * int(nt), dtype=torch.float64, device=self.device)

    def ode_tables(self, points, T_lo=None, T_hi=None, work: Optional[torch.Tensor] = None, nt: int = _native.ODE_NT,
                   nz: int = _native.LZQ_NZ, z_max: float = _native.LZQ_Z_MAX, aov=None) -> tuple:
        """BoltzmannSystem.build_tables(T_lo, T_hi, n=nt) for each point (window T_lo/T_hi per
        point, or main()'s window) with the A/V kernel's z grid (nz, z_max) and, if given, its own
        parameters `aov` (aov_to_device; y(T) stays the point's, fpy:211): returns the (n * 4 nt)
        spline workspace and the int32 status."""
        nz, z_max = _native.zgrid(nz, z_max)
        d_pts = points if isinstance(points, torch.Tensor) else self.points_to_device(points)
        n = d_pts.numel() // _native.POINT_DTYPE.itemsize
        d_aov = self.aov_to_device(aov, n)
        work = self.ode_workspace(n, nt) if work is None else work
        tl = None if T_lo is None else self._f64(T_lo).reshape(-1)
        th = None if T_hi is None else self._f64(T_hi).reshape(-1)
        status = torch.zeros(n, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_ode_tables(_vp(d_pts), n, _vp(tl), _vp(th), int(nt), nz, z_max, _vp(d_aov),
                                                _vp(work), work.numel(), _vp(status), self._stream()))
        self._keepalive_aov = d_aov
        return work, status

    def ode(self, points, ode_params, max_steps: Optional[int] = None, chunk: int = 1 << 18,
            share_tables: bool = True, method: str = "radau", group_waves: bool = True, nz: int = _native.LZQ_NZ,
            z_max: float = _native.LZQ_Z_MAX, aov=None, time_parallel: Optional[bool] = None) -> tuple:
        """fpy:385-417 for n points (POINT_DTYPE records + ODE_DTYPE records, as numpy arrays or
        as device byte tensors from points_to_device / ode_params_to_device): (n, 6) yields
        table and (n,) int32 status (enum lzq_ode_status), both on the device.  Points are
        processed in chunks so that the spline workspace stays <= chunk * 25.6 KB (6.7 GB at the
        default 2^18 points: 2 waves/SIMD on all 1024 SIMDs need >= 131072 points per launch).
        share_tables: points equal in the fields the A/V spline depends on (ODE_TABLE_KEY) share
        one table (lzq_ode_integrate_shared; bit-identical results, one A/V table per distinct
        kernel instead of per point).
        method: "radau" (default: the reference's integrator, fixed steps) or "quadrature"
        (lzq_ode_quadrature, opt-in: Y_B -- and Y_chi when sigma_v = 0 -- by the exact
        integrating-factor quadrature; with sigma_v != 0, Y_chi's Riccati equation is stepped
        alone by Radau).
        group_waves: launch the points in an order that puts points with equal stage keys
        (_native.ODE_STAGE_KEY, + deplete) next to each other, so that whole wavefronts qualify
        for the integrator's cooperative mode; results are scattered back to the input order.
        Each point's result is the same bits in either order.
        max_steps: cap on the fixed Radau steps of a point (LZQ_ODE_TOO_MANY_STEPS beyond it; the
        sweeps pass sweep.ODE_MAX_STEPS).  None (default): the batch's own largest step count
        (ode_step_counts), i.e. every window the reference accepts is integrated, however long
        (fpy:403-407): the library runs it as continuation launches of <= 2^24 steps.
        nz, z_max: the z grid of the A/V kernel behind the spline tables (fpy:141-156, 207-212).
        aov: the A/V kernel's own parameters behind each point's spline table when it is not the
        point's own (bs.aov replaced before build_tables, fpy:211; see aov_to_device); the tables are
        then built per point (no sharing).
        time_parallel: integrate by lzq_ode_integrate_tp (multiple shooting: a point's steps cut into
        intervals integrated side by side, Newton on their boundaries, the exact chains stitched
        through candidate starts) -- the latency path for a few points on long windows, with the
        sequential integration's bits.  None (default): on for a single point (the CLI's case).
        Radau only.  self.last_ode_tp_iters: the Newton updates per point of the last
        time-parallel call (<= 0: integrated sequentially)."""
        nz, z_max = _native.zgrid(nz, z_max)
        if method not in ("radau", "quadrature"):
            raise ValueError(f"method must be 'radau' or 'quadrature', got {method!r}")
        if isinstance(points, torch.Tensor):   # device records (points_to_device / ode_params_to_device)
            pts = None
            rp_, ro_ = _native.POINT_DTYPE.itemsize, _native.ODE_DTYPE.itemsize
            if not isinstance(ode_params, torch.Tensor) or points.dtype != torch.uint8 or \
                    ode_params.dtype != torch.uint8 or points.device != self.device or \
                    ode_params.device != self.device or points.numel() % rp_ or \
                    points.numel() // rp_ != ode_params.numel() // ro_ or ode_params.numel() % ro_:
                raise ValueError("device points / ode_params: uint8 record tensors of the same length on the "
                                 "engine's device (points_to_device, ode_params_to_device)")
            n = points.numel() // rp_
        else:
            pts = np.ascontiguousarray(points, dtype=_native.POINT_DTYPE).reshape(-1)
            ods = np.ascontiguousarray(ode_params, dtype=_native.ODE_DTYPE).reshape(-1)
            if pts.size != ods.size:
                raise ValueError("points and ode_params must have the same length")
            n = pts.size
        if time_parallel is None:
            time_parallel = n == 1
        time_parallel = bool(time_parallel) and method == "radau"
        tp_iters = torch.zeros(n, dtype=torch.int32, device=self.device) if time_parallel else None
        if pts is None:
            d_pts_all, d_ode_all = points.contiguous().view(-1), ode_params.contiguous().view(-1)
        else:
            d_pts_all = self.points_to_device(pts)
            d_ode_all = _to_device_bytes(ods, self.device)
        d_aov_all = self.aov_to_device(aov, n)
        if d_aov_all is not None:
            share_tables = False   # a table's key now includes the block (ODE_TABLE_KEY does not)
        # the launches cover the batch's own largest step count (or the cap, when a point needs more:
        # those points come back LZQ_ODE_TOO_MANY_STEPS), not the cap itself
        per = 1 << getattr(self, "_ode_launch_log2", 24)
        need = h_coop = coop_breaks = tab_same = n_lin = None
        if n <= 4096 and pts is not None:
            # few points (the CLI's one): on the host, no device round trip (the same values)
            need_h = ode_step_counts(pts)
            need_h = need_h[np.isfinite(need_h)]
            top = float(need_h.max()) + 64 if need_h.size else 0
        else:
            need = ode_step_counts_device(d_pts_all, n)   # same values as ode_step_counts, on the device
            # one transfer for the largest finite count (-inf: none finite), the launch order's key
            # breaks and whether every point has the first one's table key (wave_order, table_groups)
            vals = [torch.where(torch.isfinite(need), need, float("-inf")).max()]
            if group_waves and n > 64:
                h_coop = _coop_hash(d_pts_all, d_ode_all, n)
                vals.append((h_coop[1:] != h_coop[:-1]).sum().to(torch.float64))
            rows_on = share_tables and method == "radau" and not time_parallel and getattr(self, "ode_rows", True)
            if rows_on:   # points that could be in a row-table run (linear, not depleting): ode_runs' own test
                o_ = d_ode_all.view(n, _native.ODE_DTYPE.itemsize)
                sv_ = o_.view(torch.float64)[:, _native.ODE_DTYPE.fields["sigma_v_chi_GeV_m2"][1] // 8]
                dep_ = o_.view(torch.int32)[:, _native.ODE_DTYPE.fields["deplete_DM_from_source"][1] // 4]
                vals.append(((sv_ == 0.0) & (dep_ == 0)).sum().to(torch.float64))
            if share_tables:
                key = d_pts_all.view(n, _native.POINT_DTYPE.itemsize).view(torch.int64)[:, _KEY_WORDS]
                vals.append((key == key[0]).all().to(torch.float64))
            got = torch.stack(vals).tolist()
            if rows_on:
                n_lin = int(got[2 if group_waves and n > 64 else 1])
            top = got[0] + 64 if got[0] != float("-inf") else 0
            if group_waves and n > 64:
                coop_breaks = int(got[1])
            if share_tables:
                tab_same = bool(got[-1])
        longest = int(min(top, _native.ODE_MAX_LAUNCHES * per))
        max_steps = longest if max_steps is None else min(int(max_steps), longest)
        order = wave_order(d_pts_all, d_ode_all, n, h=h_coop, breaks=coop_breaks) if group_waves else None
        if need is not None and order is not None:
            need = need[order]
        if order is not None:
            d_pts_all = d_pts_all.view(n, -1)[order].contiguous().view(-1)
            d_ode_all = d_ode_all.view(n, -1)[order].contiguous().view(-1)
            if d_aov_all is not None:
                d_aov_all = d_aov_all.view(n, -1)[order].contiguous().view(-1)
        rp, ro = _native.POINT_DTYPE.itemsize, _native.ODE_DTYPE.itemsize
        out = torch.empty((n, 6), dtype=torch.float64, device=self.device)
        status = torch.zeros(n, dtype=torch.int32, device=self.device)
        keep = []
        tables = {"points": n, "tables": 0, "per_point_chunks": 0, "chunks": 0}
        # plan every chunk first (the table grouping synchronises with the host), then launch
        plan = []
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            d_pts = d_pts_all[c0 * rp:c1 * rp]
            d_ode = d_ode_all[c0 * ro:c1 * ro]
            ra = _native.AOV_DTYPE.itemsize
            d_aov = None if d_aov_all is None else d_aov_all[c0 * ra:c1 * ra]
            # (tab_same: whether every point of the batch has the first one's table key -- then every
            # chunk's does; when not, a chunk's own grouping still finds a chunk of one key)
            rep = table_groups(d_pts, c1 - c0, all_same=tab_same) if share_tables else None
            d_rep = d_idx = None
            if rep is not None:
                d_rep = d_pts.view(c1 - c0, rp)[rep[0]].contiguous()
                d_idx = rep[1].to(torch.int32)
            n_tab = (c1 - c0) if rep is None else d_rep.shape[0]
            tables["tables"] += n_tab
            tables["chunks"] += 1
            if rep is None and c1 - c0 > 1:
                tables["per_point_chunks"] += 1
                if share_tables and c1 - c0 >= 4096:
                    _log.warning(
                        "lzq ODE: %d of %d points differ in the A/V kernel or window (ODE_TABLE_KEY: %s): a spline "
                        "table per point (an A/V z-sum table build each; the integration still shares stage rows "
                        "across tables) -- ~2.6x the cost per point of a shared-table sweep on a 20000-step "
                        "window (DESIGN §4.3)", c1 - c0, c1 - c0, ", ".join(_native.ODE_TABLE_KEY))
            runs = None
            if (d_rep is not None and method == "radau" and not time_parallel and getattr(self, "ode_rows", True)
                    and (n_lin is None or n_lin >= ROWS_MIN_RUN)):
                runs = ode_runs(d_pts, d_ode, d_idx, c1 - c0, steps=None if need is None else need[c0:c1])
            if runs is not None:
                runs = runs[:3] + (runs[3], torch.empty(2 * runs[4], dtype=torch.float64, device=self.device))
                tables["row_runs"] = tables.get("row_runs", 0) + int(runs[1].numel())
            plan.append((c0, c1, d_pts, d_ode, d_rep, d_idx, n_tab, d_aov, runs))
            keep.append((d_pts, d_ode, d_rep, d_idx, d_aov) + (() if runs is None else (runs[0], runs[1], runs[2], runs[4])))
        # Two or more chunks: chunk c + 1's spline tables are built on a side stream into the other
        # of two workspaces while chunk c integrates (the table kernels fill the SIMDs the
        # integrator's tail leaves idle); events order each workspace's reuse.  One chunk: one stream.
        main = torch.cuda.current_stream(self.device)
        piped = len(plan) > 1 and getattr(self, "ode_pipeline", True)
        side = torch.cuda.Stream(self.device) if piped else main
        ws_n = max(p[6] for p in plan) if plan else 0
        works = [self.ode_workspace(ws_n) for _ in range(2 if piped else 1)] if plan else []
        if piped:
            side.wait_stream(main)          # the records and the grouping above are on the main stream
            for w in works + [status]:     # the table kernels write bad-grid statuses on the side stream
                w.record_stream(side)
            for item in keep:
                for t in item:
                    if t is not None:
                        t.record_stream(side)
        freed = [None] * len(works)
        nt = _native.ODE_NT
        with torch.cuda.device(self.device):
            for ci, (c0, c1, d_pts, d_ode, d_rep, d_idx, n_tab, d_aov, runs) in enumerate(plan):
                b = ci % len(works)
                work = works[b]
                with torch.cuda.stream(side):
                    if freed[b] is not None:
                        side.wait_event(freed[b])
                    src = d_pts if d_rep is None else d_rep
                    self._check(self.lib.lzq_ode_tables(_vp(src), n_tab, None, None, nt, nz, z_max,
                                                        _vp(d_aov if d_rep is None else None), _vp(work), work.numel(),
                                                        _vp(status[c0:c1]) if d_rep is None and method == "radau"
                                                        else None,
                                                        self._stream()))
                    built = torch.cuda.Event() if piped else None
                    if piped:
                        built.record(side)
                if piped:
                    main.wait_event(built)
                if method == "quadrature":
                    self._check(self.lib.lzq_ode_quadrature(_vp(d_pts), _vp(d_ode), c1 - c0, _vp(d_idx), n_tab,
                                                            _vp(work), work.numel(), int(max_steps), _vp(out[c0:c1]),
                                                            _vp(status[c0:c1]), self._stream()))
                elif time_parallel:
                    self._check(self.lib.lzq_ode_integrate_tp(_vp(d_pts), _vp(d_ode), c1 - c0, _vp(d_idx), n_tab,
                                                              _vp(work), work.numel(), int(max_steps),
                                                              _vp(out[c0:c1]), _vp(status[c0:c1]),
                                                              _vp(tp_iters[c0:c1]), self._stream()))
                elif d_rep is None:   # lzq_ode_batch's second half (its tables are built above)
                    self._check(self.lib.lzq_ode_integrate(_vp(d_pts), _vp(d_ode), c1 - c0, _vp(work), work.numel(),
                                                           int(max_steps), _vp(out[c0:c1]), _vp(status[c0:c1]),
                                                           self._stream()))
                elif runs is not None:   # linear runs read shared step rows (bit-identical)
                    run_of, run_rep, row_off, max_rows, rows = runs
                    nr = run_rep.numel()
                    self._check(self.lib.lzq_ode_rows(_vp(d_pts), _vp(d_ode), c1 - c0, _vp(d_idx), n_tab, _vp(work),
                                                      work.numel(), _vp(run_rep), _vp(row_off), nr, max_rows,
                                                      _vp(rows), rows.numel(), self._stream()))
                    self._check(self.lib.lzq_ode_integrate_rows(_vp(d_pts), _vp(d_ode), c1 - c0, _vp(d_idx), n_tab,
                                                                _vp(work), work.numel(), int(max_steps), _vp(run_of),
                                                                _vp(run_rep), _vp(row_off), nr, _vp(rows),
                                                                rows.numel(), _vp(out[c0:c1]), _vp(status[c0:c1]),
                                                                self._stream()))
                else:
                    self._check(self.lib.lzq_ode_integrate_shared(_vp(d_pts), _vp(d_ode), c1 - c0, _vp(d_idx),
                                                                  n_tab, _vp(work), work.numel(), int(max_steps),
                                                                  _vp(out[c0:c1]), _vp(status[c0:c1]),
                                                                  self._stream()))
                if piped:
                    freed[b] = torch.cuda.Event()
                    freed[b].record(main)
        work = works
        keep.append((d_pts_all, d_ode_all))
        self._keepalive = (keep, work)
        tables["mode"] = "shared" if tables["per_point_chunks"] == 0 else (
            "per_point" if tables["per_point_chunks"] == tables["chunks"] else "mixed")
        self.last_ode_tables = tables   # sweep summary.json "ode_tables"
        if order is not None:
            out_in, st_in = torch.empty_like(out), torch.empty_like(status)
            out_in[order], st_in[order] = out, status
            out, status = out_in, st_in
            if tp_iters is not None:
                it_in = torch.empty_like(tp_iters)
                it_in[order] = tp_iters
                tp_iters = it_in
        self.last_ode_tp_iters = tp_iters
        return out, status

    def ode_aov_T(self, point, T_lo: float, T_hi: float, work_point: torch.Tensor, Ts,
                  nt: int = _native.ODE_NT) -> torch.Tensor:
        """BoltzmannSystem.A_over_V_T (fpy:214-218) of one point at several T (nt-knot tables)."""
        T = self._f64(Ts).reshape(-1)
        out = torch.empty_like(T)
        p = to_ctypes_point(np.asarray(point, dtype=_native.POINT_DTYPE).reshape(1))
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_ode_aov_T(ctypes.byref(p), float(T_lo), float(T_hi), int(nt), _vp(work_point),
                                               _vp(T), T.numel(), _vp(out), self._stream()))
        return out

    def ode_rhs(self, point, ode_params, T_lo: float, T_hi: float, work_point: torch.Tensor, xs, Ys,
                nt: int = _native.ODE_NT) -> torch.Tensor:
        """BoltzmannSystem.rhs (fpy:270-286) of one point: (n, 2) dY/dx at (x[i], Y[i])."""
        x = self._f64(xs).reshape(-1)
        Y = self._f64(Ys).reshape(-1, 2).contiguous()
        if Y.shape[0] != x.numel():
            raise ValueError("need one (Y_chi, Y_B) pair per x")
        out = torch.empty_like(Y)
        p = to_ctypes_point(np.asarray(point, dtype=_native.POINT_DTYPE).reshape(1))
        o = to_ctypes_ode(np.asarray(ode_params, dtype=_native.ODE_DTYPE).reshape(1))
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_ode_rhs(ctypes.byref(p), ctypes.byref(o), float(T_lo), float(T_hi), int(nt),
                                             _vp(work_point), _vp(x), _vp(Y), x.numel(), _vp(out), self._stream()))
        return out

    # -- fpy:183-184 -----------------------------------------------------------------------
    def p_closed_form(self, lam) -> torch.Tensor:
        l = self._f64(lam).reshape(-1)
        out = torch.empty_like(l)
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_p_closed_form(_vp(l), l.numel(), _vp(out), self._stream()))
        return out

    # -- LZ propagator (north_star (1)) ------------------------------------------------------
    def lz_propagate(self, m_mix, dprime, xi, v_w, window_lz: float,
                     steps_per_crossing: int) -> torch.Tensor:
        """Coherent LZ conversion probability per point (arrays [n] or [n, n_cross]).  v_w: one
        wall speed for the batch, or one per point ([n]: lzq_lz_propagate_v)."""
        m = self._f64(m_mix)
        if m.dim() == 1:
            m = m.reshape(-1, 1)
        d = self._f64(dprime).reshape(m.shape)
        x = self._f64(xi).reshape(m.shape)
        out = torch.empty(m.shape[0], dtype=torch.float64, device=self.device)
        per_point = isinstance(v_w, (torch.Tensor, np.ndarray, list, tuple))
        with torch.cuda.device(self.device):
            if per_point:
                vw = self._f64(v_w).reshape(-1)
                if vw.numel() != m.shape[0]:
                    raise ValueError("v_w must be a scalar or have one entry per point")
                self._check(self.lib.lzq_lz_propagate_v(_vp(m), _vp(d), _vp(x), _vp(vw), m.shape[0], m.shape[1],
                                                          float(window_lz), int(steps_per_crossing), _vp(out),
                                                          self._stream()))
                self._keepalive_vw = vw
            else:
                self._check(self.lib.lzq_lz_propagate(_vp(m), _vp(d), _vp(x), m.shape[0], m.shape[1], float(v_w),
                                                        float(window_lz), int(steps_per_crossing), _vp(out),
                                                        self._stream()))
        return out

    # -- bounce profiles (PAPER eqs.(5)-(9); the absent modules of fpy:173) ------------------
    def profile_shapes(self, knots, phi, Phi) -> "ProfileShapes":
        """Not-a-knot cubic splines (scipy CubicSpline) of phi(xi), Phi(xi) for n_shapes profiles
        sampled on their own knots: arrays [n_knots] or [n_shapes, n_knots] (lzq_profile_splines).
        Raises ValueError for knots that are not strictly increasing, as CubicSpline does."""
        x = self._f64(knots)
        x = x.reshape(1, -1) if x.dim() == 1 else x
        a, b = self._f64(phi).reshape(x.shape), self._f64(Phi).reshape(x.shape)
        ns, nk = x.shape
        if nk < 4:
            raise ValueError("a profile needs at least 4 knots")
        coef = torch.empty((ns, nk - 1, _native.PROFILE_COEF), dtype=torch.float64, device=self.device)
        bad = torch.empty(ns, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_profile_splines(_vp(x), _vp(a), _vp(b), ns, nk, _vp(coef), _vp(bad),
                                                     self._stream()))
        nbad = int(bad.sum().item())
        if nbad:
            raise ValueError(f"{nbad} profile(s) with knots that are not strictly increasing")
        return ProfileShapes(x, coef)

    def profile_points(self, y_B, y_chi, lambda_tr_eff, v_w, shape=0) -> torch.Tensor:
        """lzq_profile_point records (broadcast arrays) -> device byte tensor [n * 40]."""
        cols = np.broadcast_arrays(*(np.asarray(v, dtype=np.float64) for v in (y_B, y_chi, lambda_tr_eff, v_w)),
                                   np.asarray(shape, dtype=np.int32))
        rec = np.zeros(cols[0].size, dtype=_native.PROFILE_POINT_DTYPE)
        for name, c in zip(("y_B", "y_chi", "lambda_tr_eff", "v_w", "shape"), cols):
            rec[name] = c.reshape(-1)
        return _to_device_bytes(rec, self.device)

    def profile_crossings(self, shapes: "ProfileShapes", points: torch.Tensor, max_cross: int = 8) -> dict:
        """eqs.(5)-(8) per point: {'xi', 'dprime', 'm_mix', 'delta_lz'} [n, max_cross] and
        'count' [n] (lzq_profile_crossings; entries past count are unspecified)."""
        n = points.numel() // _native.PROFILE_POINT_DTYPE.itemsize
        out = {k: torch.empty((n, max_cross), dtype=torch.float64, device=self.device)
               for k in ("xi", "dprime", "m_mix", "delta_lz")}
        out["count"] = torch.empty(n, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_profile_crossings(
                _vp(shapes.knots), _vp(shapes.coef), shapes.n_shapes, shapes.n_knots, _vp(points), n, int(max_cross),
                _vp(out["xi"]), _vp(out["dprime"]), _vp(out["m_mix"]), _vp(out["delta_lz"]), _vp(out["count"]),
                self._stream()))
        return out

    def lz_propagate_profile(self, shapes: "ProfileShapes", points: torch.Tensor, steps_per_radian: float = 4.0,
                             min_steps: int = 1) -> torch.Tensor:
        """Coherent conversion probability through each point's whole profile
        (lzq_lz_propagate_profile)."""
        n = points.numel() // _native.PROFILE_POINT_DTYPE.itemsize
        out = torch.empty(n, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self.lib.lzq_lz_propagate_profile(
                _vp(shapes.knots), _vp(shapes.coef), shapes.n_shapes, shapes.n_knots, _vp(points), n,
                float(steps_per_radian), int(min_steps), _vp(out), self._stream()))
        return out


def ode_step_counts(pts: np.ndarray) -> np.ndarray:
    """Fixed Radau steps of each point's fpy:385-407 window, N = ceil(|x1 - x0| / max_step) with
    max_step = min(|x1 - x0|/20000, x_p/1000, 5e-4) (fpy:403-404), on the host (the device
    computes the same; this sizes the continuation launches)."""
    m = pts["m_chi_GeV"].astype(np.float64)
    Tp = pts["T_p_GeV"]
    with np.errstate(divide="ignore", invalid="ignore"):
        x0 = m / (pts["T_max_over_Tp"] * Tp)
        x1 = m / np.maximum(pts["T_min_over_Tp"] * Tp, 1e-30)
        x_p = m / np.maximum(Tp, 1e-30)
        dx = np.abs(x1 - x0)
        ms = np.minimum(np.minimum(dx / 20000.0, x_p / 1000.0), 5e-4)
        return np.where(ms > 0.0, np.ceil(dx / ms), np.nan)


def _to_device_bytes(arr: np.ndarray, device) -> torch.Tensor:
    """A contiguous record array as a device byte tensor.  The host bytes go to the device
    straight from the caller's buffer (a host-side copy first cost ~5-40 ms per 35 MB of records,
    mostly page faults on the fresh allocation); read-only buffers are copied, since torch only
    wraps writable ones."""
    b = np.ascontiguousarray(arr).view(np.uint8)
    if not b.flags.writeable:
        b = b.copy()
    return torch.from_numpy(b).to(device)


def ode_step_counts_device(d_pts: torch.Tensor, n: int) -> torch.Tensor:
    """ode_step_counts on the device records (lzq_point bytes): the same IEEE operations in the
    same order as the numpy version, so the same values (the host version took ~20 ms per 2.6e5
    points, more than half the integrator's own time on 20000-step windows)."""
    w = d_pts.view(n, _native.POINT_DTYPE.itemsize).view(torch.float64)

    def col(f):
        return w[:, _native.POINT_DTYPE.fields[f][1] // 8]
    m, Tp = col("m_chi_GeV"), col("T_p_GeV")
    x0 = m / (col("T_max_over_Tp") * Tp)
    x1 = m / torch.clamp_min(col("T_min_over_Tp") * Tp, 1e-30)
    x_p = m / torch.clamp_min(Tp, 1e-30)
    dx = (x1 - x0).abs()
    ms = torch.minimum(torch.minimum(dx / 20000.0, x_p / 1000.0), torch.full_like(dx, 5e-4))
    return torch.where(ms > 0.0, torch.ceil(dx / ms), torch.full_like(dx, float("nan")))


class ProfileShapes:
    """Device knots [n_shapes, n_knots] and spline rows [n_shapes, n_knots - 1, 8] of bounce
    profiles (include/lzq.h lzq_profile_splines)."""

    def __init__(self, knots: torch.Tensor, coef: torch.Tensor):
        self.knots, self.coef = knots.contiguous(), coef.contiguous()
        self.n_shapes, self.n_knots = int(knots.shape[0]), int(knots.shape[1])


# fixed odd 64-bit weights of _key_hash (a wrapping weighted sum of the key words)
_HASH_W = np.random.default_rng(0x6C7A71).integers(-2 ** 63, 2 ** 63 - 1, size=32, dtype=np.int64) | 1
_hash_w_dev: dict = {}


def _hash_weights(device, k: int) -> torch.Tensor:
    w = _hash_w_dev.get(device)
    if w is None:
        w = _hash_w_dev[device] = torch.from_numpy(_HASH_W).to(device)
    return w[:k]


def _key_hash(d_pts: torch.Tensor, n: int, fields, d_ode: Optional[torch.Tensor] = None, ode_fields=(),
              extra: Optional[torch.Tensor] = None) -> torch.Tensor:
    """A 64-bit hash of each point's key words (lzq_point fields, lzq_ode_params fields and an
    optional extra int column): their bits times fixed odd 64-bit weights, summed with wrap-around
    -- a few gathers and one reduction whatever the key length (the per-field multiply-xor chain
    it replaces was ~3 kernels per field, a third of a 2.6e5-point linear ODE call's kernels).
    Equal keys hash equally; the callers treat a collision of unequal keys as a lost grouping
    only (the kernels and table_groups compare the words themselves)."""
    cols = []
    for rec, dt, fs in ((d_pts, _native.POINT_DTYPE, fields), (d_ode, _native.ODE_DTYPE, ode_fields)):
        if not fs:
            continue
        i8 = [dt.fields[f][1] // 8 for f in fs if dt.fields[f][0].itemsize == 8]
        i4 = [dt.fields[f][1] // 4 for f in fs if dt.fields[f][0].itemsize == 4]
        if i8:
            cols.append(rec.view(n, dt.itemsize).view(torch.int64)[:, i8])
        if i4:
            cols.append(rec.view(n, dt.itemsize).view(torch.int32)[:, i4].to(torch.int64))
    if extra is not None:
        cols.append(extra.to(torch.int64).view(n, 1))
    c = torch.cat(cols, 1) if len(cols) > 1 else cols[0]
    return (c * _hash_weights(c.device, c.shape[1])).sum(1)


REUSE_MAX_BYTES = 16 << 30     # Engine.sweep(reuse=True): z-sum tables beyond this run dense


def _coop_hash(d_pts: torch.Tensor, d_ode: torch.Tensor, n: int) -> torch.Tensor:
    """wave_order's key: _native.ODE_COOP_KEY, deplete and Gamma_wash."""
    return _key_hash(d_pts, n, _native.ODE_COOP_KEY, d_ode, ("deplete_DM_from_source", "Gamma_wash_over_H"))


def wave_order(d_pts: torch.Tensor, d_ode: torch.Tensor, n: int, h: Optional[torch.Tensor] = None,
               breaks: Optional[int] = None):
    """A launch order (int64 permutation tensor, on the points' device) that makes points equal
    in _native.ODE_COOP_KEY, deplete and Gamma_wash contiguous -- and within such a run, points
    equal in the whole ODE_STAGE_KEY (same spline table) -- or None when the input is already
    grouped or has no repeated keys.  Gamma_wash (round 6): a whole wave with one Gamma_wash shares
    Y_B's step maps and runs the Riccati kernel, a wave that mixes several runs the general variant
    (DESIGN §4.3).  d_pts / d_ode: the lzq_point / lzq_ode_params records as byte tensors.  A
    64-bit hash of the key fields' bits (_key_hash) is sorted stably; a hash collision only puts unequal
    points in one wavefront, which the kernel detects and runs per lane.  h, breaks: _coop_hash
    and its count of breaks in input order, when the caller has them (Engine.ode)."""
    if n <= 64:
        return None
    if h is None:
        h = _coop_hash(d_pts, d_ode, n)
    # the key's breaks in input order (none: one key, the common sweep -- no sort needed), then its
    # distinct values (from one sort)
    if breaks is None:
        breaks = int((h[1:] != h[:-1]).sum())
    if breaks == 0:
        return None
    hs = torch.sort(h).values
    distinct = 1 + int((hs[1:] != hs[:-1]).sum())
    if distinct == n or breaks <= 2 * (distinct - 1):
        return None
    ht = _key_hash(d_pts, n, ("I_p", "v_w"))
    by_table = torch.argsort(ht, stable=True)
    return by_table[torch.argsort(h[by_table], stable=True)]


ROWS_MAX_BYTES = 256 << 20     # Engine.ode: shared step-row tables per chunk (lzq_ode_rows) up to this
ROWS_MIN_RUN = 64              # a run needs a whole wavefront to be read by one


def ode_runs(d_pts: torch.Tensor, d_ode: torch.Tensor, d_idx: torch.Tensor, n: int,
             max_bytes: int = ROWS_MAX_BYTES, min_run: int = ROWS_MIN_RUN, steps: Optional[torch.Tensor] = None):
    """Runs for lzq_ode_rows / lzq_ode_integrate_rows (include/lzq.h): maximal stretches of the
    launch order whose points agree in _native.ODE_COOP_KEY, Gamma_wash and the spline table
    index d_idx, and are linear (sigma_v = 0) and not depleting -- the points whose whole
    wavefronts share Y_B's step maps.  Returns (run_of int32 [n], run_rep int64 [R], row_off int64
    [R + 1] on the device, max_rows, total_rows), or None when no run of >= min_run points fits.  Runs are
    kept longest first while their rows (16 B per step of the run's step count, ode_step_counts)
    fit in max_bytes (steps: the points' ode_step_counts_device, when the caller has them).  A
    64-bit hash of the key words (_key_hash) decides the runs; the kernel compares every
    lane with its run's representative, bit for bit, before it reads the rows, so a hash
    collision only costs the sharing."""
    if n < min_run:
        return None
    ro = _native.ODE_DTYPE.itemsize
    o64 = d_ode.view(n, ro).view(torch.int64)
    o32 = d_ode.view(n, ro).view(torch.int32)
    sv = o64[:, _native.ODE_DTYPE.fields["sigma_v_chi_GeV_m2"][1] // 8].view(torch.float64)
    elig = (sv == 0.0) & (o32[:, _native.ODE_DTYPE.fields["deplete_DM_from_source"][1] // 4] == 0)
    h = _key_hash(d_pts, n, _native.ODE_COOP_KEY, d_ode, ("Gamma_wash_over_H",), extra=d_idx)
    if steps is None:
        steps = ode_step_counts_device(d_pts, n)
    # one transfer: eligible points, points with the first point's key, the first point's step count
    n_elig, n_same, s0 = torch.stack([elig.sum().to(torch.float64), (h == h[0]).sum().to(torch.float64),
                                      steps[0]]).tolist()
    if n_elig < min_run:   # no linear run possible (e.g. Riccati sweeps)
        return None
    if n_elig == n and n_same == n:   # one run (the common linear sweep): no grouping kernels
        if not (np.isfinite(s0) and s0 > 0 and 16 * s0 <= max_bytes):
            return None
        dev = d_pts.device
        return (torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int64, device=dev),
                torch.tensor([0, int(s0)], dtype=torch.int64, device=dev), int(s0), int(s0))
    h = torch.where(elig, h, torch.full_like(h, -1))   # ineligible points: one key, never a run
    _, inv, counts = torch.unique_consecutive(h, return_inverse=True, return_counts=True)
    starts = torch.cumsum(counts, 0) - counts
    steps = steps[starts]
    ok = (counts >= min_run) & elig[starts] & torch.isfinite(steps) & (steps > 0)
    rows = torch.where(ok, steps, torch.zeros_like(steps)).to(torch.int64)
    by_len = torch.argsort(counts * ok, descending=True, stable=True)
    cap = max_bytes // 16
    keep = torch.zeros_like(ok)
    keep[by_len] = ok[by_len] & (torch.cumsum(rows[by_len], 0) <= cap)
    n_runs, max_rows, total = torch.stack([keep.sum(), (rows * keep).max(), (rows * keep).sum()]).tolist()
    if n_runs == 0:
        return None
    sel = torch.nonzero(keep).reshape(-1)               # kept runs in launch order
    run_id = torch.full_like(counts, -1)
    run_id[sel] = torch.arange(n_runs, dtype=torch.int64, device=d_pts.device)
    row_off = torch.zeros(n_runs + 1, dtype=torch.int64, device=d_pts.device)
    row_off[1:] = torch.cumsum(rows[sel], 0)
    return run_id[inv].to(torch.int32), starts[sel].contiguous(), row_off, int(max_rows), int(total)


_KEY_WORDS = [_native.POINT_DOUBLE_FIELDS.index(f) for f in _native.ODE_TABLE_KEY]  # 8-byte words of lzq_point
_ZSUM_WORDS = [_native.POINT_DOUBLE_FIELDS.index(f) for f in _native.ZSUM_KEY]


def table_groups(d_pts: torch.Tensor, n: int, words=None, all_same: Optional[bool] = None):
    """Points (device lzq_point records) that can share one ODE spline table: equal, bit for
    bit, in _native.ODE_TABLE_KEY (or in the lzq_point words `words`: _ZSUM_WORDS for the
    quadrature's z-sum tables).  Returns (representative indices, per-point table index),
    both int64 device tensors, or None when sharing would not pay (more than half the points
    distinct).  Index bookkeeping on the device: a 64-bit hash of the key words is deduplicated
    and every point's key is then compared with its representative's, so a hash collision only
    costs the sharing, never a wrong table.  all_same: the caller already knows whether every
    point has the first one's key (Engine.ode folds that test into one transfer)."""
    if n < 2:
        return None
    if all_same:
        z = torch.zeros(n, dtype=torch.int64, device=d_pts.device)
        return z[:1], z
    key = d_pts.view(n, _native.POINT_DTYPE.itemsize).view(torch.int64)[:, _KEY_WORDS if words is None else words]
    if all_same is None and bool((key == key[0]).all()):
        z = torch.zeros(n, dtype=torch.int64, device=d_pts.device)
        return z[:1], z
    h = (key * _hash_weights(key.device, key.shape[1])).sum(1)
    u, inv = torch.unique(h, return_inverse=True)
    if u.numel() * 2 > n:
        return None
    ar = torch.arange(n, dtype=torch.int64, device=d_pts.device)
    first = torch.full((u.numel(),), n, dtype=torch.int64, device=d_pts.device).scatter_reduce_(0, inv, ar, "amin")
    if not bool((key[first][inv] == key).all()):
        return None
    return first, inv


_default: Optional[Engine] = None


def default_engine() -> Engine:
    global _default
    if _default is None or _default.device.index != torch.cuda.current_device():
        _default = Engine()
    return _default


def table_to_dicts(t: torch.Tensor) -> list[dict]:
    a = t.detach().cpu().numpy()
    return [dict(zip(YIELD_FIELDS, map(float, row))) for row in a]


def as_float_list(x: Iterable) -> list[float]:
    return [float(v) for v in x]
