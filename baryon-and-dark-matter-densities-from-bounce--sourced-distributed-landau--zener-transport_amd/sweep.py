"""Parameter-sweep driver (north_star (3); the reference has no sweep code).

A sweep = a base config in the reference schema (fpy:44-79) x up to 8 Cartesian axes,
flattened in C order (last axis fastest).  Points are generated ON DEVICE from the flat
index (lzq_sweep_grid), so no parameter table ever crosses PCIe.

Multi-GPU: one process per GPU; rank r owns the contiguous shard
[r*N//W, (r+1)*N//W) and evaluates it with no communication; one all-gather of the 48-B
per-point yield records (RCCL over xGMI on GPUs, gloo in CPU tests) assembles the table on
every rank.  Each point is reduced by one wavefront, so the gathered table is bit-identical
for W = 1, 2, 4, 8.  Grid-wide statistics are reduced on the host in index order.

Checkpoint/resume: with --out, every evaluated chunk is written as
`shard_<key>_<start>_<count>.npy` (allow_pickle=False), where <key> hashes the sweep
definition (spec_key: axes, base config, n_y, crossings, library ABI); --resume reloads
existing chunks of the SAME definition instead of recomputing them, so a killed 1e8-point
run restarts where it stopped, and a directory written by another sweep is never mixed in
(manifest.json records the definition; a mismatch refuses --resume).

    python -m <package>.sweep --spec C2 --out sweep_c2          # 1 GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m <package>.sweep --spec C4 --out c4
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native
from .config import to_ode_params, to_point

YIELD_FIELDS = _native.YIELD_FIELDS

EQUAL_MASS = {  # /root/reference/yields_config_equal_mass.json
    "regime": "nonthermal", "m_chi_GeV": 0.95, "g_chi": 2, "chi_stats": "fermion",
    "sigma_v_chi_GeV_m2": 0.0, "T_p_GeV": 100.0, "beta_over_H": 100.0, "v_w": 0.30, "I_p": 0.34,
    "g_star": 106.75, "g_star_s": 106.75, "P_chi_to_B": 0.14925839040304145,
    "source_shape_sigma_y": 9.0, "Gamma_wash_over_H": 0.0, "incident_flux_scale": 1.07e-9,
    "deplete_DM_from_source": False, "T_max_over_Tp": 5.0, "T_min_over_Tp": 0.001,
    "Y_chi_init": 4.90e-10, "n_chi_at_Tp_GeV3": None,
}


@dataclass
class CrossingSpec:
    """Multi-crossing bounce profile per grid point (BASELINE config C5; no reference
    counterpart).  Crossing c of the point with grid values (m_mix, |Delta'|)
    has m_c = m_mix (1 + jitter a_c), |Delta'_c| = |Delta'| (1 + jitter b_c) and position
    xi_c = L (spacing_lz c + jitter d_c), L = sqrt(v_w/|Delta'|) max(1, sqrt(delta)), with
    (a, b, d) ~ U(-1, 1) drawn once from numpy default_rng(seed).  P is the coherent
    conversion probability through all crossings (lzq_lz_propagate)."""
    n_cross: int = 8
    spacing_lz: float = 40.0
    jitter: float = 0.1
    window_lz: float = 20.0
    steps: int = 64        # Magnus steps per crossing core (floor): <= 1e-10 from the exact solution
    seed: int = 5

    def pattern(self) -> np.ndarray:
        return np.random.default_rng(self.seed).uniform(-1.0, 1.0, (3, self.n_cross))


PROFILE_FIELDS = ("y_B", "y_chi", "lambda_tr_eff")   # PAPER eqs.(5),(7): sweep axes of a profile spec


@dataclass
class ProfileSpec:
    """P of every grid point from ONE bounce profile (PAPER p.3 eqs.(5)-(9); the plug-in path of
    fpy:170-187 as a sweep): the profile's phi, Phi (a CSV in transport_from_profile's `xi,phi,Phi`
    format, or shape `synthetic` of bounce.synthetic_shapes) with the couplings y_B, y_chi,
    lambda_tr_eff (these defaults, or sweep axes of those names) and the point's v_w.
    estimator: "auto" (one crossing -> eq.(9) of its delta_LZ; several -> the time-ordered
    propagation through the profile; none -> P = NaN, as the plug-in's Profile.probability raises
    'no avoided crossing' for it), "minimal" (eq.(9); points without exactly one crossing get
    P = NaN) or "propagate" (every point through the whole profile, crossings or not)."""
    csv: Optional[str] = None
    synthetic: int = 12     # bounce.synthetic_shapes index (12: one or three crossings across P1's couplings)
    estimator: str = "auto"
    y_B: float = 1.0
    y_chi: float = 1.0
    lambda_tr_eff: float = 0.1
    steps_per_radian: float = 4.0
    min_steps: int = 1

    def arrays(self):
        from . import bounce
        if self.csv:
            x, a, b, _ = bounce.read_bounce_csv(self.csv)
            return x, a, b
        if not 0 <= self.synthetic < 16:
            raise ValueError("profile.synthetic must index the 16-shape synthetic family (0..15)")
        X, A, B = bounce.synthetic_shapes(16)   # the family as tools/bench_profile.py draws it
        return X[self.synthetic], A[self.synthetic], B[self.synthetic]


ODE_MAX_STEPS = 1 << 26   # a sweep's default cap on one ODE point's fixed Radau steps (LZQ_ODE_TOO_MANY_STEPS beyond)


@dataclass
class SweepSpec:
    name: str
    base: dict
    axes: List[Tuple[str, np.ndarray]]
    n_y: int = 8000
    notes: str = ""
    crossings: Optional[CrossingSpec] = None
    ode_method: str = "radau"   # ODE-path points: "radau" (the reference's integrator) | "quadrature" (opt-in)
    profile: Optional[ProfileSpec] = None
    nz: int = _native.LZQ_NZ          # the A/V kernel's z grid, AoverVKernel(..., z_max, nz) (fpy:141-156)
    z_max: float = _native.LZQ_Z_MAX
    # ODE-path points needing more fixed Radau steps than this are not integrated (a NaN row counted
    # as too_many_steps in summary.json): one long window would otherwise hold its shard for hours.
    # None = no cap (every window the reference accepts, as the single-point CLI does).
    ode_max_steps: Optional[int] = ODE_MAX_STEPS

    @property
    def total(self) -> int:
        n = 1
        for _, v in self.axes:
            n *= len(v)
        return n

    def point_params(self, idx: int) -> dict:
        """Host-side decode of flat index -> axis values (for reporting / tests)."""
        out = {}
        for name, vals in reversed(self.axes):
            out[name] = float(vals[idx % len(vals)])
            idx //= len(vals)
        return out

    def to_json(self) -> dict:
        d = {"name": self.name, "base": self.base, "n_y": self.n_y, "notes": self.notes,
             "axes": [{"field": n, "values": [float(x) for x in v]} for n, v in self.axes]}
        if self.crossings is not None:
            d["crossings"] = dict(self.crossings.__dict__)
        if self.ode_method != "radau":
            d["ode_method"] = self.ode_method
        if self.profile is not None:
            d["profile"] = dict(self.profile.__dict__)
        if (self.nz, self.z_max) != (_native.LZQ_NZ, _native.LZQ_Z_MAX):
            d["nz"], d["z_max"] = int(self.nz), float(self.z_max)
        if self.ode_max_steps != ODE_MAX_STEPS:
            d["ode_max_steps"] = self.ode_max_steps
        return d

    def axis_values(self, start: int, count: int, device) -> dict:
        """{axis name: [count] torch tensor} of grid indices [start, start+count) (C order)."""
        import torch
        idx = torch.arange(start, start + count, dtype=torch.int64, device=device)
        vals, stride = {}, 1
        for name, v in reversed(self.axes):
            t = torch.as_tensor(np.asarray(v, dtype=np.float64), device=device)
            vals[name] = t[(idx // stride) % len(v)]
            stride *= len(v)
        return vals

    def crossing_arrays(self, start: int, count: int, device):
        """Per-point crossing parameters [count, n_cross] (torch, on `device`) for C5."""
        import torch
        cs = self.crossings
        names = [n for n, _ in self.axes]
        if "m_mix" not in names or "dprime" not in names:
            raise ValueError("a multi-crossing spec needs m_mix and dprime axes")
        idx = torch.arange(start, start + count, dtype=torch.int64, device=device)
        vals = {}
        stride = 1
        for name, v in reversed(self.axes):
            t = torch.as_tensor(np.asarray(v, dtype=np.float64), device=device)
            vals[name] = t[(idx // stride) % len(v)]
            stride *= len(v)
        v_w = vals["v_w"] if "v_w" in vals else torch.full_like(vals["m_mix"], float(self.base["v_w"]))
        m0, d0 = vals["m_mix"], vals["dprime"].abs()
        delta0 = m0 * m0 / (2.0 * v_w * d0)
        L = torch.sqrt(v_w / d0) * torch.clamp(torch.sqrt(delta0), min=1.0)
        a, b, dd = (torch.as_tensor(r, device=device) for r in cs.pattern())
        c = torch.arange(cs.n_cross, dtype=torch.float64, device=device)
        m = m0[:, None] * (1.0 + cs.jitter * a[None, :])
        dp = d0[:, None] * (1.0 + cs.jitter * b[None, :])
        xi = L[:, None] * (cs.spacing_lz * c[None, :] + cs.jitter * dd[None, :])
        return m.contiguous(), dp.contiguous(), xi.contiguous(), v_w


ODE_FIELDS = ("sigma_v_chi_GeV_m2", "Gamma_wash_over_H", "deplete_DM_from_source")  # fpy:372 gate


def is_ode_spec(spec: "SweepSpec") -> bool:
    """Does any point of the sweep leave the fast path (fpy:372) for the ODE fallback?"""
    b = spec.base
    base_ode = bool(b.get("deplete_DM_from_source")) or float(b.get("sigma_v_chi_GeV_m2", 0.0)) != 0.0 or \
        float(b.get("Gamma_wash_over_H", 0.0)) != 0.0
    return base_ode or any(name in ODE_FIELDS and np.any(np.asarray(v) != 0) for name, v in spec.axes)


def grid_records(spec: "SweepSpec", start: int, count: int, engine=None):
    """Explicit point records of grid indices [start, start+count): (POINT_DTYPE, ODE_DTYPE)
    numpy arrays, decoded in C order like lzq_sweep_grid.  The LZ axes set P through the
    closed form evaluated on the GPU (lzq_p_closed_form, fpy:183-184)."""
    pts = np.repeat(to_point(spec.base), count)
    ods = np.repeat(to_ode_params(spec.base), count)
    idx = np.arange(start, start + count, dtype=np.int64)
    stride = 1
    lz = {}
    for name, vals in reversed(spec.axes):
        v = np.asarray(vals, dtype=np.float64)[(idx // stride) % len(vals)]
        stride *= len(vals)
        if name in ("delta_LZ", "m_mix", "dprime"):
            lz[name] = v
        elif name in PROFILE_FIELDS:
            continue          # P comes from the profile (profile_P)
        elif name in ODE_FIELDS:
            ods[name] = v if name != "deplete_DM_from_source" else (v != 0).astype(np.int32)
        elif name == "Y_chi_init":
            pts["Y_chi_init"], pts["has_Y_chi_init"] = v, 1
        elif name == "n_chi_at_Tp_GeV3":
            pts["n_chi_at_Tp_GeV3"], pts["has_n_chi_at_Tp"] = v, 1
        else:
            pts[name] = v
    if lz:
        if "m_mix" in lz:  # PAPER eq.(8), F = 1
            delta = lz["m_mix"] * lz["m_mix"] / (2.0 * np.maximum(pts["v_w"], 1e-12) * np.abs(lz["dprime"]))
        else:
            delta = lz["delta_LZ"]
        if engine is None:
            from .engine import default_engine
            engine = default_engine()
        pts["P_chi_to_B"] = engine.p_closed_form(delta).cpu().numpy()
    return pts, ods


def _axis_from_json(a: dict) -> Tuple[str, np.ndarray]:
    if "values" in a:
        v = np.asarray(a["values"], dtype=np.float64)
    elif "logspace" in a:
        v = np.logspace(*a["logspace"][:2], int(a["logspace"][2]))
    elif "linspace" in a:
        v = np.linspace(*a["linspace"][:2], int(a["linspace"][2]))
    else:
        raise ValueError(f"axis {a!r} needs values / linspace / logspace")
    if a["field"] not in _native.FIELD and a["field"] not in ODE_FIELDS and a["field"] not in PROFILE_FIELDS:
        raise ValueError(f"unknown sweep field {a['field']!r}")
    return a["field"], v


def spec_from_json(d: dict) -> SweepSpec:
    base = dict(EQUAL_MASS)
    if "config" in d:
        with open(d["config"]) as f:
            base.update(json.load(f))
    base.update(d.get("base", {}))
    cr = CrossingSpec(**d["crossings"]) if d.get("crossings") else None
    method = d.get("ode_method", "radau")
    if method not in ("radau", "quadrature"):
        raise ValueError(f"ode_method must be 'radau' or 'quadrature', got {method!r}")
    prof = ProfileSpec(**d["profile"]) if d.get("profile") else None
    if prof is not None and prof.estimator not in ("auto", "minimal", "propagate"):
        raise ValueError(f"profile estimator must be auto / minimal / propagate, got {prof.estimator!r}")
    axes = [_axis_from_json(a) for a in d["axes"]]
    if prof is None and any(n in PROFILE_FIELDS for n, _ in axes):
        raise ValueError(f"axes {PROFILE_FIELDS} need a 'profile' section")
    if prof is not None and cr is not None:
        raise ValueError("a spec takes either 'crossings' or 'profile'")
    nz, z_max = _native.zgrid(d.get("nz", _native.LZQ_NZ), d.get("z_max", _native.LZQ_Z_MAX))
    ms = d.get("ode_max_steps", ODE_MAX_STEPS)
    if ms is not None and int(ms) < 0:
        raise ValueError("ode_max_steps must be >= 0 (0 or null: no cap)")
    # 0 means "no cap", as --ode-max-steps 0 on the command line does (one meaning in both places)
    return SweepSpec(d.get("name", "custom"), base, axes, int(d.get("n_y", 8000)), d.get("notes", ""), cr, method, prof,
                     nz, z_max, None if ms is None or int(ms) == 0 else int(ms))


def builtin_specs() -> dict:
    """BASELINE.json configs C2-C4 with the grids of SURVEY §8d."""
    ls, lin = np.logspace, np.linspace
    return {
        "C2": SweepSpec("C2", dict(EQUAL_MASS),
                        [("m_mix", ls(-3, 0, 1000)), ("dprime", ls(-3, 1, 1000))],
                        notes="equal-mass config, coupling x sweep-rate, v_w=0.30, F=1 -> delta -> P"),
        "C3": SweepSpec("C3", dict(EQUAL_MASS),
                        [("m_chi_GeV", ls(0, 3.5, 100)), ("I_p", lin(0.05, 1, 100)), ("delta_LZ", ls(-4, 0, 1000))],
                        notes="m_chi crosses T=m/3 inside the window"),
        "C5": SweepSpec("C5", dict(EQUAL_MASS),
                        [("m_mix", ls(-3, 0, 1000)), ("dprime", ls(-3, 1, 1000))],
                        notes="C2 grid, 8 jittered sequential crossings per point, coherent P (propagator)",
                        crossings=CrossingSpec()),
        "P1": SweepSpec("P1", dict(EQUAL_MASS),
                        [("y_B", lin(0.5, 2.0, 100)), ("y_chi", lin(0.5, 2.0, 100)), ("lambda_tr_eff", ls(-3, 0, 100))],
                        notes="P from a bounce profile (synthetic shape 12; PAPER eqs.(5)-(9)) over the couplings "
                              "y_B x y_chi x lambda_tr_eff, then the dense quadrature",
                        profile=ProfileSpec()),
        "C4": SweepSpec("C4", dict(EQUAL_MASS),
                        [("beta_over_H", ls(1, 3, 10)), ("I_p", lin(0.05, 1, 100)), ("v_w", lin(0.05, 0.95, 10)),
                         ("source_shape_sigma_y", lin(3, 30, 10)), ("m_chi_GeV", ls(-1, 3.5, 10)),
                         ("delta_LZ", ls(-4, 0, 100))],
                        notes="full cosmological scan, 1e8 points"),
    }


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """contiguous blocks [r*N/W, (r+1)*N/W)."""
    return rank * total // world, (rank + 1) * total // world


def spec_key(spec: SweepSpec) -> str:
    """Hash of everything a shard's contents depend on: the sweep definition (axes, base
    config, n_y, crossings, ODE method), the library's ABI version, its machine code
    (_native.library_id: any rebuild that changes a kernel changes the key) and the bit-changing
    tuning state (the inner-loop exponential).  --resume after such a change starts afresh
    instead of mixing shards of different numerics."""
    d = {"spec": spec.to_json(), "abi": _native.ABI_VERSION, "lib": _native.library_id(),
         "tune": dict(_native.TUNE_STATE)}
    d["spec"].pop("notes", None)
    return hashlib.sha256(json.dumps(d, sort_keys=True).encode()).hexdigest()[:16]


def _shard_file(out_dir: str, start: int, count: int, key: str = "") -> str:
    return os.path.join(out_dir, f"shard_{key + '_' if key else ''}{start:012d}_{count}.npy")


def prepare_out_dir(out_dir: str, spec: SweepSpec, resume: bool, rank: int = 0) -> str:
    """Create `out_dir`, check / write its manifest.json; returns the shard key.  --resume
    into a directory whose manifest describes another sweep raises instead of mixing tables."""
    os.makedirs(out_dir, exist_ok=True)
    key = spec_key(spec)
    man = os.path.join(out_dir, "manifest.json")
    if resume and os.path.exists(man):
        with open(man) as f:
            old = json.load(f).get("key")
        if old != key:
            raise RuntimeError(f"--resume: {out_dir} holds shards of another sweep (manifest key {old}, this "
                               f"sweep {key}); use a fresh --out directory")
    if rank == 0:
        tmp = man + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump({"key": key, "abi": _native.ABI_VERSION, "lib": _native.library_id(),
                       "tune": dict(_native.TUNE_STATE), "spec_def": spec.to_json()}, f, indent=1)
        os.replace(tmp, man)
    return key


ComputeFn = Callable[[int, int, "object"], None]  # (start, count, out_tensor[count, 6]) -> None
MAX_INFLIGHT_WRITES = 3   # checkpoint chunks copied out and waiting for the disk (pinned ring of <= 4)


def _status_file(shard_path: str) -> str:
    """The ODE status counts of one checkpointed chunk (int64[8] per lzq_ode_status), so a resumed
    sweep's summary counts every chunk, not only those computed by this run."""
    return shard_path[:-len(".npy")] + ".status.npy"


def _save_shard(path: str, arr: np.ndarray) -> None:
    tmp = path + ".tmp.npy"
    np.save(tmp, arr, allow_pickle=False)
    os.replace(tmp, path)


def run_local(compute: ComputeFn, start: int, end: int, make_out: Callable[[int], "object"], chunk: int,
              out_dir: Optional[str] = None, resume: bool = False, sync: Callable[[], None] = lambda: None,
              log: Callable[[str], None] = lambda s: None, key: str = ""):
    """Evaluate [start, end) in chunks into one (end-start, 6) tensor, with optional
    per-chunk checkpoint files (named by `key`, see spec_key).

    On the GPU the checkpoint of chunk i is copied out on a side stream (device -> pinned host
    memory, ordered after chunk i's kernels by an event) and written by a worker thread while
    chunk i+1 computes, so checkpointing does not serialise the sweep.  The pinned buffers are a
    small ring reused chunk after chunk, and at most MAX_INFLIGHT_WRITES writes wait for the disk
    (a slow disk throttles the sweep rather than pinning the whole shard).  On CPU tensors
    (tests) it is written inline."""
    import torch
    local = make_out(end - start)
    on_gpu = bool(getattr(local, "is_cuda", False)) and out_dir is not None
    pending = []    # (future, pinned buffer) of the writes in flight, oldest first
    ring = []       # pinned host buffers free for reuse
    if on_gpu:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=1)
        copy_stream = torch.cuda.Stream(device=local.device)

    def flush(block: bool):
        while pending and (block or pending[0][0].done()):
            fut, buf = pending.pop(0)
            fut.result()   # re-raise a failed write here
            ring.append(buf)

    try:
        for c0 in range(start, end, chunk):
            n = min(chunk, end - c0)
            view = local[c0 - start:c0 - start + n]
            path = _shard_file(out_dir, c0, n, key) if out_dir else None
            if path and resume and os.path.exists(path):
                arr = np.load(path, allow_pickle=False)
                if arr.shape != (n, 6):
                    raise RuntimeError(f"checkpoint {path} has shape {arr.shape}, expected {(n, 6)}")
                view.copy_(torch.from_numpy(arr))
                counts = getattr(compute, "ode_status", None)
                if counts is not None:   # the resumed chunk's ODE status counts (summary.json ode_status)
                    st = _status_file(path)
                    if not os.path.exists(st):
                        raise RuntimeError(f"checkpoint {path} has no ODE status record {st}")
                    counts += np.load(st, allow_pickle=False)
                log(f"resumed {path}")
                continue
            compute(c0, n, view)
            log(f"chunk [{c0}, {c0 + n}) launched")
            if not path:
                continue
            if getattr(compute, "ode_status", None) is not None:
                _save_shard(_status_file(path), np.asarray(compute.last_chunk, dtype=np.int64))
            if not on_gpu:
                sync()
                _save_shard(path, view.detach().cpu().numpy())
                continue
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(local.device))
            # at most MAX_INFLIGHT_WRITES chunks wait for the disk: when the disk is slower than the
            # GPU the sweep waits here instead of pinning the whole shard in host memory
            flush(block=False)
            while len(pending) >= MAX_INFLIGHT_WRITES:
                fut, buf = pending.pop(0)
                fut.result()
                ring.append(buf)
            full = next((b for b in ring if b.shape[0] >= n), None)
            if full is not None:
                ring.remove(full)
            else:
                full = torch.empty((chunk, 6), dtype=view.dtype, pin_memory=True)
            host = full[:n]
            with torch.cuda.stream(copy_stream):
                copy_stream.wait_event(ev)
                host.copy_(view, non_blocking=True)
                done_ev = torch.cuda.Event()
                done_ev.record(copy_stream)

            def write(path=path, host=host, done_ev=done_ev):
                done_ev.synchronize()
                _save_shard(path, host.numpy())
            pending.append((pool.submit(write), full))
            flush(block=False)
        if on_gpu:
            flush(block=True)
    finally:
        if on_gpu:
            pool.shutdown(wait=True)
    return local


def launched_distributed(world: int) -> bool:
    """True under torch.distributed.run (any world size, 1 included: its rendezvous sets
    MASTER_ADDR / MASTER_PORT) or whenever WORLD_SIZE > 1."""
    return world > 1 or ("MASTER_ADDR" in os.environ and "MASTER_PORT" in os.environ)


GATHER_ROWS = 1 << 18   # rows per rank per collective when the shards differ in size


def gather_table(local, total: int, rank: int, world: int, group=None, rows_per_round: int = GATHER_ROWS):
    """All-gather the per-rank shards (sizes differ by <= 1) into the full (total, 6) table on
    every rank (the one collective of north_star (3); every rank keeps the table, 1.7% of a
    288-GB HBM at C4, so any rank can post-process the grid without a second collective).

    Equal shards (C4 at W = 2, 4, 8): one all_gather_into_tensor straight into the output --
    rank-major order IS flat-index order -- with no padding and no concatenation: the transient
    is nothing beyond the table and the rank's own shard.  Unequal shards: the common m0 rows of
    every shard in rounds of <= rows_per_round rows per rank (transient world x rows_per_round
    x 48 B), each round's rank-major block scattered to the shards' places, then one round for
    the last row of the shards that have m0 + 1.  RCCL moves device tensors over xGMI; gloo (CPU
    tests, one-GPU rehearsals) stages through host memory.  With no process group (a plain
    single-process run) the local shard is the table; under a launcher the collective runs even
    for one rank, so a 1-rank torchrun exercises RCCL."""
    import torch
    import torch.distributed as dist
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return local
    rng = [shard_range(total, r, world) for r in range(world)]
    sizes = [e - s for s, e in rng]
    nccl = dist.get_backend(group) == "nccl"
    src = local if nccl else local.cpu()
    src = src.contiguous()
    out = torch.empty((total, 6), dtype=local.dtype, device=src.device)
    if len(set(sizes)) == 1:
        dist.all_gather_into_tensor(out, src, group=group)
        return out if nccl else out.to(local.device)
    m0 = min(sizes)
    c = max(1, min(rows_per_round, m0))
    tmp = torch.empty((world * c, 6), dtype=local.dtype, device=src.device)
    for k in range(0, m0, c):
        cc = min(c, m0 - k)
        buf = tmp[:world * cc]
        dist.all_gather_into_tensor(buf, src[k:k + cc], group=group)
        for r in range(world):
            out[rng[r][0] + k:rng[r][0] + k + cc] = buf[r * cc:(r + 1) * cc]
    last = torch.zeros((1, 6), dtype=local.dtype, device=src.device)
    if sizes[rank] > m0:
        last[0] = src[m0]
    lb = torch.empty((world, 6), dtype=local.dtype, device=src.device)
    dist.all_gather_into_tensor(lb, last, group=group)
    for r in range(world):
        if sizes[r] > m0:
            out[rng[r][0] + m0] = lb[r]
    return out if nccl else out.to(local.device)


def summarize(table: np.ndarray, spec: SweepSpec, elapsed: Optional[float] = None) -> dict:
    """Grid-wide statistics, reduced on the host in flat-index order (deterministic); keys
    match yields_out.json "final" (fpy:425-427) plus P_used."""
    stats = {}
    for j, k in enumerate(YIELD_FIELDS):
        col = table[:, j]
        fin = col[np.isfinite(col)]
        stats[k] = {"min": float(fin.min()) if fin.size else None, "max": float(fin.max()) if fin.size else None,
                    "mean": float(np.add.reduce(fin) / fin.size) if fin.size else None,
                    "n_nonfinite": int(col.size - fin.size)}
    best = int(np.nanargmin(np.abs(table[:, 4] - 5.357)))  # closest to the Planck ratio (PAPER eq.(22))
    return {"spec": spec.name, "n_points": int(table.shape[0]), "fields": list(YIELD_FIELDS), "final": stats,
            "closest_to_planck_ratio": {"index": best, "params": spec.point_params(best),
                                        "final": dict(zip(YIELD_FIELDS, map(float, table[best])))},
            "elapsed_s": elapsed}


def ode_status_summary(counts, group=None, device=None) -> Optional[dict]:
    """Grid-wide ODE point counts per lzq_ode_status (summed over ranks in rank order)."""
    if counts is None:
        return None
    import torch
    import torch.distributed as dist
    c = torch.as_tensor(np.asarray(counts, dtype=np.int64))
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend(group) == "nccl":
            c = c.to(device)
        dist.all_reduce(c, group=group)
    c = c.cpu().numpy()
    names = {_native.ODE_OK: "ok", _native.ODE_BAD_GRID: "bad_grid", _native.ODE_BAD_STEP: "bad_step",
             _native.ODE_TOO_MANY_STEPS: "too_many_steps", _native.ODE_NEWTON: "newton_failed",
             _native.ODE_NOT_LINEAR: "not_linear", _native.ODE_UNRESOLVED: "quadrature_unresolved",
             _native.ODE_BAD_TABLE: "bad_table"}
    return {names.get(k, str(k)): int(v) for k, v in enumerate(c) if v}


def run_sweep(spec: SweepSpec, engine=None, rank: int = 0, world: int = 1, chunk: int = 1 << 20,
              out_dir: Optional[str] = None, resume: bool = False, group=None, log=print, reuse: bool = False):
    """Evaluate `spec` on this rank's shard, all-gather, return the full table (torch, on
    the engine's device)."""
    import torch
    if engine is None:
        from .engine import default_engine
        engine = default_engine()
    start, end = shard_range(spec.total, rank, world)
    key = prepare_out_dir(out_dir, spec, resume, rank) if out_dir else ""

    compute = make_compute(spec, engine, reuse=reuse)
    local = run_local(compute, start, end,
                      lambda n: torch.empty((n, 6), dtype=torch.float64, device=engine.device), chunk,
                      out_dir, resume, sync=torch.cuda.synchronize, log=log, key=key)
    run_sweep.ode_status = ode_status_summary(getattr(compute, "ode_status", None), group, engine.device)
    return gather_table(local, spec.total, rank, world, group)


def coherent_P(spec: SweepSpec, s: int, n: int, engine):
    """Coherent conversion probability of grid points [s, s+n) through their crossings
    (spec.crossings; lzq_lz_propagate), a device tensor."""
    m, dp, xi, v_w = spec.crossing_arrays(s, n, engine.device)
    vw = float(v_w[0]) if bool((v_w == v_w[0]).all()) else v_w   # a v_w axis: per-point wall speeds
    return engine.lz_propagate(m, dp, xi, vw, spec.crossings.window_lz, spec.crossings.steps)


def profile_P(spec: SweepSpec, s: int, n: int, engine, cache: dict):
    """P of grid points [s, s+n) from the spec's bounce profile (ProfileSpec; PAPER eqs.(5)-(9)):
    the profile's splines once per sweep (cache), then per point the crossings and eq.(9) and/or
    the time-ordered propagation through the profile, all on the GPU; a device tensor."""
    import torch
    ps = spec.profile
    if "shape" not in cache:
        cache["shape"] = engine.profile_shapes(*ps.arrays())
    sh = cache["shape"]
    vals = spec.axis_values(s, n, engine.device)
    full = lambda k, d: vals[k] if k in vals else torch.full((n,), float(d), dtype=torch.float64, device=engine.device)
    cols = [full("y_B", ps.y_B), full("y_chi", ps.y_chi), full("lambda_tr_eff", ps.lambda_tr_eff),
            full("v_w", spec.base["v_w"])]
    rec = torch.zeros((n, 5), dtype=torch.float64, device=engine.device)
    for j, c in enumerate(cols):
        rec[:, j] = c
    pts = rec.view(torch.uint8)[:, :40].contiguous().view(-1)   # lzq_profile_point rows (shape 0, reserved 0)
    if ps.estimator == "propagate":
        return engine.lz_propagate_profile(sh, pts, ps.steps_per_radian, ps.min_steps)
    cr = engine.profile_crossings(sh, pts, 1)
    one = cr["count"] == 1
    # delta_lz[:, 0] is written only where a crossing was found: mask the rest before eq.(9)
    delta = torch.where(one, cr["delta_lz"][:, 0], torch.zeros_like(cols[0]))
    P = torch.where(one, engine.p_closed_form(delta), torch.full_like(cols[0], float("nan")))
    many = cr["count"] > 1
    if ps.estimator == "auto" and bool(many.any()):
        sel = torch.nonzero(many).reshape(-1)
        P[sel] = engine.lz_propagate_profile(sh, pts.view(n, 40)[sel].contiguous().view(-1), ps.steps_per_radian,
                                             ps.min_steps)
    return P


def grid_axes_for_kernel(spec: SweepSpec):
    """The spec's axes for lzq_sweep_grid: a profile coupling axis has no lzq_point field, so it
    rides on P_chi_to_B, which the per-point P override replaces (the flat-index decode of the
    other axes is unchanged)."""
    return [("P_chi_to_B" if n in PROFILE_FIELDS else n, v) for n, v in spec.axes]


def make_compute(spec: SweepSpec, engine, reuse: bool = False) -> ComputeFn:
    """(start, count, out) -> None on the GPU: [coherent multi-crossing P ->] quadrature, or
    the ODE fallback (lzq_ode_batch) for sweeps over sigma_v / Gamma_wash / depletion (with or
    without crossings).  reuse: the quadrature's z-sums shared across points with the same
    y-grid and A/V kernel (lzq_sweep_grid_reuse; bit-identical, not the dense headline path)."""
    pcache = {}   # the profile's device splines, built once per sweep
    if is_ode_spec(spec):
        counts = np.zeros(8, dtype=np.int64)   # ODE points per lzq_ode_status, this rank (all chunks)
        tables = {"points": 0, "tables": 0, "per_point_chunks": 0, "chunks": 0}   # this run's chunks

        def compute_ode(s, n, out):
            import torch
            pts, ods = grid_records(spec, s, n, engine)
            if spec.crossings is not None:   # coherent multi-crossing P (propagator) for every point
                pts["P_chi_to_B"] = coherent_P(spec, s, n, engine).cpu().numpy()
            if spec.profile is not None:     # P from the bounce profile
                pts["P_chi_to_B"] = profile_P(spec, s, n, engine, pcache).cpu().numpy()
            # fpy:372 per point: points with no sink/depletion take the quadrature, the rest the ODE
            ode = (ods["sigma_v_chi_GeV_m2"] != 0.0) | (ods["Gamma_wash_over_H"] != 0.0) | \
                  (ods["deplete_DM_from_source"] != 0)
            sel = np.nonzero(ode)[0]
            if sel.size:
                # (a chunk with a single ODE point integrates it parallel in time: the same bits)
                tab, status = engine.ode(pts[sel], ods[sel], method=spec.ode_method, max_steps=spec.ode_max_steps,
                                         nz=spec.nz, z_max=spec.z_max)
                for k in tables:
                    tables[k] += engine.last_ode_tables[k]
                # a point the integrator did not finish normally (a Radau Newton failure reports the
                # state where it stopped, as fpy:408-410 does for the CLI) is a NaN row in a sweep
                # table, counted per status in the summary ("ode_status")
                bad = status != 0
                tab = torch.where(bad[:, None], torch.full_like(tab, float("nan")), tab)
                chunk = np.bincount(status.clamp(0, 7).cpu().numpy(), minlength=8)[:8]
                counts[:] += chunk
                compute_ode.last_chunk = chunk.astype(np.int64)   # written beside the chunk's checkpoint
                out[torch.as_tensor(sel, device=out.device)] = tab
            else:
                compute_ode.last_chunk = np.zeros(8, dtype=np.int64)
            sel = np.nonzero(~ode)[0]
            if sel.size:
                out[torch.as_tensor(sel, device=out.device)] = engine.yields(pts[sel], n_y=spec.n_y, reuse=reuse,
                                                                             nz=spec.nz, z_max=spec.z_max)
        compute_ode.ode_status = counts
        compute_ode.ode_tables = tables
        compute_ode.last_chunk = np.zeros(8, dtype=np.int64)
        return compute_ode

    def compute(s, n, out):
        P_points = coherent_P(spec, s, n, engine) if spec.crossings is not None else None
        if spec.profile is not None:
            P_points = profile_P(spec, s, n, engine, pcache)
        engine.sweep(spec.base, grid_axes_for_kernel(spec), s, n, n_y=spec.n_y, out=out, P_points=P_points,
                     reuse=reuse, nz=spec.nz, z_max=spec.z_max)
    return compute


def main(argv=None):
    import torch
    import torch.distributed as dist
    ap = argparse.ArgumentParser(description="lzq parameter sweep (1..8 GPUs, RCCL all-gather)")
    ap.add_argument("--spec", required=True, help="C2 | C3 | C4 | C5 | P1 | path to a sweep-spec JSON")
    ap.add_argument("--out", default=None, help="directory for shard checkpoints, table.npy, summary.json")
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--limit", type=int, default=None, help="evaluate only the first N grid points")
    ap.add_argument("--reuse-zsums", action="store_true",
                    help="share the quadrature's z-sums between points with the same y-grid and A/V kernel "
                         "(lzq_sweep_grid_reuse: bit-identical, much faster; not the dense headline mode)")
    ap.add_argument("--nz", type=int, default=None, help="z nodes of the A/V kernel (AoverVKernel nz, fpy:142)")
    ap.add_argument("--z-max", type=float, default=None, help="z_max of the A/V kernel (fpy:142)")
    ap.add_argument("--ode-max-steps", type=int, default=None,
                    help=f"cap on one ODE point's Radau steps (default {ODE_MAX_STEPS}; 0 = no cap)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, default) | gloo (rehearsal: several ranks on one GPU)")
    args = ap.parse_args(argv)

    specs = builtin_specs()
    if args.spec in specs:
        spec = specs[args.spec]
    else:
        with open(args.spec) as f:
            spec = spec_from_json(json.load(f))
    if args.nz is not None or args.z_max is not None:
        spec.nz, spec.z_max = _native.zgrid(spec.nz if args.nz is None else args.nz,
                                            spec.z_max if args.z_max is None else args.z_max)
    if args.ode_max_steps is not None:
        spec.ode_max_steps = None if args.ode_max_steps == 0 else args.ode_max_steps
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_rank %= max(1, torch.cuda.device_count())  # gloo rehearsal: several ranks may share a GPU
    torch.cuda.set_device(local_rank)
    use_dist = launched_distributed(world)
    if use_dist:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(args.dist_backend)
    spec_total = spec.total if args.limit is None else min(args.limit, spec.total)

    from .engine import Engine
    eng = Engine(local_rank)
    t0 = time.perf_counter()
    start, end = shard_range(spec_total, rank, world)
    key = prepare_out_dir(args.out, spec, args.resume, rank) if args.out else ""

    compute = make_compute(spec, eng, reuse=args.reuse_zsums)
    local = run_local(compute, start, end,
                      lambda n: torch.empty((n, 6), dtype=torch.float64, device=eng.device), args.chunk,
                      args.out, args.resume, sync=torch.cuda.synchronize,
                      log=(print if rank == 0 else (lambda s: None)), key=key)
    ode_status = ode_status_summary(getattr(compute, "ode_status", None), None, eng.device)
    table = gather_table(local, spec_total, rank, world)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if rank == 0:
        tab = table.cpu().numpy()
        summ = summarize(tab, spec, elapsed)
        summ["points_per_s"] = spec_total / elapsed
        summ["n_gpus"] = world
        if ode_status is not None:
            summ["ode_status"] = ode_status   # ODE-path points per status (non-ok rows are NaN)
            t = getattr(compute, "ode_tables", None)
            if t is not None:   # rank 0's chunks computed by this run: shared A/V spline tables or one per point
                summ["ode_tables"] = dict(t, mode="shared" if t["per_point_chunks"] == 0 else (
                    "per_point" if t["per_point_chunks"] == t["chunks"] else "mixed"))
        if args.reuse_zsums:
            summ["reuse_zsums"] = eng.last_reuse
        if args.out:
            np.save(os.path.join(args.out, "table.npy"), tab, allow_pickle=False)
            with open(os.path.join(args.out, "summary.json"), "w") as f:
                json.dump({**summ, "spec_def": spec.to_json()}, f, indent=2)
        print(json.dumps({k: summ[k] for k in ("spec", "n_points", "points_per_s", "n_gpus", "elapsed_s")}))
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
