#!/usr/bin/env python3
"""Headline benchmark: LZ parameter points/s on 1..8 MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], C2): the shipped equal-mass config swept over the
(coupling m_mix, sweep-rate |Delta'|) grid, v_w = 0.30, F = 1 -> delta (PAPER eq.(8)) ->
P (eq.(9), fpy:183-184) -> dense Y_B quadrature (n_y = 8000 x nz = 1200, fpy:231-267) ->
Y_chi / densities epilogue (fpy:372-417), every point evaluated in full (no cross-point reuse,
no underflow early-exit: SURVEY §8d).  One step = one pass over 1e6 points per GPU.
Weak scaling: at N GPUs the sweep-rate axis is refined N-fold (1000 x 1000N grid) and each
rank owns a contiguous 1e6-point shard; the per-point yield tables (48 B/point) are
all-gathered over RCCL at the end of every step (north_star (3)).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no launcher (no WORLD_SIZE in the environment) starts
the N ranks itself: the parent touches no GPU, runs this same script under
`python -m torch.distributed.run --nproc-per-node N` (one process per GPU, RCCL), lets rank 0's
line through and exits with the launcher's status.  A rank count that disagrees with --gpus, or
more RCCL ranks than the node has GPUs, is an error (exit status 2), never a 1-GPU line.

Prints one JSON line (rank 0).  `roofline` = the kernel's executed FP64 FLOP (PMC
instruction mix of profiles/round6, used only if that profile's kernel ISA hash is the timed
library's) over its HIP-event time in this run, against the 78.6 TFLOP/s FP64 vector peak, with
the FP64-pipe and VALU issue fractions beside it; `kernel_ms` / `allgather_ms` decompose a step
per rank (min / max / mean); `parity_spot` checks 64 rows of the last timed step's table against
the C oracle right after the timed region, before any secondary leg reuses the buffer (the exit
status is non-zero if it, or the table's finiteness / shard placement, fails); `cpu_baseline`
times the C oracle (the CPU restatement, OpenMP) on a bounded random sample of the same grid on
every CPU of this job, and on one core.  `world_size` / `dist_backend` come from the process group
itself and `devices` holds every rank's GPU (PCI bus id, UUID, host), gathered before any timing;
two RCCL ranks reporting one device end the run (exit status 2, no line).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"

METRIC = "LZ param points/sec (node) at 1/2/4/8 MI355X; % FP64 VALU peak"
FLOP_PER_POINT = 30.0 * 8000 * 1200   # 30 FLOP per (y, z) node
PEAK_FP64_TFLOPS = 78.6               # MI355X FP64 vector: 256 CU x 2.4 GHz x 128 FLOP/clk
HBM_PEAK_BPS = 8.0e12                 # MI355X HBM3E (MI355X_MICROARCH.md)
BASE = {  # /root/reference/yields_config_equal_mass.json
    "regime": "nonthermal", "m_chi_GeV": 0.95, "g_chi": 2, "chi_stats": "fermion",
    "sigma_v_chi_GeV_m2": 0.0, "T_p_GeV": 100.0, "beta_over_H": 100.0, "v_w": 0.30, "I_p": 0.34,
    "g_star": 106.75, "g_star_s": 106.75, "P_chi_to_B": 0.14925839040304145,
    "source_shape_sigma_y": 9.0, "Gamma_wash_over_H": 0.0, "incident_flux_scale": 1.07e-9,
    "deplete_DM_from_source": False, "T_max_over_Tp": 5.0, "T_min_over_Tp": 0.001,
    "Y_chi_init": 4.90e-10, "n_chi_at_Tp_GeV3": None,
}


PMC_SUMMARY = os.path.join(ROOT, "profiles", "round6", "pmc_summary.json")
WAVE_NODES_PER_POINT = 8000 * 1200 // 64


def _pmc():
    try:
        with open(PMC_SUMMARY) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def timed_kernel_isa() -> str | None:
    """codeobj.kernel_isa_sha256 of yields_grid_kernel in the library this process loaded: its
    disassembly and descriptors with the layout-dependent PC-relative literals masked, so a
    profile stays tied to the kernel, not to the other kernels of its translation unit."""
    native = importlib.import_module(PKG + "._native")
    return importlib.import_module(PKG + ".codeobj").kernel_isa_sha256(native.LIB_PATH)


def timed_code_object() -> tuple[str | None, str | None]:
    """(kernel code sha256, whole code object sha256) of the gfx950 code object holding
    yields_grid_kernel in the library this process loaded (the one being timed).  The first hashes
    what the GPU executes (.text, kernel descriptors, metadata note: codeobj.kernel_code_sha256), so
    it survives a rebuild with another command line; the second also covers clang's per-build
    __hip_cuid symbol."""
    native = importlib.import_module(PKG + "._native")
    co = importlib.import_module(PKG + ".codeobj")
    return co.kernel_code_sha256(native.LIB_PATH), co.kernel_object_sha256(native.LIB_PATH)


def roofline(points_per_launch: int, kern_ms: float) -> dict:
    """FP64 VALU roofline of yields_grid_kernel for this run.

    achieved = EXECUTED FP64 FLOP per launch / this run's HIP-event kernel time.  The executed
    FLOP per point come from the rocprofv3 PMC pass of the same kernel (profiles/round6, tools/
    gpu_profile.sh): (2 x SQ_INSTS_VALU_FMA_F64 + SQ_INSTS_VALU_MUL_F64 + SQ_INSTS_VALU_ADD_F64)
    x 64 lanes / points; peak = 78.6 TFLOP/s (256 CU x 2.4 GHz x 128 FP64 FLOP/clk/CU, every
    issue slot an FMA).  Also reported: the FP64 pipe's busy fraction (FP64 instructions x 4
    cycles each -- the issue rate the peak is defined by -- over the SIMD cycles of this run at
    the profile's clock), and SURVEY §8d's 30-FLOP stock-exp pricing as a secondary figure."""
    d = _pmc()
    code, sha = timed_code_object()
    stock = FLOP_PER_POINT * points_per_launch / (kern_ms / 1e3) / 1e12
    out = {"bound": "fp64-valu", "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "kernel": "yields_grid_kernel",
           "kernel_ms": kern_ms, "algorithmic_bytes": 48.0 * points_per_launch,
           "stock_exp_equivalent": {"achieved": stock, "flop_per_point": FLOP_PER_POINT,
                                    "note": "SURVEY §8d prices a node at ROCm exp(double) (27 FLOP) + 3: 30 FLOP/node; "
                                            "the table exponential does the node in ~10 executed FLOP, so this "
                                            "figure exceeds the peak and is NOT a roofline fraction"}}
    out["code_object_sha256"] = sha
    out["kernel_code_sha256"] = code
    if d is None or "valu_mix_per_wave_node" not in d:
        out.update(achieved=None, frac=None, traffic=None,
                   note=f"no PMC summary at {os.path.relpath(PMC_SUMMARY, ROOT)}: executed FLOP unknown")
        return out
    isa = timed_kernel_isa() if d and d.get("kernel_isa_sha256") else None
    out["kernel_isa_sha256"] = isa
    if d and d.get("kernel_isa_sha256") and isa:
        same = d["kernel_isa_sha256"] == isa   # the kernel's own machine code and descriptors (round 6)
    else:
        same = d.get("kernel_code_sha256") == code if d.get("kernel_code_sha256") else d.get("code_object_sha256") == sha
    if not same:
        # the counters describe another build of the kernel: no fraction rather than a stale one
        out.update(achieved=None, frac=None, fp64_pipe_busy_frac=None, traffic=None,
                   profile_code_object_sha256=d.get("code_object_sha256"),
                   profile_kernel_code_sha256=d.get("kernel_code_sha256"),
                   profile_kernel_isa_sha256=d.get("kernel_isa_sha256"),
                   note=f"stale profile: {os.path.relpath(PMC_SUMMARY, ROOT)} was measured on kernel code "
                        f"{d.get('kernel_code_sha256') or d.get('code_object_sha256')}, this run timed {code}; "
                        f"re-run tools/gpu.sh profile ROUND")
        return out
    mix = d["valu_mix_per_wave_node"]
    flop_wn = 64.0 * (2.0 * mix["fma_f64"] + mix["mul_f64"] + mix["add_f64"])
    flop_pt = flop_wn * WAVE_NODES_PER_POINT
    achieved = flop_pt * points_per_launch / (kern_ms / 1e3) / 1e12
    fp64_wn = mix["fma_f64"] + mix["mul_f64"] + mix["add_f64"]
    ghz = d["clock_ghz"]
    cyc_wn = 1024 * ghz * 1e9 * (kern_ms / 1e3) / (WAVE_NODES_PER_POINT * points_per_launch)
    other_wn = d["valu_insts_per_wave_node"] - fp64_wn
    out.update({
        "achieved": achieved, "frac": achieved / PEAK_FP64_TFLOPS,
        # the same run as issue utilisation: every FP64 instruction a full 4-cycle slot (the rate
        # the peak is defined by), and with the non-FP64 VALU instructions at 2 cycles each
        "fp64_pipe_busy_frac": 4.0 * fp64_wn / cyc_wn,
        "valu_issue_busy_frac": (4.0 * fp64_wn + 2.0 * other_wn) / cyc_wn,
        "profile_code_object_sha256": d["code_object_sha256"],
        "profile_kernel_code_sha256": d.get("kernel_code_sha256"),
        "profile_kernel_isa_sha256": d.get("kernel_isa_sha256"),
        "flop_per_point_executed": flop_pt,
        "traffic": d["hbm_bytes_per_point"]["total_upper"] * points_per_launch, "traffic_unit": "bytes/launch",
        # north_star: "achieved HBM GB/s for the grid I/O" -- the path is FP64-bound, so this is small
        "grid_io": {"GB_per_s": d["hbm_bytes_per_point"]["total_upper"] * points_per_launch / (kern_ms / 1e3) / 1e9,
                    "frac_of_hbm_peak": d["hbm_bytes_per_point"]["total_upper"] * points_per_launch /
                    (kern_ms / 1e3) / HBM_PEAK_BPS, "hbm_peak_TB_per_s": HBM_PEAK_BPS / 1e12},
        "issue": {"valu_insts_per_wave_node": d["valu_insts_per_wave_node"], "fp64_insts_per_wave_node": fp64_wn,
                  "simd_cycles_per_wave_node": cyc_wn, "clock_ghz": ghz,
                  "fp64_pipe_busy_frac": 4.0 * fp64_wn / cyc_wn,
                  "valubusy_rocprof": d.get("valubusy_rocprof")},
        "source": os.path.relpath(PMC_SUMMARY, ROOT) + f" (PMC at {d['pmc_points_per_launch']} points/launch)",
        "note": "frac = executed FP64 FLOP (PMC instruction mix, FMA = 2) / kernel time / FP64 vector peak. "
                "It is below 1 because MUL/ADD fill a 2-FLOP slot with 1 FLOP and the per-node integer "
                "table address / exponent insert (and the range clamp) take VALU issue slots "
                "(DESIGN.md §4.1). fp64_pipe_busy_frac counts every FP64 instruction as a full slot; "
                "valu_issue_busy_frac adds the other VALU instructions at 2 cycles: the kernel is at its "
                "formulation's issue ceiling, so the lever left is instruction count. The counters are "
                "used only when their profile's kernel ISA hash (the kernel's disassembly and descriptors, "
                "layout-dependent PC-relative literals masked: codeobj.kernel_isa_sha256) equals the timed "
                "library's"})
    return out


def grid_axes(world: int):
    return [("m_mix", np.logspace(-3.0, 0.0, 1000)), ("dprime", np.logspace(-3.0, 1.0, 1000 * world))]


def host_cpus() -> dict:
    """The host cores this process may use: the affinity mask, capped by the cgroup CPU quota
    (cpu.max; on the GPU pool a 1-GPU job gets a 16-CPU quota on a 256-CPU machine, so more
    threads than the quota only time-slice the same 16 CPUs)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "usable": usable,
            "os_cpu_count": os.cpu_count(), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(axes, n_points_total: int, seconds: float = 12.0) -> dict:
    """C oracle (CPU restatement of fpy, OpenMP) on a bounded uniform sample of the grid, on
    every host core this job may use (host_cpus), and on one core."""
    from oracle import oracle as O
    hc = host_cpus()
    threads = hc["usable"]
    rng = np.random.default_rng(0)
    def cfgs(n):
        return [grid_config(axes, int(i), O) for i in rng.integers(0, n_points_total, n)]

    calib = cfgs(threads)
    t0 = time.perf_counter()
    O.points_batch(calib, nthreads=threads)
    per_round = max(time.perf_counter() - t0, 1e-3)
    rounds = max(1, int(seconds / per_round))
    sample = cfgs(threads * rounds)
    t0 = time.perf_counter()
    O.points_batch(sample, nthreads=threads)
    dt = time.perf_counter() - t0
    # the same restatement on one core (1 core and all cores), a short sample
    one = cfgs(max(8, int(2.0 * len(sample) / dt / threads)))
    t1 = time.perf_counter()
    O.points_batch(one, nthreads=1)
    dt1 = time.perf_counter() - t1
    # one thread per CPU of the affinity mask as well (the box's full core count), when the
    # cgroup quota is smaller: those threads time-slice the quota's CPUs, so this shows the
    # quota, not more hardware, bounds the host-side figure
    wide = None
    if hc["affinity_cpus"] > threads:
        nw = hc["affinity_cpus"]
        many = cfgs(max(nw, int(0.5 * len(sample) / nw) * nw))
        t2 = time.perf_counter()
        O.points_batch(many, nthreads=nw)
        dt2 = time.perf_counter() - t2
        wide = {"value": len(many) / dt2, "unit": "points/s", "threads": nw,
                "sample": f"{len(many)} further points, {nw} OpenMP threads (one per CPU of the affinity "
                          f"mask) under the {hc['cgroup_cpu_quota']}-CPU cgroup quota, {dt2:.1f} s"}
    return {"value": len(sample) / dt, "unit": "points/s", "cores": threads, "kind": "port",
            "host": hc, "all_affinity_cpus": wide,
            "sample": f"{len(sample)} uniformly sampled grid points (numpy default_rng(0)), full "
                      f"n_y=8000 x nz=1200 quadrature + epilogue each, C oracle (oracle/lzq_oracle.c) "
                      f"with {threads} OpenMP threads = all CPUs of this job (affinity {hc['affinity_cpus']}, "
                      f"cgroup quota {hc['cgroup_cpu_quota']}), {dt:.1f} s",
            "single_core": {"value": len(one) / dt1, "unit": "points/s", "cores": 1,
                            "sample": f"{len(one)} further points of the same sample stream, 1 thread, {dt1:.1f} s"},
            "reference_python_note": "the reference itself (numpy, fpy:231-267) ran 6.20 points/s on one core "
                                     "of the build container (SURVEY §6); it cannot travel to the GPU box"}


def grid_config(axes, i: int, O) -> dict:
    """The fpy Config of flat grid index i (last axis fastest), P by eqs.(8)-(9) as on the device."""
    m_vals, d_vals = axes[0][1], axes[1][1]
    m, d = m_vals[i // len(d_vals)], d_vals[i % len(d_vals)]
    c = dict(BASE)
    c["P_chi_to_B"] = O.p_closed_form(m * m / (2.0 * max(c["v_w"], 1e-12) * abs(d)))
    return c


def parity_spot(axes, start: int, table: torch.Tensor, n: int = 64) -> dict:
    """Outside the timed region: n default_rng(0)-sampled rows of this rank's timed table against
    the C oracle (the checker the cpu_baseline leg loads anyway), all 6 fields."""
    from oracle import oracle as O
    per = table.shape[0]
    idx = np.sort(np.random.default_rng(0).choice(per, size=min(n, per), replace=False))
    tab = table[torch.as_tensor(idx, device=table.device)].cpu().numpy()
    ref = O.points_batch([grid_config(axes, start + int(i), O) for i in idx], nthreads=host_cpus()["usable"])
    fields = importlib.import_module(PKG + "._native").YIELD_FIELDS
    err = np.where(ref != 0.0, np.abs(tab - ref) / np.where(ref != 0.0, np.abs(ref), 1.0), np.abs(tab))
    worst = float(np.nanmax(err)) if np.isfinite(ref).all() else float("nan")
    return {"n": int(len(idx)), "worst_rel": worst, "fields": list(fields), "gate": 1e-8, "guard_band": 1e-11,
            "ok": bool(worst < 1e-11),
            "sample": f"{len(idx)} rows of the last timed step's table (rank 0 shard), numpy default_rng(0), "
                      f"vs oracle/lzq_oracle.c (pinned to the reference's golden outputs)"}


class Clock:
    """Marks on the timed stream: HIP events on the GPU (elapsed on the device clock), host
    perf_counter after a synchronize otherwise (the CPU rehearsal of tests/test_bench_roofline.py)."""

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.stream = torch.cuda.current_stream() if cuda else None

    def mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record(self.stream)
            return e
        return time.perf_counter()

    def ms(self, a, b) -> float:
        return a.elapsed_time(b) if self.cuda else 1e3 * (b - a)

    def sync(self):
        if self.cuda:
            torch.cuda.synchronize()


def spread(vals) -> dict:
    v = [float(x) for x in vals]
    return {"min": min(v), "max": max(v), "mean": float(np.mean(v)), "per_rank": v}


def device_identity(eng, cuda: bool, rank: int, local: int) -> dict:
    """This rank's device as the hardware names it: PCI domain:bus:device and the HIP UUID of the
    GPU the engine runs on (torch device properties; no HIP call beyond the engine's own), the
    host, and the visibility masks the launcher set.  `key` is what must differ between RCCL
    ranks.  A stand-in engine (tests) supplies its own via eng.device_identity()."""
    rec = {"rank": rank, "local_rank": local, "host": socket.gethostname(),
           "visible": {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                      "CUDA_VISIBLE_DEVICES") if os.environ.get(k) is not None}}
    if hasattr(eng, "device_identity"):
        rec.update(eng.device_identity(rank, local))
    elif cuda:
        idx = eng.device.index if getattr(eng, "device", None) is not None and eng.device.index is not None \
            else torch.cuda.current_device()
        p = torch.cuda.get_device_properties(idx)
        pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
        uuid = str(getattr(p, "uuid", ""))
        rec.update({"device_index": idx, "name": p.name, "arch": p.gcnArchName, "pci_bus_id": pci, "uuid": uuid,
                    "cus": p.multi_processor_count})
    else:
        rec.update({"device_index": None, "pci_bus_id": None, "uuid": None})
    rec.setdefault("key", f"{rec['host']}/{rec.get('pci_bus_id')}/{rec.get('uuid')}")
    return rec


def duplicate_devices(ids: list) -> list:
    """Pairs of ranks whose device keys coincide (two ranks on one GPU)."""
    seen, dups = {}, []
    for r in ids:
        if r["key"] in seen:
            dups.append((seen[r["key"]], r["rank"]))
        else:
            seen[r["key"]] = r["rank"]
    return dups


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(argv: list, n: int) -> int:
    """--gpus N > 1 without a launcher: N ranks of this same script (sys.argv[0]: bench.py, or a
    test's stand-in) under torch.distributed.run on this node, master 127.0.0.1.  Nothing here
    touches a GPU (the ranks do); the children inherit stdout, so rank 0's JSON line is the only
    line.  Returns the launcher's exit status (non-zero if any rank failed)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(sys.argv[0]), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL needs dmabuf IPC on this pool
    print(f"[bench] --gpus {n} without a launcher: starting {n} ranks ({' '.join(cmd[1:8])} ...)", file=sys.stderr,
          flush=True)
    try:
        return subprocess.run(cmd, env=env).returncode
    except OSError as e:
        print(f"[bench] could not start the ranks: {e}", file=sys.stderr)
        return 2


def main(argv=None, engine=None) -> int:
    """The bench (one JSON line on rank 0).  engine: a stand-in with Engine.sweep's signature and a
    torch `device` (tests only: the CPU rehearsal of the timing / evidence order); None = the HIP
    engine on this rank's GPU.  Returns the exit status: non-zero when the timed table fails its
    evidence checks (non-finite rows, a misplaced shard, parity_spot beyond the guard band)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--points", type=int, default=1_000_000, help="points per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity-spot", action="store_true", help="skip the oracle check of 64 timed rows")
    ap.add_argument("--truncated", action="store_true",
                    help="also time one step with exact-underflow truncation (secondary field, not the headline)")
    ap.add_argument("--no-reuse", dest="reuse", action="store_false",
                    help="skip the secondary reuse_zsums field (one step with the z-sums shared between points, "
                         "lzq_sweep_grid_reuse; not the headline: SURVEY §8d keeps the headline dense)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, default) | gloo (rehearsal of the N>1 path on one GPU)")
    argv = list(sys.argv[1:] if argv is None else argv)
    args = ap.parse_args(argv)
    if args.gpus < 1:
        print(f"[bench] --gpus {args.gpus}: need at least 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(argv, args.gpus)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus={args.gpus}: the line would not measure --gpus GPUs",
              file=sys.stderr)
        return 2
    cuda = engine is None
    if cuda:
        ndev = torch.cuda.device_count()   # counts devices without initialising HIP
        if args.dist_backend == "nccl" and world > ndev:
            print(f"[bench] --gpus {world} over RCCL needs {world} GPUs; this node has {ndev}", file=sys.stderr)
            return 2
        local = local % max(1, ndev)  # gloo rehearsal: several ranks may share a GPU
        torch.cuda.set_device(local)
    # a process group whenever a launcher started us (torchrun sets MASTER_ADDR/PORT), so a
    # 1-rank torchrun runs the same RCCL all-gather as N ranks; plain `python bench.py` has none
    use_dist = world > 1 or ("MASTER_ADDR" in os.environ and "MASTER_PORT" in os.environ)
    nccl = cuda and args.dist_backend == "nccl"
    if use_dist:
        if nccl:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    eng = engine if engine is not None else importlib.import_module(PKG + ".engine").Engine(local)
    # every rank's device, gathered before any timing: the line names the GPUs it measured, and
    # two RCCL ranks on one GPU (or a stand-in claiming exclusive devices) end the run here
    me = device_identity(eng, cuda, rank, local)
    if use_dist:
        ids = [None] * world
        dist.all_gather_object(ids, me)
        pg = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend())}
    else:
        ids, pg = [me], {"world_size": 1, "backend": None}
    if pg["world_size"] != args.gpus:
        print(f"[bench] process group has {pg['world_size']} ranks but --gpus={args.gpus}", file=sys.stderr)
        if use_dist:
            dist.destroy_process_group()
        return 2
    dups = duplicate_devices(ids)
    if dups and (nccl or getattr(eng, "exclusive_devices", False)):
        if rank == 0:
            print(f"[bench] ranks {dups} report the same device ({[ids[a]['key'] for a, _ in dups]}): the line "
                  f"would not measure {world} GPUs", file=sys.stderr)
        if use_dist:
            dist.destroy_process_group()
        return 2
    axes = grid_axes(world)
    per = args.points
    total = per * world
    grid_total = len(axes[0][1]) * len(axes[1][1])
    assert total <= grid_total
    start = rank * per
    local_tab = torch.empty((per, 6), dtype=torch.float64, device=eng.device)
    gathered = torch.empty((total, 6), dtype=torch.float64, device=eng.device) if use_dist else local_tab
    clock = Clock(cuda)
    marks = []

    def gather():
        if nccl:
            dist.all_gather_into_tensor(gathered, local_tab)  # RCCL over xGMI
        else:
            parts = [torch.empty((per, 6), dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, local_tab.cpu())
            gathered.copy_(torch.cat(parts))

    def step(record: bool):
        k0 = clock.mark() if record else None
        eng.sweep(BASE, axes, start, per, out=local_tab)
        k1 = clock.mark() if record else None
        if use_dist:
            gather()
        if record:
            marks.append((k0, k1, clock.mark()))

    for _ in range(args.warmup):
        step(False)
    clock.sync()
    if use_dist:
        dist.barrier()
    clock.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    clock.sync()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = float(np.mean([clock.ms(a, b) for a, b, _ in marks]))          # this rank's sweep kernel
    gath = float(np.mean([clock.ms(b, c) for _, b, c in marks]))          # this rank's all-gather
    mine = torch.tensor([elapsed, kern, gath], dtype=torch.float64, device=eng.device if nccl else "cpu")
    if use_dist:
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        every = torch.stack(every).cpu().numpy()
    else:
        every = mine.cpu().numpy()[None, :]
    elapsed = float(every[:, 0].max())   # max over ranks
    kern_ms = float(every[:, 1].max())

    # Evidence on the TIMED table, before the secondary legs below overwrite local_tab: every row
    # of the gathered table finite, rank r's rows at [r*per, (r+1)*per), and parity_spot's oracle
    # rows (rank 0) from the dense table of the last timed step.
    finite = bool(torch.isfinite(gathered).all())
    placed = bool(torch.equal(gathered[start:start + per], local_tab)) if use_dist else True
    spot = parity_spot(axes, start, local_tab) if rank == 0 and not args.no_parity_spot else None
    ok = torch.tensor([1.0 if finite and placed else 0.0], dtype=torch.float64, device=eng.device if nccl else "cpu")
    if use_dist:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    evidence = {"table": "dense timed table (last timed step), checked before the secondary legs",
                "all_finite_and_placed": bool(ok.item() == 1.0), "parity_spot_ok": None if spot is None else spot["ok"]}

    # Secondary (NOT the headline): the same step with exact-underflow truncation of the
    # z-sums (LZQ_TUNE_TRUNCATE), which skips nodes whose terms cannot change the FP64 sums;
    # its table must be bit-identical to the dense one.
    dense_tab = local_tab.clone() if (args.truncated or args.reuse) else None
    trunc = None
    if args.truncated:
        eng.tune_truncate(True)
        clock.sync()
        t1 = time.perf_counter()
        eng.sweep(BASE, axes, start, per, out=local_tab)
        clock.sync()
        t_tr = time.perf_counter() - t1
        eng.tune_truncate(False)
        same = bool(torch.equal(dense_tab, local_tab))
        if use_dist:
            t = torch.tensor([t_tr, 0.0 if same else 1.0], dtype=torch.float64, device=eng.device if nccl else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t_tr, same = float(t[0]), float(t[1]) == 0.0
        trunc = {"value": total / t_tr, "unit": "points/s", "bit_identical_to_dense": same,
                 "note": "exact-underflow truncation (include/lzq.h LZQ_TUNE_TRUNCATE): nodes whose "
                         "terms are < 2^-1080 are skipped; one step, not the headline"}

    # Secondary (NOT the headline): the z-sums computed once per y-grid / A/V kernel and shared
    # by the points (lzq_sweep_grid_reuse); the table must be bit-identical to the dense one.
    reuse = None
    if args.reuse:
        eng.sweep(BASE, axes, start, per, out=local_tab, reuse=True)   # warm-up (table workspace)
        clock.sync()
        t1 = time.perf_counter()
        eng.sweep(BASE, axes, start, per, out=local_tab, reuse=True)
        clock.sync()
        t_re = time.perf_counter() - t1
        same = bool(torch.equal(dense_tab, local_tab))
        if use_dist:
            t = torch.tensor([t_re, 0.0 if same else 1.0], dtype=torch.float64, device=eng.device if nccl else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t_re, same = float(t[0]), float(t[1]) == 0.0
        reuse = {"value": total / t_re, "unit": "points/s", "bit_identical_to_dense": same,
                 "note": "z-sums shared by the points of one y-grid / A/V kernel (include/lzq.h "
                         "lzq_sweep_grid_reuse; the C2 grid has one); one step, not the headline"}

    status = 0 if evidence["all_finite_and_placed"] and (spot is None or spot["ok"]) else 1
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": total * args.steps / elapsed,
            "unit": "points/s",
            "n_gpus": world,
            "world_size": pg["world_size"],
            "dist_backend": pg["backend"],
            "devices": ids,
            "distinct_devices": len({r["key"] for r in ids}),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "C2: yields_config_equal_mass.json swept over m_mix=logspace(-3,0,1000) x "
                                   "|Delta'|=logspace(-3,1,1000*N), v_w=0.30, delta->P->dense Y_B (n_y=8000, "
                                   "nz=1200) + epilogue; 1e6 points per GPU per step",
                       "points_per_gpu": per, "global_points_per_step": total, "n_y": 8000, "nz": 1200,
                       "parallelism": f"grid-sharded x{world}, {'RCCL' if nccl else 'gloo'} "
                                      f"all-gather of 48 B/point yield tables"},
            "roofline": roofline(per, kern_ms) if cuda else None,
            # the step decomposed per rank (means over the timed steps): the sweep kernel (HIP
            # events around it) and the all-gather of the yield table (events after it), so a
            # sub-linear SCALE curve can be attributed to compute imbalance or to the collective
            "kernel_ms": spread(every[:, 1]),
            "allgather_ms": spread(every[:, 2]) if use_dist else None,
            "evidence": evidence,
        }
        if spot is not None:
            rec["parity_spot"] = spot
        if trunc is not None:
            rec["truncated"] = trunc
        if reuse is not None:
            rec["reuse_zsums"] = reuse
        if not args.no_cpu_baseline:
            # after every collective of the run (the other ranks are done), at every N (north_star:
            # the CPU path beside the throughput at 1/2/4/8 GPUs); the sample is the same grid's
            rec["cpu_baseline"] = cpu_baseline(axes, grid_total, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
        if status:
            print(f"[bench] evidence check failed: {evidence}", file=sys.stderr)
    if use_dist:
        dist.destroy_process_group()
    return status


if __name__ == "__main__":
    sys.exit(main())
