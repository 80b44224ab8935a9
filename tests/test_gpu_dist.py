"""The real engine through the multi-rank path on one GPU: fresh child
processes launched by torch.distributed.run, 2 ranks sharing cuda:0, gloo for the gather
(RCCL refuses two ranks on one device; the 8-GPU RCCL run is the driver's).  Nothing in
this module touches the GPU in the pytest process itself.

- sweep.main over a 4096-point C3 slice at world_size 2 == the single-rank table, bit for
  bit (each point is reduced by one wavefront, so sharding cannot change a result);
- bench.py under torchrun with --dist-backend gloo emits one valid JSON line whose value
  counts both ranks' points;
- the RCCL code path itself (process group on the device, all_gather_into_tensor of the
  device-resident yield tables) with ONE rank under torchrun: bench.py and sweep.main, the
  sweep table bit-identical to the plain single-process run.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG_NAME, ROOT

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(cmd, timeout):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (cmd, r.stdout[-3000:], r.stderr[-3000:])
    return r.stdout


def torchrun(n):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(free_port())]


def test_sweep_two_ranks_bit_identical_to_one(tmp_path):
    args = ["--spec", "C3", "--limit", "4096", "--chunk", "1500"]
    one, two = tmp_path / "w1", tmp_path / "w2"
    run([sys.executable, "-m", PKG_NAME + ".sweep", *args, "--out", str(one)], 300)
    out = run(torchrun(2) + ["-m", PKG_NAME + ".sweep", *args, "--out", str(two), "--dist-backend", "gloo"], 300)
    t1, t2 = np.load(one / "table.npy"), np.load(two / "table.npy")
    assert t1.shape == (4096, 6) and np.isfinite(t1).all()
    assert np.array_equal(t1, t2)
    line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["n_points"] == 4096
    # both ranks checkpointed their own chunks: rank 0 [0, 2048), rank 1 [2048, 4096)
    starts = sorted(int(f.split("_")[2]) for f in os.listdir(two) if f.startswith("shard_"))
    assert starts == [0, 1500, 2048, 3548]


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multi_rank_gloo(world):
    """bench.py's N > 1 path (rank shards of the W-fold refined grid, the per-step gather,
    barrier + max-over-ranks timing) with W ranks sharing the one GPU."""
    out = run(torchrun(world) + ["bench.py", "--gpus", str(world), "--steps", "1", "--warmup", "1", "--points",
                                 "20000", "--dist-backend", "gloo"], 300)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert len(recs) == 1
    r = recs[0]
    assert r["n_gpus"] == world and r["config"]["global_points_per_step"] == 20000 * world
    assert r["value"] > 0 and r["unit"] == "points/s" and r["scaling"] == "weak"
    assert abs(r["value"] - 20000 * world / (r["ms_per_step"] / 1e3)) <= 1e-6 * r["value"]
    assert r["cpu_baseline"]["value"] > 0 and r["cpu_baseline"]["kind"] == "port"   # rank 0, at every N


def test_bench_single_rank_line():
    """bench.py at N = 1 (small): one JSON line with the contract's fields, a roofline fraction
    in (0, 1] from executed FP64 FLOP, and the CPU baseline on every CPU of this job."""
    out = run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--points", "50000",
               "--cpu-seconds", "1"], 300)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert len(recs) == 1
    r = recs[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["dtype"] == "f64" and r["config"]["points_per_gpu"] == 50000
    rf = r["roofline"]
    assert rf["unit"] == "TFLOP/s" and rf["peak"] == 78.6
    assert rf["frac"] is not None and 0.0 < rf["frac"] <= 1.0, rf
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    assert rf["stock_exp_equivalent"]["achieved"] > rf["achieved"]
    cb = r["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == cb["host"]["usable"] and cb["value"] > 0


def test_rccl_one_rank_sweep_bit_identical(tmp_path):
    """sweep.main under a 1-rank torchrun: an RCCL process group on cuda:0 and the
    all_gather_into_tensor of gather_table (padding, placement) over the real engine's table."""
    args = ["--spec", "C4", "--limit", "3000", "--chunk", "1024"]
    one, rccl = tmp_path / "plain", tmp_path / "rccl"
    run([sys.executable, "-m", PKG_NAME + ".sweep", *args, "--out", str(one)], 300)
    run(torchrun(1) + ["-m", PKG_NAME + ".sweep", *args, "--out", str(rccl), "--dist-backend", "nccl"], 300)
    t1, t2 = np.load(one / "table.npy"), np.load(rccl / "table.npy")
    assert t1.shape == (3000, 6) and np.isfinite(t1).all()
    assert np.array_equal(t1, t2)


def test_rccl_one_rank_bench_line():
    """bench.py under a 1-rank torchrun takes the RCCL branch (process group, per-step
    all_gather_into_tensor, barrier, max-over-ranks all_reduce on the device) and still emits
    one valid line."""
    out = run(torchrun(1) + ["bench.py", "--gpus", "1", "--steps", "1", "--warmup", "1", "--points", "20000",
                             "--no-cpu-baseline"], 300)
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert len(recs) == 1
    r = recs[0]
    assert r["n_gpus"] == 1 and "RCCL" in r["config"]["parallelism"]
    assert r["value"] > 0 and abs(r["value"] - 20000 / (r["ms_per_step"] / 1e3)) <= 1e-6 * r["value"]


def test_sweep_two_ranks_reuse_equals_dense(tmp_path):
    """--reuse-zsums through the multi-rank path: 2 ranks (gloo) on a 4096-point C4 slice give the
    dense single-rank table bit for bit (each rank builds the tables it needs itself)."""
    args = ["--spec", "C4", "--limit", "4096", "--chunk", "1500"]
    one, two = tmp_path / "dense", tmp_path / "reuse2"
    run([sys.executable, "-m", PKG_NAME + ".sweep", *args, "--out", str(one)], 300)
    run(torchrun(2) + ["-m", PKG_NAME + ".sweep", *args, "--out", str(two), "--dist-backend", "gloo",
                       "--reuse-zsums"], 300)
    assert np.array_equal(np.load(one / "table.npy"), np.load(two / "table.npy"))
