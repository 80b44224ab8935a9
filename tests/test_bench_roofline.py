"""bench.py's roofline fields are reproducible by hand from the committed rocprofv3 CSVs
(profiles/round3): executed FP64 FLOP per point from the PMC instruction-mix pass, the
kernel's average duration from the kernel-trace stats of the bench command itself.  The
counters are used only for the kernel code they were measured on (codeobj.kernel_code_sha256 in
pmc_summary.json: machine code, descriptors and metadata of the code object); any other build gets
frac = null and a "stale profile" note."""
import csv
import importlib
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

PROF = os.path.dirname(bench.PMC_SUMMARY)   # this round's committed profile (profiles/round6)


def counters(path, kernel="yields_grid_kernel"):
    tot = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


def test_executed_flop_from_committed_csv():
    import pytest
    if not os.path.exists(os.path.join(PROF, "pmc_mix.csv")):
        pytest.skip(f"{os.path.relpath(PROF, ROOT)} holds no PMC pass yet")
    c = counters(os.path.join(PROF, "pmc_mix.csv"))
    points = 200_000                                     # tools/gpu.sh profile: the PMC launch size
    flop_pt = 64 * (2 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"]) / points
    stats = [r for r in csv.DictReader(open(os.path.join(PROF, "kernel_stats.csv"))) if "yields_grid_kernel" in r["Name"]]
    assert len(stats) == 1 and int(stats[0]["Calls"]) == 25     # bench.py --steps 20 --warmup 5
    kern_ms = float(stats[0]["AverageNs"]) / 1e6
    rf = bench.roofline(1_000_000, kern_ms)
    import json
    summ = json.load(open(os.path.join(PROF, "pmc_summary.json")))
    same = (rf.get("kernel_isa_sha256") == summ["kernel_isa_sha256"]) if summ.get("kernel_isa_sha256") and \
        rf.get("kernel_isa_sha256") else rf["kernel_code_sha256"] == summ.get("kernel_code_sha256")
    if not same:
        # the library here is another build of the kernel than the profiled one
        assert rf["frac"] is None and rf["note"].startswith("stale profile"), rf
        return
    assert abs(rf["flop_per_point_executed"] / flop_pt - 1) < 1e-12
    frac = flop_pt * 1e6 / (kern_ms / 1e3) / 1e12 / 78.6
    assert abs(rf["frac"] - frac) < 1e-12 and 0.5 < frac < 1.0
    # HBM traffic: FETCH_SIZE (x2, the gfx950 correction) and WRITE_SIZE passes, KiB per launch
    fetch = counters(os.path.join(PROF, "pmc_fetch.csv"))["FETCH_SIZE"] * 1024
    write = counters(os.path.join(PROF, "pmc_write.csv"))["WRITE_SIZE"] * 1024
    assert abs(rf["traffic"] / ((2 * fetch + write) / points * 1e6) - 1) < 1e-12
    assert write / points == 48.0 and rf["traffic"] < 1.2 * rf["algorithmic_bytes"]


# ---- the bench's evidence chain and step decomposition, rehearsed on the CPU -----------------
import json
import socket
import subprocess

FAKE = os.path.join(ROOT, "tests", "bench_fake.py")
SMALL = ["--points", "64", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]


def _run(cmd, env=None):
    e = dict(os.environ, **(env or {}))
    e.pop("MASTER_ADDR", None), e.pop("MASTER_PORT", None)
    return subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=600)


def _line(out):
    recs = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert len(recs) == 1, out
    return recs[0]


def test_evidence_checks_the_dense_timed_table():
    """parity_spot and the finiteness check run on the last timed step's dense table, before the
    truncated / reuse legs reuse the buffer (the stand-in engine writes NaN in those modes): the
    line's evidence is clean and the exit status 0; the secondary legs' own comparisons see the
    NaN rows and report bit_identical_to_dense = false."""
    r = _run([sys.executable, FAKE, *SMALL, "--truncated"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r.stdout)
    assert rec["parity_spot"]["ok"] and rec["parity_spot"]["n"] == 64
    assert rec["evidence"]["all_finite_and_placed"] and rec["evidence"]["parity_spot_ok"]
    assert rec["truncated"]["bit_identical_to_dense"] is False and rec["reuse_zsums"]["bit_identical_to_dense"] is False
    assert rec["kernel_ms"]["max"] >= rec["kernel_ms"]["min"] > 0 and rec["allgather_ms"] is None


def test_parity_failure_exits_nonzero():
    """One timed row off by 1e-6 relative: the line is still printed, parity_spot.ok is false and
    bench.py exits non-zero."""
    r = _run([sys.executable, FAKE, *SMALL, "--no-reuse"], env={"FAKE_BAD_ROW": "5"})
    assert r.returncode == 1
    rec = _line(r.stdout)
    assert rec["parity_spot"]["ok"] is False and rec["evidence"]["parity_spot_ok"] is False


def test_two_rank_line_is_decomposed():
    """The N > 1 path under torchrun (2 gloo ranks on the CPU): the value counts both shards, and the
    line carries per-rank kernel and all-gather times (min / max / mean / per_rank)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2", "--master-addr",
              "127.0.0.1", "--master-port", str(port), FAKE, "--gpus", "2", *SMALL, "--no-reuse", "--no-parity-spot",
              "--dist-backend", "gloo"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["global_points_per_step"] == 128
    for k in ("kernel_ms", "allgather_ms"):
        assert len(rec[k]["per_rank"]) == 2 and rec[k]["max"] >= rec[k]["mean"] >= rec[k]["min"] >= 0.0, rec[k]
    assert rec["evidence"]["all_finite_and_placed"]
    assert abs(rec["value"] - 128 / (rec["ms_per_step"] / 1e3)) <= 1e-6 * rec["value"]


def test_gpus_n_without_launcher_spawns_the_ranks():
    """`bench.py --gpus 2` with no launcher: the parent starts the 2 ranks itself
    (torch.distributed.run of the same script), and the one line it lets through measured both:
    n_gpus 2, the all-gather timed on both ranks, and the CPU baseline beside it (north_star: at
    every N)."""
    r = _run([sys.executable, FAKE, "--gpus", "2", "--points", "64", "--steps", "2", "--warmup", "1", "--no-reuse",
              "--no-parity-spot", "--dist-backend", "gloo", "--cpu-seconds", "0.5"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["global_points_per_step"] == 128
    assert rec["allgather_ms"] is not None and len(rec["allgather_ms"]["per_rank"]) == 2
    assert rec["cpu_baseline"]["value"] > 0 and rec["cpu_baseline"]["kind"] == "port"
    assert "starting 2 ranks" in r.stderr


def test_rank_count_mismatch_is_an_error():
    """A launcher's WORLD_SIZE that disagrees with --gpus exits 2 and prints no line (it would not
    measure --gpus GPUs)."""
    r = _run([sys.executable, FAKE, "--gpus", "4", *SMALL], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "WORLD_SIZE=1 but --gpus=4" in r.stderr


def test_n_rank_line_names_distinct_devices():
    """at N > 1 the line carries the process group's own world size and backend
    and one device record per rank (PCI bus id, UUID, host), and counts the distinct devices; the
    CPU baseline is still there."""
    r = _run([sys.executable, FAKE, "--gpus", "2", "--points", "64", "--steps", "2", "--warmup", "1", "--no-reuse",
              "--no-parity-spot", "--dist-backend", "gloo", "--cpu-seconds", "0.5"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["dist_backend"] == "gloo"
    assert [d["rank"] for d in rec["devices"]] == [0, 1]
    assert rec["distinct_devices"] == 2 and len({d["pci_bus_id"] for d in rec["devices"]}) == 2
    assert all(d["uuid"] and d["host"] for d in rec["devices"])
    assert rec["cpu_baseline"]["value"] > 0


def test_two_ranks_on_one_device_exit_nonzero():
    """Two ranks that report the same device (a stand-in claiming exclusive devices, as RCCL ranks
    are): exit 2 before any timing, no line."""
    r = _run([sys.executable, FAKE, "--gpus", "2", "--points", "64", "--steps", "2", "--warmup", "1", "--no-reuse",
              "--no-parity-spot", "--dist-backend", "gloo", "--no-cpu-baseline"], env={"FAKE_DUP_DEVICE": "1"})
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "report the same device" in r.stderr


def test_single_rank_line_names_its_device():
    r = _run([sys.executable, FAKE, *SMALL, "--no-reuse", "--no-parity-spot"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _line(r.stdout)
    assert rec["world_size"] == 1 and rec["dist_backend"] is None and rec["distinct_devices"] == 1
    assert len(rec["devices"]) == 1 and rec["devices"][0]["rank"] == 0
