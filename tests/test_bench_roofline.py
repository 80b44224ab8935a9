"""bench.py's roofline fields are reproducible by hand from the committed rocprofv3 CSVs
(profiles/round3): executed FP64 FLOP per point from the PMC instruction-mix pass, the
kernel's average duration from the kernel-trace stats of the bench command itself.  The
counters are used only for the code object they were measured on (its sha256 is in
pmc_summary.json); any other build gets frac = null and a "stale profile" note."""
import csv
import importlib
import os
import sys

from conftest import ROOT

PROF = os.path.join(ROOT, "profiles", "round3")


def counters(path, kernel="yields_grid_kernel"):
    tot = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


def test_executed_flop_from_committed_csv():
    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    c = counters(os.path.join(PROF, "pmc_mix.csv"))
    points = 200_000                                     # tools/gpu_profile.sh PMC launch size
    flop_pt = 64 * (2 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"]) / points
    stats = [r for r in csv.DictReader(open(os.path.join(PROF, "kernel_stats.csv"))) if "yields_grid_kernel" in r["Name"]]
    assert len(stats) == 1 and int(stats[0]["Calls"]) == 25     # bench.py --steps 20 --warmup 5
    kern_ms = float(stats[0]["AverageNs"]) / 1e6
    rf = bench.roofline(1_000_000, kern_ms)
    import json
    summ = json.load(open(os.path.join(PROF, "pmc_summary.json")))
    if rf["code_object_sha256"] != summ["code_object_sha256"]:
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
