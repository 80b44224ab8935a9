#!/usr/bin/env python3
"""Summarise `tools/gpu.sh lzprop-pmc` output (gpurun_out/lzprop-pmc) into profiles/<round>/prop_pmc.json:
per-dispatch VALU / FP64 instruction counts of lz_propagate_kernel, its rocprofv3 average
duration, the executed FP64 rate (FMA = 2 FLOP, x 64 lanes) against the 78.6 TFLOP/s peak, and
the durations of the launch-order kernels.

    python tools/summarize_prop_pmc.py [gpurun_out/lzprop-pmc] [round4]
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 78.6


def kernel_summary(src, name, n_points):
    agg, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(os.path.join(src, "pmc", "run_counter_collection.csv"))):
        if name in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    if not disp:
        return None
    per = {c: v / len(disp) for c, v in agg.items()}
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
    ks = float(next(v for n, v in stats.items() if name in n)["AverageNs"]) * 1e-9
    f64 = per["SQ_INSTS_VALU_FMA_F64"] + per["SQ_INSTS_VALU_MUL_F64"] + per["SQ_INSTS_VALU_ADD_F64"]
    flop = 64 * (2 * per["SQ_INSTS_VALU_FMA_F64"] + per["SQ_INSTS_VALU_MUL_F64"] + per["SQ_INSTS_VALU_ADD_F64"])
    return {"dispatches_counted": len(disp), "kernel_s": ks, "points_per_s": n_points / ks,
            "valu_per_dispatch": per["SQ_INSTS_VALU"], "fp64_fma_mul_add_per_dispatch": f64,
            "waves": per["SQ_WAVES"], "executed_fp64_tflops": flop / ks / 1e12,
            "frac_of_fp64_peak": flop / ks / 1e12 / PEAK,
            "valu_per_simd_cycle": per["SQ_INSTS_VALU"] / (1024 * ks * 2.4e9)}


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "lzprop-pmc")
    rnd = sys.argv[2] if len(sys.argv) > 2 else "round4"
    n_points = 4e5
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
    out = {
        "source": "tools/gpu.sh lzprop-pmc (rocprofv3 --pmc on tools/prop_only.py 400000 8 1; separate "
                  "--kernel-trace --stats pass) + tools/summarize_prop_pmc.py",
        "config": "C5 slice: 4e5 points x 8 crossings (sweep.builtin_specs()['C5']), longest-first launch order",
        "kernels": {k: kernel_summary(src, k, n_points) for k in ("lz_propagate_kernel", "lz_follow_kernel")},
        "note": "valu_per_simd_cycle: a wave64 FP64 instruction occupies a SIMD for 4 cycles, so 0.25 is the "
                "issue ceiling; lz_follow_kernel (round 3) computes the superadiabatic follow matrices, one "
                "thread per point and cell; the launch-order kernels are in launch_order_kernels_us",
        "launch_order_kernels_us": {n.split("(")[0]: float(v["AverageNs"]) * 1e-3 for n, v in stats.items()
                                    if n.startswith("lzq::") and "lz_propagate_kernel" not in n
                                    and "lz_follow_kernel" not in n},
    }
    ks = [v["kernel_s"] for v in out["kernels"].values() if v]
    out["propagator_s_total"] = sum(ks) + sum(out["launch_order_kernels_us"].values()) * 1e-6
    dst = os.path.join(ROOT, "profiles", rnd, "prop_pmc.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
