#!/usr/bin/env python3
"""Summarise the bounce-profile path's GPU runs (tools/gpu_prof_r3b.sh / tools/gpu_r3c.sh output in
gpurun_out/profprop) into profiles/<round>/: profile_pmc.json (per-dispatch VALU / FP64
instruction counts of profile_propagate_kernel, its rocprofv3 average duration, the executed
FP64 rate against the 78.6 TFLOP/s peak), profile_kernel_stats.csv and the bench lines.

    python tools/summarize_profile_pmc.py [gpurun_out/profprop] [round3]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 78.6


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "profprop")
    rnd = sys.argv[2] if len(sys.argv) > 2 else "round3"
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    agg, disp = collections.defaultdict(float), set()
    for r in csv.DictReader(open(os.path.join(src, "pmc", "run_counter_collection.csv"))):
        if "profile_propagate_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    per = {c: v / len(disp) for c, v in agg.items()}
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "profile_kernel_stats.csv"))
    ks = float(next(v for n, v in stats.items() if "profile_propagate_kernel" in n)["AverageNs"]) * 1e-9
    bench = json.load(open(os.path.join(src, "bench_traced.json")))
    n = bench["points"]
    steps = bench["magnus_steps_per_point"]["total"]
    f64 = per["SQ_INSTS_VALU_FMA_F64"] + per["SQ_INSTS_VALU_MUL_F64"] + per["SQ_INSTS_VALU_ADD_F64"]
    flop = 64 * (2 * per["SQ_INSTS_VALU_FMA_F64"] + per["SQ_INSTS_VALU_MUL_F64"] + per["SQ_INSTS_VALU_ADD_F64"])
    out = {
        "source": "rocprofv3 --pmc on tools/bench_profile.py 1000000 1 --only propagate; separate --kernel-trace "
                  "--stats pass on tools/bench_profile.py 1000000 3 (tools/gpu_r3c.sh) + tools/summarize_profile_pmc.py",
        "kernel": "profile_propagate_kernel",
        "config": f"{n} points, {bench['shapes']} synthetic bounce shapes x {bench['knots']} knots "
                  f"(bounce.synthetic_shapes / synthetic_couplings), {bench['steps_per_radian']} steps per radian, "
                  "cost-ordered launch",
        "dispatches_counted": len(disp),
        "kernel_s": ks,
        "points_per_s": n / ks,
        "magnus_steps_per_point": bench["magnus_steps_per_point"],
        "magnus_steps_per_s": steps / ks,
        "valu_per_dispatch": per["SQ_INSTS_VALU"],
        "fp64_fma_mul_add_per_dispatch": f64,
        "fp64_share_of_valu": f64 / per["SQ_INSTS_VALU"],
        "waves": per["SQ_WAVES"],
        "wave_valu_per_lane_step": 64 * per["SQ_INSTS_VALU"] / steps,
        "executed_fp64_tflops": flop / ks / 1e12,
        "frac_of_fp64_peak": flop / ks / 1e12 / PEAK,
        "valu_per_simd_cycle": per["SQ_INSTS_VALU"] / (1024 * ks * 2.4e9),
        "note": "executed FP64 counts every lane of a wave instruction (FMA = 2 FLOP); lanes idle while a "
                "wave waits for its longest lane in a knot interval count too, which wave_valu_per_lane_step "
                "(wave VALU x 64 / useful lane-steps) exposes. valu_per_simd_cycle: an FP64 wave64 instruction "
                "occupies a SIMD for 4 cycles, so 0.25 is the issue ceiling.",
        "other_kernels_us": {n.split("(")[0]: float(v["AverageNs"]) * 1e-3 for n, v in stats.items()
                             if "profile_propagate_kernel" not in n and n.startswith("lzq::")},
    }
    with open(os.path.join(dst, "profile_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    for name in ("bench.json", "bench_sorted.json", "bench_1e6.json", "bench_1e6_sorted.json", "ablate.json"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, "profile_" + name))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
