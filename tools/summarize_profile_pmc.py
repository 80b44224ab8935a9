#!/usr/bin/env python3
"""Summarise the bounce-profile path's GPU runs (`tools/gpu.sh prop-pmc`, output in
gpurun_out/prop-pmc) into profiles/<round>/: profile_pmc.json (per-dispatch VALU / FP64
instruction counts of each propagation kernel, its rocprofv3 average duration, the executed FP64
rate against the 78.6 TFLOP/s peak, and per path -- flattened (profile_steps_kernel +
profile_flat_kernel) and the interval loop (profile_key_kernel + the radix sort +
profile_propagate_kernel, the default) -- wave VALU x 64 per useful lane-step), profile_kernel_stats.csv and
the bench line.

    python tools/summarize_profile_pmc.py [gpurun_out/prop-pmc] [round4]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 78.6
KERNELS = ("profile_steps_kernel", "profile_flat_kernel", "profile_key_kernel", "profile_propagate_kernel",
           "profile_samples_kernel")
PATHS = {"flat": ("profile_steps_kernel", "profile_flat_kernel"),
         "interval_loop": ("profile_key_kernel", "profile_propagate_kernel")}


def short(name):
    return next((k for k in KERNELS if k in name), None)


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "prop-pmc")
    rnd = sys.argv[2] if len(sys.argv) > 2 else "round4"
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(src, "pmc", "run_counter_collection.csv"))):
        k = short(r["Kernel_Name"])
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    per = {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in agg.items()}
    stall = {}
    sp = os.path.join(src, "pmc_stall", "run_counter_collection.csv")
    if os.path.exists(sp):   # wave-time split of the propagation kernel (its own PMC pass)
        sa, sd = collections.defaultdict(float), set()
        for r in csv.DictReader(open(sp)):
            if "profile_propagate_kernel" in r["Kernel_Name"]:
                sa[r["Counter_Name"]] += float(r["Counter_Value"])
                sd.add(r["Dispatch_Id"])
        if sa.get("SQ_WAVE_CYCLES"):
            wc = sa["SQ_WAVE_CYCLES"]
            stall = {"kernel": "profile_propagate_kernel", "dispatches": len(sd),
                     **{c: sa[c] / wc for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS",
                                                 "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY") if c in sa},
                     "note": "fractions of the waves' cycles (SQ_WAVE_CYCLES): ACTIVE_INST_* = a wave had an "
                             "instruction of that kind in flight, WAIT_INST_ANY = waiting for an instruction's "
                             "dependency (issue/latency), WAIT_ANY = waiting on anything (memory included)"}
    stats, sort_ns = {}, 0.0
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    for r in rows:
        k = short(r["Name"])
        if k:
            stats[k] = float(r["AverageNs"]) * 1e-9
        elif "rocprim" in r["Name"] or "hipcub" in r["Name"]:
            sort_ns += float(r["TotalDurationNs"])
    calls = next((float(r["Calls"]) for r in rows if "profile_key_kernel" in r["Name"]), 0.0)
    sort_s = sort_ns * 1e-9 / calls if calls else 0.0   # the radix sort's kernels, per keyed launch
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "profile_kernel_stats.csv"))
    bench = json.load(open(os.path.join(src, "bench_traced.json")))
    n = bench["points"]
    steps = bench["magnus_steps_per_point"]["total"]
    kern = {}
    for k, c in per.items():
        f64 = c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0) + c.get("SQ_INSTS_VALU_ADD_F64", 0)
        flop = 64 * (2 * c.get("SQ_INSTS_VALU_FMA_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0)
                     + c.get("SQ_INSTS_VALU_ADD_F64", 0))
        ks = stats.get(k)
        kern[k] = {"dispatches_counted": len(disp[k]), "kernel_s": ks, "valu_per_dispatch": c["SQ_INSTS_VALU"],
                   "salu_per_dispatch": c.get("SQ_INSTS_SALU"), "trans_f64_per_dispatch": c.get("SQ_INSTS_VALU_TRANS_F64"),
                   "fp64_share_of_valu": f64 / c["SQ_INSTS_VALU"], "waves": c["SQ_WAVES"],
                   "wave_valu_per_lane_step": 64 * c["SQ_INSTS_VALU"] / steps,
                   "executed_fp64_tflops": flop / ks / 1e12 if ks else None,
                   "valu_per_simd_cycle": c["SQ_INSTS_VALU"] / (1024 * ks * 2.4e9) if ks else None}
    paths = {}
    for name, ks in PATHS.items():
        if all(k in kern and kern[k]["kernel_s"] for k in ks):
            t = sum(kern[k]["kernel_s"] for k in ks) + (sort_s if name == "interval_loop" else 0.0)
            paths[name] = {"kernels": list(ks) + (["radix sort"] if name == "interval_loop" else []), "kernel_s": t, "points_per_s": n / t, "magnus_steps_per_s": steps / t,
                           "wave_valu_per_lane_step": sum(kern[k]["wave_valu_per_lane_step"] for k in ks)}
    out = {
        "source": "tools/gpu.sh prop-pmc: rocprofv3 --pmc on tools/bench_profile.py N 1 --only propagate --ab; a "
                  "separate --kernel-trace --stats pass on tools/bench_profile.py N 3 --only propagate --ab; "
                  "tools/summarize_profile_pmc.py",
        "config": f"{n} points, {bench['shapes']} synthetic bounce shapes x {bench['knots']} knots "
                  f"(bounce.synthetic_shapes / synthetic_couplings), {bench['steps_per_radian']} steps per radian, "
                  "keyed launch order",
        "magnus_steps_per_point": bench["magnus_steps_per_point"],
        "paths": paths,
        "wave_time_split": stall or None,
        "kernels": kern,
        "bench": bench.get("propagate"),
        "note": "wave_valu_per_lane_step = 64 x wave VALU instructions / useful Magnus lane-steps; it counts the "
                "step rule (profile_steps_kernel / profile_key_kernel + the loop's per-interval rule), entering "
                "intervals and idle lanes. valu_per_simd_cycle: an FP64 wave64 instruction occupies a SIMD for 4 "
                "cycles, so 0.25 is the issue ceiling.",
    }
    with open(os.path.join(dst, "profile_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    shutil.copy(os.path.join(src, "bench_traced.json"), os.path.join(dst, "profile_bench.json"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
