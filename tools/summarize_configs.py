#!/usr/bin/env python3
"""profiles/<round>/bench_configs.jsonl from a `tools/gpu.sh configs` run: each config's timed line
(tools/bench_configs.py, one process, warm) with its executed FP64 work from its own rocprofv3 PMC
pass (every kernel of the config's run: tables, propagators, quadrature, integrators), per point:
FLOP = 64 x (2 FMA + MUL + ADD) wave-instructions / points.  The fraction is that FLOP rate at the
timed (wall-clock) throughput over the 78.6 TFLOP/s FP64 vector peak -- wall time includes the
host-side launch work, so it is a lower bound of the kernels' own fraction.

    python tools/summarize_configs.py gpurun_out/configs round6
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 78.6


def main():
    src, tag = sys.argv[1], sys.argv[2]
    timed = [json.loads(l) for l in open(os.path.join(src, "timed.jsonl")) if l.startswith("{")]
    out = []
    for rec in timed:
        c = rec["config"]
        path = os.path.join(src, f"pmc_{c}", "run_counter_collection.csv")
        pm = [json.loads(l) for l in open(os.path.join(src, f"pmc_{c}.jsonl")) if l.startswith("{")]
        if os.path.exists(path) and pm:
            tot = {}
            for r in csv.DictReader(open(path)):
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            pts = pm[0]["points"]
            flop = 64.0 * (2.0 * tot.get("SQ_INSTS_VALU_FMA_F64", 0.0) + tot.get("SQ_INSTS_VALU_MUL_F64", 0.0) +
                           tot.get("SQ_INSTS_VALU_ADD_F64", 0.0)) / pts
            rec["executed_flop_per_point"] = flop
            rec["valu_per_point"] = tot.get("SQ_INSTS_VALU", 0.0) * 64.0 / pts
            rec["executed_fp64_tflops"] = flop * rec["points_per_s"] / 1e12
            rec["frac_of_fp64_peak"] = rec["executed_fp64_tflops"] / PEAK
            rec["pmc"] = {"points": pts, "source": f"rocprofv3 --pmc of tools/bench_configs.py --pmc --only {c}",
                          "note": "every kernel of the config's run; frac at the timed wall-clock rate (a lower "
                                  "bound of the kernels' own)"}
        out.append(rec)
    dst = os.path.join(ROOT, "profiles", tag, "bench_configs.jsonl")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")
    for r in out:
        print(f"{r['config']:20s} {r['points_per_s']:12.4g} points/s  frac {r.get('frac_of_fp64_peak', float('nan')):.3f}")


if __name__ == "__main__":
    main()
