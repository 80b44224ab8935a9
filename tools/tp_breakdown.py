#!/usr/bin/env python3
"""Kernel-time breakdown of lzq_ode_integrate_tp calls from a rocprofv3 --kernel-trace of
tools/time_ode_single.py: each call is the kernels from the A/V table build before an
ode_tp_init_kernel to the last kernel before the next table build; per call, the summed duration
per kernel name and the wall span from the first kernel's start to the last one's end.

    python tools/tp_breakdown.py gpurun_out/<dir>/trace/run_kernel_trace.csv [guess_only=1]
"""
import csv
import re
import sys
from collections import OrderedDict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n.replace("lzq::", "")


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 1   # 1: only calls with the coarse guess (long Riccati windows)
    # split into calls at each ode_aov_table kernel (the table build opens every Engine.ode call)
    calls, cur = [], []
    for r in rows:
        if "ode_aov_table_kernel" in r["Kernel_Name"] and cur:
            calls.append(cur)
            cur = []
        cur.append(r)
    calls.append(cur)
    for c in calls:
        names = [short(r["Kernel_Name"]) for r in c]
        if "ode_tp_init_kernel" not in names:
            continue
        nint = names.count("ode_tp_interval_kernel")
        if want and "ode_tp_guess_kernel" not in names:
            continue
        agg = OrderedDict()
        for r in c:
            k = short(r["Kernel_Name"])
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a = agg.setdefault(k, [0, 0.0])
            a[0] += 1
            a[1] += d
        span = (int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3
        busy = [r for r in c if (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) > 4000]
        print(f"call: {len(c)} kernels ({len(busy)} over 4 us), {nint} interval launches, span {span:.0f} us, kernels {sum(v[1] for v in agg.values()):.0f} us")
        for k, (cnt, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"  {k:45s} x{cnt:3d} {d:9.1f} us")


if __name__ == "__main__":
    main()
