#!/usr/bin/env python3
"""profiles/<round>/ode_pmc.json from a `tools/gpu.sh ode-pmc` run: per config, the
ode_integrate_kernel's VALU and FP64 instructions per wave-step (PMC pass) and its duration
(kernel-trace pass), hence executed FP64 TFLOP/s against the 78.6 TFLOP/s FP64 vector peak.
bench_ode.py runs, per config, the shared-table and the per-point-table path: two
ode_integrate_kernel<false> dispatches with the same work, in that order (the quadrature
method's ode_integrate_kernel<true> dispatches are not counted)."""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def integrator(name: str) -> bool:
    """A dispatch of the Radau integrator: every ode_integrate_kernel<false, ...> variant and, since
    round 5, the three ode_riccati_kernel passes (each launch runs all of them; each steps its own
    waves)."""
    return "ode_integrate_kernel<false" in name or "ode_riccati_kernel" in name


CONFIGS = [("narrow_wash", 262144, 20000), ("stiff_thermal", 262144, 25385), ("full_window_wash", 16384, 999800)]


def main_cases(src: str, tag: str, fname: str = "ode_pmc.json") -> None:
    """`tools/gpu.sh ode-pmc` layout: tools/ode_pmc_run.py's three cases, one 262,144-point
    ode_integrate_kernel<false> dispatch each (after a 64-point warm-up), in CASES order."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from ode_pmc_run import CASES, N
    # ode_integrate_kernel<false> (one dispatch per case), or since the linear-wave variant
    # <false, false> + <false, true>, and since the split-free variant <false, false, false> +
    # <false, false, true> + <false, true, false>: one dispatch per variant and case, each stepping
    # its own wavefronts (summed)
    per = 1
    def passes(sub):
        nonlocal per
        rows = list(csv.DictReader(open(os.path.join(src, sub, "run_counter_collection.csv"))))
        disp = defaultdict(dict)
        names = set()
        for r in rows:
            if integrator(r["Kernel_Name"]):
                names.add(r["Kernel_Name"])
                per = max(per, len(names))
                d = disp[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        big = [disp[k] for k in sorted(disp) if disp[k].get("SQ_WAVES", 0) >= N // 64]
        out = []
        for j in range(0, len(big), per):
            c = {k: sum(d.get(k, 0.0) for d in big[j:j + per]) for k in big[j]}
            c["SQ_WAVES"] = big[j]["SQ_WAVES"]  # every variant launches every wavefront
            out.append(c)
        return out

    big_p = passes("pmc")
    # the optional stall pass (SQ_WAVE_CYCLES & co. count quad-cycles; GRBM_GUI_ACTIVE sums 8 XCDs)
    stall = passes("stall") if os.path.exists(os.path.join(src, "stall", "run_counter_collection.csv")) else None
    # the optional third pass (integer / conversion / scalar / LDS instructions)
    mix = passes("mix") if os.path.exists(os.path.join(src, "mix", "run_counter_collection.csv")) else None
    tr = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
          if integrator(r["Kernel_Name"]) and int(r["Grid_Size_X"]) >= N]
    d1 = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in tr]
    durs = [sum(d1[j:j + per]) for j in range(0, len(d1), per)]
    assert len(big_p) == len(CASES) and len(durs) == len(CASES), (len(big_p), len(durs))
    lines = {}
    for f in ("pmc.jsonl", "trace.jsonl"):
        for ln in open(os.path.join(src, f)):
            if ln.startswith("{"):
                j = json.loads(ln)
                lines.setdefault(j["config"], j)
    out = {"source": "tools/gpu.sh ode-pmc (tools/ode_pmc_run.py) + tools/summarize_ode_pmc.py " + tag,
           "kernel": "ode_integrate_kernel<false>" if per == 1 else
                     f"ode_integrate_kernel<false, ...> ({per} variants per launch, summed)",
           "peak_tflops": 78.6,
           "note": "executed FP64 FLOP = 64 x (2 FMA + MUL + ADD) instructions; cooperative waves evaluate a "
                   "step's stage ingredients once per wave (or per 32/16/8-lane segment), so executed FLOP "
                   "per point-step falls as sharing rises: points_per_s is the figure of merit, the executed "
                   "fraction says how busy the FP64 pipe is", "configs": {}}
    for (name, _over, steps), c, t in zip(CASES, big_p, durs):
        ws = c["SQ_WAVES"] * steps
        flop = 64.0 * (2.0 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"])
        f64 = c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"] + \
            c.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        out["configs"][name] = {
            "points": N, "steps_per_point": steps, "waves": c["SQ_WAVES"],
            "valu_per_wave_step": c["SQ_INSTS_VALU"] / ws, "fp64_per_wave_step": f64 / ws,
            "kernel_s": t, "kernel_point_steps_per_s": N * steps / t,
            "wall_points_per_s": lines.get(name, {}).get("points_per_s"),
            "executed_fp64_tflops": flop / t / 1e12, "frac_of_fp64_peak": flop / t / 1e12 / 78.6,
            # 1024 SIMDs x clock: FP64 instructions take 4 issue cycles of a SIMD (16 lanes/cycle)
            "fp64_pipe_busy_frac": f64 * 4.0 / (t * 1024 * 2.4e9)}
        if mix:
            m = mix[[n for n, _o, _s in CASES].index(name)]
            wm = m["SQ_WAVES"] * steps
            out["configs"][name]["mix_per_wave_step"] = {
                k.replace("SQ_INSTS_", "").lower(): m[k] / wm for k in
                ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT",
                 "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_SALU", "SQ_INSTS_LDS") if k in m}
        if stall:
            m = stall[[n for n, _o, _s in CASES].index(name)]
            wc = m.get("SQ_WAVE_CYCLES", 0.0)
            out["configs"][name]["wave_cycles"] = {
                "wait_any_frac": m.get("SQ_WAIT_ANY", 0.0) / wc if wc else None,
                "wait_inst_any_frac": m.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else None,
                "active_inst_any_frac": m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else None,
                "active_inst_valu_frac": m.get("SQ_ACTIVE_INST_VALU", 0.0) / wc if wc else None,
                "active_inst_sca_frac": m.get("SQ_ACTIVE_INST_SCA", 0.0) / wc if wc else None,
                "wave_quad_cycles_per_wave_step": wc / (m["SQ_WAVES"] * steps),
                "note": "fractions of SQ_WAVE_CYCLES (summed over the launch's variants); WAIT_ANY = parked on "
                        "s_waitcnt/barrier, WAIT_INST_ANY = issue stalls (dependency / pipe busy)"}
            if m.get("GRBM_GUI_ACTIVE"):
                out["configs"][name]["clock_ghz_grbm"] = m["GRBM_GUI_ACTIVE"] / 8.0 / t / 1e9
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, fname), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def main():
    if len(sys.argv) > 3 and sys.argv[3] == "cases":
        return main_cases(sys.argv[1], sys.argv[2], *sys.argv[4:5])
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "odepmc")
    tag = sys.argv[2] if len(sys.argv) > 2 else "round2"
    rows = list(csv.DictReader(open(os.path.join(src, "pmc", "run_counter_collection.csv"))))
    disp = defaultdict(dict)
    for r in rows:
        if "ode_integrate_kernel<false>" in r["Kernel_Name"]:
            disp[int(r["Dispatch_Id"])][r["Counter_Name"]] = disp[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + \
                float(r["Counter_Value"])
    tr = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
          if "ode_integrate_kernel<false>" in r["Kernel_Name"]]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in tr]
    pmc = [disp[k] for k in sorted(disp)]
    # skip the warm-up dispatches (64 points each, 2 per config): keep dispatches with the config's wave count
    out = {"source": "tools/gpu.sh ode-pmc + tools/summarize_ode_pmc.py", "kernel": "ode_integrate_kernel",
           "peak_tflops": 78.6, "configs": {}}
    big_p = [c for c in pmc if c.get("SQ_WAVES", 0) >= 256]
    big_t = [d for d, r in zip(durs, tr) if int(r["Grid_Size_X"]) >= 256 * 64]
    for i, (name, n, steps) in enumerate(CONFIGS):
        c = big_p[2 * i]
        waves = c["SQ_WAVES"]
        ws = waves * steps
        flop = 64.0 * (2.0 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"])
        t_shared, t_unshared = big_t[2 * i], big_t[2 * i + 1]
        out["configs"][name] = {
            "points": n, "steps_per_point": steps, "waves": waves,
            "valu_per_wave_step": c["SQ_INSTS_VALU"] / ws,
            "fp64_fma_mul_add_per_wave_step": (c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] +
                                               c["SQ_INSTS_VALU_ADD_F64"]) / ws,
            "kernel_s_shared_tables": t_shared, "kernel_s_per_point_tables": t_unshared,
            "executed_fp64_tflops": flop / t_shared / 1e12, "frac_of_fp64_peak": flop / t_shared / 1e12 / 78.6}
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "ode_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
