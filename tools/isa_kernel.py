#!/usr/bin/env python3
"""Device-only gfx950 compile of one lzq source to assembly (no GPU), then, for the kernels whose
mangled name contains PATTERN: registers / spills / occupancy and an instruction census of every
loop (back edge) -- VALU (FP64 / other), SALU, LDS, scratch, readlane/writelane.  The CPU-side
feedback loop for register-bound kernels.

    python tools/isa_kernel.py lzq_ode.hip ode_riccati_kernelILi0 [-DNAME=VAL ...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"


def compile_asm(src, defines, out):
    cmd = ["hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only",
           "-S", "-Rpass-analysis=kernel-resource-usage", "-I", os.path.join(ROOT, "include"), *defines,
           os.path.join(ROOT, PKG, "csrc", src), "-o", out]
    return subprocess.run(cmd, capture_output=True, text=True, check=True).stderr


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        if "readlane" in op or "writelane" in op:
            return "lane"
        if op.endswith("_f64") or "f64" in op:
            return "valu_f64"
        return "valu"
    if op.startswith("s_"):
        if op in ("s_waitcnt", "s_nop", "s_endpgm", "s_barrier"):
            return "wait"
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def census(lines):
    c = {}
    for l in lines:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":") or t.startswith("#"):
            continue
        k = classify(t)
        c[k] = c.get(k, 0) + 1
    return c


def main():
    src, pat = sys.argv[1], sys.argv[2]
    defines = [a for a in sys.argv[3:] if a.startswith("-D")]
    out = os.path.join("/tmp", "isa_" + os.path.basename(src) + ".s")
    err = compile_asm(src, defines, out)
    s = open(out).read().split("\n")
    cur = None
    res = {}
    for line in err.splitlines():
        m = re.search(r"remark:\s+(.*?):\s+(.*?)\s+\[-Rpass-analysis", line)
        if not m:
            continue
        if m.group(1) == "Function Name":
            cur = m.group(2)
            res[cur] = {}
        elif cur:
            res[cur][m.group(1)] = m.group(2)
    for name, r in res.items():
        if pat not in name:
            continue
        print(name[:90])
        print("  VGPRs %s  SGPRs %s  vspill %s  sspill %s  occ %s  scratch %s" % (
            r.get("VGPRs"), r.get("TotalSGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
            r.get("Occupancy [waves/SIMD]"), r.get("ScratchSize [bytes/lane]")))
        i0 = next(i for i, l in enumerate(s) if l.startswith(name + ":"))
        i1 = next(i for i in range(i0, len(s)) if s[i].startswith(".Lfunc_end"))
        body = s[i0:i1]
        labels = {}
        for n, l in enumerate(body):
            m = re.match(r"^(\.LBB\S+):", l)
            if m:
                labels[m.group(1)] = n
        print("  whole kernel:", census(body))
        for n, l in enumerate(body):
            m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
            if m and labels.get(m.group(2), 1 << 30) < n:
                a = labels[m.group(2)]
                print("  loop %s lines %d-%d: %s" % (m.group(2), a, n, census(body[a:n + 1])))


if __name__ == "__main__":
    main()
