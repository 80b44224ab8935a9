#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of the lzq HIP sources (hipcc
-Rpass-analysis=kernel-resource-usage, device-only compile for gfx950; no GPU needed).

    python tools/kernel_resources.py [-DNAME=VAL ...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"
SOURCES = ["lzq_kernels.hip", "lzq_aov.hip", "lzq_ode.hip", "lzq_ode_tp.hip", "lzq_propagator.hip", "lzq_profile.hip"]
KEYS = ("VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill",
        "VGPRs Spill", "LDS Size [bytes/block]")


def resources(src: str, defines: list[str]) -> list[dict]:
    out = os.path.join(ROOT, "tools", "_build", "res_" + os.path.basename(src) + ".o")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only",
           "-c", "-Rpass-analysis=kernel-resource-usage", "-I", os.path.join(ROOT, "include"), *defines,
           os.path.join(ROOT, PKG, "csrc", src), "-o", out]
    err = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark:\s+(.*?):\s+(.*?)\s+\[-Rpass-analysis", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"kernel": v}
            rows.append(cur)
        elif cur is not None and k in KEYS:
            cur[k] = v
    return rows


def main():
    defines = [a for a in sys.argv[1:] if a.startswith("-D")]
    hdr = ["VGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "VGPRs Spill", "SGPRs Spill", "Occupancy [waves/SIMD]",
           "LDS Size [bytes/block]"]
    print("%-70s %5s %5s %7s %6s %6s %4s %7s" % ("kernel", "vgpr", "sgpr", "scratch", "vspill", "sspill", "occ", "lds"))
    for src in SOURCES:
        for r in resources(src, defines):
            name = r["kernel"][:70]
            print("%-70s %5s %5s %7s %6s %6s %4s %7s" % (name, *[r.get(h, "?") for h in hdr]))


if __name__ == "__main__":
    main()
