#!/usr/bin/env python3
"""Build tuning variants of liblzq.so (compile-time knobs of csrc/lzq_kernels.hip) into
<package>/_build/variants/ for tools/ablate_builds.py.  Runs on the CPU (hipcc)."""
import importlib
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd"
B = importlib.import_module(PKG + ".build")

GRID = {"LZQ_MAGIC": [0, 1], "LZQ_KUNROLL": [4, 8], "LZQ_YB": [1, 2]}
# explicit list (overrides the full product when non-empty); keys omitted take the defaults
CONFIGS = [dict(LZQ_KUNROLL=8), dict(LZQ_KUNROLL=10), dict(LZQ_KUNROLL=12)]


def main():
    """argv: optional variant list, one 'KEY=VAL[,KEY=VAL...]' per variant (overrides CONFIGS)."""
    outdir = os.path.join(B.BUILD_DIR, "variants")
    import shutil
    shutil.rmtree(outdir, ignore_errors=True)
    keys = list(GRID)
    confs = CONFIGS or [dict(zip(keys, vals)) for vals in itertools.product(*(GRID[k] for k in keys))]
    if len(sys.argv) > 1:
        confs = [dict(kv.split("=", 1) for kv in arg.split(",")) for arg in sys.argv[1:]]
    for d in confs:
        name = "_".join(f"{k[4:].lower()}{v}" for k, v in d.items())
        B.build(defines=d, out=os.path.join(outdir, f"liblzq_{name}.so"))
        print(name)


if __name__ == "__main__":
    main()
