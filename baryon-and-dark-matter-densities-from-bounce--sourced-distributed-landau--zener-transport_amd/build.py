"""In-tree build of the HIP library (gfx950).  Used by __graft_entry__.build().

hipcc cross-compiles for gfx950 without a GPU; the resulting `_build/liblzq.so` is
git-ignored but travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.normpath(os.path.join(HERE, "..", "include"))
BUILD_DIR = os.path.join(HERE, "_build")
LIB_PATH = os.path.join(BUILD_DIR, "liblzq.so")
SOURCES = ["lzq_kernels.hip", "lzq_aov.hip", "lzq_propagator.hip", "lzq_ode.hip", "lzq_ode_tp.hip", "lzq_profile.hip"]
# every header next to the sources (tests/test_engine_host.py checks each #include "..." of the
# sources resolves to one of the build inputs)
HEADERS = sorted(os.path.basename(h) for h in glob.glob(os.path.join(CSRC, "*.h")))
ARCH = os.environ.get("LZQ_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: every a*b+c rounds twice exactly like numpy; fused ops are explicit
# __builtin_fma in the hot loops.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
         f"--offload-arch={ARCH}"]


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files.append(os.path.join(INCLUDE, "lzq.h"))
    return files


def inputs_hash(defines: dict | None = None) -> str:
    """sha256 over the build's inputs (sources, headers, flags, defines), by content: the stamp
    written next to the library, so a shipped build can be matched to its sources on any machine
    (mtimes do not survive the copy to the GPU box)."""
    h = hashlib.sha256()
    for f in _inputs():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(repr((FLAGS, sorted((defines or {}).items()))).encode())
    return h.hexdigest()


def stamp_path(lib: str = LIB_PATH) -> str:
    return lib + ".inputs.sha256"


def stamp_matches(lib: str = LIB_PATH) -> bool:
    """True when the library's stamp equals the current sources' inputs_hash()."""
    try:
        with open(stamp_path(lib)) as f:
            return f.read().strip() == inputs_hash()
    except OSError:
        return False


def up_to_date() -> bool:
    return os.path.exists(LIB_PATH) and stamp_matches(LIB_PATH)


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the lzq HIP library cannot be built")


def build(force: bool = False, verbose: bool = False, defines: dict | None = None,
          out: str | None = None) -> str:
    """Build liblzq.so (or a tuning variant with -D`defines` into `out`)."""
    target = out or LIB_PATH
    if not force and out is None and not defines and up_to_date():
        return LIB_PATH
    os.makedirs(os.path.dirname(target), exist_ok=True)
    tmp = target + ".tmp"
    dflags = [f"-D{k}={v}" for k, v in (defines or {}).items()]
    # one hipcc per translation unit, in parallel, then one link (each object embeds its own
    # gfx950 code object, exactly as the single-command build does)
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    with tempfile.TemporaryDirectory(prefix="lzq_build_") as objdir:
        objs = [os.path.join(objdir, os.path.splitext(s)[0] + ".o") for s in SOURCES]
        cflags = [f for f in FLAGS if f != "-shared"]
        cmds = [[hipcc(), *cflags, *dflags, "-I", INCLUDE, "-c", os.path.join(CSRC, s), "-o", o]
                for s, o in zip(SOURCES, objs)]
        if verbose:
            for c in cmds:
                print(" ".join(c))
        jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
        with ThreadPoolExecutor(jobs) as ex:
            for r in list(ex.map(lambda c: subprocess.run(c), cmds)):
                if r.returncode:
                    raise subprocess.CalledProcessError(r.returncode, r.args)
        link = [hipcc(), *FLAGS, "-o", tmp, *objs]
        if verbose:
            print(" ".join(link))
        subprocess.run(link, check=True)
    os.replace(tmp, target)
    with open(stamp_path(target), "w") as f:
        f.write(inputs_hash(defines) + "\n")
    return target


if __name__ == "__main__":
    print(build(force=True, verbose=True))
