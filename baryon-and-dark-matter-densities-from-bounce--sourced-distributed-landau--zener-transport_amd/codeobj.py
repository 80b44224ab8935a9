"""Identify the gfx950 code object a kernel was built into (no GPU, no ROCm tools needed).

hipcc embeds one clang offload bundle per translation unit in liblzq.so's .hip_fatbin section:
"__CLANG_OFFLOAD_BUNDLE__", u64 entry count, then per entry u64 offset, u64 size, u64 triple
length and the triple (offsets from the bundle start); the amdgcn entry is the TU's device ELF.
bench.py and tools/summarize_profile.py hash the device ELF that defines the headline kernel, so
a roofline measured by PMC on one build is never reported against another.
"""
from __future__ import annotations

import hashlib
import struct

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def device_objects(lib_path: str, arch: str = "gfx950") -> list[bytes]:
    """The amdgcn code objects for `arch` in the library's offload bundles."""
    with open(lib_path, "rb") as f:
        data = f.read()
    out, pos = [], data.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", data, pos + len(MAGIC))
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode("ascii", "replace")
            q += 24 + tlen
            if triple.startswith("hip") and "amdgcn" in triple and triple.endswith(arch):
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, q)
    return out


def kernel_object_sha256(lib_path: str, kernel: str = "yields_grid_kernel", arch: str = "gfx950") -> str | None:
    """sha256 of the device code object that defines `kernel` (a substring of its mangled
    name), or None if no code object does."""
    for obj in device_objects(lib_path, arch):
        if kernel.encode() in obj:
            return hashlib.sha256(obj).hexdigest()
    return None
