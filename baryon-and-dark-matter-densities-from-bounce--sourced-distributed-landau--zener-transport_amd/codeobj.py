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


# The sections of a device ELF that make up what the GPU executes: the kernels' machine code
# (.text), their kernel descriptors (.rodata: VGPR/SGPR/LDS/scratch settings) and the code
# object metadata note (.note: arguments, launch bounds).  The whole-object hash above also
# covers the symbol and string tables, which carry clang's per-compilation `__hip_cuid_<hash>`
# symbol -- a hash of the build COMMAND (input paths, flags, output), not of the code: building
# the same source with another command line (e.g. one hipcc per translation unit) changes it.
CODE_SECTIONS = (".note", ".rodata", ".text")


def elf_sections(obj: bytes) -> dict[str, bytes]:
    """Section name -> contents of a little-endian ELF64 object (NOBITS sections are empty)."""
    if obj[:4] != b"\x7fELF" or obj[4] != 2:
        raise ValueError("not an ELF64 object")
    (shoff,) = struct.unpack_from("<Q", obj, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", obj, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", obj, shoff + i * shentsize) for i in range(shnum)]
    str_off = hdrs[shstrndx][4]
    out = {}
    for name_off, typ, _flags, _addr, off, size, *_ in hdrs:
        end = obj.index(b"\0", str_off + name_off)
        name = obj[str_off + name_off:end].decode("ascii", "replace")
        out[name] = b"" if typ == 8 else obj[off:off + size]   # SHT_NOBITS
    return out


def kernel_code_sha256(lib_path: str, kernel: str = "yields_grid_kernel", arch: str = "gfx950") -> str | None:
    """sha256 over CODE_SECTIONS of the device code object that defines `kernel`: equal for two
    builds whose kernels execute the same machine code with the same descriptors, whatever the
    build command (the identity a PMC profile is tied to); None if no code object defines it."""
    for obj in device_objects(lib_path, arch):
        if kernel.encode() in obj:
            secs = elf_sections(obj)
            h = hashlib.sha256()
            for name in CODE_SECTIONS:
                data = secs.get(name, b"")
                h.update(name.encode() + b"\0" + struct.pack("<Q", len(data)) + data)
            return h.hexdigest()
    return None
