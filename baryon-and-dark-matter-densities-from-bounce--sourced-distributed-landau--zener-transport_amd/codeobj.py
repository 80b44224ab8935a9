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


def elf_symbols(obj: bytes) -> list[tuple[str, int, int, int]]:
    """(name, value, size, section index) of every .symtab entry of a little-endian ELF64 object."""
    (shoff,) = struct.unpack_from("<Q", obj, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", obj, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", obj, shoff + i * shentsize) for i in range(shnum)]
    str_off = hdrs[shstrndx][4]

    def sec_name(h):
        end = obj.index(b"\0", str_off + h[0])
        return obj[str_off + h[0]:end].decode("ascii", "replace")
    names = [sec_name(h) for h in hdrs]
    if ".symtab" not in names:
        return []
    sym = hdrs[names.index(".symtab")]
    strtab = hdrs[sym[6]]  # sh_link: the symbol names' string table
    out = []
    for k in range(sym[5] // 24):
        st_name, _info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", obj, sym[4] + 24 * k)
        end = obj.index(b"\0", strtab[4] + st_name)
        out.append((obj[strtab[4] + st_name:end].decode("ascii", "replace"), value, size, shndx))
    return out


OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def kernel_isa_sha256(lib_path: str, kernel: str = "yields_grid_kernel", arch: str = "gfx950") -> str | None:
    """sha256 of the disassembly of the kernels whose mangled names contain `kernel` (every template
    instantiation, in name order), with what depends on where the code object lays them out masked:
    the literal of each s_add_u32 / s_addc_u32 that forms a PC-relative address after s_getpc_b64.
    The identity of a PMC profile of those kernels that survives changes to the other kernels of the
    same translation unit (kernel_code_sha256 hashes the whole object's .text, and the raw bytes of
    a kernel change with the placement of the data it addresses).  None if the kernel or
    llvm-objdump (ROCm's) is absent."""
    import os
    import re
    import subprocess
    import tempfile
    if not os.path.exists(OBJDUMP):
        return None
    for obj in device_objects(lib_path, arch):
        if kernel.encode() not in obj:
            continue
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(obj)
            f.flush()
            r = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--no-leading-addr", f.name],
                               capture_output=True, text=True)
        if r.returncode:
            return None
        funcs, cur = {}, None
        for line in r.stdout.splitlines():
            m = re.match(r"^<(\S+)>:$", line.strip())
            if m:
                cur = m.group(1) if kernel in m.group(1) else None
                if cur:
                    funcs[cur] = []
                continue
            if cur is None:
                continue
            t = line.split("//")[0].strip()
            if t:
                funcs[cur].append(t)
        if not funcs:
            return None
        h = hashlib.sha256()
        for name in sorted(funcs):
            pcrel = set()
            out = []
            for t in funcs[name]:
                op = t.split()[0]
                args = t[len(op):].replace(" ", "").split(",")
                if op == "s_getpc_b64":
                    m = re.match(r"s\[(\d+):(\d+)\]", args[0])
                    if m:
                        pcrel = {f"s{m.group(1)}", f"s{m.group(2)}"}
                elif op in ("s_add_u32", "s_addc_u32") and args and args[0] in pcrel and len(args) == 3:
                    t = f"{op} {args[0]}, {args[1]}, PCREL"
                elif args and args[0] in pcrel:
                    pcrel.discard(args[0])  # the register is redefined: no longer a PC-relative base
                out.append(t)
            h.update(name.encode() + b"\0" + "\n".join(out).encode() + b"\0")
        # and their kernel descriptors (registers, LDS, scratch), less the code entry offset
        (shoff,) = struct.unpack_from("<Q", obj, 0x28)
        shentsize, shnum, _ = struct.unpack_from("<HHH", obj, 0x3A)
        hdrs = [struct.unpack_from("<IIQQQQIIQQ", obj, shoff + i * shentsize) for i in range(shnum)]
        for name, value, size, shndx in sorted(elf_symbols(obj)):
            if kernel in name and name.endswith(".kd") and size == 64 and 0 < shndx < shnum:
                sec = hdrs[shndx]
                kd = bytearray(obj[sec[4] + (value - sec[3]):sec[4] + (value - sec[3]) + 64])
                kd[16:24] = bytes(8)  # kernel_code_entry_byte_offset: where the code sits, not what it is
                h.update(name.encode() + b"\0" + bytes(kd))
        return h.hexdigest()
    return None
