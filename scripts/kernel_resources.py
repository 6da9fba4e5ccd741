"""Per-kernel resources of librvmcmc.so's gfx950 code object: VGPRs, AGPRs, SGPRs, spills, scratch
(private segment) and static LDS, read from the AMDGPU metadata note of the embedded code object
(no GPU needed).  The library's .hip_fatbin section holds clang offload bundles (one per translation
unit); each gfx950 entry is an ELF code object whose NT_AMDGPU_METADATA note llvm-readelf prints.

    python scripts/kernel_resources.py [path/to/librvmcmc.so] [name-regex]  -> one JSON line per kernel
"""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rvel-mcmc_amd", "rvmcmc", "librvmcmc.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = {".name": "name", ".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
          ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill",
          ".private_segment_fixed_size": "scratch", ".group_segment_fixed_size": "lds",
          ".max_flat_workgroup_size": "max_wg"}


def _section(data, name):
    """(offset, size) of an ELF64 section by name."""
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    strtab_off = struct.unpack_from("<Q", data, shoff + shstrndx * shentsize + 0x18)[0]
    for i in range(shnum):
        base = shoff + i * shentsize
        nm, = struct.unpack_from("<I", data, base)
        end = data.index(b"\0", strtab_off + nm)
        if data[strtab_off + nm:end].decode() == name:
            off, size = struct.unpack_from("<QQ", data, base + 0x18)
            return off, size
    raise KeyError(name)


def code_objects(path, arch="gfx950"):
    """The embedded code objects for `arch` (bytes), one per offload bundle."""
    data = open(path, "rb").read()
    off, size = _section(data, ".hip_fatbin")
    fat = data[off:off + size]
    out = []
    pos = fat.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if arch in triple and es > 0:
                out.append(fat[pos + eo:pos + eo + es])
        pos = fat.find(MAGIC, pos + 1)
    return out


def kernels(path=LIB, arch="gfx950"):
    """[{name, vgpr, agpr, sgpr, vgpr_spill, sgpr_spill, scratch, lds, max_wg}] of every kernel."""
    res = []
    for co in code_objects(path, arch):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True, check=True).stdout
        cur = None
        for line in txt.splitlines():
            m = re.match(r"\s*-?\s*(\.[a-z_]+):\s+(\S+)", line)
            if not m or m.group(1) not in FIELDS:
                continue
            key, val = FIELDS[m.group(1)], m.group(2)
            if line.lstrip().startswith("- "):  # a new kernel's map starts
                cur = {}
                res.append(cur)
            if cur is None:
                continue
            cur[key] = val if key == "name" else int(val)
    return [k for k in res if "name" in k]


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return list(names)


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else LIB
    rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    ks = kernels(path)
    for k, d in zip(ks, demangle([k["name"] for k in ks])):
        k["kernel"] = d.split("(")[0]
        if rx is None or rx.search(k["kernel"]):
            print(json.dumps(k))


if __name__ == "__main__":
    main()
