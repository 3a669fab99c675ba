#!/usr/bin/env python3
"""Per-kernel register and scratch use of a built HIP library, read from the
gfx950 code object's AMDGPU metadata note (no GPU, no ROCm tools needed):
the .hip_fatbin section holds a clang offload bundle, each gfx950 entry an
ELF whose NT_AMDGPU_METADATA note is a msgpack map with one record per kernel.

    python scripts/kernel_resources.py duckdb-fastlane_amd/libflsgpu.so
"""
import struct
import sys

import msgpack

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NT_AMDGPU_METADATA = 32


def _sections(elf: bytes):
    (shoff,) = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    strtab = hdrs[shstrndx]
    names = elf[strtab[4]:strtab[4] + strtab[5]]
    for h in hdrs:
        name = names[h[0]:names.index(b"\0", h[0])].decode()
        yield name, h[1], elf[h[4]:h[4] + h[5]]


def code_objects(lib: bytes):
    """gfx950 code objects inside a host library's offload bundles"""
    for name, _, data in _sections(lib):
        if name != ".hip_fatbin":
            continue
        pos = 0
        while True:
            pos = data.find(BUNDLE_MAGIC, pos)
            if pos < 0:
                break
            (n,) = struct.unpack_from("<Q", data, pos + 24)
            q = pos + 32
            for _ in range(n):
                off, size, tlen = struct.unpack_from("<QQQ", data, q)
                triple = data[q + 24:q + 24 + tlen].decode()
                q += 24 + tlen
                if "gfx950" in triple:
                    yield data[pos + off:pos + off + size]
            pos += len(BUNDLE_MAGIC)


def kernels(code_object: bytes):
    for _, stype, data in _sections(code_object):
        if stype != 7:  # SHT_NOTE
            continue
        p = 0
        while p + 12 <= len(data):
            namesz, descsz, ntype = struct.unpack_from("<III", data, p)
            p += 12
            name = data[p:p + namesz]
            p += (namesz + 3) & ~3
            desc = data[p:p + descsz]
            p += (descsz + 3) & ~3
            if ntype == NT_AMDGPU_METADATA and name.startswith(b"AMDGPU"):
                yield from msgpack.unpackb(desc, raw=False)["amdhsa.kernels"]


def resources(path: str) -> dict:
    """kernel symbol -> {vgpr, agpr, sgpr, vgpr_spill, sgpr_spill, scratch, lds}"""
    out = {}
    with open(path, "rb") as f:
        lib = f.read()
    for co in code_objects(lib):
        for k in kernels(co):
            out[k[".name"]] = {"vgpr": k.get(".vgpr_count"), "agpr": k.get(".agpr_count", 0),
                               "sgpr": k.get(".sgpr_count"), "vgpr_spill": k.get(".vgpr_spill_count", 0),
                               "sgpr_spill": k.get(".sgpr_spill_count", 0),
                               "scratch": k.get(".private_segment_fixed_size", 0),
                               "lds": k.get(".group_segment_fixed_size", 0)}
    return out


if __name__ == "__main__":
    for path in sys.argv[1:]:
        for name, r in sorted(resources(path).items()):
            print(f"{r['vgpr']:4d} vgpr {r['sgpr']:4d} sgpr {r['vgpr_spill']:3d} spill {r['scratch']:5d} B scratch  {name}")
