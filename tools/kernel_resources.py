"""Register, scratch and LDS budgets of every kernel in libart.so, read from the gfx950 code objects in its
`.hip_fatbin` section: the clang offload bundles (one per HIP object), then each code object's NT_AMDGPU_METADATA note
(msgpack, amdhsa.kernels).  No GPU needed.

    python tools/kernel_resources.py [path/to/libart.so] [name-substring]

tests/test_kernel_resources.py uses it to guard the occupancy DESIGN.md §4 relies on (k_paths: <= 128 VGPRs and no
scratch, i.e. 4 waves per SIMD)."""
import struct
import sys

import msgpack

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NT_AMDGPU_METADATA = 32


def _sections(elf):
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not a little-endian ELF64 file")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stroff = hdrs[shstrndx][4]
    out = []
    for name, typ, _flags, _addr, off, size in hdrs:
        end = elf.index(b"\0", stroff + name)
        out.append((elf[stroff + name:end].decode(), typ, off, size))
    return out


def fatbin(path):
    """The bytes of libart.so's .hip_fatbin section."""
    with open(path, "rb") as f:
        data = f.read()
    for name, _typ, off, size in _sections(data):
        if name == ".hip_fatbin":
            return data[off:off + size]
    raise ValueError("no .hip_fatbin section")


def code_objects(fb, arch="gfx950"):
    """Every `arch` code object (ELF bytes) of the concatenated offload bundles in fb."""
    objs = []
    pos = fb.find(BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fb, pos + len(BUNDLE_MAGIC))
        at = pos + len(BUNDLE_MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fb, at)
            triple = fb[at + 24:at + 24 + tlen].decode()
            at += 24 + tlen
            if triple.startswith("hip") and triple.endswith(arch) and size > 0:
                objs.append(fb[pos + off:pos + off + size])
        pos = fb.find(BUNDLE_MAGIC, pos + 1)
    return objs


def kernel_metadata(elf):
    """amdhsa.kernels of one code object: a list of dicts (.name, .vgpr_count, .sgpr_count, .vgpr_spill_count,
    .private_segment_fixed_size, .group_segment_fixed_size, ...)."""
    for _name, typ, off, size in _sections(elf):
        if typ != 7:  # SHT_NOTE
            continue
        at, end = off, off + size
        while at + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, at)
            name_at = at + 12
            desc_at = name_at + ((namesz + 3) & ~3)
            if ntype == NT_AMDGPU_METADATA and elf[name_at:name_at + namesz].rstrip(b"\0") == b"AMDGPU":
                meta = msgpack.unpackb(elf[desc_at:desc_at + descsz], raw=False, strict_map_key=False)
                return meta.get("amdhsa.kernels", [])
            at = desc_at + ((descsz + 3) & ~3)
    return []


def kernels(path):
    """{kernel symbol: metadata dict} over every gfx950 code object in the library."""
    out = {}
    for co in code_objects(fatbin(path)):
        for k in kernel_metadata(co):
            out[k[".name"]] = k
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "another_raytracer_amd/libart.so"
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, k in sorted(kernels(path).items()):
        if sub in name:
            print(f"{name}: vgpr {k.get('.vgpr_count')} agpr {k.get('.agpr_count', 0)} sgpr {k.get('.sgpr_count')} "
                  f"spill {k.get('.vgpr_spill_count', 0)} scratch {k.get('.private_segment_fixed_size')} "
                  f"lds {k.get('.group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
