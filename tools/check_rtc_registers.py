#!/usr/bin/env python3
"""Register budget of every hipRTC code object in lib/rtc_cache (CPU only).

A kernel whose registers (VGPRs + AGPRs, unified) exceed what its launch bound allows (512
registers per SIMD lane, shared by the waves of a workgroup that land on one SIMD) cannot be
dispatched at that block size. This lists every kernel with its counts and exits 1 when one
is over budget at its launch bound (the library itself caps the waves per block at launch,
polar_sc_jit.cpp fit_waves).

usage: python tools/check_rtc_registers.py [cache dir]
"""
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def read_code(path):
    """the ELF code object of a cache entry: <key>.cox ("PSCX", u64 size, xz stream) or
    <key>.coz ("PSCZ", u64 size, zlib stream) -- polar_sc_jit.cpp cache_store -- or a plain
    object file"""
    import lzma
    import struct
    import zlib
    data = open(path, "rb").read()
    if data[:4] in (b"PSCX", b"PSCZ"):
        n, = struct.unpack_from("<Q", data, 4)
        data = lzma.decompress(data[12:]) if data[:4] == b"PSCX" else zlib.decompress(data[12:])
        assert len(data) == n, path
    return data


def cache_entries(d):
    return sum((glob.glob(os.path.join(d, "*." + e)) for e in ("cox", "coz", "co")), [])


def kernels(path):
    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(read_code(path))
        f.flush()
        notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
    out = []
    for blk in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
        agpr = int(blk.split()[0])
        name = re.search(r"\.name:\s+(\S+)", blk)
        vgpr = re.search(r"\.vgpr_count:\s+(\d+)", blk)
        wg = re.search(r"\.max_flat_workgroup_size:\s+(\d+)", blk)
        if name and vgpr and wg:
            out.append((name.group(1), int(vgpr.group(1)), agpr, int(wg.group(1))))
    return out


def code_key(path):
    """polar_sc_jit.cpp code_key restated: FNV-1a (64-bit) over the PROGBITS sections that are
    executable or named .rodata, in section order, as 16 hex digits."""
    import struct
    data = read_code(path)
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    names = secs[shstrndx]
    h = 1469598103934665603
    for name, typ, flags, _, off, size, *_ in secs:
        nm = data[names[4] + name:].split(b"\0", 1)[0]
        if typ == 1 and (flags & 4 or nm == b".rodata"):
            for b in data[off:off + size]:
                h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h


def find_code(cache, key):
    """The code object in `cache` whose machine code has this code_key."""
    for co in sorted(cache_entries(cache), key=os.path.getmtime, reverse=True):
        if code_key(co) == key:
            return co
    return None


def over_budget(vgpr, agpr, wg):
    # unified register file of 512 per lane and SIMD. On gfx90a and later the metadata's
    # .vgpr_count is already the unified total (architected VGPRs padded to 4, then the
    # AGPRs: LLVM's getTotalNumVGPRs); .agpr_count is the AGPR part of it. The kernel
    # descriptor's granulated count (polar_sc_jit.cpp kernel_regs) rounds it up to 8.
    waves = -(-wg // 64)
    waves_per_simd = max(1, -(-waves // 4))
    total = -(-vgpr // 8) * 8
    return total * waves_per_simd > 512, total


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "sc_polar_decoder_hls_amd", "lib", "rtc_cache")
    bad = 0
    for co in sorted(cache_entries(d)):
        for name, vgpr, agpr, wg in kernels(co):
            over, total = over_budget(vgpr, agpr, wg)
            if over or agpr:
                print("%s %-32s vgpr %3d agpr %3d wg %4d%s" % (os.path.basename(co), name, vgpr, agpr, wg,
                                                               "  OVER BUDGET" if over else ""))
            bad += over
    print("%d kernel(s) over budget" % bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
