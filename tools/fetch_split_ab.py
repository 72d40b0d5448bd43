#!/usr/bin/env python3
"""Split channel fetch A/B of the C2 per-mask kernel (the first round's fetch).

The kernel copies a wave's 8 frames HBM -> LDS with one global_load_lds per frame and waits
for all of them (vmcnt(0)) before splitting the root words. Packed root register j holds
words j and j + 32 (lanes j and j + 32 of the copy), so registers 0..15 need only lanes
{0..15, 32..47} of each frame. The split variant issues those halves of the 8 frames first,
then the other halves, waits vmcnt(8) (the first 8 copies landed), splits registers 0..15
while the rest arrives, and waits vmcnt(0) before register 16.

build (container, CPU): python tools/fetch_split_ab.py build
    -> build_tools/fetch_base, build_tools/fetch_split (tools/wave_stamps.py's driver: launch
       median, 50 back-to-back launches, per-wave timeline)
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

WAIT0 = "__builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this batch's channel is in LDS\n"


def split_fetch(src):
    loads = re.findall(r"    \{ const int fr_ = [^\n]*\n      if \(true\) __builtin_amdgcn_global_load_lds\([^\n]*\n", src)
    assert len(loads) == 8, len(loads)
    part = lambda cond: "".join(ld.replace("if (true)", "if (" + cond + ")") for ld in loads)
    src = src.replace("".join(loads), part("(lane & 16) == 0") + part("(lane & 16) != 0"), 1)
    assert WAIT0 in src
    src = src.replace(WAIT0, WAIT0.replace("0x0F70", "0x0F78").replace("vmcnt(0)", "vmcnt(8)"), 1)
    mis = "  if (!al_) {   // input not 16-byte aligned: byte copy\n"
    assert mis in src
    src = src.replace(mis, mis + "    __builtin_amdgcn_s_waitcnt(0x0F70);\n", 1)
    r16 = "  { const u32 a0_ = chl[256],"
    assert r16 in src
    return src.replace(r16, "  __builtin_amdgcn_s_waitcnt(0x0F70);   // the other halves\n" + r16, 1)


def build():
    import sc_polar_decoder_hls_amd as pkg
    import util
    import wave_stamps
    src = pkg.Decoder(util.mask("FB_N1024_K512")).kernel_source()
    wave_stamps.build("fetch_base", src)
    # wave_stamps anchors on the vmcnt(0) line: instrument first, then split
    path = os.path.join(wave_stamps.OUT, "fetch_split.hip")
    wave_stamps.build("fetch_split", src)
    with open(path) as f:
        inst = f.read()
    with open(path, "w") as f:
        f.write(split_fetch(inst))
    exe = os.path.join(wave_stamps.OUT, "fetch_split")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", wave_stamps.CSRC, "-o", exe, path])
    print(exe)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        sys.exit(__doc__)
