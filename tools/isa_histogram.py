#!/usr/bin/env python3
"""Static instruction census of a generated per-mask kernel (CPU only, no GPU needed).

The per-mask kernels are straight-line code, so the static VALU count of the disassembly is
the dynamic count per wave (up to the REP exact-fallback branch). Compiles the plan's hipRTC
source with hipcc for gfx950 and prints VGPR / LDS figures and a mnemonic histogram, grouped
by the `// op` comment block the instruction came from when -g line info is available.

    python tools/isa_histogram.py [--mask FB_N1024_K512] [--top 40] [--env POLAR_SC_X=1 ...]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
CSRC = os.path.join(ROOT, "sc_polar_decoder_hls_amd", "csrc")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def compile_source(src, tmp):
    path = os.path.join(tmp, "k.hip")
    with open(path, "w") as f:
        f.write("#include <hip/hip_runtime.h>\n" + src)   # hipRTC includes it implicitly
    co = os.path.join(tmp, "k.co")
    res = subprocess.run(["hipcc", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output", "-O3",
                          "-std=c++17", "-I", CSRC, "-o", co, path, "-Rpass-analysis=kernel-resource-usage"],
                         check=True, capture_output=True, text=True)
    return co, res.stderr


def census(co):
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True).stdout
    hist = collections.Counter()
    for line in dis.splitlines():
        m = re.match(r"\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|flat_\w+)\b", line)
        if m:
            hist[m.group(1)] += 1
    return hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", default="FB_N1024_K512")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--env", nargs="*", default=[])
    args = ap.parse_args()
    for kv in args.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import sc_polar_decoder_hls_amd as pkg
    import util
    dec = pkg.Decoder(util.mask(args.mask))
    src = dec.kernel_source()
    with tempfile.TemporaryDirectory() as tmp:
        co, remarks = compile_source(src, tmp)
        hist = census(co)
    for line in remarks.splitlines():
        if "remark" in line and any(k in line for k in ("VGPRs:", "AGPRs", "ScratchSize", "Occupancy", "LDS Size",
                                                        "SGPRs:")):
            print(line.split("remark: ")[-1])
    valu = sum(c for k, c in hist.items() if k.startswith("v_"))
    salu = sum(c for k, c in hist.items() if k.startswith("s_"))
    lds = sum(c for k, c in hist.items() if k.startswith("ds_"))
    print("VALU %d  SALU %d  LDS %d  total %d" % (valu, salu, lds, sum(hist.values())))
    for k, c in hist.most_common(args.top):
        print("%6d  %s" % (c, k))


if __name__ == "__main__":
    main()
