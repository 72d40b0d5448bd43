#!/usr/bin/env python3
"""Instruction census of the 16-LLR leaf (polar_sc_device.h leaf_ms, Spec_P16_ext) by recursion
level and instruction class (CPU only; VERDICT r05 item 2: attribute before building).

For every distinct frozen pattern of the leaf records of a plan, one kernel per sub-block
(B, W) of the recursion calls leaf_ms<FB, B, W> on split operands loaded from memory and
stores its result; the ROCm clang driver compiles them (the flags the library uses) and the
VALU instructions between two asm markers are counted by mnemonic class. The cost of the node
at (B, W) is its kernel's count minus its two children's (W = 2: the whole base case), so every
instruction of the full leaf is attributed to exactly one node; the per-level totals add up to
the W = 16 kernel's count up to the scheduler's reshuffling across nodes (reported as `slack`).

    python tools/leaf_census.py [--mask FB_N1024_K512] [--config sigmag=0]
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
CLANG = "/opt/rocm/lib/llvm/bin/clang++"

CLASSES = [
    ("dpp-mov", re.compile(r"^v_mov_b32_dpp")),
    ("dpp-fused", re.compile(r"^v_\w+_dpp")),
    ("pk-minmax", re.compile(r"^v_pk_(min|max)_")),
    ("pk-sub/sra", re.compile(r"^v_pk_(sub|ashrrev|lshlrev|add)_")),
    ("pk-mad", re.compile(r"^v_pk_(mad|mul)_")),
    ("select", re.compile(r"^v_(bfi|bitop3|cndmask|perm|and_or|or3|xad|lshl_or)_")),
    ("logic32", re.compile(r"^v_(xor|or|and|not|lshrrev|ashrrev|lshlrev)_b32")),
    ("other", re.compile(r"^v_")),
]


def cls(ins):
    for name, rx in CLASSES:
        if rx.match(ins):
            return name
    return None


def kernels_src(fbs, ca2):
    out = ["#define POLAR_LANE_REMAP 1", "#define POLAR_Q 6"]
    if ca2:
        out.append("#define POLAR_CA2 1")
    out += ["#include <hip/hip_runtime.h>", '#include "polar_sc_device.h"', "using namespace polar;"]
    names = []
    for fb in fbs:
        W = 16
        while W >= 2:
            for B in range(0, 16, W):
                name = "k_%04x_%d_%d" % (fb, B, W)
                call = ("leaf_ca2<0x%xu, %d, %d, 0>" if ca2 else "leaf_ms<0x%xu, %d, %d>") % (fb, B, W)
                out.append('extern "C" __global__ void %s(const u32 *in, u32 *out) {\n'
                           '  int lane = threadIdx.x & 63; asm volatile("" : "+v"(lane)); Lanes ln; ln.init((u32)(lane & 15));\n'
                           '  u32 M = in[threadIdx.x], S = in[threadIdx.x + 64];\n'
                           '  asm volatile(";@@ begin" :: "v"(M), "v"(S)); __builtin_amdgcn_sched_barrier(0);\n'
                           '  u32 x = %s(M, S, ln);\n'
                           '  asm volatile(";@@ end" :: "v"(x)); __builtin_amdgcn_sched_barrier(0);\n'
                           '  out[threadIdx.x] = x; }' % (name, call))
                names.append((fb, B, W, name))
            W //= 2
    return "\n".join(out), names


def census(asm):
    per = {}
    cur, inside = None, False
    for line in asm.split("\n"):
        m = re.match(r"^(k_\w+):", line)
        if m:
            cur, inside = m.group(1), False
            per[cur] = collections.Counter()
            continue
        if ";@@ begin" in line:
            inside = True
            continue
        if ";@@ end" in line:
            inside = False
            continue
        if inside and cur:
            m = re.match(r"^\s+(v_\w+)", line)
            if m:
                c = cls(m.group(1))
                per[cur][c] += 1
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", default="FB_N1024_K512")
    ap.add_argument("--ca2", action="store_true", help="the CA2 leaf (leaf_ca2, no MIN)")
    args = ap.parse_args()
    import sc_polar_decoder_hls_amd as pkg
    import util
    cfg = None
    if args.ca2:
        cfg = pkg.default_config()
        cfg.sigmag = 0
    dec = pkg.Decoder(util.mask(args.mask), config=cfg)
    leaves = [o["fb"] & 0xFFFF for o in dec.schedule() if o["op"] in ("FLEAF", "GLEAF")]
    mult = collections.Counter(leaves)
    src, names = kernels_src(sorted(mult), args.ca2)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "k.hip")
        open(path, "w").write(src)
        s = os.path.join(tmp, "k.s")
        subprocess.run([CLANG, "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++17", "-w",
                        "-I", CSRC, "-S", "-o", s, path], check=True)
        per = census(open(s).read())
    by_level = {W: collections.Counter() for W in (16, 8, 4, 2)}
    whole = collections.Counter()
    for fb, B, W, name in names:
        k = mult[fb]
        c = per[name]
        if W == 16:
            whole.update({x: k * v for x, v in c.items()})
        own = collections.Counter(c)
        if W > 2:
            for ch in ("k_%04x_%d_%d" % (fb, B, W // 2), "k_%04x_%d_%d" % (fb, B + W // 2, W // 2)):
                own.subtract(per[ch])
        by_level[W].update({x: k * v for x, v in own.items()})
    nleaf = sum(mult.values())
    tot = sum(whole.values())
    print("%s%s: %d leaf records, %d distinct patterns; VALU per leaf %.1f (whole-leaf kernels)"
          % (args.mask, " CA2" if args.ca2 else "", nleaf, len(mult), tot / max(nleaf, 1)))
    cols = [c for c, _ in CLASSES]
    print("%-8s %8s " % ("level", "per leaf") + " ".join("%10s" % c for c in cols))
    acc = 0
    for W in (16, 8, 4, 2):
        c = by_level[W]
        n = sum(c.values())
        acc += n
        print("%-8s %8.1f " % ("W=%d" % W, n / nleaf) + " ".join("%10.1f" % (c[x] / nleaf) for x in cols))
    print("%-8s %8.1f " % ("all", tot / nleaf) + " ".join("%10.1f" % (whole[x] / nleaf) for x in cols))
    print("slack (whole - sum of nodes) per leaf: %.1f" % ((tot - acc) / nleaf))


if __name__ == "__main__":
    main()
