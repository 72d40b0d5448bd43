#!/usr/bin/env python3
"""Static instruction census of a pair plan's generated subtree decoders (CPU only).

Takes the plan's generated source (Decoder.kernel_source()), puts an asm comment marker in
front of every schedule op of every subtree decoder (`// F n 8`, `// F+leaf ...`, ...), compiles
it to assembly with the ROCm clang driver the library uses, and attributes every instruction
between two markers to that op's class (F / G / REP / R1 / SPC / H / leaf, by node width). The
markers are `asm volatile` comments, so the scheduler cannot move work across them: the counts
are those of a slightly less scheduled build, good to a few per cent.

Weighted by the number of calls of each decoder in the schedule, the totals are the static
VALU count of one frame pair's (or frame's) subtree work -- the serial instruction chain of a
long-block decode.

    python tools/pair_census.py [--mask frozen_n_262144_k_131072] [--tuning k=v,...]
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

OPLINE = re.compile(r"^(\s*)(?:u32 x\d+_;\n\s*)?\{ // (.*)$|^(\s*)const u32 (x\d+_) = .*// (H0? n \d)$")


def classify(label):
    """op class from a generated op comment"""
    m = re.match(r"(F\+leaf|G\+leaf|REP|SPC|R1|H0|H|F|G) n (\d+)", label)
    if m:
        kind, n = m.group(1), int(m.group(2))
        if kind == "H0":
            kind = "H"
        return "%s n%s" % (kind, n if n < 8 else "8+" if n < 64 else "64+")
    m = re.match(r"([FG])\+leaf", label)
    if m:
        return "leaf"
    return label.split()[0]


def mark_mask_kernel(src):
    """the per-mask kernel (N <= 1024): markers before every op block of polar_sc_mask_kernel"""
    out, n, inside = [], 0, False
    for line in src.split("\n"):
        if "polar_sc_mask_kernel(" in line:
            inside = True
        m = re.match(r"^  \{ // (\S+)(?: level \d+)? n (\d+)", line) or re.match(r"^  \{ // ([FG]\+leaf)", line)
        if inside and m:
            if "leaf" in m.group(1):
                label = "leaf"
            else:
                kind, nn = m.group(1), int(m.group(2))
                label = "%s n%s" % ("H" if kind == "H0" else kind, nn if nn < 8 else "8+")
            out.append('  asm volatile(";@@ %s"); __builtin_amdgcn_sched_barrier(0);' % label)
            n += 1
        out.append(line)
    return "\n".join(out), n


def mask_census(asm):
    valu, allc = collections.Counter(), collections.Counter()
    cur, cls = False, "prologue"
    for line in asm.split("\n"):
        if re.match(r"^polar_sc_mask_kernel:", line):
            cur = True
            continue
        if not cur:
            continue
        if re.match(r"^\.Lfunc_end", line):
            break
        m = re.match(r"^\s*;@@ (.*)$", line)
        if m:
            cls = m.group(1).strip()
            continue
        m = re.match(r"^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|scratch_\w+|flat_\w+)\b", line)
        if m:
            allc[cls] += 1
            if m.group(1).startswith("v_"):
                valu[cls] += 1
    return valu, allc


def mark(src):
    out, n = [], 0
    in_sub = False
    declared = []
    pending = []   # small-op results defined since the last marker: pinned before the next one
    def pin():
        for x in pending:
            out.append('  asm volatile("" :: "v"(%s));' % x)
        pending.clear()
    for line in src.split("\n"):
        if line.startswith("__device__") and "polar_psub_" in line:
            in_sub = True
        elif line.startswith("}") and in_sub:
            pin()
            out.append('  asm volatile(";@@ END"); __builtin_amdgcn_sched_barrier(0);')
            in_sub = False
        if in_sub:
            m = re.match(r"^\s*\{ // (.*)$", line) or re.match(r"^\s*const u32 x\d+_ = .*// (H0? n \d)\s*$", line)
            if m and not line.startswith("    "):
                label = m.group(1)
                if "leaf" in label:
                    label = label.split(" pos")[0]
                pin()
                pending.extend(declared)   # (declared before its own op's block: pinned after it)
                declared.clear()
                out.append('  asm volatile(";@@ %s"); __builtin_amdgcn_sched_barrier(0);' % classify(label))
                n += 1
        out.append(line)
        if in_sub:
            m = re.match(r"^\s*const u32 (x\d+_) =", line)
            if m:
                pending.append(m.group(1))
            m = re.match(r"^\s*u32 (x\d+_);", line)
            if m:
                declared.append(m.group(1))
    return "\n".join(out), n


def compile_asm(src, tmp):
    path = os.path.join(tmp, "k.hip")
    with open(path, "w") as f:
        f.write("#include <hip/hip_runtime.h>\n" + src)
    s = os.path.join(tmp, "k.s")
    subprocess.run([CLANG, "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++17", "-w",
                    "-I", CSRC, "-S", "-o", s, path], check=True)
    return open(s).read()


def census(asm):
    """per function: Counter(class -> VALU), Counter(class -> all instructions)"""
    funcs = {}
    cur, cls = None, None
    for line in asm.split("\n"):
        m = re.match(r"^(_Z\w*polar_psub_(\d+(?:_[FG])?(?:_L)?)\w*):", line)   # (_F / _G: fused roots; _L: CA2 leftmost)
        if m:
            cur = m.group(2)
            funcs[cur] = (collections.Counter(), collections.Counter())
            cls = "prologue"
            continue
        if cur is None:
            continue
        if line.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", line):
            cur = None
            continue
        m = re.match(r"^\s*;@@ (.*)$", line)
        if m:
            cls = m.group(1).strip()
            continue
        m = re.match(r"^\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|scratch_\w+|flat_\w+)\b", line)
        if m:
            ins = m.group(1)
            valu, allc = funcs[cur]
            allc[cls] += 1
            if ins.startswith("v_"):
                valu[cls] += 1
    return funcs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", default="frozen_n_262144_k_131072")
    ap.add_argument("--tuning", default="")
    ap.add_argument("--source", help="census of this generated source file instead of the plan's")
    ap.add_argument("--config", default="", help="polar_sc_config fields, e.g. sigmag=0,par=64")
    args = ap.parse_args()
    import sc_polar_decoder_hls_amd as pkg
    import util
    tun = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in args.tuning.split(",") if kv)
    cfg = None
    if args.config:
        cfg = pkg.default_config()
        for kv in args.config.split(","):
            setattr(cfg, kv.split("=")[0], int(kv.split("=")[1]))
    dec = pkg.Decoder(util.mask(args.mask), config=cfg, tuning=tun or None)
    src = open(args.source).read() if args.source else dec.kernel_source()
    if "polar_sc_mask_kernel(" in src:   # per-mask kernel: one straight-line function
        marked, nmark = mark_mask_kernel(src)
        with tempfile.TemporaryDirectory() as tmp:
            tot_v, tot_a = mask_census(compile_asm(marked, tmp))
        nv = sum(tot_v.values())
        print("%s: per-mask kernel, %d op markers; VALU per wave %d, all instructions %d"
              % (args.mask, nmark, nv, sum(tot_a.values())))
        for c, v in sorted(tot_v.items(), key=lambda kv: -kv[1]):
            print("%-14s %10d %5.1f%% %10d" % (c, v, 100.0 * v / max(nv, 1), tot_a[c]))
        return
    calls = collections.Counter(re.findall(r"polar_psub_(\d+(?:_[FG])?(?:_L)?)\(c\.slot_ptr", src.split("polar_sc_pair_subtest_kernel")[0]))
    marked, nmark = mark(src)
    with tempfile.TemporaryDirectory() as tmp:
        asm = compile_asm(marked, tmp)
    funcs = census(asm)
    tot_v, tot_a = collections.Counter(), collections.Counter()
    for fid, (valu, allc) in funcs.items():
        k = calls.get(fid, 0)
        for c, v in valu.items():
            tot_v[c] += k * v
        for c, v in allc.items():
            tot_a[c] += k * v
    nv, na = sum(tot_v.values()), sum(tot_a.values())
    print("%s: %d subtree kinds, %d calls, %d op markers" % (args.mask, len(funcs), sum(calls.values()), nmark))
    print("dynamic-weighted (static count x calls) per decode: VALU %d, all instructions %d" % (nv, na))
    print("%-14s %10s %6s %10s" % ("class", "VALU", "%", "all"))
    for c, v in sorted(tot_v.items(), key=lambda kv: -kv[1]):
        print("%-14s %10d %5.1f%% %10d" % (c, v, 100.0 * v / max(nv, 1), tot_a[c]))


if __name__ == "__main__":
    main()
