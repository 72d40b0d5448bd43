#!/usr/bin/env python3
"""Per-op shader-clock stamps of a pair-plan decode kernel (where does a C3 / C5 decode spend
its time: upper-level slot loops or generated subtree decoders?).

build (container, CPU):  python tools/pair_stamps.py build [--mask M] [--batch B] [--tuning k=v,..]
    Takes the plan's generated source (Decoder.kernel_source()), adds a stamps argument and
    reads s_memtime after pair_init and after every schedule op of segment 0; lane 0 of the
    lead wave of each pair writes the stamps with vector stores. Links a HIP driver (random
    channel bytes, the plan's launch shape) into build_tools/pair_stamps_<mask>_b<batch>.
run (GPU box):           ./build_tools/pair_stamps_<mask>_b<batch> > gpurun_out/pair_stamps.txt
    Prints per op (and per op class) the median over pairs of its duration in s_memtime
    ticks (shader clock) of the last of 5 launches, plus the launch's HIP-event time.
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
CSRC = os.path.join(ROOT, "sc_polar_decoder_hls_amd", "csrc")
OUT = os.path.join(ROOT, "build_tools")

DRIVER = r'''
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>
int main()
{
    const int N = P_N, batch = P_BATCH, pairs = P_BLOCKS, W = P_W;   // (solo plans: one block per frame)
    std::vector<signed char> h((size_t)batch * N);
    srand(1);
    for (auto &b : h) { int v = 4 + (rand() % 9) - 4 + ((rand() % 7) == 0 ? -8 : 0); b = (signed char)((rand() & 1) ? v : -v); }
    signed char *llr; unsigned short *out; unsigned int *scratch; unsigned long long *st;
    const int out_stride = N / 16;
    hipMalloc(&llr, h.size()); hipMalloc(&out, (size_t)batch * out_stride * 2);
    hipMalloc(&scratch, (size_t)pairs * P_PAIR_DWORDS * 4); hipMalloc(&st, (size_t)pairs * NST * 8);
    hipMemcpy(llr, h.data(), h.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float ms = 0.f;
    int n = N, b = batch, pd = P_PAIR_DWORDS, sr = P_SLOT_ROWS, l0 = P_LDS_ROW0, seg = 0;
    for (int it = 0; it < 5; it++) {
        hipMemset(st, 0, (size_t)pairs * NST * 8);
        hipEventRecord(e0);
        hipLaunchKernelGGL(polar_sc_pair_kernel, dim3(pairs), dim3(64 * W), P_LDS, 0, llr, out, scratch, n, b,
                           out_stride, pd, sr, l0, seg, st);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    std::vector<unsigned long long> s((size_t)pairs * NST);
    hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    printf("last launch %.1f us (HIP events), %d pairs, %d waves per pair; s_memtime ticks (shader clock)\n", ms * 1e3,
           pairs, W);
    std::vector<double> life(pairs);
    for (int p = 0; p < pairs; p++) life[p] = (double)(s[(size_t)p * NST + NST - 1] - s[(size_t)p * NST]);
    printf("pair lifetime median %.0f ticks\n", med(life));
    std::map<std::string, double> cls;
    double tot = 0;
    printf("%-4s %-44s %10s\n", "op", "record", "median");
    for (int k = 0; k + 1 < NST; k++) {
        std::vector<double> d(pairs);
        for (int p = 0; p < pairs; p++) d[p] = (double)(s[(size_t)p * NST + k + 1] - s[(size_t)p * NST + k]);
        const double m = med(d);
        tot += m;
        cls[CLASS[k]] += m;
        printf("%-4d %-44s %10.0f\n", k, LABEL[k], m);
    }
    printf("\nby class (sum of medians, share of their total %.0f):\n", tot);
    for (auto &kv : cls) printf("  %-22s %10.0f  %5.1f %%\n", kv.first.c_str(), kv.second, 100.0 * kv.second / tot);
    return 0;
}
'''

NAMES = {1: "F", 2: "G", 5: "REP", 6: "R1", 7: "SPC", 8: "H", 9: "H0", 13: "SUB"}


def drop_subtree_fences(src):
    """A/B variant: the generated subtree decoders without their scheduling fences (the
    sched_barrier before every op and every 8 registers), so that the machine scheduler can
    overlap an op's independent prefix with the previous op's dependent tail."""
    out, inside = [], False
    for line in src.split("\n"):
        if line.startswith("__device__ __noinline__ void polar_psub_"):
            inside = True
        elif line.startswith("}"):
            inside = False
        if inside and line.strip() == "__builtin_amdgcn_sched_barrier(0);":
            continue
        out.append(line)
    return "\n".join(out)


def synthetic_roots(src):
    """A/B variant (C3 wait attribution): every subtree decoder reads its
    root rows from a register expression of the lane and row instead of its stage slot (and,
    for fused roots, the parent's slot rows and partial sums): the same straight-line code with
    no root loads, so the subtree time left is issue time at the same occupancy, and the
    difference to the real kernel is the time the decoders wait for their root reads (LDS /
    HBM). The decoded bits are not meaningful."""
    out = []
    for line in src.split("\n"):
        if line.startswith("#define CH(j)"):
            line = "#define CH(j) ((((u32)(j) * 0x00050003u) ^ (lane_ * 0x00070009u)) & 0x801F801Fu)"
        out.append(line)
    return "\n".join(out)


def synthetic_bits(src):
    """A/B variant: the fused-root G decoders take the partial sums of their root G from a
    register expression instead of the pair's HBM bit dwords (the LDS / HBM slot reads stay)"""
    return src.replace("ubits4(hb_[((ub_ + ((j) & ~1)) >> 4) * 64], ub_ + ((j) & ~1))",
                       "ubits4(lane_ * 0x9E3779B9u ^ (u32)(j), ub_ + ((j) & ~1))")


def synthetic_slots(src):
    """A/B variant: the root rows' slot reads (SLOT(j): the parent level in LDS or HBM) from a
    register expression (the partial-sum reads of G roots stay)"""
    out = []
    for line in src.split("\n"):
        if line.startswith("#define SLOT(j)") and "su_t" not in line:
            line = "#define SLOT(j) ((((u32)(j) * 0x05030201u) ^ (lane_ * 0x01070309u)) & 0x9F9F9F9Fu)"
        out.append(line)
    return "\n".join(out)


def build(mask_name, batch, tuning, variant=""):
    import sc_polar_decoder_hls_amd as pkg
    import util
    mask = util.mask(mask_name)
    dec = pkg.Decoder(mask, tuning=dict(tuning, kernel=3))
    st = dec.stats
    assert st["kernel"] == 3 and st["tier_steps"] == 0, "pair plan without grid tier expected"
    src = dec.kernel_source()
    if variant == "nofence":
        src = drop_subtree_fences(src)
    elif variant == "synroot":
        src = synthetic_roots(src)
    elif variant == "synbits":
        src = synthetic_bits(src)
    elif variant == "synslot":
        src = synthetic_slots(src)
    N, G, S = mask.size, mask.size // 16, st["sub_words"]
    # launch shape of the library's own decision (polar_sc_plan_launch_info)
    info = dec.launch_info(batch)
    W, lds_row0, lds = info["waves_per_block"], info["lds_row0"], info["lds_bytes"]
    solo = "#define POLAR_SOLO 1" in src
    wpr = 8 if solo else 4
    fused = st["lds_bytes_per_wave"] == 2 * S // wpr * 128   # subtree roots read as F / G of the parents
    slot_rows = (G - (2 * S if fused else S)) // wpr
    blocks = batch if solo else (batch + 1) // 2
    pair_dwords = st["scratch_bytes_per_wave"] // 4
    # stamp segment 0: after pair_init, after every op
    head = "int lds_row0, int seg)\n{\n"
    k = src.index("polar_sc_pair_kernel(")
    assert src.find(head, k) > 0
    src = src[:k] + src[k:].replace(head, "int lds_row0, int seg, unsigned long long *__restrict__ stamps_)\n{\n", 1)
    stamp = ("{ const unsigned long long t_ = __builtin_amdgcn_s_memtime(); "
             "if ((threadIdx.x & 63) == 0 && wi == 0) stamps_[pair * NST + %d] = t_; }")
    init = "(lds_w32 *)smem_);\n"
    k = src.index("polar_sc_pair_kernel(")
    i = src.index(init, k) + len(init)
    src = src[:i] + "  " + stamp % 0 + "\n" + src[i:]
    lines = src[i:].split("\n")
    labels, classes, n = [], [], 0
    for j, line in enumerate(lines):
        if line.startswith("    return;"):
            break
        m = re.match(r"    c\.sync\(\); (.*;)\s+// (chain )?(\d+) level (\d+) n (\d+) pos (\d+)(.*)$", line)
        if not m:
            continue
        n += 1
        code, lev, nn, pos = (int(x) for x in m.groups()[2:6])
        name = NAMES.get(code, str(code))
        if m.group(2):   # fused F / G descent (pop_chain): the records after '|'
            recs = [name] + [NAMES.get(int(r.split()[0]), "?") for r in m.group(7).split("|")[1:]]
            labels.append("chain %s level %d n %d pos %d" % ("".join(recs), lev, nn, pos))
            classes.append("chain from level %d" % lev)
        else:
            labels.append("%s level %d n %d pos %d" % (name, lev, nn, pos))
            classes.append("SUB" if code == 13 else "%s level %d" % (name, lev) if code in (1, 2) else name)
        lines[j] = "    c.sync(); %s " % m.group(1) + stamp % n
    src = src[:i] + "\n".join(lines)
    nst = n + 1
    defs = ("#define NST %d\n#define P_N %d\n#define P_BATCH %d\n#define P_W %d\n#define P_PAIR_DWORDS %d\n"
            "#define P_SLOT_ROWS %d\n#define P_LDS_ROW0 %d\n#define P_LDS %d\n#define P_BLOCKS %d\n"
            % (nst, N, batch, W, pair_dwords, slot_rows, lds_row0, lds, blocks))
    tab = ("static const char *LABEL[] = {%s};\nstatic const char *CLASS[] = {%s};\n"
           % (", ".join('"%s"' % s for s in labels), ", ".join('"%s"' % s for s in classes)))
    os.makedirs(OUT, exist_ok=True)
    tag = "pair_stamps_%s_b%d%s%s" % (mask_name, batch, "_solo" if solo else "", "_" + variant if variant else "")
    path = os.path.join(OUT, tag + ".hip")
    with open(path, "w") as f:
        f.write("#include <hip/hip_runtime.h>\n" + defs + src + tab + DRIVER)
    exe = os.path.join(OUT, tag)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", CSRC, "-o", exe, path])
    print(exe, "ops", n, "W", W, "lds_row0", lds_row0, "of", slot_rows)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build"])
    ap.add_argument("--mask", default="frozen_n_65536_k_32768")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--tuning", default="")
    ap.add_argument("--variant", default="", choices=["", "nofence", "synroot", "synbits", "synslot"])
    a = ap.parse_args()
    tun = {k: int(v) for k, v in (kv.split("=") for kv in filter(None, a.tuning.split(",")))}
    build(a.mask, a.batch, tun, a.variant)
