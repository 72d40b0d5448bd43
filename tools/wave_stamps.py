#!/usr/bin/env python3
"""Per-wave phase stamps of the C2 per-mask kernel (where does a launch spend its time?
DESIGN.md 3.1).

build (container, CPU):  python tools/wave_stamps.py build
    Takes the plan's generated kernel source (Decoder.kernel_source()), adds a stamps
    argument and reads s_memtime (shader clock) at the wave's start, when its channel is in
    LDS, after the presplit, after the decode and at the end, plus s_memrealtime (100 MHz,
    one clock for the whole device) at start and end; lane 0 of each wave writes them with
    vector stores. Links a small HIP driver (random channel bytes, 65536 frames, 5 rotated
    input batches, 40 launches) into build_tools/wave_stamps.
run (GPU box):           ./build_tools/wave_stamps > gpurun_out/wave_stamps.txt
    Prints, for the last launch, per-phase quantiles in shader ticks, and from the real-time
    stamps the live-wave count, starts and ends per time bin of the launch.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
CSRC = os.path.join(ROOT, "sc_polar_decoder_hls_amd", "csrc")
OUT = os.path.join(ROOT, "build_tools")

NS = 7   # per wave: s_memtime at start, channel in LDS, presplit done, decode done, end; s_memrealtime start / end

DRIVER = r"""
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
int main()
{
    const int N = 1024, batch = 65536, G = N / 16, waves = batch / 8;
    std::vector<unsigned char> h((size_t)batch * N);
    srand(1);
    for (auto &b : h) b = (unsigned char)(rand() % 63 - 31);
    unsigned char *llr; unsigned short *out; unsigned long long *st;
    // 5 distinct input batches (> 256 MB Infinity Cache, as bench.py rotates them)
    const int NB = 5;
    hipMalloc(&llr, h.size() * NB); hipMalloc(&out, (size_t)batch * G * 2); hipMalloc(&st, (size_t)waves * NS * 8);
    for (int b = 0; b < NB; b++) hipMemcpy(llr + (size_t)b * h.size(), h.data(), h.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float ms = 0.f;
    std::vector<double> lms;
    for (int it = 0; it < 40; it++) {
        hipMemset(st, 0, (size_t)waves * NS * 8);
        hipEventRecord(e0);
        polar_sc_mask_kernel<<<waves / 4, 256>>>(llr + (size_t)(it % NB) * h.size(), out, batch, G, st);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        if (it >= 10) lms.push_back(ms * 1e3);
    }
    // back-to-back launches without the stamp reset in between (the bench's loop shape)
    hipEventRecord(e0);
    for (int it = 0; it < 50; it++)
        polar_sc_mask_kernel<<<waves / 4, 256>>>(llr + (size_t)(it % NB) * h.size(), out, batch, G, st);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float bb = 0.f;
    hipEventElapsedTime(&bb, e0, e1);
    std::sort(lms.begin(), lms.end());
    printf("launch median over 30: %.2f us; 50 back-to-back launches: %.2f us each\n", lms[lms.size() / 2],
           bb * 1e3 / 50);
    std::vector<unsigned long long> s((size_t)waves * NS);
    hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
    auto q = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
    printf("last launch %.2f us (HIP events), %d waves\n", ms * 1e3, waves);
    const char *ph[] = {"channel fetch wait", "presplit (qconv + root split)", "decode", "output"};
    std::vector<double> life(waves);
    printf("per-wave phases, s_memtime ticks (shader clock): quantiles 0.1 / 0.5 / 0.9, mean\n");
    for (int k = 0; k < 4; k++) {
        std::vector<double> d(waves);
        double m = 0;
        for (int w = 0; w < waves; w++) { d[w] = (double)(s[(size_t)w * NS + k + 1] - s[(size_t)w * NS + k]); m += d[w]; }
        printf("  %-32s %9.0f %9.0f %9.0f  mean %9.0f\n", ph[k], q(d, 0.1), q(d, 0.5), q(d, 0.9), m / waves);
    }
    for (int w = 0; w < waves; w++) life[w] = (double)(s[(size_t)w * NS + 4] - s[(size_t)w * NS]);
    printf("  %-32s %9.0f %9.0f %9.0f\n", "lifetime", q(life, 0.1), q(life, 0.5), q(life, 0.9));
    // global timeline from s_memrealtime (100 MHz, one clock for the device)
    unsigned long long r0 = ~0ull, r1 = 0;
    for (int w = 0; w < waves; w++) { r0 = std::min(r0, s[(size_t)w * NS + 5]); r1 = std::max(r1, s[(size_t)w * NS + 6]); }
    const double span = (double)(r1 - r0) * 10.0;   // ns
    printf("s_memrealtime span of the waves: %.2f us (first start -> last end)\n", span / 1e3);
    const int BINS = 24;
    printf("live waves per time bin (%.2f us each):", span / BINS / 1e3);
    for (int b = 0; b < BINS; b++) {
        const double t = r0 + (b + 0.5) * (double)(r1 - r0) / BINS;
        int n = 0;
        for (int w = 0; w < waves; w++) n += (double)s[(size_t)w * NS + 5] <= t && t < (double)s[(size_t)w * NS + 6];
        printf(" %d", n);
    }
    printf("\nstarts per time bin:");
    for (int b = 0; b < BINS; b++) {
        const double a = r0 + b * (double)(r1 - r0) / BINS, c = r0 + (b + 1) * (double)(r1 - r0) / BINS;
        int n = 0;
        for (int w = 0; w < waves; w++) n += (double)s[(size_t)w * NS + 5] >= a && (double)s[(size_t)w * NS + 5] < c;
        printf(" %d", n);
    }
    printf("\nends per time bin:");
    for (int b = 0; b < BINS; b++) {
        const double a = r0 + b * (double)(r1 - r0) / BINS, c = r0 + (b + 1) * (double)(r1 - r0) / BINS;
        int n = 0;
        for (int w = 0; w < waves; w++) n += (double)s[(size_t)w * NS + 6] >= a && (double)s[(size_t)w * NS + 6] <= c;
        printf(" %d", n);
    }
    printf("\n");
    return 0;
}
"""


def build(out_name="wave_stamps", src=None):
    """src: a per-mask kernel source (default: the C2 plan's) to instrument."""
    import sc_polar_decoder_hls_amd as pkg
    import util
    if src is None:
        src = pkg.Decoder(util.mask("FB_N1024_K512")).kernel_source()
    sig = "int batch, int out_stride)\n{\n"
    assert sig in src
    src = src.replace(sig, "int batch, int out_stride, unsigned long long *__restrict__ stamps_)\n{\n", 1)
    stamp = "  const unsigned long long t%d_ = __builtin_amdgcn_s_memtime();\n"
    ret = "  if (wave >= nw_) return;\n"
    assert ret in src
    src = src.replace(ret, ret + stamp % 0 + "  const unsigned long long r0_ = __builtin_amdgcn_s_memrealtime();\n", 1)
    wait = "  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this batch's channel is in LDS\n"
    assert wait in src
    src = src.replace(wait, wait + stamp % 1, 1)
    first = "  __builtin_amdgcn_sched_barrier(0);\n  { // F level 0"
    assert first in src
    src = src.replace(first, stamp % 2 + first, 1)
    outp = "  const long f_lo = wave * 8"
    assert outp in src
    src = src.replace(outp, stamp % 3 + outp, 1)
    tail = "  }\n}\n"
    assert src.endswith(tail)
    # (inside the decode block, whose locals t1_ .. t3_ are)
    src = src[: -len(tail)] + (stamp % 4 + "  const unsigned long long r1_ = __builtin_amdgcn_s_memrealtime();\n"
                               "  if ((threadIdx.x & 63) == 0) { unsigned long long *p_ = stamps_ + wave * NS;\n"
                               "    p_[0] = t0_; p_[1] = t1_; p_[2] = t2_; p_[3] = t3_; p_[4] = t4_; p_[5] = r0_; p_[6] = r1_; }\n"
                               + tail)
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, out_name + ".hip")
    with open(path, "w") as f:
        f.write("#include <hip/hip_runtime.h>\n#define NS %d\n" % NS + src + DRIVER)
    exe = os.path.join(OUT, out_name)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", CSRC, "-o", exe, path])
    print(exe)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        # optional: an output name and a saved per-mask kernel source (same-box A/B of variants)
        name = sys.argv[2] if len(sys.argv) > 2 else "wave_stamps"
        build(name, open(sys.argv[3]).read() if len(sys.argv) > 3 else None)
    else:
        sys.exit("usage: tools/wave_stamps.py build [name [kernel source]]   (then run build_tools/<name> on the GPU box)")
