#!/usr/bin/env python3
"""Per-wave start / end shader-clock stamps of the C2 per-mask kernel (where does a launch
spend the time no wave is alive? DESIGN.md 3.1 / 9).

build (container, CPU):  python tools/wave_stamps.py build
    Takes the plan's generated kernel source (Decoder.kernel_source()), adds a stamps
    argument, reads s_memtime after the early exit and again at the end, and lane 0 of each
    wave writes both with a vector store under a lane mask; links a small HIP driver
    (random channel bytes, 65536 frames, 20 launches) into build_tools/wave_stamps.
run (GPU box):           ./build_tools/wave_stamps > gpurun_out/wave_stamps.txt
    Prints, for the last launch, quantiles of wave start / end / lifetime relative to the
    first start, in s_memtime ticks, plus the launch's HIP-event time.
"""
import os
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
#include <vector>
int main()
{
    const int N = 1024, batch = 65536, G = N / 16, waves = batch / 8;
    std::vector<unsigned char> h((size_t)batch * N);
    srand(1);
    for (auto &b : h) b = (unsigned char)(rand() % 63 - 31);
    unsigned char *llr; unsigned short *out; unsigned long long *st;
    hipMalloc(&llr, h.size()); hipMalloc(&out, (size_t)batch * G * 2); hipMalloc(&st, (size_t)waves * 16);
    hipMemcpy(llr, h.data(), h.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float ms = 0.f;
    for (int it = 0; it < 20; it++) {
        hipMemset(st, 0, (size_t)waves * 16);
        hipEventRecord(e0);
        polar_sc_mask_kernel<<<waves / 4, 256>>>(llr, out, batch, G, st);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    std::vector<unsigned long long> s((size_t)waves * 2);
    hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull;
    for (int w = 0; w < waves; w++) t0 = std::min(t0, s[2 * w]);
    std::vector<double> start(waves), end(waves), life(waves);
    for (int w = 0; w < waves; w++) {
        start[w] = (double)(s[2 * w] - t0); end[w] = (double)(s[2 * w + 1] - t0); life[w] = end[w] - start[w];
    }
    auto q = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
    printf("last launch %.2f us (HIP events), %d waves; s_memtime ticks relative to the first wave start\n", ms * 1e3, waves);
    const double ps[] = {0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0};
    printf("quantile   start      end        lifetime\n");
    for (double p : ps) printf("%5.2f  %9.0f  %9.0f  %9.0f\n", p, q(start, p), q(end, p), q(life, p));
    // starts by wave index blocks (dispatch order)
    printf("mean start by wave-index decile:");
    for (int d = 0; d < 10; d++) {
        double a = 0; int n = 0;
        for (int w = d * waves / 10; w < (d + 1) * waves / 10; w++) { a += start[w]; n++; }
        printf(" %.0f", a / n);
    }
    printf("\n");
    return 0;
}
'''


def build():
    import sc_polar_decoder_hls_amd as pkg
    import util
    src = pkg.Decoder(util.mask("FB_N1024_K512")).kernel_source()
    sig = "int batch, int out_stride)\n{\n"
    assert sig in src
    src = src.replace(sig, "int batch, int out_stride, unsigned long long *__restrict__ stamps_)\n{\n", 1)
    ret = "  if (wave >= nw_) return;\n"
    assert ret in src
    src = src.replace(ret, ret + "  const unsigned long long t0_ = __builtin_amdgcn_s_memtime();\n", 1)
    tail = "  }\n}\n"
    assert src.endswith(tail)
    src = src[: -len("}\n")] + ("  { const unsigned long long t1_ = __builtin_amdgcn_s_memtime();\n"
                                "    if ((threadIdx.x & 63) == 0) { stamps_[2 * wave] = t0_; stamps_[2 * wave + 1] = t1_; } }\n"
                                "}\n")
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, "wave_stamps.hip")
    with open(path, "w") as f:
        f.write("#include <hip/hip_runtime.h>\n" + src + DRIVER)
    exe = os.path.join(OUT, "wave_stamps")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", CSRC, "-o", exe, path])
    print(exe)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        sys.exit("usage: tools/wave_stamps.py build   (then run build_tools/wave_stamps on the GPU box)")
