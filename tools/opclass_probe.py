#!/usr/bin/env python3
"""Where does the schedule interpreter spend its time? Timing-only experiment.

build (container):  python tools/opclass_probe.py build
    Builds variants of libpolar_sc.so into build_tools/opclass/ from a patched temporary
    copy of csrc/polar_sc_interp.h in which one class of ops is skipped (results are
    wrong; the product sources are not modified). The patched header is also embedded for
    hipRTC, so hybrid plans (N > 1024) run the patched loop too.
run (GPU box):      python tools/opclass_probe.py run [--mask M --batch B]
    Times the decode with every variant (each in its own process) and prints JSON lines.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUTD = os.path.join(ROOT, "build_tools", "opclass")
# op codes: F 1, G 2, FLEAF 3, GLEAF 4, REP 5, R1 6, SPC 7, H 8, H0 9
VARIANTS = {
    "base": "",
    "no_leaf": "if (code == OP_FLEAF || code == OP_GLEAF) continue;",
    "no_rep_r1_spc": "if (code == OP_REP || code == OP_R1 || code == OP_SPC) continue;",
    "no_h": "if (code == OP_H || code == OP_H0) continue;",
    "no_narrow_fg": "if ((code == OP_F || code == OP_G) && !split) continue;",
    "no_wide_fg": "if ((code == OP_F || code == OP_G) && split) continue;",
    # hybrid plans (POLAR_SC_JIT=1, N > 1024): the generated subtree calls vs the rest
    "no_sub": "if (code == OP_SUB) continue;",
    "only_sub": "if (code != OP_SUB) continue;",
}
ANCHOR = "        if (!split && wi != lead) continue;\n"
# cycle-accounting variant: s_memtime around every op and barrier; wave 0 of group 0 prints
# the totals. (gfx950 has no SHADER_CYCLES hwreg: s_getreg id 29 reads 0.) Reading s_memtime
# waits for lgkmcnt(0), so an op's outstanding LDS traffic is charged to that op.
CYC_PATCHES = [
    ("namespace polar {\n",
     "namespace polar {\n__device__ __forceinline__ long long cyc_now_() {\n"
     "    return (long long)__builtin_amdgcn_s_memtime(); }\n"),
    ("    bool prev_split = true;\n",
     "    bool prev_split = true;\n"
     "    long long c1_ = 0, c2_ = 0, c3_ = 0, c4_ = 0, c5_ = 0, c6_ = 0, c7_ = 0, c8_ = 0, c9_ = 0;\n"
     "    long long bar_ = 0, loop_ = 0, lt_ = cyc_now_(), t00_ = lt_;\n"),
    ("        if (wpg > 1 && (split || prev_split)) __syncthreads();\n",
     "        { const long long b0_ = cyc_now_();\n"
     "          if (wpg > 1 && (split || prev_split)) __syncthreads();\n"
     "          bar_ += cyc_now_() - b0_; }\n"),
    ("        switch (code) {\n        case OP_F: op_fg<false>",
     "        const long long t0_ = cyc_now_();\n        switch (code) {\n        case OP_F: op_fg<false>"),
    ("        default: break;\n        }\n    }\n",
     "        default: break;\n        }\n"
     "        { const long long d_ = cyc_now_() - t0_;\n"
     "          if (code == 1) c1_ += d_; else if (code == 2) c2_ += d_; else if (code == 3) c3_ += d_;\n"
     "          else if (code == 4) c4_ += d_; else if (code == 5) c5_ += d_; else if (code == 6) c6_ += d_;\n"
     "          else if (code == 7) c7_ += d_; else if (code == 8) c8_ += d_; else c9_ += d_; }\n"
     "    }\n"
     "    loop_ = cyc_now_() - t00_;\n"
     "    if (group == 0 && lane == 0) {\n"
     "        printf(\"CYC wave %d loop %lld barrier %lld F %lld G %lld FLEAF %lld GLEAF %lld REP %lld R1 %lld SPC %lld H %lld H0 %lld\\n\",\n"
     "               wi, loop_, bar_, c1_, c2_, c3_, c4_, c5_, c6_, c7_, c8_, c9_);\n"
     "    }\n"),
]


def copy_sources(tmp, name):
    """csrc/ and include/ in the repository layout (polar_sc_plan.hpp includes ../../include)."""
    from sc_polar_decoder_hls_amd import _build
    base = os.path.join(tmp, name)
    kdir = os.path.join(base, "pkg", "csrc")
    shutil.copytree(os.path.join(_build.PKG, "csrc"), kdir)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(base, "include"))
    return kdir


def build_cycles():
    """libpolar_sc_cycles.so: the interpreter with per-op-type cycle accounting (printf)."""
    sys.path.insert(0, ROOT)
    from sc_polar_decoder_hls_amd import _build
    os.makedirs(OUTD, exist_ok=True)
    tmp = tempfile.mkdtemp()
    src = open(os.path.join(_build.PKG, "csrc", "polar_sc_interp.h")).read()
    for a, b in CYC_PATCHES:
        assert a in src, a
        src = src.replace(a, b, 1)
    kdir = copy_sources(tmp, "cyc")
    with open(os.path.join(kdir, "polar_sc_interp.h"), "w") as f:
        f.write(src)
    out = os.path.join(OUTD, "libpolar_sc_cycles.so")
    srcs = [os.path.join(kdir, f) for f in ("polar_sc_kernels.hip", "polar_sc_host.cpp", "polar_sc_jit.cpp",
                                             "polar_sc_channel.hip")]
    subprocess.check_call([_build.hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-I" + os.path.join(ROOT, "include"), "-I" + _build.GEN_DIR] + srcs +
                          ["-o", out, "-lhiprtc"])
    shutil.rmtree(tmp)
    print("built", out)


def build():
    sys.path.insert(0, ROOT)
    from sc_polar_decoder_hls_amd import _build
    os.makedirs(OUTD, exist_ok=True)
    tmp = tempfile.mkdtemp()
    src = open(os.path.join(_build.PKG, "csrc", "polar_sc_interp.h")).read()
    assert ANCHOR in src
    for name, skip in VARIANTS.items():
        kdir = copy_sources(tmp, name)
        patched = src.replace(ANCHOR, ANCHOR + ("        " + skip + "\n" if skip else ""))
        with open(os.path.join(kdir, "polar_sc_interp.h"), "w") as f:
            f.write(patched)
        # the hybrid kernel compiles the embedded header text with hipRTC: embed the patched one
        gen = os.path.join(kdir, "gen")
        os.makedirs(gen)
        shutil.copy(os.path.join(_build.GEN_DIR, "polar_sc_device_src.inc"), gen)
        with open(os.path.join(gen, "polar_sc_interp_src.inc"), "w") as f:
            f.write("static const char kPolarInterpSrc[] = R\"POLARSRC(" + patched + ")POLARSRC\";\n")
        out = os.path.join(OUTD, "libpolar_sc_%s.so" % name)
        cmd = [_build.hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-I" + os.path.join(ROOT, "include"), "-I" + gen,
               os.path.join(kdir, "polar_sc_kernels.hip"), os.path.join(kdir, "polar_sc_host.cpp"),
               os.path.join(kdir, "polar_sc_jit.cpp"), os.path.join(kdir, "polar_sc_channel.hip"), "-o", out,
               "-lhiprtc"]
        subprocess.check_call(cmd)
        print("built", out)
    shutil.rmtree(tmp)


def one(name, mask_name, batch, reps):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from sc_polar_decoder_hls_amd import _build
    _build.LIB = os.path.join(OUTD, "libpolar_sc_%s.so" % name)
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    import util
    mask = util.mask(mask_name)
    dev = torch.device("cuda", 0)
    dec = pkg.Decoder(mask)
    dec.prepare(batch)
    llr, _ = bench.gen_frames_torch(torch, mask, batch, 2.5, 1, dev)
    out = torch.empty((batch, dec.words), dtype=torch.int64, device=dev)
    dec.decode(llr, out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        dec.decode(llr, out)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"variant": name, "mask": mask_name, "batch": batch, "ms": a.elapsed_time(b) / reps}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["build", "build_cycles", "run", "one"])
    ap.add_argument("--variant", default="base")
    ap.add_argument("--mask", default="frozen_n_65536_k_32768")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    if a.what == "build":
        build()
    elif a.what == "build_cycles":
        build_cycles()
    elif a.what == "one":
        one(a.variant, a.mask, a.batch, a.reps)
    else:
        for name in VARIANTS:
            subprocess.check_call([sys.executable, __file__, "one", "--variant", name, "--mask", a.mask,
                                   "--batch", str(a.batch), "--reps", str(a.reps)], timeout=300)


if __name__ == "__main__":
    main()
