#!/usr/bin/env python3
"""Where does the schedule interpreter spend its time? Timing-only experiment.

build (container):  python tools/opclass_probe.py build
    Builds variants of libpolar_sc.so into build_tools/opclass/ from a patched temporary
    copy of csrc/polar_sc_kernels.hip in which one class of ops is skipped (results are
    wrong; the product sources are not modified).
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
}
ANCHOR = "        if (!split && wi != 0) continue;\n"


def build():
    sys.path.insert(0, ROOT)
    from sc_polar_decoder_hls_amd import _build
    os.makedirs(OUTD, exist_ok=True)
    tmp = tempfile.mkdtemp()
    src = open(os.path.join(_build.PKG, "csrc", "polar_sc_kernels.hip")).read()
    assert ANCHOR in src
    for name, skip in VARIANTS.items():
        kdir = os.path.join(tmp, name)
        shutil.copytree(os.path.join(_build.PKG, "csrc"), kdir)
        with open(os.path.join(kdir, "polar_sc_kernels.hip"), "w") as f:
            f.write(src.replace(ANCHOR, ANCHOR + ("        " + skip + "\n" if skip else "")))
        out = os.path.join(OUTD, "libpolar_sc_%s.so" % name)
        cmd = [_build.hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-I" + os.path.join(ROOT, "include"), "-I" + _build.GEN_DIR,
               os.path.join(kdir, "polar_sc_kernels.hip"), os.path.join(kdir, "polar_sc_host.cpp"),
               os.path.join(kdir, "polar_sc_jit.cpp"), "-o", out, "-lhiprtc"]
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
    ap.add_argument("what", choices=["build", "run", "one"])
    ap.add_argument("--variant", default="base")
    ap.add_argument("--mask", default="frozen_n_65536_k_32768")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    if a.what == "build":
        build()
    elif a.what == "one":
        one(a.variant, a.mask, a.batch, a.reps)
    else:
        for name in VARIANTS:
            subprocess.check_call([sys.executable, __file__, "one", "--variant", name, "--mask", a.mask,
                                   "--batch", str(a.batch), "--reps", str(a.reps)], timeout=300)


if __name__ == "__main__":
    main()
