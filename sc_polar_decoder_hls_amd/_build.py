"""Build libpolar_sc.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

The shared library is the product: HIP kernels (csrc/polar_sc_kernels.hip) + host plan /
schedule compiler / C ABI (csrc/polar_sc_host.cpp) behind include/polar_sc.h.
"""
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "lib", "libpolar_sc.so")
SOURCES = [os.path.join(PKG, "csrc", "polar_sc_kernels.hip"), os.path.join(PKG, "csrc", "polar_sc_host.cpp"),
           os.path.join(PKG, "csrc", "polar_sc_jit.cpp"), os.path.join(PKG, "csrc", "polar_sc_pairgen.cpp"),
           os.path.join(PKG, "csrc", "polar_sc_channel.hip"),
           os.path.join(PKG, "csrc", "polar_sc_tables.cpp")]
DEVICE_H = os.path.join(PKG, "csrc", "polar_sc_device.h")
INTERP_H = os.path.join(PKG, "csrc", "polar_sc_interp.h")
PAIR_H = os.path.join(PKG, "csrc", "polar_sc_pair.h")
HEADERS = [os.path.join(ROOT, "include", "polar_sc.h"), DEVICE_H, INTERP_H, PAIR_H, os.path.join(PKG, "csrc", "polar_sc_plan.hpp"),
           os.path.join(PKG, "csrc", "polar_sc_glibcf.h")]
GEN_DIR = os.path.join(PKG, "build")
CLI_SRC = os.path.join(ROOT, "examples", "polar_decode_cli.c")
CLI = os.path.join(PKG, "lib", "polar_decode_cli")
ARCH = os.environ.get("POLAR_SC_ARCH", "gfx950")


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    return "hipcc"


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in SOURCES + HEADERS)


def build_cli(verbose=False):
    """Plain-C example caller (examples/polar_decode_cli.c) linked against the library."""
    if os.path.exists(CLI) and os.path.getmtime(CLI) > max(os.path.getmtime(CLI_SRC), os.path.getmtime(LIB)):
        return CLI
    cmd = ["gcc", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"), CLI_SRC, "-o", CLI,
           "-L" + os.path.dirname(LIB), "-lpolar_sc", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return CLI


def build(force=False, verbose=False):
    """Compile the library if stale; returns its path. Raises on compiler errors."""
    if not force and not needs_build():
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    os.makedirs(GEN_DIR, exist_ok=True)
    # embed the device headers for hipRTC (per-mask kernels are compiled at plan time)
    for path, inc, name in ((DEVICE_H, "polar_sc_device_src.inc", "kPolarDeviceSrc"),
                            (INTERP_H, "polar_sc_interp_src.inc", "kPolarInterpSrc"),
                            (PAIR_H, "polar_sc_pair_src.inc", "kPolarPairSrc")):
        with open(path) as f:
            src = f.read()
        assert ")POLARSRC\"" not in src
        with open(os.path.join(GEN_DIR, inc), "w") as f:
            f.write("static const char " + name + "[] = R\"POLARSRC(" + src + ")POLARSRC\";\n")
    tmp = LIB + ".tmp.%d" % os.getpid()
    cmd = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-I" + os.path.join(ROOT, "include"), "-I" + GEN_DIR] + SOURCES + ["-o", tmp, "-lhiprtc"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


def prewarm_plans(plans, threads=8, verbose=False):
    """Compile the hipRTC kernels of [(name, info mask, tuning dict)] into the code-object cache
    (host only, in parallel, largest first)."""
    import time
    from concurrent.futures import ThreadPoolExecutor
    import sc_polar_decoder_hls_amd as pkg

    def one(item):
        name, m, tun = item
        t0 = time.time()
        dec = pkg.Decoder(m, tuning=tun)
        ok = dec.compile()
        dec.close()
        return name, tun, ok, time.time() - t0

    items = sorted(plans, key=lambda it: -it[1].size)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        for name, tun, ok, dt in ex.map(one, items):
            if verbose:
                print("prewarm %-28s %s %s %.1f s" % (name, tun, "compiled" if ok else "(no hipRTC kernel)", dt))


def prewarm(masks, configs=(None,), threads=8, verbose=False):
    """Compile the hipRTC kernels of the plans of `masks` ({name: info mask}) x `configs`
    into the on-disk code-object cache next to the library (lib/rtc_cache/), host only, in
    parallel. A GPU box then loads them instead of compiling (the C5 hybrid kernel takes about
    two minutes of hipRTC)."""
    import time
    from concurrent.futures import ThreadPoolExecutor
    import sc_polar_decoder_hls_amd as pkg

    def one(item):
        name, m, cfg = item
        t0 = time.time()
        dec = pkg.Decoder(m, cfg)
        ok = dec.compile()
        dec.close()
        return name, ok, time.time() - t0

    items = [(n, m, c) for n, m in masks.items() for c in configs]
    # largest first: the long compiles overlap the short ones
    items.sort(key=lambda it: -it[1].size)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        for name, ok, dt in ex.map(one, items):
            if verbose:
                print("prewarm %-28s %s %.1f s" % (name, "compiled" if ok else "(no hipRTC kernel)", dt))
