"""Build libpolar_sc.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

The shared library is the product: HIP kernels (csrc/polar_sc_kernels.hip) + host plan /
schedule compiler / C ABI (csrc/polar_sc_host.cpp) behind include/polar_sc.h.
"""
import os
import shutil
import subprocess
import sys

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


def strip_comments(src):
    """the device header as embedded for run-time compiles: without its // comments and blank
    lines, so that editing a comment does not change the code-object cache keys (polar_sc_jit.cpp
    source_key hashes the embedded text); the headers hold no string literal with '//'"""
    import re
    lines = (re.sub(r"\s*//.*$", "", line).rstrip() for line in src.split("\n"))
    return "\n".join(line for line in lines if line) + "\n"


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
            src = strip_comments(f.read())
        assert ")POLARSRC\"" not in src
        with open(os.path.join(GEN_DIR, inc), "w") as f:
            f.write("static const char " + name + "[] = R\"POLARSRC(" + src + ")POLARSRC\";\n")
    tmp = LIB + ".tmp.%d" % os.getpid()
    # the ROCm clang driver next to this hipcc: whole-module compiles of generated kernels
    # (polar_sc_jit.cpp offline_compile)
    hc = shutil.which(hipcc()) or hipcc()
    clang = os.path.join(os.path.dirname(os.path.dirname(os.path.realpath(hc))), "lib", "llvm", "bin", "clang++")
    # the driver's version text, fixed at library build time: part of the cache key of the
    # objects it builds (identical on every machine the library and its cache travel to)
    try:
        ver = subprocess.run([clang, "--version"], capture_output=True, text=True, timeout=60).stdout.split("\n")[0]
    except (OSError, subprocess.SubprocessError):
        ver = "unknown"
    ver = "".join(ch for ch in ver if ch.isalnum() or ch in " .-_()/+:")
    cmd = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           '-DPOLAR_ROCM_CLANG="%s"' % clang, '-DPOLAR_ROCM_CLANG_VERSION="%s"' % ver,
           "-I" + os.path.join(ROOT, "include"), "-I" + GEN_DIR] + SOURCES + ["-o", tmp, "-lhiprtc", "-lz"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


def _cfg_fields(cfg):
    if cfg is None:
        return None
    return {f: int(getattr(cfg, f)) for f, _ in cfg._fields_}


def _compile_item(item):
    """Worker of the prewarm pool: one plan's hipRTC kernels into the code-object cache."""
    import sys
    import time
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import sc_polar_decoder_hls_amd as pkg
    name, m, cfg, tun = item
    t0 = time.time()
    c = None
    if cfg is not None:
        c = pkg.default_config()
        for k, v in cfg.items():
            setattr(c, k, v)
    dec = pkg.Decoder(m, c, tuning=tun)
    ok = dec.compile()
    dec.close()
    return name, tun, ok, time.time() - t0


def _run_pool(items, procs, verbose):
    """hipRTC serialises compilations inside one process (a single thread makes progress at a
    time), so the prewarm fans out over worker PROCESSES (spawned: nothing of the parent's HIP
    runtime state is inherited). Largest codes first: the long compiles overlap the short ones."""
    import multiprocessing as mp
    items = sorted(items, key=lambda it: -it[1].size)
    procs = max(1, min(procs, len(items)))
    if procs == 1:
        res = map(_compile_item, items)
        for r in res:
            _report(r, verbose)
        return
    # (a pool whose workers cannot start -- e.g. the parent runs a script from stdin, which
    # spawned children cannot re-import -- raises BrokenProcessPool instead of hanging: then
    # compile in-process)
    from concurrent.futures import ProcessPoolExecutor, as_completed
    from concurrent.futures.process import BrokenProcessPool
    # (python -c has no __main__ file and spawns fine; python - / a REPL names one that is
    # not a file, which spawned children would try to import)
    main = sys.modules.get("__main__")
    mfile = getattr(main, "__file__", None)
    if mfile is not None and not os.path.isfile(mfile):
        for r in map(_compile_item, items):
            _report(r, verbose)
        return
    done = set()
    try:
        with ProcessPoolExecutor(procs, mp_context=mp.get_context("spawn")) as ex:
            futs = {ex.submit(_compile_item, it): i for i, it in enumerate(items)}
            for f in as_completed(futs):
                _report(f.result(), verbose)
                done.add(futs[f])
    except BrokenProcessPool:
        for i, it in enumerate(items):
            if i not in done:
                _report(_compile_item(it), verbose)


def _report(r, verbose):
    name, tun, ok, dt = r
    if verbose:
        print("prewarm %-28s %s %s %.1f s" % (name, tun or "", "compiled" if ok else "(no hipRTC kernel)", dt),
              flush=True)


def _default_procs():
    # a C5 hybrid / pair compile holds a few GB: bounded by memory as well as cores
    return int(os.environ.get("POLAR_SC_PREWARM_PROCS", min(6, os.cpu_count() or 1)))


def prewarm_plans(plans, procs=None, verbose=False):
    """Compile the hipRTC kernels of [(name, info mask, tuning dict)] into the code-object cache
    (host only, in parallel worker processes, largest first)."""
    _run_pool([(n, m, None, t) for n, m, t in plans], procs or _default_procs(), verbose)


def prewarm_items(items, procs=None, verbose=False):
    """Compile the hipRTC kernels of [(name, info mask, config fields dict or None, tuning dict
    or None)] into the code-object cache (host only, in parallel)."""
    _run_pool(list(items), procs or _default_procs(), verbose)


def prewarm(masks, configs=(None,), procs=None, verbose=False):
    """Compile the hipRTC kernels of the plans of `masks` ({name: info mask}) x `configs`
    into the on-disk code-object cache next to the library (lib/rtc_cache/), host only, in
    parallel. A GPU box then loads them instead of compiling (the C5 hybrid kernel takes about
    two minutes of hipRTC)."""
    items = [(n, m, _cfg_fields(c), None) for n, m in masks.items() for c in configs]
    _run_pool(items, procs or _default_procs(), verbose)
