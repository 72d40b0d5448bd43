"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the CPU code:

* the oracle (oracle/polar_oracle.c, polar_channel_oracle.c; gcc), driven by
  tests/sanitize/oracle_san.c: random masks / LLRs through the literal FSM and the recursive
  restatement at every swept configuration, which must agree;
* the host half of libpolar_sc.so (schedule compiler, plans, source generators, loaders,
  frozen-table tooling; hipcc with the sanitizers on the host side only), driven by
  tests/sanitize/host_san.c through the C ABI without touching a GPU.

Any sanitizer report aborts the driver (-fno-sanitize-recover=all), failing the test.
"""
import os
import subprocess

import numpy as np
import pytest

import util

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")
OUT = os.path.join(SAN, "build")
CSRC = os.path.join(ROOT, "sc_polar_decoder_hls_amd", "csrc")
FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer"]


def _stale(target, deps):
    return not os.path.exists(target) or os.path.getmtime(target) < max(os.path.getmtime(d) for d in deps)


def _env():
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    return env


def test_oracle_asan_ubsan():
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "oracle_san")
    srcs = [os.path.join(SAN, "oracle_san.c"), os.path.join(ROOT, "oracle", "polar_oracle.c"),
            os.path.join(ROOT, "oracle", "polar_channel_oracle.c")]
    if _stale(exe, srcs):
        subprocess.check_call(["gcc", "-std=c99", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]
                              + FLAGS + ["-o", exe] + srcs + ["-lm"])
    r = subprocess.run([exe], capture_output=True, text=True, env=_env(), timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout


def test_host_library_asan_ubsan(pkg, tmp_path):
    from sc_polar_decoder_hls_amd import _build
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, "libpolar_sc_san.so")
    exe = os.path.join(OUT, "host_san")
    deps = _build.SOURCES + _build.HEADERS
    if _stale(lib, deps):
        pkg.build()   # refreshes the embedded hipRTC headers under build/
        san = []
        for f in ("address", "undefined"):
            san += ["-Xarch_host", "-fsanitize=" + f]
        subprocess.check_call([_build.hipcc(), "--offload-arch=" + _build.ARCH, "-std=c++17", "-fPIC", "-shared"]
                              + FLAGS + san + ["-Xarch_host", "-fno-sanitize-recover=all",
                                               "-I" + os.path.join(ROOT, "include"), "-I" + _build.GEN_DIR]
                              + _build.SOURCES + ["-o", lib, "-lhiprtc"])
    if _stale(exe, [lib, os.path.join(SAN, "host_san.c")]):
        # host-only C driver (no device code): -fno-gpu-sanitize keeps the sanitizers off any GPU target
        subprocess.check_call([_build.hipcc(), "-x", "c", "-fno-gpu-sanitize", "-fsanitize=address,undefined",
                               "-fno-sanitize-recover=all"]
                              + FLAGS + ["-I" + os.path.join(ROOT, "include"), os.path.join(SAN, "host_san.c"),
                                         "-o", exe, "-L" + OUT, "-lpolar_sc_san", "-Wl,-rpath," + OUT])
    # table files in both reference formats, written from the repo's mask fixtures
    m1 = util.mask("FB_N1024_K512")
    order = np.concatenate([np.flatnonzero(m1), np.flatnonzero(m1 == 0)])
    tab = tmp_path / "FB_N1024_K512.txt"
    tab.write_text(pkg.frozen_tab_text(order, 1024))
    m2 = util.mask("frozen_n_4096_k_2048")
    gen = tmp_path / "frozen_n_4096_k_2048.txt"
    gen.write_text(" ".join(str(int(v)) for v in m2))
    r = subprocess.run([exe, str(tab), str(gen)], capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_san: ok" in r.stdout
