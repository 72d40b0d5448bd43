#!/usr/bin/env python3
"""Wave-priority A/B of the C2 per-mask kernel (the launch tail).

The SIMD arbiter issues from the oldest wave first among equal priorities, so the four waves
of a SIMD finish staggered (the end clusters of profiles/r04_c2_wave_timeline.txt) and the
last-dispatched waves form the launch's tail. These variants set the wave priority
(s_setprio) at fractions of the op list of the straight-line decode (at existing
sched_barrier points, so the instruction schedule is unchanged):
  dec4  3 at the start, 2 / 1 / 0 after 1/4, 1/2, 3/4 of the ops (waves further along yield)
  dec2  1 at the start, 0 after half of the ops
  inc4  0 / 1 / 2 / 3 (oldest-first made explicit; the control)
  young 3 until the channel is split, then 0 (a new wave's fetch + presplit go first)
Each variant is built with tools/wave_stamps.py's driver (launch median, 50 back-to-back
launches, per-wave timeline): build_tools/prio_<variant>; the baseline is build_tools/prio_base.

build (container, CPU): python tools/prio_ab.py build
run (GPU box):          for v in base dec4 dec2 inc4 young; do ./build_tools/prio_$v; done
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

VARIANTS = {"dec4": (3, [(0.25, 2), (0.5, 1), (0.75, 0)]), "dec2": (1, [(0.5, 0)]),
            "inc4": (0, [(0.25, 1), (0.5, 2), (0.75, 3)]),
            # a new wave outranks the others only until its channel is split (fetch + presplit)
            "young": (3, "decode")}
BARRIER = "  __builtin_amdgcn_sched_barrier(0);\n"


def with_priorities(src, start, steps):
    ret = "  if (wave >= nw_) return;\n"
    assert ret in src
    src = src.replace(ret, ret + "  __builtin_amdgcn_s_setprio(%d);\n" % start, 1)
    if steps == "decode":
        first = BARRIER + "  { // F level 0"
        assert first in src
        return src.replace(first, "  __builtin_amdgcn_s_setprio(0);\n" + first, 1)
    pos = [m.start() for m in re.finditer(re.escape(BARRIER), src)]
    assert len(pos) > 8
    inserts = sorted(((pos[int(f * (len(pos) - 1))], p) for f, p in steps), reverse=True)
    for at, p in inserts:
        at += len(BARRIER)
        src = src[:at] + "  __builtin_amdgcn_s_setprio(%d);\n" % p + src[at:]
    return src


def build():
    import sc_polar_decoder_hls_amd as pkg
    import util
    import wave_stamps
    src = pkg.Decoder(util.mask("FB_N1024_K512")).kernel_source()
    wave_stamps.build("prio_base", src)
    for name, (start, steps) in VARIANTS.items():
        wave_stamps.build("prio_" + name, with_priorities(src, start, steps))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        sys.exit(__doc__)
