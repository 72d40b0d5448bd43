#!/usr/bin/env python3
"""Regression fixtures: LLR frames and the decoded x^ of the CPU restatement (oracle/,
orc_decode_fsm) -> tests/golden/decode_vectors.npz.

These vectors are produced by the restatement, not by the reference (which cannot be
built here). They freeze its current behaviour so that any change to the
oracle, or a GPU path that drifts, is caught without rebuilding anything. The parity pin
of the restatement itself stays the reference's KAT codewords (tests/golden/
kat_codewords.json).

Cases (SURVEY.md 8c "fixtures to create"):
  c1      FB_N128_K64, 1 AWGN frame at 2.5 dB (BASELINE config C1)
  c2_snr  FB_N1024_K512, 64 frames at each Eb/N0 in {0, 1, 2.5, 4} dB
  c2_edge FB_N1024_K512: all-zero LLRs, saturated +-31, -32 only, {-1, 0, 1}, int8 wrap
  c3      frozen_n_65536_k_32768, 1 frame at 1 dB (BASELINE config C3 mask)

usage: python tools/make_decode_vectors.py   (rewrites the fixture)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

OUT = os.path.join(ROOT, "tests", "golden", "decode_vectors.npz")


def cases():
    import util
    rng = np.random.default_rng(20261015)
    out = {}
    m = util.mask("FB_N128_K64")
    out["c1"] = ("FB_N128_K64", util.synth_frames(m, 1, ebn0_db=2.5, seed=0xF0)[0])
    m = util.mask("FB_N1024_K512")
    out["c2_snr"] = ("FB_N1024_K512", np.concatenate(
        [util.synth_frames(m, 64, ebn0_db=e, seed=100 + i)[0] for i, e in enumerate((0.0, 1.0, 2.5, 4.0))]))
    shape = (8, m.size)
    edge = [np.zeros(shape, int), rng.choice([-31, 31], shape), np.full(shape, -32),
            rng.integers(-1, 2, shape), rng.integers(-128, 128, shape)]
    out["c2_edge"] = ("FB_N1024_K512", np.concatenate(edge).astype(np.int8))
    m = util.mask("frozen_n_65536_k_32768")
    out["c3"] = ("frozen_n_65536_k_32768", util.synth_frames(m, 1, ebn0_db=1.0, seed=65536)[0])
    return out


def main():
    import util
    from oracle import oracle
    oracle.build()
    arrays = {}
    for key, (mask_name, llr) in cases().items():
        mask = util.mask(mask_name)
        x = oracle.decode_fsm(mask, llr)
        arrays[key + "__llr"] = llr.astype(np.int8)
        arrays[key + "__xhat"] = np.packbits(x.astype(np.uint8), axis=1, bitorder="little")
        arrays[key + "__mask"] = np.array(mask_name)
    np.savez_compressed(OUT, **arrays)
    print("wrote %s (%d bytes)" % (OUT, os.path.getsize(OUT)))


if __name__ == "__main__":
    main()
