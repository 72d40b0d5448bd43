#!/usr/bin/env python3
"""Diagnostics of the pair kernel against the oracle on small cases: which frames / 16-LLR
words differ, for masks and tunings chosen to isolate one feature each (root F / G and the
output layout with all-information masks, noiseless codewords, small subtrees ...).
Prints one line per case."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import sc_polar_decoder_hls_amd as pkg
    import util
    from oracle import oracle
    oracle.build()
    t = pkg.selftest_lanes()
    lanes = np.arange(64)
    print("selftest permlane16", (t[4] == (lanes & ~16)).all(), (t[5] == (lanes | 16)).all(),
          "permlane32", (t[6] == (lanes & ~32)).all(), (t[7] == (lanes | 32)).all())
    print("p16a", t[4][::8].tolist(), "p16b", t[5][::8].tolist())
    print("p32a", t[6][::8].tolist(), "p32b", t[7][::8].tolist())
    rng = np.random.default_rng(1)
    cases = []
    N = 2048
    allinfo = np.ones(N, np.uint8)
    cases.append(("allinfo_noiseless_S64", allinfo, {"sub_words": 64}, "noiseless"))
    cases.append(("allinfo_noiseless_S32", allinfo, {"sub_words": 32}, "noiseless"))
    m = util.mask("frozen_n_2048_k_1024")
    cases.append(("n2048_noiseless_S64", m, {"sub_words": 64}, "noiseless"))
    cases.append(("n2048_awgn_S64", m, {"sub_words": 64}, "awgn"))
    cases.append(("n2048_awgn_S32", m, {"sub_words": 32}, "awgn"))
    half = np.zeros(N, np.uint8)
    half[N // 2:] = 1
    cases.append(("upperhalf_noiseless_S64", half, {"sub_words": 64}, "noiseless"))
    # one mixed 16-bit group pattern everywhere (leaves only below R1/R0 structure)
    cases.append(("n2048_noiseless_S64_W1", m, {"sub_words": 64, "waves_per_group": 1}, "noiseless"))
    cases.append(("n2048_noiseless_S64_W2", m, {"sub_words": 64, "waves_per_group": 2}, "noiseless"))
    cases.append(("n2048_noiseless_S32", m, {"sub_words": 32}, "noiseless"))
    cases.append(("n2048_noiseless_S32_W1", m, {"sub_words": 32, "waves_per_group": 1}, "noiseless"))
    rh = m.copy()
    rh[N // 2:] = 1
    cases.append(("n2048_left_rightR1_S64", rh, {"sub_words": 64}, "noiseless"))
    lh = m.copy()
    lh[:N // 2] = 0
    cases.append(("n2048_leftR0_right_S64", lh, {"sub_words": 64}, "noiseless"))
    for pat in (0xfee8, 0x8000, 0xfffe, 0xe880):
        mm = np.array([(pat >> k) & 1 for k in range(16)] * (N // 16), np.uint8)
        cases.append(("pat%04x_awgn_S64" % pat, mm, {"sub_words": 64}, "awgn"))
    for name, mask, tun, kind in cases:
        B = 4
        if kind == "noiseless":
            u = rng.integers(0, 2, size=(B, mask.size), dtype=np.uint8) & mask[None, :]
            x = util.encode_np(u)
            llr = np.where(x == 1, -9, 9).astype(np.int8)
        else:
            llr, _ = util.synth_frames(mask, B, ebn0_db=1.0, seed=7)
        dec = pkg.Decoder(mask, tuning=dict(tun, kernel=3))
        out = dec.decode(torch.from_numpy(llr).cuda())
        torch.cuda.synchronize()
        got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
        ref = oracle.decode_fsm(mask, llr)
        bad = (got != ref).any(axis=1)
        words = np.nonzero((got[0] != ref[0]).reshape(-1, 16).any(axis=1))[0]
        print("%-26s frames bad %d/%d  frame0 bad words %d: %s" % (name, int(bad.sum()), B, words.size,
                                                                  words[:24].tolist()), flush=True)
        if words.size:
            w = int(words[0])
            print("   word %d got %s ref %s" % (w, got[0, 16 * w:16 * w + 16].tolist(), ref[0, 16 * w:16 * w + 16].tolist()))


if __name__ == "__main__":
    main()
