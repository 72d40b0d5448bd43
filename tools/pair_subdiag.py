#!/usr/bin/env python3
"""Every generated subtree decoder of a few pair plans on the GPU (polar_sc_debug_subtree)
against its CPU emulation (tests/pair_emu.py) on random root LLRs; prints mismatches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import sc_polar_decoder_hls_amd as pkg
    import util
    import pair_emu
    rng = np.random.default_rng(5)
    for name, sw in (("frozen_n_2048_k_1024", 64), ("frozen_n_2048_k_1024", 32)):
        dec = pkg.Decoder(util.mask(name), tuning={"kernel": 3, "sub_words": sw})
        subs = pair_emu.Sub(dec.kernel_source(), dec.stats["n_sub_kinds"])
        bad = 0
        for sid in range(dec.stats["n_sub_kinds"]):
            for t in range(3):
                rows = pair_emu.random_rows(rng, sw)
                got = dec.debug_subtree(sid, rows)
                ref = pair_emu.run_sub(dec, sid, rows, subs)
                if not (got == ref).all():
                    bad += 1
                    diff = got ^ ref
                    dw, ln = np.nonzero(diff)
                    print("%s S=%d sub %d try %d: %d lanes differ; dwords %s lanes %s bits %s" % (
                        name, sw, sid, t, len(ln), sorted(set(dw.tolist())), ln[:16].tolist(),
                        [hex(int(diff[a, b])) for a, b in zip(dw[:8], ln[:8])]), flush=True)
        print("%s S=%d: %d subs, %d mismatching runs" % (name, sw, dec.stats["n_sub_kinds"], bad), flush=True)


if __name__ == "__main__":
    main()
