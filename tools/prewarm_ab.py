#!/usr/bin/env python3
"""hipRTC code objects of the C3 / C5 pair plans with the chain fusion off (tuning chain_max =
1), for same-box A/Bs (tools/pair_ab.py --tuning chain_max=1). Host only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

if __name__ == "__main__":
    import util
    from sc_polar_decoder_hls_amd import _build
    _build.prewarm_plans([(n, util.mask(n), {"kernel": 3, "chain_max": 1})
                          for n in ("frozen_n_65536_k_32768", "frozen_n_262144_k_131072")], verbose=True)
    # subtree size at C5 (N = 262144): 64 and 128 words against the automatic 256
    _build.prewarm_plans([("frozen_n_262144_k_131072", util.mask("frozen_n_262144_k_131072"), {"kernel": 3, "sub_words": s})
                          for s in (64, 128)], verbose=True)
