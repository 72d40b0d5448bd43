#!/usr/bin/env python3
"""Build the library and prewarm the hipRTC cache for the C3 / C5 masks only (fast
iteration on the large-N kernels; __graft_entry__.build() prewarms everything)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import sc_polar_decoder_hls_amd as pkg  # noqa: E402
from sc_polar_decoder_hls_amd import _build  # noqa: E402
import util  # noqa: E402

pkg.build(verbose=False)
names = sys.argv[1:] or ["frozen_n_262144_k_131072", "frozen_n_65536_k_32768"]
_build.prewarm({n: util.mask(n) for n in names}, verbose=True)
