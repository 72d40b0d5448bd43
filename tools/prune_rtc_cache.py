#!/usr/bin/env python3
"""Drop stale hipRTC code objects from lib/rtc_cache: run every prewarm of
__graft_entry__.build() (a cache hit marks its file as used), then delete the files no plan
loaded. Keeps the tree gpurun sends small."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__
    from sc_polar_decoder_hls_amd import _build
    cache = os.path.join(os.path.dirname(_build.LIB), "rtc_cache")
    t0 = time.time() - 1
    __graft_entry__.prewarm_all()
    gone = 0
    for f in os.listdir(cache):
        p = os.path.join(cache, f)
        if os.path.getmtime(p) < t0:
            os.remove(p)
            gone += 1
    print("pruned %d stale code objects; %d kept" % (gone, len(os.listdir(cache))))


if __name__ == "__main__":
    main()
