#!/usr/bin/env python3
"""Drop stale code objects from lib/rtc_cache: run every prewarm of __graft_entry__.build()
(a cache hit marks its file as used), then delete the files no plan loaded. Keeps the tree
gpurun sends small. --compress first rewrites plain <key>.co entries as <key>.coz (zlib,
polar_sc_jit.cpp cache_store), which the library loads the same way."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__
    from sc_polar_decoder_hls_amd import _build
    cache = os.path.join(os.path.dirname(_build.LIB), "rtc_cache")
    if "--compress" in sys.argv:
        import struct
        import zlib
        for f in os.listdir(cache):
            if f.endswith(".co"):
                p = os.path.join(cache, f)
                data = open(p, "rb").read()
                with open(p + "z.tmp", "wb") as o:
                    o.write(b"PSCZ" + struct.pack("<Q", len(data)) + zlib.compress(data, 6))
                os.replace(p + "z.tmp", p + "z")
                os.remove(p)
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
