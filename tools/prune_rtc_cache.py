#!/usr/bin/env python3
"""Drop stale code objects from lib/rtc_cache: run every prewarm of __graft_entry__.build()
(a cache hit marks its file as used), then delete the files no plan loaded. Keeps the tree
gpurun sends small. --compress first rewrites <key>.co / <key>.coz entries as <key>.cox (xz,
polar_sc_jit.cpp cache_store), which the library loads the same way; --compress-only stops
there (no prewarm)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def to_xz(p):
    import lzma
    import struct
    import zlib
    data = open(p, "rb").read()
    if data[:4] == b"PSCZ":
        n, = struct.unpack_from("<Q", data, 4)
        data = zlib.decompress(data[12:])
        assert len(data) == n, p
    base = p[:-1] if p.endswith(".coz") else p
    out = base + "x"
    with open(out + ".tmp", "wb") as o:
        o.write(b"PSCX" + struct.pack("<Q", len(data)) + lzma.compress(data, preset=6))
    os.replace(out + ".tmp", out)
    st = os.stat(p)
    os.utime(out, (st.st_atime, st.st_mtime))   # (keeps the entry's age for pruning)
    os.remove(p)
    return out


def main():
    from sc_polar_decoder_hls_amd import _build
    cache = os.path.join(os.path.dirname(_build.LIB), "rtc_cache")
    if "--compress" in sys.argv or "--compress-only" in sys.argv:
        from concurrent.futures import ProcessPoolExecutor
        todo = [os.path.join(cache, f) for f in os.listdir(cache) if f.endswith(".co") or f.endswith(".coz")]
        with ProcessPoolExecutor(int(os.environ.get("POLAR_SC_PREWARM_PROCS", "6"))) as ex:
            list(ex.map(to_xz, todo, chunksize=4))
        print("compressed %d entries" % len(todo))
        if "--compress-only" in sys.argv:
            return
    import __graft_entry__
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
