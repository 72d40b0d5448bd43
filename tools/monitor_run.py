#!/usr/bin/env python3
"""Run the per-op monitor (Decoder.trace) on a committed mask and print the report + the
ten most expensive op kinds by (function, node size). GPU box.

usage: tools/monitor_run.py <mask name in data/frozen_masks.json> [--batch B] [--ebn0 dB]
"""
import argparse
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mask")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ebn0", type=float, default=2.5)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    from sc_polar_decoder_hls_amd import monitor
    import util
    mask = util.mask(a.mask)
    dec = pkg.Decoder(mask)
    llr, _ = bench.gen_frames_torch(torch, mask, a.batch, a.ebn0, 0xF0, torch.device("cuda", 0))
    dec.trace(llr)                       # warm-up (module load, schedule upload)
    rows, info = dec.trace(llr)
    rep = monitor.report(rows, info)
    print("mask %s N=%d batch %d kernel %d" % (a.mask, mask.size, a.batch, dec.stats["kernel"]))
    print(monitor.format_report(rep))
    agg = defaultdict(lambda: [0, 0])
    for r in rows:
        k = (r["op"], r["nodeN"])
        agg[k][0] += r["cycles"]
        agg[k][1] += 1
    print("\ntop op kinds (op, node LLRs): cycles, count, share")
    for (op, nn), (c, k) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:14]:
        print("  %-6s %7d : %10d  %6d  %5.1f%%" % (op, nn, c, k, 100.0 * c / max(1, info["total_cycles"])))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(mask=a.mask, batch=a.batch, kernel=dec.stats["kernel"], report=rep), f)


if __name__ == "__main__":
    main()
