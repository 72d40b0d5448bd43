#!/usr/bin/env python3
"""Dump the per-op monitor records (Decoder.trace) of a mask at a batch to JSON, for the
per-op latency analysis of the large-N kernels. GPU box.

usage: tools/op_latency_probe.py <mask> --batch B --out file.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mask")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    import util
    mask = util.mask(a.mask)
    dec = pkg.Decoder(mask)
    llr, _ = bench.gen_frames_torch(torch, mask, a.batch, 2.5, 0xF0, torch.device("cuda", 0))
    dec.trace(llr)
    rows, info = dec.trace(llr)
    info.pop("out", None)
    with open(a.out, "w") as f:
        json.dump(dict(mask=a.mask, batch=a.batch, stats={k: v for k, v in dec.stats.items() if isinstance(v, (int, float))},
                       info=info, rows=rows), f)
    print(a.mask, a.batch, info)


if __name__ == "__main__":
    main()
