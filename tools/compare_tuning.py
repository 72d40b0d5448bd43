#!/usr/bin/env python3
"""Decode one batch with two tunings of the same plan and compare the outputs bit for bit
(a tuning never changes results; a same-box check before an A/B is believed).

usage: python tools/compare_tuning.py --mask M --batch B --tuning k=v[,k=v] [--base k=v,..]
prints one JSON line: frames, differing frames."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(s):
    out = {"kernel": 3}
    for kv in filter(None, s.split(",")):
        k, v = kv.split("=")
        out[k] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--tuning", required=True)
    ap.add_argument("--base", default="")
    args = ap.parse_args()
    import torch
    import sc_polar_decoder_hls_amd as pkg
    from sc_polar_decoder_hls_amd import _plansets
    mask = _plansets.mask(args.mask)
    N, K = mask.size, int(mask.sum())
    llr, _ = pkg.csim_frames(N, args.batch, pkg.csim_sigma(1.5, K / N), seed=0xF1)
    outs = []
    for t in (parse(args.base), parse(args.tuning)):
        dec = pkg.Decoder(mask, tuning=t)
        outs.append(dec.decode(llr))
        torch.cuda.synchronize()
    diff = int((outs[0] != outs[1]).any(dim=1).sum())
    print(json.dumps({"mask": args.mask, "frames": args.batch, "base": args.base, "tuning": args.tuning,
                      "differing_frames": diff}), flush=True)
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main())
