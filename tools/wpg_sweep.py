#!/usr/bin/env python3
"""Interpreter launch-shape sweep (timing only): decode time vs batch and waves per group.

python tools/wpg_sweep.py [--mask M] [--batches 1024,2048,4096,8192] [--wpg 1,2,4,8,16]
Prints one JSON line per (batch, wpg) with the mean kernel time over --reps launches."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", default="frozen_n_65536_k_32768")
    ap.add_argument("--batches", default="1024,2048,4096,8192")
    ap.add_argument("--wpg", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    import util
    mask = util.mask(a.mask)
    dev = torch.device("cuda", 0)
    dec = pkg.Decoder(mask)
    for batch in [int(x) for x in a.batches.split(",")]:
        dec.prepare(batch)
        llr, _ = bench.gen_frames_torch(torch, mask, batch, 2.5, 1, dev)
        out = torch.empty((batch, dec.words), dtype=torch.int64, device=dev)
        ref = None
        for w in [int(x) for x in a.wpg.split(",")]:
            os.environ["POLAR_SC_WAVES_PER_GROUP"] = str(w)
            dec.decode(llr, out)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            same = bool(torch.equal(ref, out))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                dec.decode(llr, out)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"mask": a.mask, "batch": batch, "wpg": w, "ms": round(e0.elapsed_time(e1) / a.reps, 4),
                              "same_as_first": same}), flush=True)
        os.environ.pop("POLAR_SC_WAVES_PER_GROUP", None)


if __name__ == "__main__":
    main()
