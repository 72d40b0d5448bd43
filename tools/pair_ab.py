#!/usr/bin/env python3
"""Same-box A/B of the large-N decode kernels: the hybrid kernel (8-frame groups, tuning
kernel 2) against the pair kernel (frame pairs, tuning kernel 3) on the bench's resident
C-sim batches, HIP-event timed, outputs compared frame for frame.

usage: python tools/pair_ab.py [--steps 10] [--configs c3,c5,c5_64] [--tuning key=val,...]
prints one JSON line per config."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CONFIGS = {"c3": ("frozen_n_65536_k_32768", 4096), "c5": ("frozen_n_262144_k_131072", 512),
           "c5_64": ("frozen_n_262144_k_131072", 64), "n524288_32": ("frozen_n_524288_k_262144", 32),
           "n16384_4096": ("frozen_n_16384_k_8192", 4096), "n4096_16384": ("frozen_n_4096_k_2048", 16384)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--configs", default="c3,c5,c5_64")
    ap.add_argument("--tuning", default="", help="extra pair tuning, e.g. waves_per_group=4,tier_words=1024")
    ap.add_argument("--kernels", default="2,3")
    args = ap.parse_args()
    import torch
    import sc_polar_decoder_hls_amd as pkg
    import util
    extra = {}
    for kv in filter(None, args.tuning.split(",")):
        k, v = kv.split("=")
        extra[k] = int(v)
    for name in args.configs.split(","):
        mname, batch = CONFIGS[name]
        mask = util.mask(mname)
        N, K = mask.size, int(mask.sum())
        llr, _ = pkg.csim_frames(N, batch, pkg.csim_sigma(2.5, K / N), seed=0xF0)
        res = {"config": name, "mask": mname, "frames": batch}
        outs = {}
        for kern in [int(k) for k in args.kernels.split(",")]:
            tun = dict(extra, kernel=kern) if kern == 3 else {"kernel": kern}
            dec = pkg.Decoder(mask, tuning=tun)
            dec.prepare(batch)
            out = dec.decode(llr)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                dec.decode(llr, out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            outs[kern] = out.cpu()
            res["k%d_ms" % kern] = ms
            res["k%d_info_bits_per_s" % kern] = batch * K / (ms * 1e-3)
            res["k%d_stats" % kern] = {k: dec.stats[k] for k in ("kernel", "sub_words", "n_sub_kinds", "tier_steps")}
            dec.close()
        if len(outs) == 2:
            a, b = list(outs.values())
            res["equal"] = bool(torch.equal(a, b))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
