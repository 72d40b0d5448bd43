#!/usr/bin/env python3
"""Same-box A/B of pair-plan variants (tuning dicts: layout, sub_words, ...) on the bench's
resident C-sim batches: interleaved rounds of HIP-event-timed decodes, every variant's output
compared frame for frame with the first variant's and, on a sample, with the oracle.

build (container):  python tools/layout_ab.py --prewarm [--configs ...] [--variants ...]
run (GPU box):      python tools/layout_ab.py [--steps 10] [--rounds 2] [--configs c3,c5,c5_64]
                        [--variants "layout=1;layout=2;layout=2,sub_words=512"]
prints one JSON line per config and round."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CONFIGS = {"c3": ("frozen_n_65536_k_32768", 4096), "c5": ("frozen_n_262144_k_131072", 512),
           "c5_64": ("frozen_n_262144_k_131072", 64), "c3_2048": ("frozen_n_65536_k_32768", 2048),
           "c3_1024": ("frozen_n_65536_k_32768", 1024), "c3_3072": ("frozen_n_65536_k_32768", 3072),
           "c5_1024": ("frozen_n_262144_k_131072", 1024), "c5_2048": ("frozen_n_262144_k_131072", 2048),
           "n16384_4096": ("frozen_n_16384_k_8192", 4096),
           "n16384_256": ("frozen_n_16384_k_8192", 256), "n65536_256": ("frozen_n_65536_k_32768", 256),
           # (bench.py's secondary entries: polar_sc_config fields as a third element)
           "q8_4096": ("frozen_n_16384_k_14746", 4096, {"llr_bits": 8}),
           "par64_4096": ("frozen_n_16384_k_8192", 4096, {"par": 64})}


def config_of(pkg, name):
    """the polar_sc_config of a CONFIGS entry (None: the reference's default)"""
    fields = CONFIGS[name][2] if len(CONFIGS[name]) > 2 else None
    if not fields:
        return None
    c = pkg.default_config()
    for k, v in fields.items():
        setattr(c, k, v)
    return c
DEFAULT_VARIANTS = "layout=1;layout=2;layout=2,sub_words=512"


def parse_variants(s):
    out = []
    for v in s.split(";"):
        t = {"kernel": 3}
        for kv in filter(None, v.split(",")):
            k, x = kv.split("=")
            t[k] = int(x)
        out.append(t)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--configs", default="c3,c5,c5_64")
    ap.add_argument("--variants", default=DEFAULT_VARIANTS)
    ap.add_argument("--check", type=int, default=4, help="frames checked against the oracle")
    ap.add_argument("--prewarm", action="store_true", help="compile the variants' code objects (host only)")
    args = ap.parse_args()
    import numpy as np
    import sc_polar_decoder_hls_amd as pkg
    import util
    variants = parse_variants(args.variants)
    if args.prewarm:
        for name in args.configs.split(","):
            mask = util.mask(CONFIGS[name][0])
            for t in variants:
                d = pkg.Decoder(mask, config=config_of(pkg, name), tuning=t)
                d.compile()
                print("prewarmed", name, t, flush=True)
        return
    import torch
    from oracle import oracle
    for name in args.configs.split(","):
        mname, batch = CONFIGS[name][:2]
        cfg = config_of(pkg, name)
        mask = util.mask(mname)
        N, K = mask.size, int(mask.sum())
        llr, _ = pkg.csim_frames(N, batch, pkg.csim_sigma(2.5, K / N), seed=0xF0)
        decs = []
        for t in variants:
            d = pkg.Decoder(mask, config=cfg, tuning=t)
            d.prepare(batch)
            out = d.decode(llr)
            torch.cuda.synchronize()
            decs.append((t, d, out))
        ref = decs[0][2].cpu()
        sample = llr[: args.check].cpu().numpy()
        want = oracle.decode_fsm(mask, sample, **(CONFIGS[name][2] if len(CONFIGS[name]) > 2 else {}))
        checks = []
        for t, d, out in decs:
            got = pkg.unpack_bits(out[: args.check].cpu().numpy(), N)
            checks.append({"equal_to_first": bool(torch.equal(out.cpu(), ref)),
                           "oracle_frames_bad": int((got != want).any(axis=1).sum()),
                           "launch": d.launch_info(batch)})
        for r in range(args.rounds):
            res = {"config": name, "mask": mname, "frames": batch, "round": r, "variants": []}
            for (t, d, out), chk in zip(decs, checks):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                d.decode(llr, out)
                e0.record()
                for _ in range(args.steps):
                    d.decode(llr, out)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.steps
                res["variants"].append(dict(tuning=t, ms=round(ms, 4), info_bits_per_s=batch * K / (ms * 1e-3), **chk))
            print(json.dumps(res), flush=True)
        for _, d, _ in decs:
            d.close()


if __name__ == "__main__":
    main()
