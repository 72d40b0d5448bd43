#!/usr/bin/env python3
"""Hybrid kernel vs schedule interpreter on the GPU: bit-exact comparison and timing.

python tools/hybrid_check.py [--masks a,b] [--batch B] [--reps R]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def timed(torch, dec, llr, out, reps):
    dec.decode(llr, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dec.decode(llr, out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--masks", default="FB_N2048_K1024,frozen_n_65536_k_32768")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    import util
    dev = torch.device("cuda", 0)
    for name in a.masks.split(","):
        mask = util.mask(name)
        os.environ["POLAR_SC_JIT"] = "0"
        ref = pkg.Decoder(mask)
        os.environ.pop("POLAR_SC_JIT")
        hyb = pkg.Decoder(mask)
        t = time.time()
        hyb.compile()
        tc = time.time() - t
        llr, _ = bench.gen_frames_torch(torch, mask, a.batch, 2.0, 1, dev)
        o_ref = torch.empty((a.batch, ref.words), dtype=torch.int64, device=dev)
        o_hyb = torch.empty_like(o_ref)
        t_ref = timed(torch, ref, llr, o_ref, a.reps)
        t_hyb = timed(torch, hyb, llr, o_hyb, a.reps)
        same = bool(torch.equal(o_ref, o_hyb))
        bad = int((o_ref != o_hyb).any(dim=1).sum().item())
        st = hyb.stats
        print(json.dumps({"mask": name, "batch": a.batch, "same": same, "frames_differ": bad,
                          "compile_s": round(tc, 2), "interp_ms": round(t_ref, 4), "hybrid_ms": round(t_hyb, 4),
                          "kernel": st["kernel"], "sub_kinds": st["n_sub_kinds"], "sub_calls": st["n_sub_calls"]}),
              flush=True)


if __name__ == "__main__":
    main()
