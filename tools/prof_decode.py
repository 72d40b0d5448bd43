#!/usr/bin/env python3
"""Decode-only driver for rocprofv3 runs: generates frames once, then launches the decode
kernel `--reps` times (no other kernels in the loop)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", default="FB_N1024_K512")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ebn0", type=float, default=2.5)
    ap.add_argument("--rotate", type=int, default=0,
                    help="distinct input batches cycled through (0: as bench.py, >= 300 MB in total)")
    ap.add_argument("--tuning", default="", help="polar_sc_tuning fields, e.g. kernel=3,tier_words=2048")
    ap.add_argument("--config", default="", help="polar_sc_config fields other than the shipped, e.g. par=64")
    a = ap.parse_args()
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    import util
    mask = util.mask(a.mask)
    dev = torch.device("cuda", 0)
    tun = {k: int(v) for k, v in (kv.split("=") for kv in filter(None, a.tuning.split(",")))}
    fmt = {k: int(v) for k, v in (kv.split("=") for kv in filter(None, a.config.split(",")))}
    cfg = None
    if fmt:
        cfg = pkg.default_config()
        for k, v in fmt.items():
            setattr(cfg, k, v)
    dec = pkg.Decoder(mask, config=cfg, tuning=tun or None)
    dec.prepare(a.batch)
    # the launch shape and code object being profiled (tools/pmc_summary.py copies it into the
    # summary; bench.py uses a profile's traffic only for the code object it times)
    print("launch_info " + json.dumps(dict(dec.launch_info(a.batch), mask=a.mask, batch=a.batch, tuning=tun,
                                           config=fmt)), flush=True)
    nb = a.rotate if a.rotate > 0 else max(1, min(8, -(-bench.ROTATE_BYTES // (a.batch * mask.size))))
    llrs = [bench.widen_q9(torch, bench.gen_frames_torch(torch, mask, a.batch, a.ebn0, 0xF0 + b, dev)[0], fmt)
            for b in range(nb)]
    out = torch.empty((a.batch, dec.words), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for i in range(a.reps):
        dec.decode(llrs[i % nb], out)
    torch.cuda.synchronize()
    print("decoded %d x %d frames (N=%d)" % (a.reps, a.batch, mask.size))


if __name__ == "__main__":
    main()
