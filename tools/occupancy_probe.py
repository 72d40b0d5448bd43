#!/usr/bin/env python3
"""Kernel time vs batch size (HIP events around the decode launch): steps in the curve
show how many waves per SIMD are resident at once (8 frames per wave, 1024 SIMDs)."""
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
    ap.add_argument("--max-waves-per-simd", type=int, default=12)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    import util
    mask = util.mask(a.mask)
    dev = torch.device("cuda", 0)
    dec = pkg.Decoder(mask)
    simds = torch.cuda.get_device_properties(0).multi_processor_count * 4
    top = 8 * simds * a.max_waves_per_simd
    llr, _ = bench.gen_frames_torch(torch, mask, top, 2.5, 1, dev)
    out = torch.empty((top, dec.words), dtype=torch.int64, device=dev)
    rows = []
    for k in range(1, 4 * a.max_waves_per_simd + 1):
        wps = k / 4.0
        batch = int(8 * simds * wps)
        dec.decode(llr[:batch], out[:batch])
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            dec.decode(llr[:batch], out[:batch])
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        rows.append({"waves_per_simd": wps, "batch": batch, "ms": ms})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
