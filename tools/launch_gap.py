#!/usr/bin/env python3
"""Host wall time vs HIP-event time of back-to-back decode launches (timing diagnostic).

python tools/launch_gap.py [--mask M] [--batch B] [--steps 1,5,20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", default="frozen_n_65536_k_32768")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", default="1,5,20")
    ap.add_argument("--jit", default="1")
    a = ap.parse_args()
    os.environ["POLAR_SC_JIT"] = a.jit
    import torch
    import bench
    import sc_polar_decoder_hls_amd as pkg
    import util
    mask = util.mask(a.mask)
    dev = torch.device("cuda", 0)
    dec = pkg.Decoder(mask)
    dec.prepare(a.batch)
    llr, _ = bench.gen_frames_torch(torch, mask, a.batch, 2.5, 1, dev)
    out = torch.empty((a.batch, dec.words), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(3):
        dec.decode(llr, out, stream)
    torch.cuda.synchronize()
    for steps in [int(x) for x in a.steps.split(",")]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        host = []
        for _ in range(steps):
            h0 = time.perf_counter()
            dec.decode(llr, out, stream)
            host.append(time.perf_counter() - h0)
        e1.record(stream)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(json.dumps({"jit": a.jit, "steps": steps, "wall_ms_per_step": wall / steps * 1e3,
                          "event_ms_per_step": e0.elapsed_time(e1) / steps, "enqueue_ms_total": t_enq * 1e3,
                          "host_call_ms_max": max(host) * 1e3, "host_call_ms_mean": sum(host) / steps * 1e3}),
              flush=True)


if __name__ == "__main__":
    main()
