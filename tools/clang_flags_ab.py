#!/usr/bin/env python3
"""Same-box A/B of clang driver flags for the generated kernels (POLAR_SC_CLANG_FLAGS, part of
the code-object cache key): C2 / C3 / C5 / C5-share decoded by the default plans, HIP-event
timed, one child process per variant and round (the parent never touches the GPU), outputs
hashed so a variant that changes the bits shows up.

usage: python tools/clang_flags_ab.py --prewarm          (here: compile every variant, host only)
       python tools/clang_flags_ab.py [--rounds 2]       (GPU box: time every variant)
prints one JSON line per variant and round."""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

VARIANTS = {
    "base": "",
    "max_ilp": "-mllvm --amdgpu-sched-strategy=max-ilp",
    "bias0": "-mllvm --amdgpu-schedule-metric-bias=0",
    "no_cluster_resched": "-mllvm --amdgpu-disable-clustered-low-occupancy-reschedule "
                          "-mllvm --amdgpu-disable-unclustered-high-rp-reschedule",
}
CONFIGS = {"c2": ("FB_N1024_K512", 65536), "c3": ("frozen_n_65536_k_32768", 4096),
           "c5": ("frozen_n_262144_k_131072", 512), "c5_64": ("frozen_n_262144_k_131072", 64)}


def prewarm(names, configs):
    import sc_polar_decoder_hls_amd as pkg
    import util
    for v in names:
        os.environ["POLAR_SC_CLANG_FLAGS"] = VARIANTS[v]
        for c in sorted({"c5" if c == "c5_64" else c for c in configs}):
            dec = pkg.Decoder(util.mask(CONFIGS[c][0]))
            ok = dec.compile()
            print(v, c, ok, dec.launch_info(CONFIGS[c][1])["code_key"], flush=True)
            dec.close()


def child(steps, configs):
    import torch
    import sc_polar_decoder_hls_amd as pkg
    import util
    res = {"flags": os.environ.get("POLAR_SC_CLANG_FLAGS", "")}
    for name in configs:
        mname, batch = CONFIGS[name]
        mask = util.mask(mname)
        N, K = mask.size, int(mask.sum())
        llr, _ = pkg.csim_frames(N, batch, pkg.csim_sigma(2.5, K / N), seed=0xF0)
        dec = pkg.Decoder(mask)
        dec.prepare(batch)
        out = dec.decode(llr)
        for _ in range(3):
            dec.decode(llr, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            dec.decode(llr, out)
        e1.record()
        torch.cuda.synchronize()
        res[name] = {"ms": e0.elapsed_time(e1) / steps, "code_key": dec.launch_info(batch)["code_key"],
                     "out_sha1": hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12],
                     "kernel": dec.stats["kernel"]}
        dec.close()
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prewarm", action="store_true")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--configs", default="c2,c3,c5,c5_64")
    args = ap.parse_args()
    if args.prewarm:
        return prewarm(args.variants.split(","), args.configs.split(","))
    if args.child:
        return child(args.steps, args.configs.split(","))
    for r in range(args.rounds):
        for v in args.variants.split(","):
            env = dict(os.environ, POLAR_SC_CLANG_FLAGS=VARIANTS[v])
            p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", "--steps",
                                str(args.steps), "--configs", args.configs], env=env, capture_output=True,
                               text=True, timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("{")]
            if p.returncode != 0 or not line:
                print(json.dumps({"variant": v, "round": r, "rc": p.returncode, "err": p.stderr[-2000:]}), flush=True)
                return p.returncode or 1
            d = json.loads(line[0])
            d.update(variant=v, round=r)
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    sys.exit(main())
