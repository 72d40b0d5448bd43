#!/usr/bin/env python3
"""Decode speed of the reference's swept datapath formats: every
format of the GPU format matrix (_plansets.FORMATS: PAR 4..64, SIGMAG / CA2, EXTENDED 0 / 1,
LLR_BITS 6..9) and PRUNING_LEVEL 0 / 1 of the shipped format, on one mask and batch, HIP-event
timed on resident C-sim frames. Prints one JSON line per format with the kernel family that
ran (stats["kernel"]: 0 interpreter, 1 per-mask, 2 hybrid, 3 pair) and the time relative to the
shipped format (SIGMAG, PAR 16, EXTENDED, LLR_BITS 6, PRUNING_LEVEL 2). Parity of the same
formats is tests/test_gpu_formats.py / test_gpu_configs.py; nothing is checked here.

usage: python tools/format_speed.py [--mask frozen_n_16384_k_8192] [--frames 4096] [--steps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def formats():
    from sc_polar_decoder_hls_amd import _plansets
    out = [dict(par=16, sigmag=1, extended=1, llr_bits=6)]
    out += [dict(par=p, sigmag=s, extended=e, llr_bits=q) for p, s, e, q in _plansets.FORMATS]
    out += [dict(par=16, sigmag=1, extended=1, llr_bits=6, pruning_level=lvl) for lvl in (1, 0)]
    # PRUNING_LEVEL 1 with every leaf decoder (the format matrix's configuration): PAR 64 / 32
    # (PAR-word decoders) and CA2 at PAR 16 / 64 (round 6: on the pair kernel)
    pl1 = dict(zip(("pruning_level", "elag_r1", "elag_rep", "elag_spc", "elag_rep2", "elag_spc2", "elag_h0"),
                   (1, 1, 1, 1, 1, 1, 0)))
    out += [dict(pl1, par=p, sigmag=sg, extended=1, llr_bits=6) for p, sg in ((16, 1), (64, 1), (32, 1), (16, 0), (64, 0))]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mask", default="frozen_n_16384_k_8192")
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--formats", default="",
                    help="only these formats: 'par,sigmag,extended,llr_bits;...' (the shipped one is always first)")
    ap.add_argument("--pl1-only", action="store_true", help="only the PRUNING_LEVEL 1 entries (and the shipped one)")
    ap.add_argument("--kernel", type=int, default=0, help="polar_sc_tuning.kernel for the non-shipped formats "
                    "(1: the schedule interpreter, for before / after comparisons)")
    args = ap.parse_args()
    import torch
    import sc_polar_decoder_hls_amd as pkg
    from sc_polar_decoder_hls_amd import _plansets
    mask = _plansets.mask(args.mask)
    N, K = mask.size, int(mask.sum())
    llr8, _ = pkg.csim_frames(N, args.frames, pkg.csim_sigma(2.5, K / N), seed=0xF0)
    base_ms = None
    fmts = formats()
    if args.formats:
        keep = [tuple(int(x) for x in f.split(",")) for f in args.formats.split(";")]
        fmts = [fmts[0]] + [dict(par=p, sigmag=sg, extended=e, llr_bits=q) for p, sg, e, q in keep]
    if args.pl1_only:
        fmts = [fmts[0]] + [f for f in fmts if f.get("elag_rep2")]
    for fmt in fmts:
        cfg = pkg.default_config()
        for k, v in fmt.items():
            setattr(cfg, k, v)
        dec = pkg.Decoder(mask, cfg, tuning={"kernel": args.kernel} if args.kernel and fmt is not fmts[0] else None)
        # LLR_BITS 9 takes the int16 channel (polar_sc_decode_i16)
        llr = llr8.to(torch.int16) if fmt["llr_bits"] > 8 else llr8
        dec.prepare(args.frames)
        out = dec.decode(llr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            dec.decode(llr, out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        if base_ms is None:
            base_ms = ms
        st = dec.stats
        lay = dec.launch_info(args.frames).get("layout") if st["kernel"] == 3 else None
        print(json.dumps({"mask": args.mask, "frames": args.frames, "format": fmt, "kernel": st["kernel"], "layout": lay,
                          "ms": round(ms, 4), "info_bits_per_s": args.frames * K / (ms * 1e-3),
                          "vs_shipped": round(ms / base_ms, 3)}), flush=True)
        dec.close()


if __name__ == "__main__":
    main()
