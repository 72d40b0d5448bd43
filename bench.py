#!/usr/bin/env python3
"""Benchmark: decoded information bits/s of the MI355X SC polar decoder.

Workload (BASELINE.json configs[1], "C2"): N=1024, K=512 (Frozen_Bit_Tab/FB_N1024_K512.txt),
65536 AWGN frames per GPU (Eb/N0 = 2.5 dB, seed 0xF0 as in src/testbench/main.cpp:86-104),
int8 LLRs already resident in HBM. One step = one decode of the whole per-GPU batch.

Multi-GPU (torchrun, one process per GPU, RCCL): every rank generates and decodes its own
shard of frames (weak scaling, no data-path collective); timing is max over ranks.

Prints ONE JSON line (rank 0). Extra fields:
  roofline     -- HBM roofline of the decode kernel: algorithmic bytes per launch
                  (1.125 N bytes per frame: N int8 LLRs in + N/8 bytes of x^ out) / mean
                  kernel duration (HIP events on the launch stream)
  cpu_baseline -- the CPU oracle (literal C restatement of my_module::do_action, one thread)
                  timed on a bounded sample on this host, rank 0 / N=1 only
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# PMC summaries (tools/profile_gpu.sh + tools/pmc_summary.py) of the current kernels: the HBM
# bytes they report (FETCH_SIZE x2 on gfx950 + WRITE_SIZE, separate passes) fill
# roofline.traffic when the benchmarked (mask, frames per GPU) is the profiled one.
PROFILE_DIR = os.path.join(ROOT, "profiles")


def find_traffic_profile(mask_name, per_gpu, key):
    """The committed PMC summary (profiles/<round>_<tag>_pmc.json, tools/pmc_summary.py) of this
    workload and machine code: same mask and batch in its launch_info and the same code_key
    (the hash of the kernels' instructions and descriptors, polar_sc_plan_launch_info); the
    newest round's when several match. (None, None) if there is none; (None, path) if profiles
    of the workload exist only for other machine code."""
    import glob
    other = None
    for path in sorted(glob.glob(os.path.join(PROFILE_DIR, "r*_pmc.json")), reverse=True):
        try:
            with open(path) as f:
                prof = json.load(f)
        except (OSError, ValueError):
            continue
        info = prof.get("launch_info") or {}
        if info.get("mask") != mask_name or info.get("batch") != per_gpu:
            continue
        if prof.get("code_key") == key:
            return prof, path
        other = other or path
    return None, other


# Rotated input: the timed loop cycles through distinct resident batches of at least this
# many bytes in total, so the LLR reads come from HBM and not from the 256 MB Infinity Cache
# (MI355X_MICROARCH.md) that would hold one C2 batch (67 MB).
ROTATE_BYTES = 300 << 20
EBN0_SWEEP = (1.0, 2.5, 4.0)   # throughput depends weakly on the SNR
# VALU issue cost on gfx950, timed in-kernel with the shader clock (s_memtime) by
# tools/valu_microbench.hip (profiles/r02_valu_microbench.log): SIMD cycles per wave64
# instruction of the packed-16 / DPP / v_perm classes the decoder issues, by waves per SIMD
# (independent chains). 8 waves: 2.62 (32-bit ALU 1.45); 4: 3.25; 2: 4.45; 1: 5.20. The
# roofline peak is the full-occupancy figure; the per-mask kernel runs at 4 waves per SIMD
# (123 VGPRs with the packed root and the LDS-DMA channel fetch, 33 KB of LDS per 4-wave block).
VALU_CYCLES_PER_INST = 2.62
VALU_CYCLES_BY_WAVES = {1: 5.20, 2: 4.45, 4: 3.25, 8: 2.62}
NOMINAL_CLOCK_GHZ = 2.4   # fallback when the PMC profile has no measured clock

CONFIGS = {
    # name: (mask fixture, per-GPU frames at N=1 semantics, description)
    "c1": ("FB_N128_K64", 1, "N=128 K=64 single frame (plumbing)"),
    "c2": ("FB_N1024_K512", 65536, "N=1024 K=512, 65536-frame batch per GPU"),
    "c3": ("frozen_n_65536_k_32768", 4096, "N=65536 K=32768, 4096-frame batch per GPU"),
    "c4": ("FB_N1024_K512", None, "N=1024 K=512, 2^20 frames sharded over the GPUs"),
    "c5": ("frozen_n_262144_k_131072", None, "N=262144 K=131072, 512 frames sharded over the GPUs"),
}


# kernel that carries the decode for each plan storage class (polar_sc_plan_stats.storage)
def kernel_name(stats, info=None):
    """The kernel that carries the decode of a plan (polar_sc_plan_stats.kernel / .storage;
    info: polar_sc_plan_launch_info of the timed batch -- the layout an automatic pair plan
    takes for it)."""
    if stats["kernel"] == 1:
        return "polar_sc_mask_kernel (per-mask generated kernel)"
    if stats["kernel"] == 3 and info and info.get("layout") == 2:
        return ("polar_sc_pair_kernel, solo layout (generated: one frame per wave, eight words per register, "
                "%d-LLR subtree decoders, upper levels over stage-slot rows; %d waves per frame)"
                % (16 * info["sub_words"], info["waves_per_block"]))
    if stats["kernel"] == 3:
        k = ("polar_sc_pair_kernel (generated: one frame pair per wave, %d generated %d-LLR subtree decoders, "
             "upper levels over stage-slot rows)" % (stats["n_sub_kinds"], 16 * stats["sub_words"]))
        if stats.get("tier_steps"):
            k += " + grid tier (%d launches per decode)" % stats["tier_steps"]
        return k
    store = "HBM-scratch" if stats["storage"] == 1 else "LDS"
    if stats["kernel"] == 2:
        k = ("polar_sc_hybrid_kernel (generated: %s interpreter + %d generated %d-LLR subtree decoders)"
             % (store, stats["n_sub_kinds"], 16 * stats["sub_words"]))
        if stats.get("tier_steps"):
            k = ("grid tier: polar_sc_tier_kernel (upper-level F / G over all frame groups) + segments of "
                 + k + "; %d launches per decode at the deep cut (F / G >= %d words), the root-only cut when "
                 "the batch has a frame group per CU" % (stats["tier_steps"], stats["tier_words"]))
        return k
    return "polar_sc_decode_kernel<%s> (%s interpreter)" % ("true" if stats["storage"] == 1 else "false", store)


def gen_frames_torch(torch, mask, batch, ebn0_db, seed, device):
    """Synthetic AWGN frames on the GPU (reference C-sim chain semantics)."""
    N = mask.size
    K = int(mask.sum())
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    m = torch.from_numpy(mask.astype(np.uint8)).to(device)
    u = torch.randint(0, 2, (batch, N), generator=g, device=device, dtype=torch.uint8) & m
    x = u.clone()
    h = 1
    while h < N:
        v = x.view(batch, N // (2 * h), 2, h)
        v[:, :, 0, :] ^= v[:, :, 1, :]
        h *= 2
    sigma = 1.0 / np.sqrt(2.0 * (K / N) * 10.0 ** (ebn0_db / 10.0))
    y = (1.0 - 2.0 * x.float()) + sigma * torch.randn((batch, N), generator=g, device=device)
    llr = torch.clamp(torch.trunc(4.0 * y), -31, 31).to(torch.int8).contiguous()
    return llr, x


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(mask, seconds, ebn0_db, llr, threads=None, runs=5):
    """Time the CPU oracle (literal FSM restatement) on a bounded sample of the workload
    (runs of >= 1 s, median of 5, the same LLR buffers as the GPU run):
    `llr` is the head of the first resident batch the GPU decoded, copied to the host. One
    thread, then `threads` threads over disjoint frame chunks (the ctypes call releases the
    GIL). Returns the multi-thread median with the single-thread one beside it."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle
    oracle.build()
    N, K = mask.size, int(mask.sum())
    if threads is None:
        # the GPU box grants 16 CPUs per GPU (os.cpu_count() shows the whole machine)
        threads = max(1, min(16, os.cpu_count() or 1))
    sample = llr.shape[0]
    oracle.decode_fsm(mask, llr[:2])   # warm
    per_run = max(1.0, seconds / (2 * runs))

    def timed(fn, budget):
        frames, t0 = 0, time.perf_counter()
        while True:
            frames += fn()
            el = time.perf_counter() - t0
            if el >= budget:
                return frames / el

    fps1 = [timed(lambda: (oracle.decode_fsm(mask, llr), sample)[1], per_run) for _ in range(runs)]
    chunks = np.array_split(llr, threads)
    with ThreadPoolExecutor(threads) as ex:
        def all_threads():
            list(ex.map(lambda c: oracle.decode_fsm(mask, c), chunks))
            return sample
        fpsn = [timed(all_threads, per_run) for _ in range(runs)]
    med1, medn = float(np.median(fps1)), float(np.median(fpsn))
    return {"value": medn * K, "unit": "info_bits/s", "frames_per_sec": medn, "cores": threads,
            "kind": "port", "value_1thread": med1 * K, "runs": runs, "run_seconds": per_run,
            "values_nthreads": [v * K for v in fpsn], "values_1thread": [v * K for v in fps1],
            "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": "the first %d frames of the GPU run's first resident batch (N=%d K=%d, Eb/N0=%.1f dB, "
                      "copied to the host) decoded repeatedly by oracle/polar_oracle.c orc_decode_fsm (literal "
                      "my_module FSM): median of %d runs of %.1f s on 1 thread, then on %d threads (frame chunks)"
                      % (sample, N, K, ebn0_db, runs, per_run, threads)}


def make_batches(pkg, torch, args, mask, per_gpu, frame0, stride, dev, ebn0, nb):
    """nb distinct resident batches of per_gpu frames (batch b: frames frame0 + b * stride ...
    of the testbench's frame stream, stride = frames of all ranks; or torch AWGN):
    [(llr, xref or None, x or None)]"""
    N, K = mask.size, int(mask.sum())
    out = []
    for b in range(nb):
        if args.data == "csim":
            kat_key = {8: "cw8x4", 512: "cw512x256", 1024: "cw1024x512"}.get(N)
            import util
            cws = np.array(util.kat()[kat_key], dtype=np.uint8) if kat_key else None
            llr, xref = pkg.csim_frames(N, per_gpu, pkg.csim_sigma(ebn0, K / N), seed=0xF0,
                                        frame0=frame0 + b * stride, codewords=cws, device=dev)
            out.append((llr, xref, None))
        else:
            from sc_polar_decoder_hls_amd import sharding
            rank = int(os.environ.get("RANK", "0"))
            llr, x = gen_frames_torch(torch, mask, per_gpu, ebn0, sharding.frame_seed(0xF0 + 104729 * b, rank), dev)
            out.append((llr, None, x))
    return out


def timed_decodes(torch, sharding, dist, coll_dev, dec, batches, outs, steps, warmup, stream, settle_s=0.0):
    """Warm-up, then `steps` back-to-back decode launches on one stream cycling through the
    resident batches, bracketed by a barrier + synchronize and by one HIP event pair on the
    launch stream (per-step event records would add ~5 us of stream markers to every step).
    settle_s: before the warm-up, untimed decodes for this long, so that the timed steps see
    the GPU clock of a continuous stream of batches and not its ramp out of idle.
    Returns (wall seconds, mean ms per launch from the events), both max over ranks."""
    nb = len(batches)
    t_end = time.perf_counter() + settle_s
    i = 0
    while time.perf_counter() < t_end:
        for _ in range(8):
            dec.decode(batches[i % nb][0], outs[i % nb], stream)
            i += 1
        torch.cuda.synchronize()
    for i in range(warmup):
        dec.decode(batches[i % nb][0], outs[i % nb], stream)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(steps):
        dec.decode(batches[i % nb][0], outs[i % nb], stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    return sharding.max_over_ranks([elapsed, kern_ms], dist, coll_dev)


def pipelined_decodes(torch, sharding, dist, coll_dev, dec, batches, steps, dev, nstreams=2):
    """The same `steps` decodes with consecutive batches on `nstreams` HIP streams (each with
    its own output buffers): a serving loop keeps two batches in flight, so one launch's tail
    overlaps the next one's start. Per-mask plans hold no shared scratch (polar_sc.h: storage
    2 plans may overlap on streams). Informative; `value` stays the one-stream loop.
    Returns wall seconds (max over ranks)."""
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    nb = len(batches)
    outs = [torch.empty((batches[0][0].shape[0], dec.words), dtype=torch.int64, device=dev)
            for _ in range(nstreams * nb)]
    torch.cuda.synchronize()
    for i in range(2 * nstreams):
        dec.decode(batches[i % nb][0], outs[i % len(outs)], streams[i % nstreams])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        dec.decode(batches[i % nb][0], outs[i % len(outs)], streams[i % nstreams])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return sharding.max_over_ranks([elapsed], dist, coll_dev)[0]


# Secondary entries of the same JSON line (BASELINE.json configs[2] and [4], and the formats of
# the reference's own sweep script): timed in the same process after the headline C2 region,
# each with its own roofline and a 4-frame oracle check.
# name: (mask, frames per GPU or None = the 512-frame C5 batch sharded over the ranks, datapath
# fields of polar_sc_config that differ from the shipped one, note)
SWEEP_FRAMES = 4096
SECONDARY = (
    ("c3", "frozen_n_65536_k_32768", 4096, {}, "BASELINE configs[2]: N=65536 K=32768, 4096-frame batch per GPU"),
    ("c5", "frozen_n_262144_k_131072", None, {}, "BASELINE configs[4]: N=262144 K=131072, 512 frames sharded over the GPUs"),
    ("c5_share64", "frozen_n_262144_k_131072", 64, {},
     "C5's 8-GPU share (64 frames) on one GPU: the per-GPU latency of configs[4] at 8 GPUs"),
    ("c4_share", "FB_N1024_K512", 131072, {},
     "C4's 8-GPU share (2^20 / 8 = 131072 frames of N=1024 K=512) on one GPU: the per-GPU work of configs[3] at 8 GPUs"),
    # script/script_tests.sh:11,124 runs PAR 16 and PAR 64; :7-9 the rate-0.9 codes at QUANT 8
    ("par16_n16384", "frozen_n_16384_k_8192", SWEEP_FRAMES, {},
     "PAR 16 (the shipped datapath) on N=16384 K=8192, %d frames per GPU: the PAR 64 entry's baseline" % SWEEP_FRAMES),
    ("par64_n16384", "frozen_n_16384_k_8192", SWEEP_FRAMES, {"par": 64},
     "PAR 64 (script_tests.sh:11,124) on N=16384 K=8192, %d frames per GPU" % SWEEP_FRAMES),
    ("q8_n16384_k14746", "frozen_n_16384_k_14746", SWEEP_FRAMES, {"llr_bits": 8},
     "QUANT 8 (LLR_BITS 8) on the rate-0.9 code N=16384 K=14746 of script_tests.sh:7-9, %d frames per GPU"
     % SWEEP_FRAMES),
    # parser_comp.sh:12 sweeps LLR_BITS up to 9: the int16 channel (the C-sim LLRs x 8)
    ("q9_n16384", "frozen_n_16384_k_8192", SWEEP_FRAMES, {"llr_bits": 9},
     "LLR_BITS 9 (parser_comp.sh:12; int16 channel, C-sim LLRs x 8) on N=16384 K=8192, %d frames per GPU"
     % SWEEP_FRAMES),
)


def widen_q9(torch, llr, fmt):
    """LLR_BITS 9 frames: the C-sim int8 LLRs (6-bit range) as int16 scaled into the 9-bit range"""
    return llr.to(torch.int16) * 8 if fmt and fmt.get("llr_bits", 6) > 8 else llr


def channel_bytes(fmt):
    """input bytes per LLR: int8, or int16 for 9-bit LLRs (polar_sc_decode_i16)"""
    return 2 if fmt and fmt.get("llr_bits", 6) > 8 else 1


def roofline_entry(name, N, per_gpu, kern_ms, dec, fmt=None):
    """HBM roofline of one decode launch sequence: algorithmic bytes (1.125 N per frame) over
    the event-timed kernel time; traffic from the committed PMC summary of the same workload,
    used only when that profile is of the machine code timed here (its code_key -- the hash of
    the kernels' instructions and descriptors, polar_sc_plan_launch_info -- equals this plan's)."""
    bytes_per_launch = (channel_bytes(fmt) + 0.125) * N * per_gpu   # (1.125 N per frame; int16 channel 2.125 N)
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src, note = None, None, None
    info = dec.launch_info(per_gpu)
    key = info["code_key"]
    prof, prof_path = find_traffic_profile(name, per_gpu, key)
    if prof is None:
        note = ("profile %s is of other machine code than this run's %s: traffic not reported"
                % (os.path.relpath(prof_path, ROOT), key) if prof_path else
                "no committed PMC profile of this workload's code object %s" % key)
    elif "hbm_read_bytes_corrected" in prof and "hbm_write_bytes" in prof:
        traffic = prof["hbm_read_bytes_corrected"] + prof["hbm_write_bytes"]
        traffic_src = os.path.relpath(prof_path, ROOT)
    ent = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
           "traffic_source": traffic_src, "kernel_ms": kern_ms, "code_key": key,
           # which compiler built the timed kernel: the ROCm clang driver (prewarmed code
           # objects) or hipRTC (a cache miss on this machine)
           "compiler": {1: "ROCm clang driver", 2: "hipRTC"}.get(info.get("compiler"), None),
           "algorithmic_bytes_per_launch": bytes_per_launch}
    if note:
        ent["traffic_note"] = note
    return ent, prof


def secondary_entry(torch, pkg, sharding, dist, coll_dev, args, key, mask_name, per_gpu, fmt, note, rank, world,
                    dev, stream):
    """One secondary configuration: resident rotated C-sim batches, a short timed loop (same
    barrier / synchronize / max-over-ranks bracket as the headline), roofline, and a 4-frame
    bit-exact check against the oracle on rank 0. fmt: polar_sc_config fields that differ from
    the shipped datapath (par, llr_bits)."""
    import util
    mask = util.mask(mask_name)
    N, K = mask.size, int(mask.sum())
    cfg = None
    if fmt:
        cfg = pkg.default_config()
        for f, v in fmt.items():
            setattr(cfg, f, v)
    if per_gpu is None:
        per_gpu = sharding.shard_bounds(512, world, rank)[1]
    counts = [per_gpu]
    if dist is not None:
        t = torch.zeros(world, dtype=torch.float64, device=coll_dev)
        t[rank] = per_gpu
        dist.all_reduce(t)
        counts = [int(v) for v in t.tolist()]
    frame0 = int(sum(counts[:rank]))
    dec = pkg.Decoder(mask, config=cfg)
    dec.prepare(per_gpu)
    nb = max(1, min(8, -(-ROTATE_BYTES // (per_gpu * N))))
    batches = make_batches(pkg, torch, args, mask, per_gpu, frame0, sum(counts), dev, args.ebn0, nb)
    batches = [(widen_q9(torch, b[0], fmt),) + tuple(b[1:]) for b in batches]
    outs = [torch.empty((per_gpu, dec.words), dtype=torch.int64, device=dev) for _ in range(nb)]
    # at least 20 steps and ~30 ms of decodes (a 0.13 ms launch timed over 20 steps read 12 %
    # slow against the same kernel over 200: profiles/r06_final_bench.json c4_share vs
    # r06_final_bench_c4share_traced.json), at most --steps; after the headline's settle period,
    # so that short launches are timed at the clock of a continuous stream
    steps = max(3, min(args.steps, 20))
    if args.steps > steps:
        for i in range(3):
            dec.decode(batches[i % nb][0], outs[i % nb], stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(3):
            dec.decode(batches[i % nb][0], outs[i % nb], stream)
        torch.cuda.synchronize()
        est = (time.perf_counter() - t0) / 3
        want = [float(min(args.steps, max(steps, int(0.03 / max(est, 1e-6)) + 1)))]
        steps = int(sharding.max_over_ranks(want, dist, coll_dev)[0])   # (the same count on every rank)
    warm = 3
    elapsed, kern_ms = timed_decodes(torch, sharding, dist, coll_dev, dec, batches, outs, steps, warm, stream,
                                     settle_s=args.settle_ms * 1e-3)
    frames_all = int(sum(counts))
    ent = {"workload": note, "mask": mask_name, "N": N, "K": K, "datapath": dict(fmt), "frames_per_gpu": per_gpu,
           "frames_all_ranks": frames_all, "steps": steps, "warmup": warm, "rotated_batches": nb,
           "ms_per_step": elapsed / steps * 1e3, "info_bits_per_s": frames_all * steps / elapsed * K,
           "frames_per_sec": frames_all * steps / elapsed, "kernel": kernel_name(dec.stats, dec.launch_info(per_gpu))}
    ent["roofline"], _ = roofline_entry(mask_name, N, per_gpu, kern_ms, dec, fmt)
    if rank == 0 and args.check > 0:
        from oracle import oracle
        last = (steps - 1) % nb
        nchk = min(4, per_gpu)
        got = pkg.unpack_bits(outs[last][:nchk].cpu().numpy(), N)
        ref = oracle.decode_fsm(mask, batches[last][0][:nchk].cpu().numpy(), **fmt)
        ent["parity_check"] = {"frames": nchk, "bit_exact": bool((got == ref).all())}
    dec.close()
    del batches, outs
    torch.cuda.empty_cache()
    return ent


def time_scatter_gather(torch, pkg, sharding, dist, dec, mask, total, rank, dev, cdev, args):
    """C4 flow: rank 0 holds `total` frames in HBM; per step RCCL scatters the LLR shards,
    every rank decodes its shard, RCCL gathers x^ to rank 0. Returns timing (max over ranks)."""
    N, K = mask.size, int(mask.sum())
    full = None
    if rank == 0:
        full, _ = gen_frames_torch(torch, mask, total, args.ebn0, 0xF0, dev)
        full = full.to(cdev)
    steps = max(1, min(args.steps, 20))

    def step():
        shard = sharding.scatter_shards(full, total, (N,), torch.int8, dist, cdev).to(dev)
        out = dec.decode(shard)
        return sharding.gather_to_root(out.to(cdev), total, dist, cdev)

    got = step()   # warm-up (and a correctness spot check of the reassembled batch on rank 0)
    ok = None
    if rank == 0:
        ref = dec.decode(full.to(dev))
        ok = bool(torch.equal(got.to(dev), ref))
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    el = sharding.max_over_ranks([time.perf_counter() - t0], dist, cdev)[0]
    fps = total * steps / el
    return {"ms_per_step": el / steps * 1e3, "frames_per_sec": fps, "info_bits_per_s": fps * K,
            "frames_per_step": total, "steps": steps, "gathered_equals_single_decode": ok,
            "flow": "rank 0 batch in HBM -> RCCL scatter (LLRs) -> decode on every rank -> RCCL gather (x^) to rank 0"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU frames")
    ap.add_argument("--ebn0", type=float, default=2.5)
    ap.add_argument("--data", choices=["csim", "torch"], default="csim",
                    help="csim: the reference testbench's own frame chain on the GPU (KAT codewords for "
                         "N in {8, 512, 1024}, else all-zero; xorshift128 seed 0xF0; Box-Muller; beta 4, +-31), "
                         "each rank taking the next frames of the global stream; torch: random information "
                         "bits + torch AWGN")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-io", action="store_true",
                    help="also time polar_sc_decode_host (PCIe-inclusive, host buffers) on the batch")
    ap.add_argument("--check", type=int, default=64, help="frames checked vs the oracle (rank 0)")
    ap.add_argument("--rotate", type=int, default=0,
                    help="distinct resident input batches cycled through by the timed loop (0: enough for "
                         "%d MB, so the inputs do not sit in the Infinity Cache)" % (ROTATE_BYTES >> 20))
    ap.add_argument("--no-ebn0-sweep", dest="ebn0_sweep", action="store_false",
                    help="skip the Eb/N0 {1, 2.5, 4} dB sweep of the timed loop")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false",
                    help="skip the C3 / C5 / C5-share entries timed after the headline region")
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed decodes before the warm-up so that the timed steps run at the clock of "
                         "a continuous stream (reported as settle_ms)")
    ap.add_argument("--io", choices=["resident", "scatter"], default="resident",
                    help="scatter: also time the C4 flow -- rank 0 holds the whole batch in HBM, "
                         "RCCL scatters the LLR shards, every rank decodes, RCCL gathers x^ to rank 0 "
                         "(reported as 'scatter_gather'; 'value' stays the resident-input decode)")
    args = ap.parse_args()

    import torch
    import sc_polar_decoder_hls_amd as pkg
    from sc_polar_decoder_hls_amd import sharding
    import util

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("--gpus %d needs torchrun with %d processes" % (args.gpus, args.gpus))
    # one process per GPU; local ranks beyond the visible devices wrap (rehearsals on a
    # 1-GPU box: POLAR_BENCH_BACKEND=gloo torchrun --nproc-per-node 2 bench.py --gpus 2)
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    dist = None
    coll_dev = dev
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("POLAR_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
            coll_dev = torch.device("cpu")

    name, per_gpu, desc = CONFIGS[args.config]
    mask = util.mask(name)
    N, K = mask.size, int(mask.sum())
    strong = per_gpu is None     # c4 / c5: a fixed total batch sharded over the ranks
    if args.config == "c4":
        per_gpu = sharding.shard_bounds(1 << 20, world, rank)[1]
    elif args.config == "c5":
        per_gpu = sharding.shard_bounds(512, world, rank)[1]
    if args.batch:
        per_gpu = args.batch

    dec = pkg.Decoder(mask)
    dec.prepare(per_gpu)
    # frames of this rank: the next per_gpu frames of the testbench's single stream
    counts = [per_gpu]
    if dist is not None:
        t = torch.zeros(world, dtype=torch.float64, device=coll_dev)
        t[rank] = per_gpu
        dist.all_reduce(t)
        counts = [int(v) for v in t.tolist()]
    frame0 = int(sum(counts[:rank]))
    nb = args.rotate if args.rotate > 0 else max(1, min(8, -(-ROTATE_BYTES // (per_gpu * N))))
    batches = make_batches(pkg, torch, args, mask, per_gpu, frame0, sum(counts), dev, args.ebn0, nb)
    outs = [torch.empty((per_gpu, dec.words), dtype=torch.int64, device=dev) for _ in range(nb)]
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()

    elapsed, kern_ms = timed_decodes(torch, sharding, dist, coll_dev, dec, batches, outs, args.steps, args.warmup,
                                     stream, settle_s=args.settle_ms * 1e-3)
    # the CPU baseline decodes the head of the first resident batch (the GPU run's own LLRs)
    cpu_llr = batches[0][0][: max(8, min(4096, int(2 ** 22 // N)))].cpu().numpy() if rank == 0 else None
    if dist is not None:   # frames decoded by all ranks (shards may differ by a few frames)
        cnt = torch.tensor([per_gpu], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(cnt)
        frames_all = int(cnt.item())
    else:
        frames_all = per_gpu

    total_frames = frames_all * args.steps
    fps = total_frames / elapsed
    value = fps * K
    # the last launch of the timed loop decoded batch (steps - 1) % nb into its output
    last = (args.steps - 1) % nb
    llr, xref, x = batches[last]
    out = outs[last]

    scatter_res = None
    if args.io == "scatter" and dist is not None:
        scatter_res = time_scatter_gather(torch, pkg, sharding, dist, dec, mask, frames_all, rank, dev,
                                          coll_dev, args)

    # parity spot check (rank 0) vs the CPU oracle on the first frames of the batch; after the
    # timed region, so the oracle's CPU threads cannot perturb it
    check = {}
    if rank == 0 and args.check > 0:
        from oracle import oracle
        nchk = min(args.check, per_gpu)
        got = pkg.unpack_bits(out[:nchk].cpu().numpy(), N)
        ref = oracle.decode_fsm(mask, llr[:nchk].cpu().numpy())
        check = {"frames": nchk, "bit_exact": bool((got == ref).all())}

    # error rates of the last decoded batch vs the transmitted codewords (informative)
    errors_all = None
    if xref is not None:
        # sc_error_counter semantics on the device (per-frame count mod 1024), whole batch
        cnt = pkg.count_errors(out, xref, N)
        torch.cuda.synchronize()
        c = [float(v) for v in cnt.cpu().tolist()]
        fer, ber = c[1] / per_gpu, c[2] / (per_gpu * N)
        if dist is not None:
            # every rank's own counts (reported beside the total, so that the sum can be checked)
            mine = cnt.to(coll_dev, torch.float64)
            per_rank = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(per_rank, mine)
            # the job's error totals: device counts summed over the ranks (RCCL all-reduce)
            sharding.sum_over_ranks(cnt, dist, coll_dev)
            t = [int(v) for v in cnt.cpu().tolist()]
            errors_all = {"frames": frames_all, "frame_errors": t[1], "bit_errors": t[2],
                          "bit_errors_mod1024_sum": t[0], "frame_error_rate": t[1] / frames_all,
                          "bit_error_rate": t[2] / (frames_all * N),
                          "per_rank": [{"frames": counts[r], "frame_errors": int(v[1].item()),
                                        "bit_errors": int(v[2].item())} for r, v in enumerate(per_rank)]}
    else:
        xhat = pkg.unpack_bits(out[: min(per_gpu, 4096)].cpu().numpy(), N)
        xs = x[: xhat.shape[0]].cpu().numpy()
        fer = float((xhat != xs).any(axis=1).mean())
        ber = float((xhat != xs).mean())

    # (after the parity check and the error counts: the sweep reuses the output buffers)
    # Eb/N0 sweep: the same timed loop on frames at each SNR
    sweep = None
    if args.ebn0_sweep:
        sweep = []
        for e in EBN0_SWEEP:
            bs = make_batches(pkg, torch, args, mask, per_gpu, frame0, sum(counts), dev, e, nb)
            el, km = timed_decodes(torch, sharding, dist, coll_dev, dec, bs, outs, max(1, args.steps // 2),
                                   max(1, args.warmup // 4), stream)
            ent = {"ebn0_db": e, "value": frames_all * max(1, args.steps // 2) / el * K,
                   "ms_per_step": el / max(1, args.steps // 2) * 1e3, "kernel_ms": km}
            if bs[0][1] is not None:
                cnt = pkg.count_errors(outs[(max(1, args.steps // 2) - 1) % nb], bs[(max(1, args.steps // 2) - 1) % nb][1], N)
                torch.cuda.synchronize()
                ent["frame_error_rate"] = float(cnt[1].item()) / per_gpu
            sweep.append(ent)
            del bs
        torch.cuda.synchronize()

    # two batches in flight (after the sweep, before the secondary plans allocate)
    pipelined = None
    if dec.stats["storage"] != 1:
        el2 = pipelined_decodes(torch, sharding, dist, coll_dev, dec, batches, args.steps, dev)
        pipelined = {"streams": 2, "ms_per_step": el2 / args.steps * 1e3,
                     "value": frames_all * args.steps / el2 * K, "vs_one_stream": elapsed / el2,
                     "note": "consecutive batches alternate two HIP streams (a serving loop): one launch's "
                             "tail overlaps the next one's start; value above is the one-stream loop"}

    secondary = None
    if args.secondary and args.config == "c2" and not args.batch:
        secondary = {}
        for key, mname, pg, fmt, note in SECONDARY:
            if key in ("c5_share64", "c4_share") and world != 1:
                continue   # 8-GPU shares, timed on one GPU (at N > 1 each rank's own share is the c2 / c5 work)
            secondary[key] = secondary_entry(torch, pkg, sharding, dist, coll_dev, args, key, mname, pg, fmt, note,
                                             rank, world, dev, stream)
        if "par16_n16384" in secondary and "par64_n16384" in secondary:
            # script_tests.sh sweeps PAR 16 and 64 on the same codes: PAR 64's cost relative to 16
            secondary["par64_over_par16_time"] = (secondary["par64_n16384"]["ms_per_step"] /
                                                  secondary["par16_n16384"]["ms_per_step"])

    if rank == 0:
        roof, prof = roofline_entry(name, N, per_gpu, kern_ms, dec)
        prof_path = os.path.join(ROOT, roof["traffic_source"]) if roof.get("traffic_source") else None
        valu = None
        if prof is not None:
            if "valu_insts_per_wave" in prof:
                # supplementary: the bound that actually limits this kernel
                simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
                waves = (per_gpu + 7) // 8
                rate = waves * prof["valu_insts_per_wave"] / (kern_ms * 1e-3)
                ghz = prof.get("effective_clock_ghz") or NOMINAL_CLOCK_GHZ
                peak = simds * ghz * 1e9 / VALU_CYCLES_PER_INST
                valu = {"insts_per_wave": prof["valu_insts_per_wave"], "waves_per_launch": waves,
                        "achieved": rate, "peak": peak, "unit": "wave-instructions/s", "frac": rate / peak,
                        "peak_basis": "%d SIMDs x %.2f GHz (PMC clock) / %.2f SIMD cycles per wave64 packed-16 "
                                      "VALU instruction at 8 waves/SIMD (profiles/r02_valu_microbench.log)"
                                      % (simds, ghz, VALU_CYCLES_PER_INST),
                        # the per-mask kernel's occupancy (123 VGPRs, 33 KB LDS per 4-wave block)
                        "peak_at_4_waves_per_simd": simds * ghz * 1e9 / VALU_CYCLES_BY_WAVES[4],
                        "source": os.path.relpath(prof_path, ROOT)}
        res = {
            "metric": "decoded info bits/sec + frames/sec, N=1024 K=512 batch, 1/2/4/8 MI355X",
            "value": value,
            "unit": "info_bits/s",
            "frames_per_sec": fps,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "int16 sign-magnitude (6-bit LLRs, u8 in / bit-packed out)",
            "data": (("synthetic: the reference testbench's C-sim chain generated on-device (KAT codewords, "
                      "xorshift128 seed 0xF0, Box-Muller, Eb/N0=%.1f dB, beta 4, +-31)" if args.data == "csim" else
                      "synthetic AWGN frames generated on-device (random info bits, BPSK, Eb/N0=%.1f dB, "
                      "4x quantizer, +-31)") % args.ebn0),
            "config": {"workload": desc, "N": N, "K": K, "frames_per_gpu": per_gpu,
                       "mask": name, "parallelism": "frames sharded, dp%d" % world,
                       "rotated_batches": nb, "rotated_bytes": nb * per_gpu * N},
            "roofline": dict(roof, kernel=kernel_name(dec.stats, dec.launch_info(per_gpu))),
            "valu_roofline": valu,
            "settle_ms": args.settle_ms,
            "secondary": secondary,
            "scatter_gather": scatter_res,
            "ebn0_sweep": sweep,
            "pipelined": pipelined,
            "frame_error_rate": fer,
            "bit_error_rate": ber,
            "errors_all_ranks": errors_all,
            "parity_check": check,
        }
        if world == 1 and args.host_io:
            # PCIe-inclusive rate of the host-buffer entry point (polar_sc_decode_host):
            # pageable host int8 frames in, packed x^ out, synchronous
            host_llr = llr.cpu().numpy()
            dec.decode_host(host_llr)
            reps = 5
            t0h = time.perf_counter()
            for _ in range(reps):
                dec.decode_host(host_llr)
            elh = (time.perf_counter() - t0h) / reps
            res["host_io"] = {"ms_per_step": elh * 1e3, "frames_per_sec": per_gpu / elh,
                              "info_bits_per_s": per_gpu * K / elh,
                              "note": "polar_sc_decode_host: %d frames from pageable host memory "
                                      "(%.1f MB in, %.1f MB out), copies + decode, synchronous"
                                      % (per_gpu, per_gpu * N / 1e6, per_gpu * dec.words * 8 / 1e6)}
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(mask, args.cpu_seconds, args.ebn0, cpu_llr)
        print(json.dumps(res))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
