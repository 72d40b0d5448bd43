#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh run: per decode-kernel dispatch averages of every PMC
counter, kernel duration from the trace, and derived figures (issue rate, wait shares,
effective clock, HBM bytes per launch with the gfx950 FETCH_SIZE correction).

usage: tools/pmc_summary.py gpurun_out/prof_<tag> [--kernel REGEX] [--json out.json] [--reps R]

--reps R: the driver ran R decodes of a multi-launch plan (grid tier: grid F / G launches +
segment launches per decode); counters and kernel time are then totals per decode (all
matching dispatches / R) instead of per-dispatch averages.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def load_counters(d, kre, reps=0):
    per = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> value (sum over instances)
    for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if not kre.search(r["Kernel_Name"]):
                    continue
                per[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    if reps > 0:
        return {k: sum(v.values()) / reps for k, v in per.items() if v}
    return {k: sum(v.values()) / len(v) for k, v in per.items() if v}


def load_trace(d, kre):
    durs = []
    for f in glob.glob(os.path.join(d, "trace", "*_kernel_trace.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kre.search(r["Kernel_Name"]):
                    durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return durs


def load_launch_info(d):
    """The 'launch_info {...}' line tools/prof_decode.py prints (any pass's log), or None."""
    for f in sorted(glob.glob(os.path.join(d, "*.log"))):
        with open(f, errors="replace") as fh:
            for line in fh:
                if line.startswith("launch_info "):
                    return json.loads(line[len("launch_info "):])
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="polar_sc")
    ap.add_argument("--json")
    ap.add_argument("--skip-first", type=int, default=1, help="trace dispatches to drop (warm-up)")
    ap.add_argument("--reps", type=int, default=0, help="decodes per run of a multi-launch plan")
    a = ap.parse_args()
    kre = re.compile(a.kernel)
    c = load_counters(a.dir, kre, a.reps)
    durs = load_trace(a.dir, kre)
    if a.reps > 0 and durs:
        durs = [sum(durs) / a.reps]   # kernel time per decode (all its launches)
        d = durs
    else:
        d = durs[a.skip_first:] if len(durs) > a.skip_first else durs
    res = {"kernel_regex": a.kernel, "dispatches": len(durs), "counters": c}
    info = load_launch_info(a.dir)
    if info:
        # the profiled plan's launch shape and code-object key (tools/prof_decode.py)
        res["launch_info"] = info
        res["code_key"] = info["code_key"]
    if a.reps > 0:
        res["per_decode_of_reps"] = a.reps
    if d:
        res["kernel_s_mean"] = sum(d) / len(d)
        res["kernel_s_min"] = min(d)
    if "SQ_WAVE_CYCLES" in c and "SQ_WAVES" in c:
        # SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles (MI355X_MICROARCH.md)
        wc = c["SQ_WAVE_CYCLES"]
        res["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
        res["salu_insts_per_wave"] = c.get("SQ_INSTS_SALU", 0) / c["SQ_WAVES"]
        res["lds_insts_per_wave"] = c.get("SQ_INSTS_LDS", 0) / c["SQ_WAVES"]
        res["wave_cycles_per_wave"] = 4 * wc / c["SQ_WAVES"]
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_ACTIVE_INST_LDS"):
            if k in c:
                res["share_" + k] = c[k] / wc
    if "GRBM_GUI_ACTIVE" in c and d:
        res["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / res["kernel_s_mean"] / 1e9
    if "FETCH_SIZE" in c:
        res["fetch_kb"] = c["FETCH_SIZE"]
        res["hbm_read_bytes_corrected"] = 2 * 1024 * c["FETCH_SIZE"]   # gfx950: FETCH_SIZE = 1/2 of wide reads
    if "WRITE_SIZE" in c:
        res["hbm_write_bytes"] = 1024 * c["WRITE_SIZE"]
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
