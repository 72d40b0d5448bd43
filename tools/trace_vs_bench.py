#!/usr/bin/env python3
"""bench.py's HIP-event kernel time against rocprofv3's kernel-trace average of the same command
(tools/gpu_round.sh benchprof): per config the decode kernel's trace average, the bench line's
kernel_ms, and the roofline fraction recomputed from each.

usage: python tools/trace_vs_bench.py gpurun_out/<tag> [--out profiles/<tag>_bench_trace.txt]"""
import argparse
import csv
import glob
import json
import os


def trace_avg(d):
    """(name, calls, average ns, min ns) of the polar_sc decode kernel in a kernel_stats csv."""
    path = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Name"].startswith("polar_sc_") and row["Name"] != "polar_sc_tier_kernel":
                return row["Name"], int(row["Calls"]), float(row["AverageNs"]), float(row["MinNs"])
    raise SystemExit("no polar_sc kernel in " + path)


def timed_avg(d, kname, steps):
    """Average ns of the last `steps` dispatches of `kname` on the stream of its first dispatch
    (bench.py's timed loop; the two-stream entry that follows runs on streams of its own and
    overlaps its launches)."""
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if r["Kernel_Name"] == kname]
    main = [r for r in rows if r["Stream_Id"] == rows[0]["Stream_Id"]][-steps:]
    return sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in main) / len(main)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    args = ap.parse_args()
    lines = ["config | kernel | trace calls | all-dispatch avg (us) | timed-loop avg (us) | bench kernel_ms (us) | "
             "timed avg / bench | frac (bench) | frac (trace, timed loop)"]
    for name in ("c2", "c3", "c5", "c5b64", "c4share"):
        jpath = os.path.join(args.dir, "bench_%s.json" % name)
        if not os.path.exists(jpath):
            continue
        r = json.loads([l for l in open(jpath) if l.startswith("{")][0])
        ro = r["roofline"]
        kname, calls, avg, mn = trace_avg(os.path.join(args.dir, "bench_" + name))
        bench_us = ro["kernel_ms"] * 1e3
        tavg = timed_avg(os.path.join(args.dir, "bench_" + name), kname, r["steps"])
        frac_trace = ro["algorithmic_bytes_per_launch"] / (tavg * 1e-9) / 1e9 / ro["peak"]
        lines.append("%s | %s | %d | %.2f | %.2f | %.2f | %.3f | %.4f | %.4f" % (
            name, kname, calls, avg / 1e3, tavg / 1e3, bench_us, tavg / 1e3 / bench_us, ro["frac"], frac_trace))
    text = "\n".join(lines) + "\n"
    print(text, end="")
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
