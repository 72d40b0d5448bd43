#!/usr/bin/env python3
"""BASELINE.md section 5 results table from a committed bench line (profiles/<tag>_bench.json):
the C2 headline, the C3 / C5 / C5-share secondary entries, and the CPU baseline beside them.

usage: python tools/baseline_table.py profiles/r03_v3_bench.json
"""
import json
import sys


def main():
    path = sys.argv[1]
    with open(path) as f:
        d = json.loads(f.read().strip().splitlines()[-1])
    rows = []
    rf = d["roofline"]
    rows.append(("C2 N=1024 K=512", "65536 frames", "%.1f µs" % (d["ms_per_step"] * 1e3), "%.3g" % d["value"],
                 "%.3g" % d["frames_per_sec"], "%.3f" % rf["frac"],
                 "%.1f MB / %.1f MB" % (rf["traffic"] / 1e6, rf["algorithmic_bytes_per_launch"] / 1e6)
                 if rf.get("traffic") else "—"))
    for key, e in (d.get("secondary") or {}).items():
        r = e["roofline"]
        rows.append(("%s N=%d K=%d" % (key.upper().replace("_SHARE64", " (8-GPU share)"), e["N"], e["K"]),
                     "%d frames" % e["frames_per_gpu"], "%.3f ms" % e["ms_per_step"], "%.3g" % e["info_bits_per_s"],
                     "%.3g" % e["frames_per_sec"], "%.4f" % r["frac"],
                     "%.2f GB / %.3f GB" % (r["traffic"] / 1e9, r["algorithmic_bytes_per_launch"] / 1e9)
                     if r.get("traffic") else "—"))
    print("| config (1 × MI355X) | batch | time per decode | info bits/s | frames/s | HBM roofline frac | "
          "PMC traffic / algorithmic bytes per decode |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        print("| " + " | ".join(r) + " |")
    cb = d.get("cpu_baseline")
    if cb:
        print()
        print("CPU baseline (`%s`, %s): %.3g info bits/s on %d threads, %.3g on 1 thread; nproc %s, %s. Sample: %s."
              % (cb["kind"], "the oracle's literal my_module FSM" if cb["kind"] == "port" else "oracle/_ref",
                 cb["value"], cb["cores"], cb["value_1thread"], cb.get("nproc"), cb.get("cpu_model"), cb["sample"]))
        print("GPU / CPU (all threads) at C2: %.0f×." % (d["value"] / cb["value"]))


if __name__ == "__main__":
    main()
