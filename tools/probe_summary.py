#!/usr/bin/env python3
"""Summarise op_latency_probe.py dumps: cycles by (op, n) with counts, median, share."""
import json
import statistics as st
import sys
from collections import defaultdict

for fn in sys.argv[1:]:
    d = json.load(open(fn))
    rows, tot = d["rows"], d["info"]["total_cycles"]
    agg = defaultdict(list)
    for r in rows:
        agg[(r["op"], r["n"])].append(r["cycles"])
    print("%s  total %d cycles, %d ops" % (fn, tot, len(rows)))
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:int(d.get("top", 18))]:
        print("  %-7s n=%-6d cnt %4d  sum %9d (%4.1f%%) med %7d min %7d" % (k[0], k[1], len(v), sum(v), 100 * sum(v) / tot,
                                                                          st.median(v), min(v)))
