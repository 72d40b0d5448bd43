#!/usr/bin/env python3
"""Per-dispatch PMC sums of the pair kernel from a rocprofv3 counter-collection directory.
usage: python tools/pmc_pair.py gpurun_out/<tag>/<pass dir> [kernel substring]"""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "pair"
    per = collections.defaultdict(list)
    for path in glob.glob(d + "/*counter_collection.csv"):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if key in r["Kernel_Name"]:
                agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in sorted(agg.items()):
            per[c].append(v)
    for c, v in sorted(per.items()):
        print("%-22s %s" % (c, " ".join("%.4g" % x for x in v)))


if __name__ == "__main__":
    main()
