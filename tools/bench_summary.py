#!/usr/bin/env python3
"""One line per bench JSON file: value, ms/step, kernel ms (HIP events), roofline frac."""
import json
import sys

for fn in sys.argv[1:]:
    try:
        d = json.loads(open(fn).read().strip().splitlines()[-1])
        r = d.get("roofline", {})
        print("%-44s value %.4g  ms/step %.4f  kernel_ms %s  frac %.4f  parity %s" % (
            fn, d["value"], d["ms_per_step"], r.get("kernel_ms"), r.get("frac", 0), d.get("parity_check")))
    except Exception as e:  # noqa: BLE001
        print(fn, "unreadable:", e)
