"""Per-op latency monitor report.

The reference measures its decoder with sc_monitor (src/rtl_simu_testbench/sc_monitor/
sc_monitor.h:50-140): while `busy` is high it counts clock cycles per tree level
(N_value) and per function (Fct_ID: F 0x88, G 0x48, H 0x28, R 0x18, H_R0 0x20, F_REP 0x82,
G_R1 0x4F, G_SPC 0x44, my_module.h:21-30), plus the occurrences of each (function, level)
run. report() builds the same tables from Decoder.trace() records: shader-clock cycles of
frame group 0's lead wave per device op, grouped by function and by level (node size).

    python -m sc_polar_decoder_hls_amd.monitor <mask file> [K] [--batch B] [--json]
"""
import argparse
import json
from collections import OrderedDict, defaultdict

# schedule op -> the reference monitor's function name
FUNCTION = OrderedDict([
    ("F", "F"), ("G", "G"), ("H", "H"), ("FLEAF", "R"), ("GLEAF", "R"), ("H0", "H_R0"), ("REP", "F_REP"),
    ("R1", "G_R1"), ("SPC", "G_SPC"), ("SUB", "SUBTREE"), ("WOPEN", "WINDOW"), ("WFLUSH", "WINDOW"),
])


def report(rows, info):
    """Aggregate trace rows: {'total_cycles', 'clock_ghz', 'us', 'by_level': {nodeN: cycles},
    'by_function': {name: cycles}, 'occurrences': {(name, nodeN): runs}, 'ops': {name: count}}."""
    by_level = defaultdict(int)
    by_fn = OrderedDict((v, 0) for v in FUNCTION.values())
    occ = defaultdict(int)
    ops = defaultdict(int)
    last = None
    for r in rows:
        if r["op"] == "END":
            continue
        fn = FUNCTION.get(r["op"], str(r["op"]))
        by_level[r["nodeN"]] += r["cycles"]
        by_fn[fn] += r["cycles"]
        ops[fn] += 1
        key = (fn, r["nodeN"])
        if key != last:          # sc_monitor.h: a new run starts when function or level changes
            occ[key] += 1
        last = key
    return dict(total_cycles=info["total_cycles"], clock_ghz=info["clock_ghz"], us=info["us"],
                by_level=dict(sorted(by_level.items(), reverse=True)),
                by_function={k: v for k, v in by_fn.items() if v or ops.get(k)},
                occurrences={"%s@%d" % k: v for k, v in sorted(occ.items())}, ops=dict(ops))


def format_report(rep):
    ghz = rep["clock_ghz"] or 0.0
    lines = ["[MONITOR] PROCESS latency : %d cycles (%.2f us at %.2f GHz, frame group 0)"
             % (rep["total_cycles"], rep["us"] or 0.0, ghz), "", "\t\t*** Latency by Level ***"]
    for lvl, c in rep["by_level"].items():
        lines.append("\t\t\t\tnode %7d LLRs : %10d cycles" % (lvl, c))
    lines += ["", "\t\t*** Latency by Function ***"]
    for fn, c in rep["by_function"].items():
        lines.append("\t\t\t\tfunction %-8s: %10d cycles  (%d ops)" % (fn, c, rep["ops"].get(fn, 0)))
    return "\n".join(lines)


def main(argv=None):
    import numpy as np
    import torch

    from . import Decoder, load_frozen_tab, load_mask_file
    ap = argparse.ArgumentParser()
    ap.add_argument("table")
    ap.add_argument("K", nargs="?", type=int, default=0, help="Frozen_Bit_Tab K (0: Generated_Frozen_Bit file)")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    mask = load_frozen_tab(a.table, a.K) if a.K else load_mask_file(a.table)
    dec = Decoder(mask)
    rng = np.random.default_rng(a.seed)
    llr = torch.from_numpy(rng.integers(-31, 32, size=(a.batch, mask.size)).astype(np.int8)).cuda()
    rows, info = dec.trace(llr)
    rep = report(rows, info)
    print(json.dumps(rep) if a.json else format_report(rep))


if __name__ == "__main__":
    main()
