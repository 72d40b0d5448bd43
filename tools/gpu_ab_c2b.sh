#!/bin/bash
# Same-box A/B of the packed-root per-mask kernel at C2: 3 interleaved rounds of bench +
# kernel-trace means.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-abc2b}
OUT=$ROOT/gpurun_out/$T
mkdir -p "$OUT"
B="python bench.py --steps 300 --warmup 50 --no-ebn0-sweep --no-cpu-baseline"
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 env POLAR_SC_ROOT_PACK=$v $B > "$OUT/bench_pack${v}_$r.json"
  done
done
cd /tmp
export TMPDIR=/tmp
for v in 1 0; do
  POLAR_SC_ROOT_PACK=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace_pack$v" -o t --output-format csv -- python3 $ROOT/tools/prof_decode.py --reps 20 > "$OUT/trace_pack$v.log" 2>&1
done
echo ok
