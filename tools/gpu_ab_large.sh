#!/bin/bash
# Same-box A/B of hybrid-plan knobs at C3 / C5 (interleaved rounds). Every bench line carries
# its own 64-frame parity check against the oracle.
# usage: bash tools/gpu_ab_large.sh <tag> <rounds> <config> <batch|0> "<env a>" "<env b>" ...
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=$1; R=$2; C=$3; NB=$4; shift 4
mkdir -p gpurun_out
B="bench.py --config $C --steps 20 --warmup 5 --no-ebn0-sweep --no-cpu-baseline"
if [ "$NB" != "0" ]; then B="$B --batch $NB"; fi
for r in $(seq 1 "$R"); do
  i=0
  for v in "$@"; do
    timeout -k 10 300 env $v python $B > gpurun_out/${T}_v${i}_$r.json
    i=$((i + 1))
  done
  echo "round $r done"
done
python tools/bench_summary.py gpurun_out/${T}_v*.json > gpurun_out/${T}_summary.txt 2>&1 || true
echo "ok"
