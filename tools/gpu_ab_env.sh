#!/bin/bash
# Same-box A/B of environment knobs of the C2 bench (interleaved rounds), parity first.
# usage: bash tools/gpu_ab_env.sh <tag> <rounds> "<env of variant a>" "<env of variant b>" ...
#   (an empty string is the default build; e.g. "POLAR_SC_MASK_WPB=1")
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=$1; R=$2; shift 2
mkdir -p gpurun_out
B="bench.py --steps 200 --warmup 30 --no-ebn0-sweep --no-cpu-baseline --check 256"
i=0
for v in "$@"; do
  timeout -k 10 300 env $v python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "awgn or edge or misaligned or full_size or ragged" > gpurun_out/${T}_v${i}_pytest.log 2>&1
  echo "parity v$i ($v) ok"
  i=$((i + 1))
done
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
