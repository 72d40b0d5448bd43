#!/bin/bash
# Same-box A/B of per-mask kernel variants at C2 (interleaved, two rounds).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-abc2}
mkdir -p gpurun_out
B="python bench.py --steps 200 --warmup 30 --no-ebn0-sweep --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 300 $B > gpurun_out/${T}_base_$r.json
  timeout -k 10 300 env POLAR_SC_ROOT_PACK=1 $B > gpurun_out/${T}_pack_$r.json
done
timeout -k 10 300 env POLAR_SC_ROOT_PACK=1 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "awgn or edge or kat or full_size or committed" > gpurun_out/${T}_pack_pytest.log 2>&1
echo "ok"
