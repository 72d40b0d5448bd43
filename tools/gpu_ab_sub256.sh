#!/bin/bash
# Same-box A/B: 64-word vs 128-word generated subtrees (POLAR_SC_SUB_WORDS), C5 / C5-64 / C3,
# plus parity of the 128-word variant on the C3 / C5 samples.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-s128}
mkdir -p gpurun_out
timeout -k 10 500 env POLAR_SC_SUB_WORDS=256 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c3_mask or c5_mask" > gpurun_out/${T}_pytest.log 2>&1
echo "pytest ok"
B="python bench.py --steps 10 --warmup 3 --no-ebn0-sweep --no-cpu-baseline"
for r in 1 2; do
  for sw in 128 256; do
    timeout -k 10 300 env POLAR_SC_SUB_WORDS=$sw $B --config c5 > gpurun_out/${T}_c5_sw${sw}_$r.json
    timeout -k 10 300 env POLAR_SC_SUB_WORDS=$sw $B --config c5 --batch 64 > gpurun_out/${T}_c5b64_sw${sw}_$r.json
    timeout -k 10 300 env POLAR_SC_SUB_WORDS=$sw $B --config c3 > gpurun_out/${T}_c3_sw${sw}_$r.json
  done
done
echo "ab ok"
