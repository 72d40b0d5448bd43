#!/bin/bash
# Grid-tier iteration: parity subset + C3 / C5 bench variants (POLAR_SC_TIER_WORDS).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-tier}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_hybrid.py -m gpu -x -v --timeout 300 --timeout-method thread -k "hbm_scratch or waves_per_group or c3_mask or c5_mask or full_c3 or grid_tier" > gpurun_out/${T}_pytest.log 2>&1
echo "pytest ok"
B="python bench.py --steps 10 --warmup 3 --no-ebn0-sweep --no-cpu-baseline"
timeout -k 10 300 $B --config c3 > gpurun_out/${T}_bench_c3.json
timeout -k 10 300 env POLAR_SC_TIER_WORDS=2048 $B --config c3 > gpurun_out/${T}_bench_c3_tw2048.json
timeout -k 10 300 $B --config c5 > gpurun_out/${T}_bench_c5.json
timeout -k 10 300 $B --config c5 --batch 64 > gpurun_out/${T}_bench_c5_b64.json
timeout -k 10 300 env POLAR_SC_TIER_WORDS=0 $B --config c5 --batch 64 > gpurun_out/${T}_bench_c5_b64_tw0.json
timeout -k 10 300 env POLAR_SC_TIER_WORDS=512 $B --config c5 > gpurun_out/${T}_bench_c5_tw512.json
echo "bench ok"
