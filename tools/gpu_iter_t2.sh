#!/bin/bash
# SPC split + C2 occupancy A/B.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-t2}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hbm_scratch or waves_per_group or c3_mask or c5_mask or full_c3 or grid_tier" > gpurun_out/${T}_pytest.log 2>&1
echo "pytest ok"
timeout -k 10 200 python tools/op_latency_probe.py frozen_n_262144_k_131072 --batch 64 --out gpurun_out/${T}_probe_c5.json
B="python bench.py --steps 10 --warmup 3 --no-ebn0-sweep --no-cpu-baseline"
timeout -k 10 300 $B --config c3 > gpurun_out/${T}_bench_c3.json
timeout -k 10 300 $B --config c5 > gpurun_out/${T}_bench_c5.json
timeout -k 10 300 $B --config c5 --batch 64 > gpurun_out/${T}_bench_c5_b64.json
B2="python bench.py --steps 200 --warmup 30 --no-ebn0-sweep --no-cpu-baseline"
timeout -k 10 300 $B2 > gpurun_out/${T}_bench_c2.json
timeout -k 10 300 env POLAR_SC_MASK_MIN_WAVES=4 $B2 > gpurun_out/${T}_bench_c2_w4.json
timeout -k 10 300 env POLAR_SC_MASK_MIN_WAVES=5 $B2 > gpurun_out/${T}_bench_c2_w5.json
echo "bench ok"
