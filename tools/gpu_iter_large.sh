#!/bin/bash
# Large-N iteration: interpreter/hybrid parity subset, per-op probe, C3/C5 bench lines.
# usage: tools/gpu_iter_large.sh <tag>
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-iter}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_hybrid.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hbm_scratch or waves_per_group or c3_mask or c5_mask or full_c3" > gpurun_out/${T}_pytest.log 2>&1
echo "pytest ok"
timeout -k 10 200 python tools/op_latency_probe.py frozen_n_262144_k_131072 --batch 512 --out gpurun_out/${T}_probe_c5.json
timeout -k 10 200 python tools/op_latency_probe.py frozen_n_65536_k_32768 --batch 4096 --out gpurun_out/${T}_probe_c3.json
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 --no-ebn0-sweep --no-cpu-baseline > gpurun_out/${T}_bench_c3.json
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-ebn0-sweep --no-cpu-baseline > gpurun_out/${T}_bench_c5.json
echo "bench ok"
