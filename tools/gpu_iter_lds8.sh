#!/bin/bash
# LDS8 region iteration: GPU suite subset (interpreter, hybrid, formats, tier) + C3 / C5 A/B
# of the LDS region size on the same box.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-l8}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_hybrid.py tests/test_gpu_formats.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
echo "pytest ok"
B="python bench.py --steps 10 --warmup 3 --no-ebn0-sweep --no-cpu-baseline"
timeout -k 10 300 $B --config c3 > gpurun_out/${T}_bench_c3.json
timeout -k 10 300 env POLAR_SC_LDS_SLOTS=256 $B --config c3 > gpurun_out/${T}_bench_c3_w256.json
timeout -k 10 300 $B --config c5 > gpurun_out/${T}_bench_c5.json
timeout -k 10 300 env POLAR_SC_LDS_SLOTS=512 $B --config c5 > gpurun_out/${T}_bench_c5_w512.json
timeout -k 10 300 env POLAR_SC_LDS_SLOTS=256 $B --config c5 > gpurun_out/${T}_bench_c5_w256.json
timeout -k 10 300 $B --config c5 --batch 64 > gpurun_out/${T}_bench_c5_b64.json
timeout -k 10 300 env POLAR_SC_LDS_SLOTS=256 $B --config c5 --batch 64 > gpurun_out/${T}_bench_c5_b64_w256.json
echo "bench ok"
B2="python bench.py --steps 200 --warmup 30 --no-ebn0-sweep --no-cpu-baseline"
timeout -k 10 300 $B2 > gpurun_out/${T}_bench_c2.json
timeout -k 10 300 env POLAR_SC_ROOT_RESPLIT=1 $B2 > gpurun_out/${T}_bench_c2_resplit.json
timeout -k 10 300 $B2 > gpurun_out/${T}_bench_c2_again.json
timeout -k 10 300 env POLAR_SC_ROOT_RESPLIT=1 $B2 > gpurun_out/${T}_bench_c2_resplit_again.json
echo "c2 ok"
