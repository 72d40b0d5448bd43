#!/bin/bash
# Whole GPU suite at HEAD + C3 waves-per-group A/B.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
echo "pytest ok"
B="python bench.py --steps 10 --warmup 3 --no-ebn0-sweep --no-cpu-baseline --config c3"
timeout -k 10 300 $B > gpurun_out/${T}_c3_w4.json
timeout -k 10 300 env POLAR_SC_WAVES_PER_GROUP=2 $B > gpurun_out/${T}_c3_w2.json
timeout -k 10 300 env POLAR_SC_WAVES_PER_GROUP=1 $B > gpurun_out/${T}_c3_w1.json
echo "ab ok"
