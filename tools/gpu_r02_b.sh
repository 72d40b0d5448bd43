#!/bin/bash
# Round 2: the datapath-format GPU tests, then the whole GPU suite, then the VALU microbench.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_formats.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b_formats.log 2>&1
echo "formats ok"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_formats.py > gpurun_out/r02b_pytest.log 2>&1
echo "suite ok"
timeout -k 10 120 ./build_tools/valu_mb > gpurun_out/r02b_valu_mb.log 2>&1
echo "valu ok"
