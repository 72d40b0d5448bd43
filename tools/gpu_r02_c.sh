#!/bin/bash
# Round 2: script_tests.sh sweep tests (PAR 16/64 at QUANT 8), the re-run VALU microbench.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_formats.py -m gpu -x -v --timeout 300 --timeout-method thread -k script_tests > gpurun_out/r02c_sweep.log 2>&1
echo "sweep ok"
timeout -k 10 120 ./build_tools/valu_mb > gpurun_out/r02c_valu_mb.log 2>&1
echo "valu ok"
