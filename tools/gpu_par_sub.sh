#!/bin/bash
# PAR 4 / 8 format tests on the GPU.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_formats.py -m gpu -v --timeout 300 --timeout-method thread -k "p8 or p4 or sweep" > gpurun_out/parsub_formats.log 2>&1 || true
echo done
