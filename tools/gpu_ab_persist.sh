#!/bin/bash
# Same-box A/B of the per-mask kernel (C2): the previous kernel (VGPR-staged channel copy,
# built from HEAD into build_tools/old) vs the LDS-DMA channel fetch (default) vs the
# persistent batch loop with the next channel prefetched HBM -> LDS (POLAR_SC_MASK_PERSIST=1).
# GPU parity first (the new kernels must be bit-exact before they are timed).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-abp}
mkdir -p gpurun_out
timeout -k 10 300 env POLAR_SC_VERBOSE=1 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
echo "parity ok"
B="bench.py --steps 200 --warmup 30 --no-ebn0-sweep --no-cpu-baseline --check 256"
timeout -k 10 300 env POLAR_SC_MASK_PERSIST=1 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "awgn or edge or misaligned or full_size" > gpurun_out/${T}_pytest_p1.log 2>&1
echo "parity (persistent) ok"
for r in 1 2 3; do
  timeout -k 10 300 python build_tools/old/$B > gpurun_out/${T}_old_$r.json
  timeout -k 10 300 python $B > gpurun_out/${T}_new_$r.json
  timeout -k 10 300 env POLAR_SC_VERBOSE=1 POLAR_SC_MASK_PERSIST=1 python $B > gpurun_out/${T}_p1_$r.json 2> gpurun_out/${T}_p1_$r.err
  echo "round $r done"
done
python tools/bench_summary.py gpurun_out/${T}_*.json > gpurun_out/${T}_summary.txt 2>&1 || true
echo "ok"
