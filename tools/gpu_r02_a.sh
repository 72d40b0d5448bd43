#!/bin/bash
# Round 2, first box call: new GPU tests, bench lines (C2 with the CPU baseline and the Eb/N0
# sweep, C3, C5), and PMC passes of the C2 / C3 / C5 decode kernels with rotated inputs.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_c4_gpu.py tests/test_monitor.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest.log 2>&1
echo "pytest ok"
timeout -k 10 400 python -u bench.py > gpurun_out/r02a_bench_c2.json 2> gpurun_out/r02a_bench_c2.err
echo "bench c2 ok"
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r02a_bench_c3.json 2> gpurun_out/r02a_bench_c3.err
echo "bench c3 ok"
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r02a_bench_c5.json 2> gpurun_out/r02a_bench_c5.err
echo "bench c5 ok"
bash tools/profile_gpu.sh r02a_c2 --reps 10
bash tools/profile_gpu.sh r02a_c3 --mask frozen_n_65536_k_32768 --batch 4096 --reps 5
bash tools/profile_gpu.sh r02a_c5 --mask frozen_n_262144_k_131072 --batch 512 --reps 5
echo "profiles ok"
