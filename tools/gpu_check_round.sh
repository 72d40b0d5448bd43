#!/bin/bash
# One GPU call: the whole -m gpu suite, the default bench line, the VALU issue-rate probe and the
# profiles of tools/gpu_profile_round.sh. usage: bash tools/gpu_check_round.sh <tag>
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${1:?tag}_pytest.log 2>&1 && echo pytest ok &&
timeout -k 10 300 python -u bench.py > gpurun_out/${1:?tag}_bench_c2.json 2> gpurun_out/${1:?tag}_bench_c2.err && echo bench ok &&
timeout -k 10 120 ./build_tools/valu_rate_probe > gpurun_out/${1:?tag}_valu_rate.log 2>&1 && echo probe ok &&
bash tools/gpu_profile_round.sh ${1} && echo prof ok
