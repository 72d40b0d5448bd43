#!/bin/bash
# GPU check after an interpreter / hybrid storage change: the HBM-scratch and hybrid parity
# tests first, then timing of C3 / C5 and the per-op monitor. usage: bash tools/gpu_hbm_check.sh <tag>
set -o pipefail
TAG=${1:?tag}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hybrid.py tests/test_monitor.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
echo tests ok
timeout -k 10 200 python -u tools/wpg_sweep.py --mask frozen_n_65536_k_32768 --batches 4096 --wpg 4 --reps 5 > gpurun_out/${TAG}_sweep.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/wpg_sweep.py --mask frozen_n_262144_k_131072 --batches 512,64 --wpg 8 --reps 3 >> gpurun_out/${TAG}_sweep.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/${TAG}_sweep.log
timeout -k 10 120 python -u tools/monitor_run.py frozen_n_65536_k_32768 --batch 4096 > gpurun_out/${TAG}_mon_c3.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/monitor_run.py frozen_n_262144_k_131072 --batch 512 > gpurun_out/${TAG}_mon_c5.txt 2>&1 || exit 1
echo monitor ok
