#!/bin/bash
# A/B of the root-op channel staging (POLAR_SC_ROOT_STAGE) on C3 / C5 timing and the C3
# per-op monitor at batch 4096 and 8. usage: bash tools/ab_root_stage.sh <tag>
set -o pipefail
TAG=${1:?tag}
for rs in 1 0; do
  POLAR_SC_ROOT_STAGE=$rs timeout -k 10 200 python -u tools/wpg_sweep.py --mask frozen_n_65536_k_32768 --batches 4096 --wpg 4 --reps 5 >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  POLAR_SC_ROOT_STAGE=$rs timeout -k 10 200 python -u tools/wpg_sweep.py --mask frozen_n_262144_k_131072 --batches 512 --wpg 8 --reps 3 >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  POLAR_SC_ROOT_STAGE=$rs timeout -k 10 120 python -u tools/monitor_run.py frozen_n_65536_k_32768 --batch 4096 > gpurun_out/${TAG}_mon_rs${rs}.txt 2>&1 || exit 1
  POLAR_SC_ROOT_STAGE=$rs timeout -k 10 120 python -u tools/monitor_run.py frozen_n_65536_k_32768 --batch 8 > gpurun_out/${TAG}_mon8_rs${rs}.txt 2>&1 || exit 1
  echo "rs=$rs done"
done
grep -v amdgpu gpurun_out/${TAG}_ab.log
