#!/bin/bash
# Instruction-cache PMC of the pair kernel at C5 (512 frames, the 64-frame share) and C3: do
# lone waves of straight-line subtree code stall on instruction fetch?
set -euo pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/r04_ic
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
PMC="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES"
for c in "c5 frozen_n_262144_k_131072 512 3" "c5b64 frozen_n_262144_k_131072 64 3" "c3 frozen_n_65536_k_32768 4096 4"; do
  set -- $c
  timeout -s KILL 120 rocprofv3 --pmc $PMC -d $OUT/$1 -o ic --output-format csv -- python3 $ROOT/tools/prof_decode.py --mask $2 --batch $3 --reps $4 > $OUT/$1.log 2>&1
  echo "$1 ok"
done
