#!/bin/bash
# Pair kernel: GPU tests, then C3 / C5 timing (pair kernel only) and a C3 profile.
# usage: bash tools/gpu_pair_quick.sh <tag> [configs]
set -euo pipefail
TAG=${1:?tag}
CFGS=${2:-c3,c5,c5_64}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_pair.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_pair.log" 2>&1
echo "pair tests ok"
timeout -k 10 300 python -u tools/pair_ab.py --kernels 3 --configs "$CFGS" > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
echo "ab ok"
cd /tmp
export TMPDIR=/tmp
DRV="$ROOT/tools/prof_decode.py --mask frozen_n_65536_k_32768 --batch 4096 --reps 4 --tuning kernel=3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/sq" -o sq --output-format csv -- python3 $DRV > "$OUT/sq.log" 2>&1
echo "prof ok"
