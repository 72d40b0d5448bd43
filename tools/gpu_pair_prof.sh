#!/bin/bash
# Pair-kernel tuning sweep + C3 profile: pair_ab over tunings (pair kernel only), then a
# kernel trace, HBM traffic and SQ counter passes of the C3 decode.
# usage: bash tools/gpu_pair_prof.sh <tag> [tuning of the profiled plan]
set -euo pipefail
TAG=${1:?tag}
TUN=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
AB="timeout -k 10 300 python -u tools/pair_ab.py --kernels 3 --steps 10"
$AB --configs c3,c5,c5_64 > "$OUT/ab_default.jsonl" 2> "$OUT/ab.err"
$AB --configs c3 --tuning sub_words=128 > "$OUT/ab_c3_s128.jsonl" 2>> "$OUT/ab.err"
$AB --configs c3 --tuning tier_words=2048 > "$OUT/ab_c3_t2048.jsonl" 2>> "$OUT/ab.err"
$AB --configs c5,c5_64 --tuning tier_words=1024 > "$OUT/ab_c5_t1024.jsonl" 2>> "$OUT/ab.err"
$AB --configs c5,c5_64 --tuning tier_words=2048 > "$OUT/ab_c5_t2048.jsonl" 2>> "$OUT/ab.err"
echo "sweep ok"
cd /tmp
export TMPDIR=/tmp
DRV="$ROOT/tools/prof_decode.py --mask frozen_n_65536_k_32768 --batch 4096 --reps 4 --tuning kernel=3${TUN:+,$TUN}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/trace.log" 2>&1
echo "trace ok"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 $DRV > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 $DRV > "$OUT/write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/sq" -o sq --output-format csv -- python3 $DRV > "$OUT/sq.log" 2>&1
echo "pmc ok"
