#!/bin/bash
# C5 (64 frames) profile: kernel trace of the grid-tier launches, and instruction-fetch /
# wait counters of the single hybrid kernel (POLAR_SC_TIER_WORDS=0) when available.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/ic
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
DRV="$ROOT/tools/prof_decode.py --mask frozen_n_262144_k_131072 --batch 64 --reps 3 --rotate 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/trace.log" 2>&1
echo "trace ok"
C=""
for k in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU; do
  if grep -qw "$k" "$OUT/avail.txt"; then C="$C $k"; fi
done
echo "counters:$C" > "$OUT/counters.txt"
if [ -n "$C" ]; then
  POLAR_SC_TIER_WORDS=0 timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc" -o pmc --output-format csv -- python3 $DRV > "$OUT/pmc.log" 2>&1
fi
echo "pmc ok"
