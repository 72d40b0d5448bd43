#!/bin/bash
# C3 profile at HEAD: kernel trace (tier launches), HBM traffic passes, per-op probe.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-c3p}
OUT=$ROOT/gpurun_out/$T
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
DRV="$ROOT/tools/prof_decode.py --mask frozen_n_65536_k_32768 --batch 4096 --reps 4"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/trace.log" 2>&1
echo "trace ok"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 $DRV > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 $DRV > "$OUT/write.log" 2>&1
echo "pmc ok"
cd "$ROOT"
timeout -k 10 200 python tools/op_latency_probe.py frozen_n_65536_k_32768 --batch 4096 --out $OUT/probe.json
echo "probe ok"
