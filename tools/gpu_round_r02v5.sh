#!/bin/bash
# Round 2 (v5) measurement at HEAD: GPU suite, bench lines (C2 headline with CPU baseline +
# Eb/N0 sweep; C3, C5, C5 64-frame share), kernel-trace stats and PMC traffic passes.
# usage: bash tools/gpu_round_r02v2.sh <tag> [skip-tests]
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  echo "pytest ok"
fi
timeout -k 10 400 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
echo "bench c2 ok"
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-ebn0-sweep > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
done
timeout -k 10 300 python bench.py --config c5 --batch 64 --steps 20 --warmup 5 --no-cpu-baseline --no-ebn0-sweep > "$OUT/bench_c5_b64.json" 2> "$OUT/bench_c5_b64.err"
echo "bench c3 c5 ok"
cd /tmp
export TMPDIR=/tmp
prof() {   # name mask batch reps
  local name=$1 mask=$2 batch=$3 reps=$4
  local DRV="$ROOT/tools/prof_decode.py --mask $mask --batch $batch --reps $reps"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$name/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/$name.trace.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$name/fetch" -o fetch --output-format csv -- python3 $DRV > "$OUT/$name.fetch.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/$name/write" -o write --output-format csv -- python3 $DRV > "$OUT/$name.write.log" 2>&1
  echo "$name profiled"
}
prof c2 FB_N1024_K512 65536 10
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d "$OUT/c2/sq1" -o sq1 --output-format csv -- python3 $ROOT/tools/prof_decode.py --mask FB_N1024_K512 --batch 65536 --reps 10 > "$OUT/c2.sq1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/c2/sq2" -o sq2 --output-format csv -- python3 $ROOT/tools/prof_decode.py --mask FB_N1024_K512 --batch 65536 --reps 10 > "$OUT/c2.sq2.log" 2>&1
echo "c2 sq ok"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/c2/tcc" -o tcc --output-format csv -- python3 $ROOT/tools/prof_decode.py --mask FB_N1024_K512 --batch 65536 --reps 10 > "$OUT/c2.tcc.log" 2>&1
echo "c2 tcc ok"
prof c3 frozen_n_65536_k_32768 4096 4
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/c3/tcc" -o tcc --output-format csv -- python3 $ROOT/tools/prof_decode.py --mask frozen_n_65536_k_32768 --batch 4096 --reps 4 > "$OUT/c3.tcc.log" 2>&1
echo "c3 tcc ok"
prof c5 frozen_n_262144_k_131072 512 3
prof c5b64 frozen_n_262144_k_131072 64 3
echo "all ok"
