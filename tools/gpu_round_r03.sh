#!/bin/bash
# Round 3 measurement at HEAD: the whole -m gpu suite, smoke(), the default bench line (C2
# headline + C3 / C5 / C5-share secondary entries + CPU baseline), kernel-trace stats and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of every config, SQ passes of C2 and C3.
# usage: bash tools/gpu_round_r03.sh <tag> [skip-tests|tests] [c5ab]
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "head $(cat "$ROOT/.head" 2>/dev/null || echo unknown)" > "$OUT/head.txt"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  echo "pytest ok"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  echo "smoke ok"
fi
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_steps20.json" 2> "$OUT/bench_steps20.err"
echo "bench steps20 ok"
cd /tmp
export TMPDIR=/tmp
prof() {   # name mask batch reps
  local name=$1 mask=$2 batch=$3 reps=$4
  local DRV="$ROOT/tools/prof_decode.py --mask $mask --batch $batch --reps $reps"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$name/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/$name.trace.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$name/fetch" -o fetch --output-format csv -- python3 $DRV > "$OUT/$name.fetch.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/$name/write" -o write --output-format csv -- python3 $DRV > "$OUT/$name.write.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d "$OUT/$name/sq1" -o sq1 --output-format csv -- python3 $DRV > "$OUT/$name.sq1.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/$name/sq2" -o sq2 --output-format csv -- python3 $DRV > "$OUT/$name.sq2.log" 2>&1
  echo "$name profiled"
}
prof c2 FB_N1024_K512 65536 10
prof c3 frozen_n_65536_k_32768 4096 4
prof c5 frozen_n_262144_k_131072 512 3
prof c5b64 frozen_n_262144_k_131072 64 3
echo "all ok"
for b in "$ROOT"/build_tools/pair_stamps_*; do
  case "$b" in *.hip) continue;; esac
  timeout -k 10 60 "$b" > "$OUT/$(basename "$b").txt" 2>&1
done
echo "stamps ok"
if [ "${3:-}" = "c5ab" ]; then
  cd "$ROOT"
  for r in 1 2; do
    timeout -k 10 300 python -u tools/pair_ab.py --kernels 3 --configs c5,c5_64 > "$OUT/ab_default_r$r.jsonl" 2>> "$OUT/ab.err"
    timeout -k 10 300 python -u tools/pair_ab.py --kernels 3 --configs c5,c5_64 --tuning chain_max=1 > "$OUT/ab_nochain_r$r.jsonl" 2>> "$OUT/ab.err"
  done
  echo "c5 ab ok"
fi
