#!/bin/bash
# Pair-kernel iteration: GPU pair tests, same-box timing of C3 / C5 / C5-share (pair kernel),
# per-op stamps of C3 and the C5 64-frame share (build_tools/pair_stamps_*, built on the CPU).
# usage: bash tools/gpu_pair_iter.sh <tag> [bench]
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_pair.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_pair.log" 2>&1
echo "pair tests ok"
timeout -k 10 300 python -u tools/pair_ab.py --kernels 3 --configs c3,c5,c5_64,n16384_4096 > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
echo "ab ok"
for b in build_tools/pair_stamps_*; do
  case "$b" in *.hip) continue;; esac
  timeout -k 10 60 "./$b" > "$OUT/$(basename "$b").txt" 2>&1
done
echo "stamps ok"
if [ "${2:-}" = "bench" ]; then
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
  echo "bench ok"
fi
