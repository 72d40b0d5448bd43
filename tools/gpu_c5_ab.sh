#!/bin/bash
# Pair GPU tests, then same-box A/Bs at C5 / C5-share: chain fusion on / off, subtree size.
# usage: bash tools/gpu_c5_ab.sh <tag>
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_pair.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_pair.log" 2>&1
echo "pair tests ok"
AB="timeout -k 10 300 python -u tools/pair_ab.py --kernels 3"
for r in 1 2; do
  $AB --configs c3,c5,c5_64 > "$OUT/ab_default_r$r.jsonl" 2>> "$OUT/ab.err"
  $AB --configs c3,c5,c5_64 --tuning chain_max=1 > "$OUT/ab_nochain_r$r.jsonl" 2>> "$OUT/ab.err"
done
$AB --configs c5,c5_64 --tuning sub_words=128 > "$OUT/ab_s128.jsonl" 2>> "$OUT/ab.err"
$AB --configs c5,c5_64 --tuning sub_words=64 > "$OUT/ab_s64.jsonl" 2>> "$OUT/ab.err"
echo "ab ok"
