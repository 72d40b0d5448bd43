#!/bin/bash
# Pair-kernel check: its GPU parity tests, then the same-box hybrid / pair A/B.
# usage: bash tools/gpu_pair_check.sh <tag> [configs]
set -euo pipefail
TAG=${1:?tag}
CFGS=${2:-c3,c5,c5_64,n16384_4096,n4096_16384}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_pair.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_pair.log" 2>&1
echo "pair tests ok"
timeout -k 10 400 python -u tools/pair_ab.py --configs "$CFGS" > "$OUT/pair_ab.jsonl" 2> "$OUT/pair_ab.err"
echo "pair ab ok"
