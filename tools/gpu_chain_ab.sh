#!/bin/bash
# Same-box A/B of the chain fusion (tuning chain_max = 1 vs automatic) on the pair kernel,
# two interleaved rounds, after the pair GPU tests.
# usage: bash tools/gpu_chain_ab.sh <tag>
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
[ "${2:-}" = "skip-tests" ] || timeout -k 10 600 python -u -m pytest tests/test_pair.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_pair.log" 2>&1
echo "pair tests ok"
for r in 1 2; do
  timeout -k 10 300 python -u tools/pair_ab.py --kernels 3 --configs c3,c5,c5_64 > "$OUT/ab_chain_r$r.jsonl" 2>> "$OUT/ab.err"
  timeout -k 10 300 python -u tools/pair_ab.py --kernels 3 --configs c3,c5,c5_64 --tuning chain_max=1 > "$OUT/ab_nochain_r$r.jsonl" 2>> "$OUT/ab.err"
done
echo "ab ok"
