#!/bin/bash
# Round 3 check at HEAD: the whole -m gpu suite, smoke(), and the default bench line (C2
# headline + C3 / C5 / C5-share secondary entries + CPU baseline). Logs under gpurun_out/<tag>.
# usage: bash tools/gpu_r03_check.sh <tag> [skip-tests]
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
git_head=$(cat "$ROOT/.head" 2>/dev/null || echo unknown)
echo "head $git_head" > "$OUT/head.txt"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  echo "pytest ok"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  echo "smoke ok"
fi
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
