#!/bin/bash
# Short end-of-session check at HEAD: the whole -m gpu suite, smoke(), the default bench line.
# usage: bash tools/gpu_final_check.sh <tag>
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "head $(cat "$ROOT/.head" 2>/dev/null || echo unknown)" > "$OUT/head.txt"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
echo "pytest ok"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke ok"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
