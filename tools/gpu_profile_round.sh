#!/bin/bash
# One GPU call: rocprofv3 kernel-trace stats of the default bench command (C2), the PMC
# passes of tools/profile_gpu.sh for C2, and kernel-trace stats for the C3 / C5 hybrid kernel.
# usage: bash tools/gpu_profile_round.sh <tag>
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/bench_c2" -o bench_c2 --output-format csv \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
echo "bench c2 traced"
bash "$ROOT/tools/profile_gpu.sh" "${TAG}_c2" --reps 10
for c in c3 c5; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/bench_$c" -o bench_$c --output-format csv \
        -- python3 "$ROOT/bench.py" --config $c --no-cpu-baseline --steps 20 --warmup 5 \
        > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
    echo "bench $c traced"
done
