#!/bin/bash
# Same-box A/B of the large-N launch knobs (tier cut, waves per group, subtree size).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-ab}
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-ebn0-sweep --no-cpu-baseline"
run() { local name=$1; shift; local e=$1; shift; timeout -k 10 300 env $e $B "$@" > gpurun_out/${T}_$name.json; echo "$name"; }
run c3_tw2048 POLAR_SC_TIER_WORDS=2048 --config c3
run c5 POLAR_X=0 --config c5
run c5_tw2048 POLAR_SC_TIER_WORDS=2048 --config c5
run c5_b64 POLAR_X=0 --config c5 --batch 64
run c5_b64_tw2048 POLAR_SC_TIER_WORDS=2048 --config c5 --batch 64
run c5_sub32 POLAR_SC_SUB_WORDS=32 --config c5
