#!/bin/bash
# Per-op latency A/B: hybrid vs plain interpreter, 8 vs 1 waves per group (C5 mask).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=${1:-ab}
mkdir -p gpurun_out
M=frozen_n_262144_k_131072
timeout -k 10 200 env POLAR_SC_WAVES_PER_GROUP=1 python tools/op_latency_probe.py $M --batch 512 --out gpurun_out/${T}_hyb_w1.json
timeout -k 10 300 env POLAR_SC_JIT=0 python tools/op_latency_probe.py $M --batch 512 --out gpurun_out/${T}_interp_w8.json
timeout -k 10 300 env POLAR_SC_JIT=0 POLAR_SC_WAVES_PER_GROUP=1 python tools/op_latency_probe.py $M --batch 512 --out gpurun_out/${T}_interp_w1.json
