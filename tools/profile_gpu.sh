#!/bin/bash
# Profile the decode kernel on the GPU box: kernel-trace stats, SQ issue/stall counters,
# and HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes, per the gfx950 PMC slot
# limits). Usage: tools/profile_gpu.sh <tag> [prof_decode.py args...]
# Output: gpurun_out/prof_<tag>/{trace,sq1,sq2,fetch,write}/...
set -euo pipefail
TAG=${1:?tag}
shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
DRV=("$ROOT/tools/prof_decode.py" "$@")
run() {
    local name=$1
    shift
    timeout -k 10 240 rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- python3 "${DRV[@]}" \
        > "$OUT/$name.log" 2>&1
    echo "$name done"
}
run trace --kernel-trace --stats
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
