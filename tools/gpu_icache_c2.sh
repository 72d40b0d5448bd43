#!/bin/bash
# Instruction-cache PMC of the C2 per-mask kernel, default vs the two-batch straight-line
# variant (POLAR_SC_MASK_DUAL=1): is the doubled code the cost of the dual kernel?
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/icc2
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
DRV="$ROOT/tools/prof_decode.py --mask FB_N1024_K512 --batch 65536 --reps 10"
PMC="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES"
[ "${1:-}" = clock ] || POLAR_SC_MASK_DUAL=0 timeout -s KILL 120 rocprofv3 --pmc $PMC -d "$OUT/single/ic" -o ic --output-format csv -- python3 $DRV > "$OUT/single.log" 2>&1
echo "single ok"
[ "${1:-}" = clock ] || POLAR_SC_MASK_DUAL=1 timeout -s KILL 120 rocprofv3 --pmc $PMC -d "$OUT/dual/ic" -o ic --output-format csv -- python3 $DRV > "$OUT/dual.log" 2>&1
echo "dual ok"
# clock: GRBM_GUI_ACTIVE per dispatch against the kernel-trace duration, both variants
for v in 0 1; do
  POLAR_SC_MASK_DUAL=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/clk$v/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/clk$v.trace.log" 2>&1
  POLAR_SC_MASK_DUAL=$v timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES -d "$OUT/clk$v/grbm" -o grbm --output-format csv -- python3 $DRV > "$OUT/clk$v.grbm.log" 2>&1
  echo "clock $v ok"
done
