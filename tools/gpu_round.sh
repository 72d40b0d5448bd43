#!/bin/bash
# GPU measurement at HEAD (one script for every round; run from gpurun):
#   tests   -- the whole -m gpu suite and smoke()
#   bench   -- the default bench line (C2 headline + secondary entries + CPU baseline) and a
#              driver-shaped short run (--steps 20 --warmup 5)
#   prof    -- per config: kernel-trace stats, FETCH_SIZE and WRITE_SIZE (separate passes, the
#              gfx950 PMC slot limits), two SQ passes; tools/prof_decode.py records the launch
#              shape and code-object key each profile is of (bench.py reads traffic only for it)
#   benchprof -- bench.py itself under rocprofv3 --kernel-trace --stats, one config per run
#              (C2, C3, C5, C5 share; no secondary entries, so each trace holds one decode
#              kernel): the trace average next to the HIP-event kernel_ms of the same command
#   stamps  -- per-op s_memtime stamps of the pair kernels built by tools/pair_stamps.py
# usage: bash tools/gpu_round.sh <tag> <step> [<step> ...]
set -euo pipefail
TAG=${1:?tag}
shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "head $(cat "$ROOT/.head" 2>/dev/null || echo unknown)" > "$OUT/head.txt"
prof() {   # name mask batch reps [polar_sc_config fields]
  local name=$1 mask=$2 batch=$3 reps=$4 cfg=${5:-}
  local DRV="$ROOT/tools/prof_decode.py --mask $mask --batch $batch --reps $reps${cfg:+ --config $cfg}"
  ( cd /tmp && export TMPDIR=/tmp &&
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$name/trace" -o trace --output-format csv -- python3 $DRV > "$OUT/$name/trace.log" 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$name/fetch" -o fetch --output-format csv -- python3 $DRV > "$OUT/$name/fetch.log" 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/$name/write" -o write --output-format csv -- python3 $DRV > "$OUT/$name/write.log" 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d "$OUT/$name/sq1" -o sq1 --output-format csv -- python3 $DRV > "$OUT/$name/sq1.log" 2>&1 &&
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/$name/sq2" -o sq2 --output-format csv -- python3 $DRV > "$OUT/$name/sq2.log" 2>&1 )
  echo "$name profiled"
}
for step in "$@"; do
  case "$step" in
  tests)
    timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1
    echo "pytest ok"
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    echo "smoke ok" ;;
  bench)
    timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
    echo "bench ok"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_steps20.json" 2> "$OUT/bench_steps20.err"
    echo "bench steps20 ok" ;;
  prof)
    for c in "c2 FB_N1024_K512 65536 10" "c4share FB_N1024_K512 131072 10" "c3 frozen_n_65536_k_32768 4096 4" "c5 frozen_n_262144_k_131072 512 3" \
             "c5b64 frozen_n_262144_k_131072 64 3" "par16 frozen_n_16384_k_8192 4096 5" \
             "par64 frozen_n_16384_k_8192 4096 5 par=64" "q8 frozen_n_16384_k_14746 4096 5 llr_bits=8" \
             "q9 frozen_n_16384_k_8192 4096 5 llr_bits=9"; do
      set -- $c
      case " ${PROF_ONLY:-$1} " in *" $1 "*) ;; *) continue ;; esac   # PROF_ONLY="c2 c4share": a subset
      mkdir -p "$OUT/$1"
      prof "$@"
    done ;;
  benchprof)
    for c in "c2 --config c2" "c3 --config c3" "c5 --config c5" "c5b64 --config c5 --batch 64" \
             "c4share --config c2 --batch 131072"; do
      set -- $c
      name=$1; shift
      case " ${PROF_ONLY:-$name} " in *" $name "*) ;; *) continue ;; esac
      ( cd /tmp && export TMPDIR=/tmp &&
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/bench_$name" -o trace --output-format csv -- \
          python3 "$ROOT/bench.py" --no-secondary --no-ebn0-sweep --no-cpu-baseline "$@" \
          > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" )
      echo "bench $name traced"
    done ;;
  formats)
    # every swept datapath format on N = 16384 x 4096 frames (CA2 on the pair kernel), then the
    # C5 8-GPU share shape at LLR_BITS 9 (the solo layout)
    timeout -k 10 600 python -u tools/format_speed.py > "$OUT/format_speed.jsonl" 2> "$OUT/format_speed.err"
    timeout -k 10 300 python -u tools/format_speed.py --mask frozen_n_262144_k_131072 --frames 64 --steps 5 \
      --formats "16,1,1,9;16,1,0,9" > "$OUT/format_speed_c5b64_q9.jsonl" 2> "$OUT/format_speed_c5b64_q9.err"
    echo "formats ok" ;;
  layout)
    # pair vs solo around the automatic switch point (2 frames per SIMD = 2048 frames)
    timeout -k 10 900 python -u tools/layout_ab.py --steps 10 --rounds 2 \
      --configs "${LAYOUT_CONFIGS:-c3_2048,c3_3072,c3,c5_1024,c5_2048}" \
      --variants "layout=1;layout=2" > "$OUT/layout_ab.jsonl" 2> "$OUT/layout_ab.err"
    echo "layout ok" ;;
  stamps)
    for b in "$ROOT"/build_tools/pair_stamps_*; do
      case "$b" in *.hip) continue;; esac
      timeout -k 10 60 "$b" > "$OUT/$(basename "$b").txt" 2>&1
    done
    echo "stamps ok" ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all ok"
