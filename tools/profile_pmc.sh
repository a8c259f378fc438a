#!/bin/bash
# Collects the rocprofv3 evidence for one bench configuration on the GPU box:
#   pass 0: --kernel-trace --stats (durations)
#   pass 1..: one --pmc group per run (counters never combined with tracing
#             domains other than --kernel-trace)
# Usage (on the box, from the repo root):
#   tools/profile_pmc.sh <out_dir> [bench args...]
# PASSES="stats fetch write" limits the passes (default: all)
set -e -o pipefail
OUT=$(realpath -m "$1"); shift
REPO=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-north-star $*"
PASSES=${PASSES:-"stats fetch write valu wait lds icache"}
run() {   # name, rocprof args...
    local name=$1; shift
    case " $PASSES " in *" $name "*) ;; *) return 0 ;; esac
    timeout -k 10 300 rocprofv3 "$@" --kernel-include-regex "strip|pair|long" -d "$OUT/$name" -o run --output-format csv \
        -- python3 "$REPO/bench.py" $ARGS > "$OUT/$name.log" 2>&1
}
run stats --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
run valu --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run wait --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run lds --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE
run icache --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SMEM
echo "profiles in $OUT"
