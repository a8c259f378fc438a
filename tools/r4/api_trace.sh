#!/bin/bash
# HIP API + kernel + copy trace of a short C2 run: where the ~150 us between
# two searches' pair kernels go (host issue, filter, copies).  No counters.
set -e -o pipefail
OUT=$(realpath -m gpurun_out/r4/api); mkdir -p "$OUT"
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d "$OUT" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-north-star > "$OUT/bench.log" 2>&1
echo "api trace in $OUT"
