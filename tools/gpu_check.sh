#!/bin/bash
# One GPU round trip: parity tests, then the given bench variants.
# usage (on the GPU box): bash tools/gpu_check.sh [tests|notests] "<bench args>" ...
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = "tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
shift
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star $a > gpurun_out/b$i.json 2> gpurun_out/b$i.err || { tail -20 gpurun_out/b$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b$i.json')); print('$a', d['value'], d['kernel']['name'], d['kernel']['avg_ms'], d['kernel']['kernel_gcups'], d['kernel']['wide_count'], d['kernel']['wide_ms_avg'], d['top_hit'], d.get('topk_vs_reference'))"
done
