#!/bin/bash
# wave timelines of the ref shape at long-split thresholds on both sides of a dip
set -o pipefail
mkdir -p gpurun_out/r4/tljag
for p in 50 52 54 58; do
  timeout -k 10 300 python bench.py --config ref --steps 5 --warmup 2 --no-north-star --no-cpu-baseline --option long_share_pct=$p --timeline gpurun_out/r4/tljag/p$p.npy > gpurun_out/r4/tljag/p$p.json 2> gpurun_out/r4/tljag/p$p.err || exit 1
  python tools/timeline.py gpurun_out/r4/tljag/p$p.npy > gpurun_out/r4/tljag/p$p.txt || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r4/tljag/p$p.json').read().strip().splitlines()[-1]); print('p$p', d['kernel']['kernel_gcups'])"
  grep -E "span|per SIMD" gpurun_out/r4/tljag/p$p.txt
done
