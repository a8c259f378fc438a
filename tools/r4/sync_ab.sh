#!/bin/bash
# host-side timing of a C2 search: trace lines, then sync_spin on/off A/B
set -o pipefail
mkdir -p gpurun_out/r4/sync
SSA_AMD_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/r4/sync/trace.json 2> gpurun_out/r4/sync/trace.err || exit 1
grep "trace:" gpurun_out/r4/sync/trace.err | tail -12
for i in 1 2 3; do
  for sp in 1 0; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --option sync_spin=$sp > gpurun_out/r4/sync/s${sp}_$i.json 2> gpurun_out/r4/sync/s${sp}_$i.err || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/r4/sync/s${sp}_$i.json').read().strip().splitlines()[-1]); print('spin $sp', d['value'], d['kernel']['kernel_gcups'], d['host_ms'])"
  done
done
