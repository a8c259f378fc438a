#!/bin/bash
# filter / strip-part / batch tests, then the API trace and two C2 benches
set -o pipefail
mkdir -p gpurun_out/r4/post
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu \
    -k "filter or part or batch or fullsize_matches_reference_hash" > gpurun_out/r4/post/tests.log 2>&1 || { tail -30 gpurun_out/r4/post/tests.log; exit 1; }
tail -2 gpurun_out/r4/post/tests.log
bash tools/r4/api_trace.sh || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-north-star > gpurun_out/r4/post/c2_$i.json 2> gpurun_out/r4/post/c2_$i.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r4/post/c2_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel']['kernel_gcups'], d['host_ms'], d.get('topk_vs_reference'))"
done
