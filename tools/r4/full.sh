#!/bin/bash
# round 4: the whole GPU suite, then C2 (+ north star), sprot x2, C5 whole at N = 1
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r4/full_tests.log 2>&1 || { tail -60 gpurun_out/r4/full_tests.log; exit 1; }
tail -2 gpurun_out/r4/full_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r4/c2.json 2> gpurun_out/r4/c2.err || { tail -30 gpurun_out/r4/c2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4/c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'), 'ns', d['north_star']['value'], d['north_star'].get('topk_vs_reference'))"
for i in 1 2; do
timeout -k 10 300 python bench.py --config sprot --steps 20 --warmup 3 --no-north-star --no-cpu-baseline > gpurun_out/r4/sprot$i.json 2> gpurun_out/r4/sprot$i.err || { tail -30 gpurun_out/r4/sprot$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4/sprot$i.json').read().strip().splitlines()[-1]); print('sprot', d['value'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'))"
done
timeout -k 10 900 python bench.py --config c5 --steps 2 --warmup 1 --no-north-star > gpurun_out/r4/c5_bench.json 2> gpurun_out/r4/c5_bench.err || { tail -30 gpurun_out/r4/c5_bench.err; exit 1; }
tail -1 gpurun_out/r4/c5_bench.json
