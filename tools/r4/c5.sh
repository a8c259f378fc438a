#!/bin/bash
# round 4: the new tests (int32 tier, whole-DB fixtures incl. c5full, rare merge), bench c5 / sprot at N = 1
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "int32_rescore or rare_merge or large_db or sprot" > gpurun_out/r4/c5_tests.log 2>&1 || { tail -60 gpurun_out/r4/c5_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r4/c5_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --config sprot --steps 20 --warmup 3 --no-north-star --no-cpu-baseline > gpurun_out/r4/sprot$i.json 2> gpurun_out/r4/sprot$i.err || { tail -30 gpurun_out/r4/sprot$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4/sprot$i.json').read().strip().splitlines()[-1]); print('sprot', d['value'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'))"
done
timeout -k 10 900 python bench.py --config c5 --steps 2 --warmup 1 --no-north-star > gpurun_out/r4/c5_bench.json 2> gpurun_out/r4/c5_bench.err || { tail -30 gpurun_out/r4/c5_bench.err; exit 1; }
tail -1 gpurun_out/r4/c5_bench.json
