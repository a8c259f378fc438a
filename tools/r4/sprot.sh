#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "rare_merge or sprot or sp25 or u28 or residue_classes" > gpurun_out/r4/rm_tests.log 2>&1 || { tail -60 gpurun_out/r4/rm_tests.log; exit 1; }
tail -2 gpurun_out/r4/rm_tests.log
for opt in 5000 0 5000 0; do
timeout -k 10 300 python bench.py --config sprot --steps 20 --warmup 3 --no-north-star --no-cpu-baseline --option rare_merge_ppm=$opt > gpurun_out/r4/sprot_$opt.json 2> gpurun_out/r4/sprot_$opt.err || { tail -30 gpurun_out/r4/sprot_$opt.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4/sprot_$opt.json').read().strip().splitlines()[-1]); print('sprot ppm $opt', d['value'], d['kernel']['kernel_gcups'], d['ms_per_step'], d.get('topk_vs_reference'))"
done
