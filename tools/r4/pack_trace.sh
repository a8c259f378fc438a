#!/bin/bash
# where DB packing time goes (trace lines), c4full and c5 setup
set -o pipefail
mkdir -p gpurun_out/r4/pack
for cfg in ${CFGS:-north_star c5}; do
  SSA_AMD_TRACE=1 timeout -k 10 400 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-north-star > gpurun_out/r4/pack/$cfg.json 2> gpurun_out/r4/pack/$cfg.err || exit 1
  grep "trace: pack" gpurun_out/r4/pack/$cfg.err
  python -c "import json; d=json.loads(open('gpurun_out/r4/pack/$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['setup'])"
done
