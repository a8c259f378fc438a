#!/bin/bash
# where the reference-shape gap goes: alphabet, tail, rare merge (SW and NW), same box alternating
set -o pipefail
mkdir -p gpurun_out/r4/sprot3
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/sprot3/$n.json 2> gpurun_out/r4/sprot3/$n.err || { tail -20 gpurun_out/r4/sprot3/$n.err; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4/sprot3/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['ms_per_step'], d.get('topk_vs_reference'))"
}
for i in 1 2; do
run ref$i --config ref &&
run sprot_notail$i --config sprot --long-tail 0 &&
run sprot_notail_m0_$i --config sprot --long-tail 0 --option rare_merge_ppm=0 &&
run sprot$i --config sprot &&
run sprot_m0_$i --config sprot --option rare_merge_ppm=0 &&
run sprotnw$i --config sprot --algo nw &&
run sprotnw_m0_$i --config sprot --algo nw --option rare_merge_ppm=0 || exit 1
done
