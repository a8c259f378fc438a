#!/bin/bash
# A/B: pair_kernel workgroups of 4 waves (A) vs 6 waves (B, libssa_amd/lib_w6)
set -o pipefail
mkdir -p gpurun_out/r4/ab_w6
run() {  # name, lib, args
  local n=$1 lib=$2; shift 2
  SSA_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/ab_w6/$n.json 2> gpurun_out/r4/ab_w6/$n.err || { tail -20 gpurun_out/r4/ab_w6/$n.err; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4/ab_w6/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
}
A=$PWD/libssa_amd/lib/libssa_amd.so
B=$PWD/libssa_amd/lib_w6/libssa_amd.so
for i in 1 2; do
  for cfg in sprot c2 ref; do
    run ${cfg}_w4_$i $A --config $cfg && run ${cfg}_w6_$i $B --config $cfg || exit 1
  done
done
