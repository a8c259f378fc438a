#!/bin/bash
# A/B of two library builds on the same box, alternating: $1 = name of B's lib dir under libssa_amd/
set -o pipefail
B=${1:-lib_ab}
mkdir -p gpurun_out/r4/ab
run() {  # name, lib, args
  local n=$1 lib=$2; shift 2
  SSA_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/ab/$n.json 2> gpurun_out/r4/ab/$n.err || { tail -20 gpurun_out/r4/ab/$n.err; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4/ab/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
}
A=$PWD/libssa_amd/lib/libssa_amd.so
BB=$PWD/libssa_amd/$B/libssa_amd.so
for i in 1 2 3; do
  for cfg in c2 c3 sprot; do
    run ${cfg}_new$i $A --config $cfg && run ${cfg}_old$i $BB --config $cfg || exit 1
  done
done
