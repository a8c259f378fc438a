#!/bin/bash
# long-entry split threshold (option long_share_pct; long_groups=0: none) on ref, c2 at 548 k, c2, sprot
set -o pipefail
mkdir -p gpurun_out/r4/lsweep
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/lsweep/$n.json 2> gpurun_out/r4/lsweep/$n.err || { tail -20 gpurun_out/r4/lsweep/$n.err; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4/lsweep/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
}
if [ -n "$CFG" ]; then CFGLIST=("$CFG"); else CFGLIST=("ref --config ref" "c2s --config c2 --seqs 548208" "c2 --config c2" "sprot --config sprot"); fi
for cfg in "${CFGLIST[@]}"; do
  set -- $cfg; n=$1; shift
  for p in ${PCTS:-50 80 120 200}; do run ${n}_p$p "$@" --option long_share_pct=$p || exit 1; done
  [ -n "$PCTS" ] || run ${n}_none "$@" --option long_groups=0 || exit 1
done
