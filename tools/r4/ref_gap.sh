#!/bin/bash
# what separates the ref shape (548 k seqs, q 513, BLOSUM50 -3/-1) from C2 (1 M, q 400, BLOSUM62 -11/-1)
set -o pipefail
mkdir -p gpurun_out/r4/refgap
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/refgap/$n.json 2> gpurun_out/r4/refgap/$n.err || { tail -20 gpurun_out/r4/refgap/$n.err; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4/refgap/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['kernel'].get('name'))"
}
run ref --config ref &&
run ref_q480 --config ref --qlen 480 &&
run ref_q400 --config ref --qlen 400 &&
run ref_1m --config ref --seqs 1000000 &&
run ref_b62 --config ref --matrix blosum62 --gap-open -11 --gap-extend -1 &&
run c2_q513 --config c2 --qlen 513 &&
run c2_548k --config c2 --seqs 548208 &&
run c2 --config c2
