#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4/tl
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-north-star --no-cpu-baseline --option pair_parts=1 --timeline gpurun_out/r4/tl/$n.npy "$@" > gpurun_out/r4/tl/$n.json 2> gpurun_out/r4/tl/$n.err || { tail -20 gpurun_out/r4/tl/$n.err; return 1; }
  python tools/timeline.py gpurun_out/r4/tl/$n.npy > gpurun_out/r4/tl/$n.txt && grep -E "peak|span" gpurun_out/r4/tl/$n.txt
}
run ref --config ref && run sprot_notail_m --config sprot --long-tail 0 && run c2 --config c2
