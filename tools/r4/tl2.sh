#!/bin/bash
# wave timelines at the default settings (strip parts on): the launch tail of ref vs c2
set -o pipefail
mkdir -p gpurun_out/r4/tl2
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-north-star --no-cpu-baseline --timeline gpurun_out/r4/tl2/$n.npy "$@" > gpurun_out/r4/tl2/$n.json 2> gpurun_out/r4/tl2/$n.err || { tail -20 gpurun_out/r4/tl2/$n.err; return 1; }
  python tools/timeline.py gpurun_out/r4/tl2/$n.npy > gpurun_out/r4/tl2/$n.txt && grep -E "peak|span|per SIMD|per 10" gpurun_out/r4/tl2/$n.txt
}
run ref --config ref && run c2 --config c2 && run c5share1m --config c5 --seqs 1000000 --steps 2
