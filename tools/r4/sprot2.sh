#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python tools/r4/sprot_diag.py 5000 0 5000 0 > gpurun_out/r4/sprot_diag2.log 2>&1 || { tail -20 gpurun_out/r4/sprot_diag2.log; exit 1; }
grep ppm gpurun_out/r4/sprot_diag2.log
for opt in 5000 0; do
timeout -k 10 300 python bench.py --config sprot --steps 10 --warmup 3 --no-north-star --no-cpu-baseline --option rare_merge_ppm=$opt --option pair_parts=1 --timeline gpurun_out/r4/tl_sprot_$opt.npy > gpurun_out/r4/tl_sprot_$opt.json 2> gpurun_out/r4/tl_sprot_$opt.err || { tail -30 gpurun_out/r4/tl_sprot_$opt.err; exit 1; }
python tools/timeline.py gpurun_out/r4/tl_sprot_$opt.npy > gpurun_out/r4/tl_sprot_$opt.txt
head -30 gpurun_out/r4/tl_sprot_$opt.txt
done
