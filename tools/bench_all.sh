#!/bin/bash
# The BASELINE.json configurations at N = 1 (plus the reference's benchmark shape and
# its Swiss-Prot form), with the CPU baseline where it is cheap; one JSON line per
# config into gpurun_out/bench_all/<name>.json.
# usage (on the GPU box): bash tools/bench_all.sh
set -o pipefail
mkdir -p gpurun_out/bench_all
run() {   # name, args...
    local name=$1; shift
    timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_all/$name.json 2> gpurun_out/bench_all/$name.err || { tail -5 gpurun_out/bench_all/$name.err; return 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bench_all/$name.json').read().strip().splitlines()[-1]); c=d.get('cpu_baseline') or {}; print('$name', d['value'], d['kernel']['avg_ms'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'), d['roofline']['traffic'], c.get('value'), c.get('cores'))"
}
run c2 --steps 10 --no-north-star &&
run c3 --config c3 --steps 5 --no-north-star &&
run c4share --config c4 --seqs 1250000 --steps 10 --no-north-star &&
run c5share1m --config c5 --seqs 1000000 --steps 3 --no-cpu-baseline --no-north-star &&
run c5share --config c5 --seqs 6250000 --steps 2 --warmup 1 --no-north-star &&
run ref --config ref --steps 10 --no-cpu-baseline --no-north-star &&
run sprot --config sprot --steps 10 --no-cpu-baseline --no-north-star &&
run u28 --alphabet uniform28 --steps 10 --no-cpu-baseline --no-north-star &&
run c4full --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-north-star &&
run north_star --config north_star --steps 5 --warmup 1 --no-cpu-baseline --no-north-star &&
run c5 --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-north-star
