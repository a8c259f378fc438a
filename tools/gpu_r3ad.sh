set -o pipefail
# round-3 final check of the current build: smoke, default bench (C2, with cpu_baseline),
# medians of 5 x 20 steps for C2 / sprot / ref, C3, the 2-rank gloo rehearsal of --gpus 2
O=$PWD/gpurun_out/r3ad
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/c2_default.json 2> $O/c2_default.err || { tail -20 $O/c2_default.err; exit 1; }
cat $O/c2_default.json
b() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$tag $*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2 3 4 5; do b c2 --steps 20 --warmup 3 || exit 1; b sprot --config sprot --steps 20 --warmup 3 || exit 1; b ref --config ref --steps 20 --warmup 3 || exit 1; done
b c3 --config c3 --steps 10 --warmup 2 || exit 1
SSA_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/gloo2.json 2> $O/gloo2.err || { tail -20 $O/gloo2.err; exit 1; }
cat $O/gloo2.json
