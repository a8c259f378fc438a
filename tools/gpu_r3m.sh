set -o pipefail
O=$PWD/gpurun_out/r3m
mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do
b --config sprot --steps 20 --warmup 3 --option long16=0 || exit 1
b --config sprot --steps 20 --warmup 3 || exit 1
b --config ref --steps 20 --warmup 3 --option long16=0 || exit 1
b --config ref --steps 20 --warmup 3 || exit 1
done
for s in 25 35 70; do
b --config sprot --steps 20 --warmup 3 --option long_share_pct=$s || exit 1
b --config ref --steps 20 --warmup 3 --option long_share_pct=$s || exit 1
done
b --config c2 --steps 20 --warmup 3 || exit 1
b --config sprot --steps 20 --warmup 3 --timeline $O/tl_sprot.npy || exit 1
python tools/timeline.py $O/tl_sprot.npy | head -8
