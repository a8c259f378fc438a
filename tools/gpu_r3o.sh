set -o pipefail
O=$PWD/gpurun_out/r3o
mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do
b --config sprot --steps 10 --warmup 3 --alphabet bg20 || exit 1
b --config sprot --steps 10 --warmup 3 || exit 1
b --config sprot --steps 10 --warmup 3 --option pair_np=16 || exit 1
done
