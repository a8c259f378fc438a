set -o pipefail
O=$PWD/gpurun_out/r3k
mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'), d['config']['pair_strip_rows'])" | tee -a $O/sweep.txt; }
for i in 1 2; do
b --config sprot --steps 20 --warmup 3 || exit 1
b --config sprot --steps 20 --warmup 3 --pair-np 16 || exit 1
b --alphabet sprot25 --steps 20 --warmup 3 || exit 1
b --alphabet sprot25 --steps 20 --warmup 3 --pair-np 16 || exit 1
done
b --config c3 --long-tail 100 --steps 10 --warmup 2 || exit 1
python -c "import json; d=json.load(open('$O/b.json')); print('C3 long tail: value', d['value'], 'kernel', d['kernel']['kernel_gcups'], 'wide_ms', d['kernel']['wide_ms_avg'], d['host_ms'])"
