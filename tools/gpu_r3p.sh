set -o pipefail
O=$PWD/gpurun_out/r3p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "six_waves or strip_parts or sprot" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do
b --config sprot --steps 10 --warmup 3 --option pair_waves=4 || exit 1
b --config sprot --steps 10 --warmup 3 || exit 1
done
b --config sprot --steps 10 --warmup 3 --option pair_waves=6 --option pair_parts=1 || exit 1
b --config c2 --steps 10 --warmup 3 || exit 1
