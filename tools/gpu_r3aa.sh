set -o pipefail
# 12-wave (SW) / 8-wave (NW) pair workgroups for 25-letter tables: targeted tests, full suite, sprot A/B
O=$PWD/gpurun_out/r3aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "large_table or strip_parts or pair_row_stream" > $O/t0.log 2>&1 || { tail -30 $O/t0.log; exit 1; }
tail -1 $O/t0.log
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
b() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$tag $*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do
  b auto --config sprot --steps 20 --warmup 3 || exit 1
  b w4 --config sprot --steps 20 --warmup 3 --option pair_waves=4 || exit 1
  b auto --config sprot --steps 20 --warmup 3 --algo nw || exit 1
  b w4 --config sprot --steps 20 --warmup 3 --algo nw --option pair_waves=4 || exit 1
done
b auto --steps 20 --warmup 3 || exit 1
