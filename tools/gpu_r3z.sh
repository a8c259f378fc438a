set -o pipefail
# full GPU suite on the non-temporal row-buffer build, then C2 / sprot / C3 benches
O=$PWD/gpurun_out/r3z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
b() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$tag $*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do b new --steps 20 --warmup 3 || exit 1; b new --config sprot --steps 20 --warmup 3 || exit 1; b new --config c3 --steps 10 --warmup 2 || exit 1; done
