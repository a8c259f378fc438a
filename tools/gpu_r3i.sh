# round 3: full GPU suite, C2 default bench (3x), ref/sprot (5x each), PMC C2 + C3
set -o pipefail
O=$PWD/gpurun_out/r3i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/c2_full.json 2> $O/c2_full.err || { tail -20 $O/c2_full.err; exit 1; }
cut -c1-400 $O/c2_full.json
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do b --steps 20 --warmup 5 || exit 1; done
for i in 1 2 3 4 5; do b --config ref --steps 20 --warmup 5 || exit 1; done
for i in 1 2 3 4 5; do b --config sprot --steps 20 --warmup 5 || exit 1; done
for i in 1 2; do b --config c3 --steps 10 --warmup 2 || exit 1; done
PASSES="stats fetch write valu lds" bash tools/profile_pmc.sh $O/pmc_c2 || exit 1
PASSES="stats fetch write valu" bash tools/profile_pmc.sh $O/pmc_c3 --config c3 || exit 1
python tools/pmc_summary.py $O/pmc_c2 > $O/pmc_c2.txt; python tools/pmc_summary.py $O/pmc_c3 > $O/pmc_c3.txt
