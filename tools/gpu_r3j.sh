set -o pipefail
O=$PWD/gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch or strip_parts or fullsize_matches_reference_hash" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for c in c2 ref sprot c3; do for p in 1 2 1 2; do b --config $c --steps 20 --warmup 3 --option pair_parts=$p || exit 1; done; done
for p in 1 2; do b --qlen 64 --steps 20 --warmup 3 --option pair_parts=$p || exit 1; b --qlen 100 --steps 20 --warmup 3 --option pair_parts=$p || exit 1; b --qlen 200 --steps 20 --warmup 3 --option pair_parts=$p || exit 1; done
PASSES="fetch write" bash tools/profile_pmc.sh $O/pmc_c2 || exit 1
python tools/pmc_summary.py $O/pmc_c2 | grep pair
