# round 3, first GPU pass: parity tests, C2 bench, gloo 2-rank rehearsal,
# strip-part sweeps (C2, ref, sprot)
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
cut -c1-700 $O/c2.json
SSA_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > $O/gloo2.json 2> $O/gloo2.err || { tail -20 $O/gloo2.err; exit 1; }
cat $O/gloo2.json
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for p in 1 2 3 4 1 2 3 4; do b --steps 20 --warmup 3 --option pair_parts=$p || exit 1; done
for p in 1 2 3 4; do b --config ref --steps 20 --warmup 3 --option pair_parts=$p || exit 1; done
for p in 1 2 3 4; do b --config sprot --steps 20 --warmup 3 --option pair_parts=$p || exit 1; done
for p in 1 2 3 5; do b --config c3 --steps 10 --warmup 2 --option pair_parts=$p || exit 1; done
