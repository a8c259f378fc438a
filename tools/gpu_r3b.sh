# round 3, second pass: fused batches (tests + batch bench), strip parts, timelines
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch or strip_parts or kat_public or counters_skipped" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u tools/batch_bench.py --qlen 30 64 100 400 --nq 16 --reps 3 > $O/batch_sw.txt 2> $O/batch_sw.err || { tail -20 $O/batch_sw.err; exit 1; }
cat $O/batch_sw.txt
timeout -k 10 300 python -u tools/batch_bench.py --algo nw --qlen 30 100 --nq 16 --reps 2 > $O/batch_nw.txt 2> $O/batch_nw.err || { tail -20 $O/batch_nw.err; exit 1; }
cat $O/batch_nw.txt
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for c in c2 ref sprot c3; do for p in 1 2 1 2; do b --config $c --steps 20 --warmup 3 --option pair_parts=$p || exit 1; done; done
b --steps 20 --warmup 3 --timeline $O/tl_c2.npy || exit 1
b --config ref --steps 20 --warmup 3 --timeline $O/tl_ref.npy || exit 1
b --config sprot --steps 20 --warmup 3 --timeline $O/tl_sprot.npy || exit 1
