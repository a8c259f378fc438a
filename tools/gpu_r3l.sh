set -o pipefail
O=$PWD/gpurun_out/r3l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "long_entry or fullsize_matches_reference_hash or overflow_counters_long" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do
SSA_AMD_LIB=$PWD/libssa_amd/lib_prev/libssa_amd.so b --config sprot --steps 20 --warmup 3 || exit 1
b --config sprot --steps 20 --warmup 3 || exit 1
SSA_AMD_LIB=$PWD/libssa_amd/lib_prev/libssa_amd.so b --config ref --steps 20 --warmup 3 || exit 1
b --config ref --steps 20 --warmup 3 || exit 1
done
b --config sprot --steps 20 --warmup 3 --timeline $O/tl_sprot.npy || exit 1
python tools/timeline.py $O/tl_sprot.npy | head -6
