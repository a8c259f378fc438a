# A/B: round-2 library vs current on C2 (same box, alternating), + timelines
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do
SSA_AMD_LIB=$PWD/libssa_amd/lib_r02/libssa_amd.so b --steps 20 --warmup 3 --timeline $O/tl_c2_r02_$i.npy || exit 1
b --steps 20 --warmup 3 --timeline $O/tl_c2_new_$i.npy || exit 1
done
b --config ref --steps 20 --warmup 3 --option pair_parts=2 --timeline $O/tl_ref_p2.npy || exit 1
