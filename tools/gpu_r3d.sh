# A/B of pair-kernel variants on C2 (same box, alternating)
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2 3; do
for v in ${VARIANTS:-lib_r02 lib}; do
echo -n "$v " | tee -a $O/sweep.txt
SSA_AMD_LIB=$PWD/libssa_amd/$v/libssa_amd.so b --steps 20 --warmup 3 $BARGS || exit 1
done; done
