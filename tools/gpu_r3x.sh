set -o pipefail
# Diagnostic variants of pair_kernel on C2 (timing only; e1-e3 give wrong scores):
#  e1: uniform pair-row address per column (no LDS bank conflicts)
#  e2: no row-buffer loads or stores
#  e3: no SW anti-diagonal maxima (12 fewer max3 per column)
O=$PWD/gpurun_out/r3x
mkdir -p $O
b() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$tag $*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2; do
  b cur --steps 20 --warmup 3 || exit 1
  for v in e1 e2 e3; do SSA_AMD_LIB=$PWD/libssa_amd/lib_$v/libssa_amd.so b $v --steps 20 --warmup 3 || exit 1; done
done
