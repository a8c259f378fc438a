set -o pipefail
# pair_kernel variants, same box alternating: cur (HEAD), e4 SW prefetch distance 2 quads,
# e5 non-temporal row-buffer loads/stores, e6 both
O=$PWD/gpurun_out/r3y
mkdir -p $O
b() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$tag $*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for cfg in "--steps 20 --warmup 3" "--config c3 --steps 10 --warmup 2"; do
for i in 1 2; do
  b cur $cfg || exit 1
  for v in e4 e5 e6; do SSA_AMD_LIB=$PWD/libssa_amd/lib_$v/libssa_amd.so b $v $cfg || exit 1; done
done; done
