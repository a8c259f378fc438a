set -o pipefail
# cache-policy variants of the pair kernel, same box alternating: cur (row buffer nt loads + stores),
# f1 + pair-row stream loads nt, f2 row-buffer stores nt only, f3 row-buffer loads nt only
O=$PWD/gpurun_out/r3ac
mkdir -p $O
b() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$tag $*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for cfg in "--steps 20 --warmup 3" "--config c3 --steps 10 --warmup 2"; do
for i in 1 2; do
  b cur $cfg || exit 1
  for v in f1 f2 f3; do SSA_AMD_LIB=$PWD/libssa_amd/lib_$v/libssa_amd.so b $v $cfg || exit 1; done
done; done
