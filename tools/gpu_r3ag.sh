set -o pipefail
# round-3 kernel: C2 and sprot wave timelines (launch ramp/tail), then option re-check, same box alternating
O=$PWD/gpurun_out/r3ag
mkdir -p $O
b() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$tag $*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
b tl --steps 20 --warmup 3 --timeline $O/tl_c2.npy || exit 1
b tl --config sprot --steps 20 --warmup 3 --timeline $O/tl_sprot.npy || exit 1
python tools/timeline.py $O/tl_c2.npy > $O/timeline_c2.txt 2>&1 || true
python tools/timeline.py $O/tl_sprot.npy > $O/timeline_sprot.txt 2>&1 || true
for i in 1 2; do
  for p in 50 40 60; do b lsp$p --config sprot --steps 20 --warmup 3 --option long_share_pct=$p || exit 1; done
  for p in 0 1; do b parts$p --steps 20 --warmup 3 --option pair_parts=$p || exit 1; done
done
