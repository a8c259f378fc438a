set -o pipefail
O=$PWD/gpurun_out/r3n
mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
t() { n=$1; shift; b "$@" --timeline $O/tl_$n.npy && python tools/timeline.py $O/tl_$n.npy > $O/tl_$n.txt && sed -n 1,7p $O/tl_$n.txt; }
t sprot --config sprot --steps 10 --warmup 3 || exit 1
t sprot_parts1 --config sprot --steps 10 --warmup 3 --option pair_parts=1 || exit 1
t sprot_noticket --config sprot --steps 10 --warmup 3 --option pair_ticket=0 || exit 1
t ref --config ref --steps 10 --warmup 3 || exit 1
t sprot_lg0 --config sprot --steps 10 --warmup 3 --option long_groups=0 || exit 1
b --config sprot --steps 10 --warmup 3 --alphabet bg20 || exit 1
b --config sprot --steps 10 --warmup 3 --option pair_np=16 || exit 1
