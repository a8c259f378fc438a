set -o pipefail
O=$PWD/gpurun_out/r3s
mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }; python -c "import json; d=json.load(open('$O/b.json')); print('$*', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['ms_per_step'], d.get('topk_vs_reference'))" | tee -a $O/sweep.txt; }
for i in 1 2 3 4 5; do b --config sprot --steps 20 --warmup 3 || exit 1; b --config ref --steps 20 --warmup 3 || exit 1; done
timeout -k 10 300 python bench.py > $O/c2_full.json 2> $O/c2_full.err || { tail -20 $O/c2_full.err; exit 1; }
cat $O/c2_full.json
bash tools/profile_pmc.sh $O/pmc_c2 || exit 1
python tools/pmc_summary.py $O/pmc_c2 > $O/pmc_c2_summary.txt || exit 1
cat $O/pmc_c2_summary.txt | head -30
