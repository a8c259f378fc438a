set -o pipefail
# every BASELINE.json configuration at N = 1 on the round-3 build (tools/bench_all.sh), + sprot and the 28-symbol DB
bash tools/bench_all.sh || exit 1
mkdir -p gpurun_out/bench_all
for a in "sprot --config sprot --steps 10 --no-cpu-baseline" "u28 --alphabet uniform28 --steps 10 --no-cpu-baseline"; do
  set -- $a; name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_all/$name.json 2> gpurun_out/bench_all/$name.err || { tail -5 gpurun_out/bench_all/$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_all/$name.json')); print('$name', d['value'], d['kernel']['avg_ms'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'))"
done
