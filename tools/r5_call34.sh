set -o pipefail
bash tools/r5_runs.sh tests "filter or topk or tie_band or fullsize or batch or multiview or sharded or driver_cuts or kat or golden" && \
mkdir -p gpurun_out/r5/trace && \
SSA_AMD_TRACE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-north-star > gpurun_out/r5/trace/bench_seed.json 2> gpurun_out/r5/trace/trace_seed.err && \
bash tools/r5_runs.sh kgap seed && \
bash tools/r5_runs.sh kgap seed_sprot --config sprot
