set -o pipefail
mkdir -p gpurun_out/r5/trace
SSA_AMD_TRACE=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-north-star > gpurun_out/r5/trace/bench.json 2> gpurun_out/r5/trace/trace.err
