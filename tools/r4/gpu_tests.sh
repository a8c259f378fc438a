#!/bin/bash
# round 4: the GPU suite (optionally a -k selection), then the given bench args
set -o pipefail
mkdir -p gpurun_out/r4
SEL=${1:-}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${SEL:+-k "$SEL"} > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4/gpu_tests.log
