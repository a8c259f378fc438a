set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "rare_code_merge or sp25 or sprot or tie_band or long" > gpurun_out/r5/merge_tests.log 2>&1 || { tail -60 gpurun_out/r5/merge_tests.log; exit 1; }
tail -3 gpurun_out/r5/merge_tests.log
bash tools/r5_runs.sh ab merge_sprot2 sprot "" "--option rare_merge=0" 3 && \
bash tools/r5_runs.sh ab side_tier c2 "" "--option side_tier=0" 3 && \
bash tools/r5_runs.sh ab filter_host3 c2 "--option filter_host=3" "" 2 && \
bash tools/r5_runs.sh api_trace c2
