set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "rare_code_merge or sp25 or sprot or tie_band or candidate_count or strip_part or fused or pair_np or kat" > gpurun_out/r5/merge_tests.log 2>&1 || { tail -60 gpurun_out/r5/merge_tests.log; exit 1; }
tail -3 gpurun_out/r5/merge_tests.log
REPS=2 bash tools/r5_runs.sh libab floors c2 c3 ref sprot && \
bash tools/r5_runs.sh ab merge_sprot sprot "" "--option rare_merge=0" 2 && \
bash tools/r5_runs.sh ab split_ref_first50 ref "--option pair_split=50" "" 2 && \
bash tools/r5_runs.sh ab split_ref_last50 ref "--option pair_split=-50" "" 2
