set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "rare_code_merge or sp25 or sprot or u28 or tie_band or residue_classes or candidate_count or strip_part or fused" > gpurun_out/r5/merge_tests.log 2>&1 || { tail -60 gpurun_out/r5/merge_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r5/merge_tests.log | tail -60 | cut -c1-150
bash tools/r5_runs.sh ab merge_sprot sprot "" "--option rare_merge=0" 3 && \
bash tools/r5_runs.sh ab split_ref_first50 ref "--option pair_split=50" "" 2 && \
bash tools/r5_runs.sh ab split_ref_last50 ref "--option pair_split=-50" "" 2 && \
bash tools/r5_runs.sh ab split_c2_first25 c2 "--option pair_split=25" "" 2
