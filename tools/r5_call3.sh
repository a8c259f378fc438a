set -o pipefail
bash tools/r5_runs.sh tests && \
bash tools/r5_runs.sh ab filter_host c2 "--option filter_host=1" "--option filter_host=0" 3 && \
bash tools/r5_runs.sh ab parts_c2 c2 "" "--option pair_parts=1" 2 && \
bash tools/r5_runs.sh ab parts_ref ref "" "--option pair_parts=1" 2 && \
bash tools/r5_runs.sh ab parts_sprot sprot "" "--option pair_parts=1" 2 && \
bash tools/r5_runs.sh ab parts_c3 c3 "" "--option pair_parts=1" 2 && \
bash tools/r5_runs.sh clock
