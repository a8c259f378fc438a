set -o pipefail
bash tools/r5_runs.sh tests && \
bash tools/r5_runs.sh ab filter_host2 c2 "--option filter_host=2" "--option filter_host=0" 3 && \
bash tools/r5_runs.sh ab sprot_np16 sprot "--pair-np 16" "" 2 && \
bash tools/r5_runs.sh ab rowdrop_c2 c2 "" "" 1
