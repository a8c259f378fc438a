set -o pipefail
bash tools/r5_runs.sh kgap unread && \
bash tools/r5_runs.sh kgap unread_sprot --config sprot && \
bash tools/r5_runs.sh ab unread_c2 c2 "" "" 2
