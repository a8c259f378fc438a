set -o pipefail
bash tools/r5_runs.sh tests "tail_strip or query_length_edges or fullsize or long16_kernel_vs or tie_band" && \
bash tools/r5_runs.sh ab tail4_sprot sprot "" "--option tail_rows4=0" 3 && \
bash tools/r5_runs.sh ab tail4_ref ref "" "--option tail_rows4=0" 2 && \
bash tools/r5_runs.sh ab prio_sprot sprot "" "--option long_prio=0" 2
