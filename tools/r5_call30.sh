set -o pipefail
bash tools/r5_runs.sh tests "long16_kernel_vs or long_entries_without or fullsize or long_entry_kernel or strip_parts or query_length_edges or tie_band" && \
bash tools/r5_runs.sh kgap jp25 && \
bash tools/r5_runs.sh kgap jp0 --option join_poll=0 && \
bash tools/r5_runs.sh kgap jp25b && \
bash tools/r5_runs.sh kgap jp0b --option join_poll=0 && \
bash tools/r5_runs.sh kgap jp25_sprot --config sprot && \
bash tools/r5_runs.sh kgap jp0_sprot --config sprot --option join_poll=0
