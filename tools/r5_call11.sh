set -o pipefail
bash tools/r5_runs.sh tests "filter or rescore or batch or multiview or tier or long16 or long_entry or tie_band or boundary or edge" && \
bash tools/r5_runs.sh kgap lean2 && \
bash tools/r5_runs.sh kgap sprot2 --config sprot && \
bash tools/r5_runs.sh ab rows_sprot sprot "" "--option long16_rows=0" 3 && \
bash tools/r5_runs.sh ab rows_ref ref "" "--option long16_rows=0" 2
