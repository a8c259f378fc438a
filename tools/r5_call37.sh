set -o pipefail
bash tools/r5_runs.sh kgap pf0 && \
bash tools/r5_runs.sh kgap pf1 --option pair_first=1 && \
bash tools/r5_runs.sh kgap pf0b && \
bash tools/r5_runs.sh kgap pf1b --option pair_first=1 && \
bash tools/r5_runs.sh kgap pf0_sprot --config sprot && \
bash tools/r5_runs.sh kgap pf1_sprot --config sprot --option pair_first=1 && \
bash tools/r5_runs.sh ab pf_c2 c2 "--option pair_first=1" "" 4 && \
bash tools/r5_runs.sh ab pf_sprot sprot "--option pair_first=1" "" 3
