set -o pipefail
bash tools/r5_runs.sh tests "long16 or long_entry or overflow_reroute or rescore or filter" && \
bash tools/r5_runs.sh ab tier_c2 c2 "" "--option tier_defer=0" 2 && \
bash tools/r5_runs.sh ab rows2_sprot sprot "" "--option long16_rows=2" 3
