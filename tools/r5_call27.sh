set -o pipefail
bash tools/r5_runs.sh tests "long16_kernel_vs" && \
bash tools/r5_runs.sh ab prio_sprot sprot "" "--option long_prio=0" 3 && \
bash tools/r5_runs.sh ab prio_c2 c2 "" "--option long_prio=0" 2
