set -o pipefail
bash tools/r5_runs.sh tests long16 && \
bash tools/r5_runs.sh ab l16w8_sprot sprot "" "--option long16_waves=8" 3 && \
bash tools/r5_runs.sh ab l16w8_c2 c2 "" "--option long16_waves=8" 2
