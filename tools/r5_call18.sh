set -o pipefail
bash tools/r5_runs.sh tests "nw or NW" && \
REPS=3 bash tools/r5_runs.sh libab nwnop c3
