set -o pipefail
bash tools/r5_runs.sh tests && \
bash tools/r5_runs.sh medians && \
bash tools/r5_runs.sh final
