set -o pipefail
bash tools/r5_runs.sh tests && \
bash tools/r5_runs.sh final && \
bash tools/r5_runs.sh kgap final4 && \
bash tools/r5_runs.sh kgap final4_sprot --config sprot
