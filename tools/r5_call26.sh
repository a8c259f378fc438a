set -o pipefail
bash tools/r5_runs.sh tests && \
bash tools/r5_runs.sh final && \
bash tools/r5_runs.sh kgap final3 && \
bash tools/r5_runs.sh kgap final3_sprot --config sprot && \
bash tools/r5_runs.sh medians && \
bash tools/r5_runs.sh rehearse
