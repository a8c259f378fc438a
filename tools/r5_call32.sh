set -o pipefail
bash tools/r5_runs.sh medians && \
bash tools/r5_runs.sh rehearse
