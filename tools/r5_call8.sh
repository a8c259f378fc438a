set -o pipefail
bash tools/r5_runs.sh ab sync_spin c2 "" "--option sync_spin=0" 3 && \
bash tools/r5_runs.sh api_trace c2spin && \
bash tools/r5_runs.sh tests
