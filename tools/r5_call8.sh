set -o pipefail
bash tools/r5_runs.sh ab sync_spin c2 "" "--option sync_spin=0" 3 && \
bash tools/r5_runs.sh ab lean_events c2 "" "--option lean_events=1" 3 && \
bash tools/r5_runs.sh api_trace c2lean --option lean_events=1 && \
bash tools/r5_runs.sh tests
