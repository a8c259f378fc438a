set -o pipefail
bash tools/r5_runs.sh kgap pj0 && \
bash tools/r5_runs.sh kgap pj1 --option probe_join=1 && \
bash tools/r5_runs.sh kgap pj2 --option probe_join=2 && \
bash tools/r5_runs.sh kgap pj3 --option probe_join=3 && \
bash tools/r5_runs.sh kgap pj0b
