set -o pipefail
bash tools/r5_runs.sh tests "filter or rescore or batch or multiview or tier or fullsize or tie_band" && \
bash tools/r5_runs.sh kgap lean2 && \
bash tools/r5_runs.sh kgap sprot2 --config sprot
