set -o pipefail
bash tools/r5_runs.sh tests "filter or batch or multiview or upload_kernel or rescore or overflow_reroute" && \
bash tools/r5_runs.sh kgap cand && \
bash tools/r5_runs.sh kgap cand_sprot --config sprot
