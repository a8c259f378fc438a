set -o pipefail
bash tools/r5_runs.sh tests "long or gate or filter or batch or multiview or upload_kernel or staging or piped or fused" && \
bash tools/r5_runs.sh kgap devrel && \
bash tools/r5_runs.sh kgap devrel_sprot --config sprot && \
bash tools/r5_runs.sh ab devrel_sprot sprot "" "" 2 && \
bash tools/r5_runs.sh ab devrel_c2 c2 "" "" 2
