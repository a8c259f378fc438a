set -o pipefail
bash tools/r5_runs.sh tests "long or gate or timeline or fullsize or batch" && \
bash tools/r5_runs.sh kgap order && \
bash tools/r5_runs.sh kgap order_sprot --config sprot && \
bash tools/r5_runs.sh ab order_sprot sprot "" "" 2
