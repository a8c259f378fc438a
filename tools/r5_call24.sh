set -o pipefail
bash tools/r5_runs.sh tests && \
bash tools/r5_runs.sh final && \
bash tools/r5_runs.sh kgap final2 && \
bash tools/r5_runs.sh kgap final2_r4seq --option lean_events=0 --option filter_prefix_regs=0 --option tier_defer=0 --option upload_kernel=0 && \
bash tools/r5_runs.sh medians
