set -o pipefail
bash tools/r5_runs.sh tests && \
bash tools/r5_runs.sh final && \
bash tools/r5_runs.sh kgap final_lean && \
bash tools/r5_runs.sh kgap final_nolean --option lean_events=0 && \
bash tools/r5_runs.sh kgap final_r4seq --option lean_events=0 --option filter_prefix_regs=0 --option tier_defer=0
