set -o pipefail
bash tools/r5_runs.sh kgap lean && \
bash tools/r5_runs.sh kgap nolean --option lean_events=0 && \
bash tools/r5_runs.sh ab np16_sprot sprot "" "--pair-np 16" 2 && \
REPS=1 bash tools/r5_runs.sh sprot_decomp && \
PASSES="stats valu lds" bash tools/profile_pmc.sh gpurun_out/r5/pmc_final/c2 --config c2 && \
PASSES="stats valu lds" bash tools/profile_pmc.sh gpurun_out/r5/pmc_final/c3 --config c3 && \
python3 tools/pmc_shapes.py gpurun_out/r5/pmc_final/c2 gpurun_out/r5/pmc_final/c3 2>&1 | tail -8
