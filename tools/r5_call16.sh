set -o pipefail
bash tools/r5_runs.sh medians && \
bash tools/r5_runs.sh rehearse && \
PASSES="stats valu lds fetch write" bash tools/profile_pmc.sh gpurun_out/r5/pmc_final2/c2 --config c2 && \
PASSES="stats valu" bash tools/profile_pmc.sh gpurun_out/r5/pmc_final2/sprot --config sprot && \
python3 tools/pmc_shapes.py gpurun_out/r5/pmc_final2/c2 gpurun_out/r5/pmc_final2/sprot 2>&1 | tail -4
