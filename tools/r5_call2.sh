set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 120 tools/ubench/lds_occ > gpurun_out/r5/lds_occ.txt 2>&1 || { cat gpurun_out/r5/lds_occ.txt; exit 1; }
cat gpurun_out/r5/lds_occ.txt
bash tools/r5_runs.sh tests && bash tools/r5_runs.sh bench && bash tools/r5_runs.sh pmc_shapes
