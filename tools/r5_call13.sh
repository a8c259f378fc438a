set -o pipefail
bash tools/r5_runs.sh ab share_sprot sprot "" "--option long_share_pct=100" 2 && \
bash tools/r5_runs.sh ab share2_sprot sprot "--option long_share_pct=200" "--option long_share_pct=25" 2 && \
mkdir -p gpurun_out/r5/sprot && \
timeout -k 10 300 python bench.py --config sprot --steps 10 --warmup 2 --no-north-star --no-cpu-baseline --option pair_parts=1 \
    --timeline gpurun_out/r5/sprot/sprot_noparts.npy > gpurun_out/r5/sprot/sprot_noparts.json 2> gpurun_out/r5/sprot/sprot_noparts.err && \
python3 tools/timeline.py gpurun_out/r5/sprot/sprot_noparts.npy | head -14
