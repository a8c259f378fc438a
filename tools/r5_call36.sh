set -o pipefail
mkdir -p gpurun_out/r5/last
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/last/smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py > gpurun_out/r5/last/bench.json 2> gpurun_out/r5/last/bench.err
