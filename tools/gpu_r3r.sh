set -o pipefail
O=$PWD/gpurun_out/r3r
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
