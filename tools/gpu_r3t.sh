set -o pipefail
# Session-start check on HEAD: full GPU suite, default bench, sprot bench
O=$PWD/gpurun_out/r3t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
cat $O/c2.json
timeout -k 10 300 python bench.py --no-cpu-baseline --config sprot --steps 20 --warmup 3 > $O/sprot.json 2> $O/sprot.err || { tail -20 $O/sprot.err; exit 1; }
cat $O/sprot.json
