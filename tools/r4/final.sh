#!/bin/bash
# the default bench line, the same command under rocprofv3 --kernel-trace --stats, and smoke()
set -o pipefail
OUT=$PWD/gpurun_out/r4/final; mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json; echo
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $REPO/bench.py > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -20 $OUT/prof_bench.err; exit 1; }
cd $REPO
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
