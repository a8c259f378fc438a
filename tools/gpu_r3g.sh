set -o pipefail
O=$PWD/gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch or strip_parts or device_topk or multiview" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u tools/batch_bench.py --qlen 30 64 100 400 --nq 16 --reps 3 > $O/batch_sw.txt 2> $O/batch_sw.err || { tail -20 $O/batch_sw.err; exit 1; }
cat $O/batch_sw.txt
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_batch30 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/batch_bench.py --qlen 30 --nq 16 --reps 2 > $O/prof_batch30.log 2>&1 || { tail -20 $O/prof_batch30.log; exit 1; }
head -12 $O/prof_batch30/*/run_kernel_stats.csv 2>/dev/null || find $O/prof_batch30 -name "*stats*"
