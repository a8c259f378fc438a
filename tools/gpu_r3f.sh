set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch or strip_parts" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
VARIANTS="lib_r02 lib_varH lib" bash tools/gpu_r3d.sh || exit 1
timeout -k 10 400 python -u tools/batch_bench.py --qlen 30 100 400 --nq 16 --reps 3 > $O/batch_sw.txt 2> $O/batch_sw.err || { tail -20 $O/batch_sw.err; exit 1; }
cat $O/batch_sw.txt
