set -o pipefail
O=$PWD/gpurun_out/r3h
mkdir -p $O
for opt in "pair_parts=2" "pair_parts=1"; do
for nq in 16 8; do
timeout -k 10 400 python -u tools/batch_bench.py --qlen 64 100 --nq $nq --reps 2 --option $opt >> $O/batch.txt 2> $O/batch.err || { tail -20 $O/batch.err; exit 1; }
done; done
cat $O/batch.txt
