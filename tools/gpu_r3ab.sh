set -o pipefail
# rocprofv3 evidence of the current build on C2 (kernel trace + PMC passes), and C3
O=$PWD/gpurun_out/r3ab
mkdir -p $O
timeout -k 10 120 tools/ubench/bank_rates > $O/bank_rates.txt 2>&1 || { cat $O/bank_rates.txt; exit 1; }
cat $O/bank_rates.txt
mkdir -p $O
bash tools/profile_pmc.sh $O/pmc_c2 || exit 1
python tools/pmc_summary.py $O/pmc_c2 > $O/pmc_c2/summary.txt || exit 1
grep pair_kernel $O/pmc_c2/summary.txt
PASSES="stats fetch write valu" bash tools/profile_pmc.sh $O/pmc_c3 --config c3 || exit 1
python tools/pmc_summary.py $O/pmc_c3 > $O/pmc_c3/summary.txt || exit 1
grep pair_kernel $O/pmc_c3/summary.txt
