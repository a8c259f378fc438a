# PMC comparison of the round-2 pair kernel and the current one (C2)
set -o pipefail
O=$PWD/gpurun_out/r3e
mkdir -p $O
PASSES="stats valu wait icache" SSA_AMD_LIB=$PWD/libssa_amd/lib_r02/libssa_amd.so bash tools/profile_pmc.sh $O/r02 || exit 1
PASSES="stats valu wait icache" bash tools/profile_pmc.sh $O/new || exit 1
python tools/pmc_summary.py $O/r02 > $O/r02.txt 2>&1; python tools/pmc_summary.py $O/new > $O/new.txt 2>&1
cat $O/r02.txt $O/new.txt
