set -o pipefail
# PMC of the pair-row-stream build vs the previous build (lib_ab) on C2: VALU, waits, LDS
O=$PWD/gpurun_out/r3w
mkdir -p $O
PASSES="valu wait lds" bash tools/profile_pmc.sh $O/new || exit 1
SSA_AMD_LIB=$PWD/libssa_amd/lib_ab/libssa_amd.so PASSES="valu wait lds" bash tools/profile_pmc.sh $O/base || exit 1
python tools/pmc_summary.py $O/new > $O/new_summary.txt || exit 1
python tools/pmc_summary.py $O/base > $O/base_summary.txt || exit 1
grep pair_kernel $O/new_summary.txt; grep pair_kernel $O/base_summary.txt
