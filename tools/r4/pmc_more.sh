#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4/pmc
P=$PWD/tools/profile_pmc.sh
prof() {  # name, passes, bench args...
  local n=$1 passes=$2; shift 2
  PASSES="$passes" timeout -k 10 1000 bash $P gpurun_out/r4/pmc/$n "$@" > gpurun_out/r4/pmc/$n.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/r4/pmc/$n.log; return 1; }
  echo "ok $n"
}
prof c5share "stats fetch write" --config c5 --seqs 6250000 &&
prof c4full "stats fetch write" --config c4 &&
prof north_star "stats fetch write" --config north_star &&
prof c5 "stats fetch write" --config c5
