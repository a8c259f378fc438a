#!/bin/bash
# round 4: rocprofv3 kernel-trace/stats + PMC passes (tools/profile_pmc.sh) for every
# bench_all configuration; outputs under gpurun_out/r4/pmc/<name>
set -o pipefail
mkdir -p gpurun_out/r4/pmc
P=$PWD/tools/profile_pmc.sh
prof() {  # name, passes, bench args...
  local n=$1 passes=$2; shift 2
  PASSES="$passes" timeout -k 10 900 bash $P gpurun_out/r4/pmc/$n "$@" > gpurun_out/r4/pmc/$n.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/r4/pmc/$n.log; return 1; }
  echo "ok $n"
}
prof c2 "stats fetch write valu wait lds" &&
prof c3 "stats fetch write valu lds" --config c3 &&
prof c4share "stats fetch write" --config c4 --seqs 1250000 &&
prof c5share1m "stats fetch write" --config c5 --seqs 1000000 &&
prof ref "stats fetch write" --config ref &&
prof sprot "stats fetch write" --config sprot
