set -o pipefail
bash tools/r5_runs.sh tests "long16 or long_entry or gate or timeline" && \
bash tools/r5_runs.sh ab gate_sprot sprot "" "--option long_gate=0" 3 && \
bash tools/r5_runs.sh ab gate_c2 c2 "" "--option long_gate=0" 2 && \
bash tools/r5_runs.sh kgap sprot_nogate --config sprot --option long_gate=0
