set -o pipefail
bash tools/r5_runs.sh tests "gate or long16" && \
bash tools/r5_runs.sh kgap g50_sprot --config sprot --option long_gate=50 && \
bash tools/r5_runs.sh kgap g100_sprot --config sprot && \
bash tools/r5_runs.sh kgap spin --option sync_spin=1 && \
bash tools/r5_runs.sh kgap nospin && \
bash tools/r5_runs.sh ab g50_sprot sprot "" "--option long_gate=50" 3
