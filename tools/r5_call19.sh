set -o pipefail
bash tools/r5_runs.sh tests "upload_kernel or batch or multiview or filter_candidate" && \
bash tools/r5_runs.sh kgap upk --option upload_kernel=1 && \
bash tools/r5_runs.sh kgap upk_fh3 --option upload_kernel=1 --option filter_host=3 && \
bash tools/r5_runs.sh kgap base && \
bash tools/r5_runs.sh ab upk_c2 c2 "" "--option upload_kernel=1 --option filter_host=3" 3
