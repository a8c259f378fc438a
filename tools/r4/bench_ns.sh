#!/bin/bash
# round 4: the default bench line (C2 + north_star) and a 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 400 python bench.py > gpurun_out/r4/default.json 2> gpurun_out/r4/default.err || { tail -30 gpurun_out/r4/default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4/default.json')); print(d['value'], d.get('topk_vs_reference'), json.dumps(d.get('north_star')))"
SSA_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/r4/gloo2.json 2> gpurun_out/r4/gloo2.err || { tail -30 gpurun_out/r4/gloo2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4/gloo2.json')); print(d['value'], d['n_gpus'], d.get('rehearsal'), d.get('topk_vs_reference'), json.dumps(d.get('north_star')))"
