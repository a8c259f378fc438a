set -o pipefail
# final full GPU suite on the round-3 tree, then the default bench line
O=$PWD/gpurun_out/r3af
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python bench.py > $O/c2_default.json 2> $O/c2_default.err || { tail -20 $O/c2_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/c2_default.json')); print(d['value'], d['kernel']['kernel_gcups'], d['topk_vs_reference'], d['roofline'])"
