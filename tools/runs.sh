#!/bin/bash
# GPU runs, one function per run (the command lines the profiles and
# DESIGN.md cite; rounds 4-5 used tools/r4_runs.sh, tools/r5_runs.sh and
# one-off r5_call*.sh chains, now in git history).  Usage, on the GPU box
# from the repo root, several runs chained with &&:
#   RUN=r6 bash tools/runs.sh <name> [args] && bash tools/runs.sh <name2> ...
# Output goes under gpurun_out/$RUN (default r6).  Every GPU step runs under
# its own timeout; a failing step ends the function and the chain.
set -o pipefail
R=${RUN:-r6}

run_tests() (
    # the GPU parity suite (optionally -k filter as $1)
    mkdir -p gpurun_out/$R
    K=()
    [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
        > gpurun_out/$R/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$R/gpu_tests.log; exit 1; }
    tail -3 gpurun_out/$R/gpu_tests.log
)

run_bench() (
    # the default bench line (C2 + north_star + cpu_baseline)
    mkdir -p gpurun_out/$R
    timeout -k 10 600 python bench.py > gpurun_out/$R/default.json 2> gpurun_out/$R/default.err \
        || { tail -30 gpurun_out/$R/default.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$R/default.json')); c=d.get('cpu_baseline',{}); print(d['value'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'), d['north_star']['value'], d['north_star'].get('topk_vs_reference'), c.get('value'), c.get('one_thread_gcups'))"
)

run_rehearse() (
    # gloo rehearsals of the N > 1 line: 2 and 4 ranks on the one GPU
    mkdir -p gpurun_out/$R
    for n in 2 4; do
        SSA_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus $n --no-cpu-baseline \
            > gpurun_out/$R/gloo$n.json 2> gpurun_out/$R/gloo$n.err || { tail -30 gpurun_out/$R/gloo$n.err; exit 1; }
        python -c "import json; d=json.load(open('gpurun_out/$R/gloo$n.json')); print($n, d['value'], d.get('rehearsal'), d.get('topk_vs_reference'), json.dumps(d.get('ranks_split',{}).get('step_split_ms')), d['north_star'].get('topk_vs_reference'), json.dumps(d['north_star'].get('ranks_split',{}).get('step_split_ms')), json.dumps({x: d.get('drop_in',{}).get(x) for x in ('value','devices','slot_kernel_ms','step_split_ms','topk_vs_reference','vs_multi_process')}))"
    done
)

run_pmc_shapes() (
    # valu / lds / stats PMC passes for C2, the reference's benchmark shape
    # with its own scoring (BLOSUM50 -3/-1) and with BLOSUM62 -11/-1, and the
    # Swiss-Prot form: effective clock, VALU per cell, LDS conflicts
    for cfg in "c2:--config c2" "ref:--config ref" "ref_b62:--config ref --matrix blosum62 --gap-open -11 --gap-extend -1" "sprot:--config sprot"; do
        name=${cfg%%:*}; args=${cfg#*:}
        PASSES="stats valu lds" bash tools/profile_pmc.sh gpurun_out/$R/pmc/$name $args || exit 1
        echo "$name done"
    done
)

run_pmc_sprot() (
    # the Swiss-Prot form's factors on one box: stats/valu/lds passes of the
    # 20-letter ref shape, the 25-letter form without and with its length
    # tail, each 25-letter case also with the rare-code merge (three pair
    # workgroups per CU); summary by tools/pmc_shapes.py
    for cfg in "ref:--config ref" "notail:--config sprot --long-tail 0" \
               "notail_merge:--config sprot --long-tail 0 --option rare_merge=1" \
               "sprot:--config sprot" "sprot_merge:--config sprot --option rare_merge=1"; do
        name=${cfg%%:*}; args=${cfg#*:}
        PASSES="stats valu lds" bash tools/profile_pmc.sh gpurun_out/$R/pmc_sprot/$name $args || exit 1
        echo "$name done"
    done
    python3 tools/pmc_shapes.py gpurun_out/$R/pmc_sprot/* > gpurun_out/$R/pmc_sprot/summary.txt && cat gpurun_out/$R/pmc_sprot/summary.txt
)

run_medians() (
    # 5 x 20 steps of C2, ref, sprot (kernel and end-to-end TCUPS)
    mkdir -p gpurun_out/$R/medians
    for i in 1 2 3 4 5; do
        for cfg in c2 ref sprot; do
            timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-north-star --no-cpu-baseline \
                > gpurun_out/$R/medians/${cfg}_$i.json 2> gpurun_out/$R/medians/${cfg}_$i.err || { tail -20 gpurun_out/$R/medians/${cfg}_$i.err; exit 1; }
        done
    done
    python - <<'EOF'
import json, glob, os, statistics as st
R = os.environ.get("RUN", "r6")
for cfg in ("c2", "ref", "sprot"):
    v, k = [], []
    for f in sorted(glob.glob(f"gpurun_out/{R}/medians/{cfg}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        v.append(d["value"]); k.append(d["kernel"]["kernel_gcups"])
    print(cfg, "median end-to-end", st.median(v), "kernel", st.median(k), v)
EOF
)

run_ab() (
    # alternating A/B of bench options on one box: $1 = name, $2 = config,
    # $3 = option string A, $4 = option string B, $5 = repeats (default 3)
    mkdir -p gpurun_out/$R/ab/$1
    for i in $(seq 1 ${5:-3}); do
        for v in A B; do
            if [ $v = A ]; then o="$3"; else o="$4"; fi
            timeout -k 10 300 python bench.py --config $2 --steps 20 --warmup 3 --no-north-star --no-cpu-baseline $o \
                > gpurun_out/$R/ab/$1/${v}_$i.json 2> gpurun_out/$R/ab/$1/${v}_$i.err || { tail -20 gpurun_out/$R/ab/$1/${v}_$i.err; exit 1; }
            python -c "import json; d=json.loads(open('gpurun_out/$R/ab/$1/${v}_$i.json').read().strip().splitlines()[-1]); print('$1 $v$i', d['value'], d['kernel']['kernel_gcups'], d['ms_per_step'], d['kernel']['avg_ms'], d['host_ms']['search_call'], d['host_ms']['sync_wait'], d.get('topk_vs_reference'))"
        done
    done
)

run_clock() (
    # valu passes alternating between two configurations (effective clock)
    for i in 1 2; do
        for cfg in "ref:--config ref" "ref_b62:--config ref --matrix blosum62 --gap-open -11 --gap-extend -1"; do
            name=${cfg%%:*}; args=${cfg#*:}
            PASSES="valu" bash tools/profile_pmc.sh gpurun_out/$R/clock/${name}_$i $args || exit 1
            cp gpurun_out/$R/clock/${name}_$i/valu.log gpurun_out/$R/clock/${name}_$i/stats.log 2>/dev/null
        done
    done
)

run_api_trace() (
    # HIP API + kernel + copy trace of a short C2 run (bench args as $@): the
    # time between two searches' pair kernels (tools/api_gap.py).  No counters.
    OUT=$(realpath -m gpurun_out/$R/api${1:+_$1}); mkdir -p "$OUT"; shift
    REPO=$PWD
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d "$OUT" -o run --output-format csv \
        -- python3 "$REPO/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-north-star "$@" > "$OUT/bench.log" 2>&1
    python3 "$REPO/tools/api_gap.py" "$OUT" > "$OUT/gap.txt" && head -3 "$OUT/gap.txt"
)

run_libab() (
    # alternating A/B of two library builds: A = libssa_amd/lib (this tree),
    # B = libssa_amd/lib_ab; $1 = name, $2.. = configs, REPS (default 2)
    name=$1; shift
    mkdir -p gpurun_out/$R/libab/$name
    A=$PWD/libssa_amd/lib/libssa_amd.so
    B=$PWD/libssa_amd/lib_ab/libssa_amd.so
    for i in $(seq 1 ${REPS:-2}); do
        for cfg in "$@"; do
            for v in A B; do
                if [ $v = A ]; then L=$A; else L=$B; fi
                SSA_AMD_LIB=$L timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-north-star --no-cpu-baseline \
                    > gpurun_out/$R/libab/$name/${cfg}_${v}_$i.json 2> gpurun_out/$R/libab/$name/${cfg}_${v}_$i.err || { tail -20 gpurun_out/$R/libab/$name/${cfg}_${v}_$i.err; exit 1; }
                python -c "import json; d=json.loads(open('gpurun_out/$R/libab/$name/${cfg}_${v}_$i.json').read().strip().splitlines()[-1]); print('$name $cfg $v$i', d['value'], d['kernel']['kernel_gcups'], d['ms_per_step'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
            done
        done
    done
)

run_sprot_decomp() (
    # the Swiss-Prot form's factors, one at a time, on one box (2 rounds,
    # alternating), each with a wave timeline of one extra step
    mkdir -p gpurun_out/$R/sprot
    for i in $(seq 1 ${REPS:-2}); do
        for v in "sprot:--config sprot" "sprot_bg20:--config sprot --alphabet bg20" "sprot_notail:--config sprot --long-tail 0" "ref:--config ref" "c2_548k:--config c2 --seqs 548208" "c2:--config c2"; do
            name=${v%%:*}; args=${v#*:}
            timeout -k 10 300 python bench.py $args --steps 20 --warmup 3 --no-north-star --no-cpu-baseline \
                --timeline gpurun_out/$R/sprot/${name}_$i.npy > gpurun_out/$R/sprot/${name}_$i.json 2> gpurun_out/$R/sprot/${name}_$i.err \
                || { tail -20 gpurun_out/$R/sprot/${name}_$i.err; exit 1; }
            python -c "import json; d=json.loads(open('gpurun_out/$R/sprot/${name}_$i.json').read().strip().splitlines()[-1]); print('$name $i', d['value'], d['kernel']['kernel_gcups'], d['ms_per_step'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
        done
    done
)

run_kgap() (
    # kernel + copy trace only (no API trace: its own cost inflates the gap)
    # of 30 C2 searches: the median time from one pair kernel's end to the
    # next one's start.  $1 = name, bench args after it
    OUT=$(realpath -m gpurun_out/$R/kgap_$1); mkdir -p "$OUT"; shift
    REPO=$PWD
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT" -o run --output-format csv \
        -- python3 "$REPO/bench.py" --steps 30 --warmup 2 --no-cpu-baseline --no-north-star "$@" > "$OUT/bench.log" 2>&1
    python3 "$REPO/tools/api_gap.py" "$OUT" > "$OUT/gap.txt" && head -2 "$OUT/gap.txt"
)

run_htrace() (
    # host marks (SSA_AMD_TRACE) over a kernel + copy trace of 30 C2 searches:
    # tools/host_device_timeline.py.  $1 = name, bench args after it
    OUT=$(realpath -m gpurun_out/$R/htrace_$1); mkdir -p "$OUT"; shift
    REPO=$PWD
    cd /tmp && export TMPDIR=/tmp && export SSA_AMD_TRACE=1
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT" -o run --output-format csv \
        -- python3 "$REPO/bench.py" --steps 30 --warmup 2 --no-cpu-baseline --no-north-star "$@" > "$OUT/bench.log" 2> "$OUT/trace.log"
    python3 "$REPO/tools/host_device_timeline.py" "$OUT" "$OUT/trace.log" > "$OUT/timeline.txt" && cat "$OUT/timeline.txt"
)

run_nsslice() (
    # the north-star N = 8 rank-0 slice on one GPU (the first 1.25 M IDs of
    # the 10 M DB): end to end vs kernel (5 x 20 steps) and the kernel trace's
    # per-search gap
    mkdir -p gpurun_out/$R/nsslice
    for i in 1 2 3 4 5; do
        timeout -k 10 300 python bench.py --config north_star --seqs 1250000 --steps 20 --warmup 3 --no-north-star \
            --no-cpu-baseline "$@" > gpurun_out/$R/nsslice/run_$i.json 2> gpurun_out/$R/nsslice/run_$i.err \
            || { tail -20 gpurun_out/$R/nsslice/run_$i.err; exit 1; }
    done
    python - <<'PYEOF'
import json, glob, statistics as st, os
R = os.environ.get("RUN", "r6")
v, k = [], []
for f in sorted(glob.glob(f"gpurun_out/{R}/nsslice/run_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    v.append(d["value"]); k.append(d["kernel"]["kernel_gcups"])
print("nsslice median end-to-end", st.median(v), "kernel", st.median(k), "gap %", round(100 * (1 - st.median(v) / st.median(k)), 3), v)
PYEOF
)

run_refresh_pmc() (
    # this build's PMC figures for the bench lines' roofline (profiles/
    # traffic.json, keyed by workload and kernel-source hash): stats / fetch /
    # write / valu / lds passes of C2 and the north-star shard, filed under
    # $PDIR/pmc2 (default profiles/r06; copied back from gpurun_out by the
    # caller as well, with the same command)
    for cfg in "c2:--config c2" "north_star:--config north_star"; do
        name=${cfg%%:*}; args=${cfg#*:}
        PASSES="stats fetch write valu lds" bash tools/profile_pmc.sh gpurun_out/$R/pmc2/$name $args || exit 1
        P=${PDIR:-profiles/r06}/pmc2
        mkdir -p $P && rm -rf $P/$name && cp -r gpurun_out/$R/pmc2/$name $P/ || exit 1
        python3 tools/traffic_from_pmc.py $P/$name || exit 1
    done
)

run_nwshapes() (
    # NW on the reference's shape and the Swiss-Prot form (with and without
    # its tail, with the rare-code merge): per-kernel time under rocprofv3
    # --kernel-trace --stats
    for cfg in "ref_nw:--config ref --algo nw" "sprot_nw:--config sprot --algo nw" \
               "sprot_nw_notail:--config sprot --algo nw --long-tail 0" \
               "sprot_nw_merge:--config sprot --algo nw --option rare_merge=1"; do
        name=${cfg%%:*}; args=${cfg#*:}
        OUT=$(realpath -m gpurun_out/$R/nwshapes/$name); mkdir -p "$OUT"
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
            -- python3 "$OLDPWD/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-north-star $args > "$OUT/bench.json" 2> "$OUT/bench.err" ) || exit 1
        python3 - "$OUT" <<'PYEOF'
import csv, glob, json, sys
d = sys.argv[1]
b = json.loads(open(d + "/bench.json").read().strip().splitlines()[-1])
print(d.rsplit("/", 1)[1], b["value"], b["kernel"]["kernel_gcups"], b["kernel"]["name"], b["kernel"].get("strip_rows"), b.get("topk_vs_reference"))
for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0])):
    if float(r["Percentage"]) > 0.5:
        print("   ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Percentage"])
PYEOF
    done
)

run_kshapes() (
    # per-kernel time of any bench shapes under rocprofv3 --kernel-trace
    # --stats: SHAPES="name:bench args;name2:args2"
    IFS=';' read -ra CFGS <<< "$SHAPES"
    for cfg in "${CFGS[@]}"; do
        name=${cfg%%:*}; args=${cfg#*:}
        OUT=$(realpath -m gpurun_out/$R/kshapes/$name); mkdir -p "$OUT"
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
            -- python3 "$OLDPWD/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-north-star $args > "$OUT/bench.json" 2> "$OUT/bench.err" ) || exit 1
        python3 - "$OUT" <<'PYEOF'
import csv, glob, json, sys
d = sys.argv[1]
b = json.loads(open(d + "/bench.json").read().strip().splitlines()[-1])
print(d.rsplit("/", 1)[1], b["value"], b["kernel"]["kernel_gcups"], b["kernel"]["name"], b.get("topk_vs_reference"))
for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0])):
    if float(r["Percentage"]) > 1.0:
        print("   ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Percentage"])
PYEOF
    done
)

run_final() (
    # the default bench line (python bench.py: C2 headline, north_star,
    # cpu_baseline) under rocprofv3 --kernel-trace --stats: the summary whose
    # pair-kernel average the line's roofline must agree with
    OUT=$(realpath -m gpurun_out/$R/final); mkdir -p "$OUT"
    REPO=$PWD
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
        -- python3 "$REPO/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
    tail -1 "$OUT/bench.json" | cut -c1-400
)

"run_$@"
