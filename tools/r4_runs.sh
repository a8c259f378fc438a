#!/bin/bash
# Round-4 GPU experiments, one function per run (the command lines the round-4
# profiles and DESIGN.md cite).  Usage, on the GPU box from the repo root:
#   bash tools/r4_runs.sh <name> [args]      names: ab ab_w6 api_trace bench_ns c5 final full gpu_tests long_sweep medians pack_trace pmc_all np_sweep parts3 parts3b parts3c pmc_more post_check prio ref_gap sprot sprot2 sprot3 sync_ab tl tl2 tl_jag
set -o pipefail

r4_ab() (
    # A/B of two library builds on the same box, alternating: $1 = name of B's lib dir under libssa_amd/
    B=${1:-lib_ab}
    mkdir -p gpurun_out/r4/ab
    run() {  # name, lib, args
      local n=$1 lib=$2; shift 2
      SSA_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/ab/$n.json 2> gpurun_out/r4/ab/$n.err || { tail -20 gpurun_out/r4/ab/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/ab/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
    }
    A=$PWD/libssa_amd/lib/libssa_amd.so
    BB=$PWD/libssa_amd/$B/libssa_amd.so
    for i in 1 2 3; do
      for cfg in c2 c3 sprot; do
        run ${cfg}_new$i $A --config $cfg && run ${cfg}_old$i $BB --config $cfg || exit 1
      done
    done
)

r4_ab_w6() (
    # A/B: pair_kernel workgroups of 4 waves (A) vs 6 waves (B, libssa_amd/lib_w6)
    mkdir -p gpurun_out/r4/ab_w6
    run() {  # name, lib, args
      local n=$1 lib=$2; shift 2
      SSA_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/ab_w6/$n.json 2> gpurun_out/r4/ab_w6/$n.err || { tail -20 gpurun_out/r4/ab_w6/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/ab_w6/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
    }
    A=$PWD/libssa_amd/lib/libssa_amd.so
    B=$PWD/libssa_amd/lib_w6/libssa_amd.so
    for i in 1 2; do
      for cfg in sprot c2 ref; do
        run ${cfg}_w4_$i $A --config $cfg && run ${cfg}_w6_$i $B --config $cfg || exit 1
      done
    done
)

r4_api_trace() (
    # HIP API + kernel + copy trace of a short C2 run: where the ~150 us between
    # two searches' pair kernels go (host issue, filter, copies).  No counters.
    OUT=$(realpath -m gpurun_out/r4/api); mkdir -p "$OUT"
    REPO=$PWD
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d "$OUT" -o run --output-format csv \
        -- python3 "$REPO/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-north-star > "$OUT/bench.log" 2>&1
    echo "api trace in $OUT"
)

r4_bench_ns() (
    # round 4: the default bench line (C2 + north_star) and a 2-rank gloo rehearsal
    mkdir -p gpurun_out/r4
    timeout -k 10 400 python bench.py > gpurun_out/r4/default.json 2> gpurun_out/r4/default.err || { tail -30 gpurun_out/r4/default.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4/default.json')); print(d['value'], d.get('topk_vs_reference'), json.dumps(d.get('north_star')))"
    SSA_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/r4/gloo2.json 2> gpurun_out/r4/gloo2.err || { tail -30 gpurun_out/r4/gloo2.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4/gloo2.json')); print(d['value'], d['n_gpus'], d.get('rehearsal'), d.get('topk_vs_reference'), json.dumps(d.get('north_star')))"
)

r4_c5() (
    # round 4: the new tests (int32 tier, whole-DB fixtures incl. c5full, rare merge), bench c5 / sprot at N = 1
    mkdir -p gpurun_out/r4
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "int32_rescore or rare_merge or large_db or sprot" > gpurun_out/r4/c5_tests.log 2>&1 || { tail -60 gpurun_out/r4/c5_tests.log; exit 1; }
    grep -E "PASS|FAIL" gpurun_out/r4/c5_tests.log
    for i in 1 2; do
    timeout -k 10 300 python bench.py --config sprot --steps 20 --warmup 3 --no-north-star --no-cpu-baseline > gpurun_out/r4/sprot$i.json 2> gpurun_out/r4/sprot$i.err || { tail -30 gpurun_out/r4/sprot$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4/sprot$i.json').read().strip().splitlines()[-1]); print('sprot', d['value'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'))"
    done
    timeout -k 10 900 python bench.py --config c5 --steps 2 --warmup 1 --no-north-star > gpurun_out/r4/c5_bench.json 2> gpurun_out/r4/c5_bench.err || { tail -30 gpurun_out/r4/c5_bench.err; exit 1; }
    tail -1 gpurun_out/r4/c5_bench.json
)

r4_final() (
    # the default bench line, the same command under rocprofv3 --kernel-trace --stats, and smoke()
    OUT=$PWD/gpurun_out/r4/final; mkdir -p $OUT
    timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    tail -c 600 $OUT/bench.json; echo
    REPO=$PWD
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $REPO/bench.py > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -20 $OUT/prof_bench.err; exit 1; }
    cd $REPO
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
    tail -1 $OUT/smoke.log
)

r4_full() (
    # round 4: the whole GPU suite, then C2 (+ north star), sprot x2, C5 whole at N = 1
    mkdir -p gpurun_out/r4
    timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r4/full_tests.log 2>&1 || { tail -60 gpurun_out/r4/full_tests.log; exit 1; }
    tail -2 gpurun_out/r4/full_tests.log
    timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r4/c2.json 2> gpurun_out/r4/c2.err || { tail -30 gpurun_out/r4/c2.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4/c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'), 'ns', d['north_star']['value'], d['north_star'].get('topk_vs_reference'))"
    for i in 1 2; do
    timeout -k 10 300 python bench.py --config sprot --steps 20 --warmup 3 --no-north-star --no-cpu-baseline > gpurun_out/r4/sprot$i.json 2> gpurun_out/r4/sprot$i.err || { tail -30 gpurun_out/r4/sprot$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4/sprot$i.json').read().strip().splitlines()[-1]); print('sprot', d['value'], d['kernel']['kernel_gcups'], d.get('topk_vs_reference'))"
    done
    timeout -k 10 900 python bench.py --config c5 --steps 2 --warmup 1 --no-north-star > gpurun_out/r4/c5_bench.json 2> gpurun_out/r4/c5_bench.err || { tail -30 gpurun_out/r4/c5_bench.err; exit 1; }
    tail -1 gpurun_out/r4/c5_bench.json
)

r4_gpu_tests() (
    # round 4: the GPU suite (optionally a -k selection), then the given bench args
    mkdir -p gpurun_out/r4
    SEL=${1:-}
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${SEL:+-k "$SEL"} > gpurun_out/r4/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4/gpu_tests.log; exit 1; }
    tail -3 gpurun_out/r4/gpu_tests.log
)

r4_long_sweep() (
    # long-entry split threshold (option long_share_pct; long_groups=0: none) on ref, c2 at 548 k, c2, sprot
    mkdir -p gpurun_out/r4/lsweep
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/lsweep/$n.json 2> gpurun_out/r4/lsweep/$n.err || { tail -20 gpurun_out/r4/lsweep/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/lsweep/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
    }
    if [ -n "$CFG" ]; then CFGLIST=("$CFG"); else CFGLIST=("ref --config ref" "c2s --config c2 --seqs 548208" "c2 --config c2" "sprot --config sprot"); fi
    for cfg in "${CFGLIST[@]}"; do
      set -- $cfg; n=$1; shift
      for p in ${PCTS:-50 80 120 200}; do run ${n}_p$p "$@" --option long_share_pct=$p || exit 1; done
      [ -n "$PCTS" ] || run ${n}_none "$@" --option long_groups=0 || exit 1
    done
)

r4_pack_trace() (
    # where DB packing time goes (trace lines), c4full and c5 setup
    mkdir -p gpurun_out/r4/pack
    for cfg in ${CFGS:-north_star c5}; do
      SSA_AMD_TRACE=1 timeout -k 10 400 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-north-star > gpurun_out/r4/pack/$cfg.json 2> gpurun_out/r4/pack/$cfg.err || exit 1
      grep "trace: pack" gpurun_out/r4/pack/$cfg.err
      python -c "import json; d=json.loads(open('gpurun_out/r4/pack/$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['setup'])"
    done
)

r4_pmc_all() (
    # round 4: rocprofv3 kernel-trace/stats + PMC passes (tools/profile_pmc.sh) for every
    # bench_all configuration; outputs under gpurun_out/r4/pmc/<name>
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
)

r4_pmc_more() (
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
)

r4_post_check() (
    # filter / strip-part / batch tests, then the API trace and two C2 benches
    mkdir -p gpurun_out/r4/post
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu \
        -k "filter or part or batch or fullsize_matches_reference_hash" > gpurun_out/r4/post/tests.log 2>&1 || { tail -30 gpurun_out/r4/post/tests.log; exit 1; }
    tail -2 gpurun_out/r4/post/tests.log
    r4_api_trace || exit 1
    for i in 1 2; do
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-north-star > gpurun_out/r4/post/c2_$i.json 2> gpurun_out/r4/post/c2_$i.err || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/r4/post/c2_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel']['kernel_gcups'], d['host_ms'], d.get('topk_vs_reference'))"
    done
)

r4_ref_gap() (
    # what separates the ref shape (548 k seqs, q 513, BLOSUM50 -3/-1) from C2 (1 M, q 400, BLOSUM62 -11/-1)
    mkdir -p gpurun_out/r4/refgap
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/refgap/$n.json 2> gpurun_out/r4/refgap/$n.err || { tail -20 gpurun_out/r4/refgap/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/refgap/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['kernel'].get('name'))"
    }
    run ref --config ref &&
    run ref_q480 --config ref --qlen 480 &&
    run ref_q400 --config ref --qlen 400 &&
    run ref_1m --config ref --seqs 1000000 &&
    run ref_b62 --config ref --matrix blosum62 --gap-open -11 --gap-extend -1 &&
    run c2_q513 --config c2 --qlen 513 &&
    run c2_548k --config c2 --seqs 548208 &&
    run c2 --config c2
)

r4_sprot() (
    # (historical: the rare-merge runs of profiles/r04/rare_merge; option rare_merge_ppm
    # left with the feature)
    mkdir -p gpurun_out/r4
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "rare_merge or sprot or sp25 or u28 or residue_classes" > gpurun_out/r4/rm_tests.log 2>&1 || { tail -60 gpurun_out/r4/rm_tests.log; exit 1; }
    tail -2 gpurun_out/r4/rm_tests.log
    for opt in 5000 0 5000 0; do
    timeout -k 10 300 python bench.py --config sprot --steps 20 --warmup 3 --no-north-star --no-cpu-baseline --option rare_merge_ppm=$opt > gpurun_out/r4/sprot_$opt.json 2> gpurun_out/r4/sprot_$opt.err || { tail -30 gpurun_out/r4/sprot_$opt.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r4/sprot_$opt.json').read().strip().splitlines()[-1]); print('sprot ppm $opt', d['value'], d['kernel']['kernel_gcups'], d['ms_per_step'], d.get('topk_vs_reference'))"
    done
)

r4_sprot2() (
    # (historical: the rare-merge runs of profiles/r04/rare_merge; option rare_merge_ppm
    # left with the feature)
    mkdir -p gpurun_out/r4
    timeout -k 10 300 python tools/sprot_diag.py 5000 0 5000 0 > gpurun_out/r4/sprot_diag2.log 2>&1 || { tail -20 gpurun_out/r4/sprot_diag2.log; exit 1; }
    grep ppm gpurun_out/r4/sprot_diag2.log
    for opt in 5000 0; do
    timeout -k 10 300 python bench.py --config sprot --steps 10 --warmup 3 --no-north-star --no-cpu-baseline --option rare_merge_ppm=$opt --option pair_parts=1 --timeline gpurun_out/r4/tl_sprot_$opt.npy > gpurun_out/r4/tl_sprot_$opt.json 2> gpurun_out/r4/tl_sprot_$opt.err || { tail -30 gpurun_out/r4/tl_sprot_$opt.err; exit 1; }
    python tools/timeline.py gpurun_out/r4/tl_sprot_$opt.npy > gpurun_out/r4/tl_sprot_$opt.txt
    head -30 gpurun_out/r4/tl_sprot_$opt.txt
    done
)

r4_sprot3() (
    # (historical: the rare-merge runs of profiles/r04/rare_merge; option rare_merge_ppm
    # left with the feature)
    # where the reference-shape gap goes: alphabet, tail, rare merge (SW and NW), same box alternating
    mkdir -p gpurun_out/r4/sprot3
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/sprot3/$n.json 2> gpurun_out/r4/sprot3/$n.err || { tail -20 gpurun_out/r4/sprot3/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/sprot3/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['ms_per_step'], d.get('topk_vs_reference'))"
    }
    for i in 1 2; do
    run ref$i --config ref &&
    run sprot_notail$i --config sprot --long-tail 0 &&
    run sprot_notail_m0_$i --config sprot --long-tail 0 --option rare_merge_ppm=0 &&
    run sprot$i --config sprot &&
    run sprot_m0_$i --config sprot --option rare_merge_ppm=0 &&
    run sprotnw$i --config sprot --algo nw &&
    run sprotnw_m0_$i --config sprot --algo nw --option rare_merge_ppm=0 || exit 1
    done
)

r4_sync_ab() (
    # host-side timing of a C2 search: trace lines, then sync_spin on/off A/B
    mkdir -p gpurun_out/r4/sync
    SSA_AMD_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-north-star > gpurun_out/r4/sync/trace.json 2> gpurun_out/r4/sync/trace.err || exit 1
    grep "trace:" gpurun_out/r4/sync/trace.err | tail -12
    for i in 1 2 3; do
      for sp in 1 0; do
        timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --option sync_spin=$sp > gpurun_out/r4/sync/s${sp}_$i.json 2> gpurun_out/r4/sync/s${sp}_$i.err || exit 1
        python -c "import json; d=json.loads(open('gpurun_out/r4/sync/s${sp}_$i.json').read().strip().splitlines()[-1]); print('spin $sp', d['value'], d['kernel']['kernel_gcups'], d['host_ms'])"
      done
    done
)

r4_tl() (
    mkdir -p gpurun_out/r4/tl
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-north-star --no-cpu-baseline --option pair_parts=1 --timeline gpurun_out/r4/tl/$n.npy "$@" > gpurun_out/r4/tl/$n.json 2> gpurun_out/r4/tl/$n.err || { tail -20 gpurun_out/r4/tl/$n.err; return 1; }
      python tools/timeline.py gpurun_out/r4/tl/$n.npy > gpurun_out/r4/tl/$n.txt && grep -E "peak|span" gpurun_out/r4/tl/$n.txt
    }
    run ref --config ref && run sprot_notail_m --config sprot --long-tail 0 && run c2 --config c2
)

r4_tl2() (
    # wave timelines at the default settings (strip parts on): the launch tail of ref vs c2
    mkdir -p gpurun_out/r4/tl2
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-north-star --no-cpu-baseline --timeline gpurun_out/r4/tl2/$n.npy "$@" > gpurun_out/r4/tl2/$n.json 2> gpurun_out/r4/tl2/$n.err || { tail -20 gpurun_out/r4/tl2/$n.err; return 1; }
      python tools/timeline.py gpurun_out/r4/tl2/$n.npy > gpurun_out/r4/tl2/$n.txt && grep -E "peak|span|per SIMD|per 10" gpurun_out/r4/tl2/$n.txt
    }
    run ref --config ref && run c2 --config c2 && run c5share1m --config c5 --seqs 1000000 --steps 2
)

r4_tl_jag() (
    # wave timelines of the ref shape at long-split thresholds on both sides of a dip
    mkdir -p gpurun_out/r4/tljag
    for p in 50 52 54 58; do
      timeout -k 10 300 python bench.py --config ref --steps 5 --warmup 2 --no-north-star --no-cpu-baseline --option long_share_pct=$p --timeline gpurun_out/r4/tljag/p$p.npy > gpurun_out/r4/tljag/p$p.json 2> gpurun_out/r4/tljag/p$p.err || exit 1
      python tools/timeline.py gpurun_out/r4/tljag/p$p.npy > gpurun_out/r4/tljag/p$p.txt || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/r4/tljag/p$p.json').read().strip().splitlines()[-1]); print('p$p', d['kernel']['kernel_gcups'])"
      grep -E "span|per SIMD" gpurun_out/r4/tljag/p$p.txt
    done
)

r4_np_sweep() (
    # pair-kernel strip height (bench --pair-np) on C2, C3 and the DNA C5 share
    mkdir -p gpurun_out/r4/np
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/np/$n.json 2> gpurun_out/r4/np/$n.err || { tail -20 gpurun_out/r4/np/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/np/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d['config'].get('pair_strip_rows'), d.get('topk_vs_reference'))"
    }
    for np_ in ${NPS:-0 24 32 36 40}; do
      run c5s_np$np_ --config c5 --seqs 1000000 --steps 3 --pair-np $np_ || exit 1
      run c2_np$np_ --config c2 --pair-np $np_ || exit 1
    done
)

r4_parts3() (
    # three strip parts: the parts tests, then pair_parts 3 against the default (2) on five shapes
    mkdir -p gpurun_out/r4/parts3
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
        -k "strip_part or batch_fused" > gpurun_out/r4/parts3/tests.log 2>&1 || { tail -30 gpurun_out/r4/parts3/tests.log; exit 1; }
    tail -1 gpurun_out/r4/parts3/tests.log
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps ${STEPS:-15} --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/parts3/$n.json 2> gpurun_out/r4/parts3/$n.err || { tail -20 gpurun_out/r4/parts3/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/parts3/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
    }
    for i in 1 2; do
      for cfg in ref sprot c2 c3; do
        run ${cfg}_p2_$i --config $cfg && run ${cfg}_p3_$i --config $cfg --option pair_parts=3 || exit 1
      done
    done
    run c5s_p2 --config c5 --seqs 1000000 --steps 3 && run c5s_p3 --config c5 --seqs 1000000 --steps 3 --option pair_parts=3 || exit 1
)

r4_parts3b() (
    # pair_parts 3 vs 2, repeated on the headline (C2) and the north-star DB
    mkdir -p gpurun_out/r4/parts3b
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/parts3b/$n.json 2> gpurun_out/r4/parts3b/$n.err || { tail -20 gpurun_out/r4/parts3b/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/parts3b/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
    }
    for i in 1 2 3 4; do
      run c2_p2_$i --steps 20 --option pair_parts=2 && run c2_p3_$i --steps 20 --option pair_parts=3 || exit 1
    done
    run ns_p2 --config north_star --steps 4 --option pair_parts=2 && run ns_p3 --config north_star --steps 4 --option pair_parts=3 || exit 1
    run c4s_p2 --config c4 --seqs 1250000 --steps 15 --option pair_parts=2 && run c4s_p3 --config c4 --seqs 1250000 --steps 15 --option pair_parts=3 || exit 1
)

r4_parts3c() (
    # pair_parts 3 vs 2 on the C5 shapes (209 strips per group)
    mkdir -p gpurun_out/r4/parts3c
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 600 python bench.py --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/parts3c/$n.json 2> gpurun_out/r4/parts3c/$n.err || { tail -20 gpurun_out/r4/parts3c/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/parts3c/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
    }
    for i in 1 2; do
      run c5share_p2_$i --config c5 --seqs 6250000 --steps 3 --warmup 1 --option pair_parts=2 &&
      run c5share_p3_$i --config c5 --seqs 6250000 --steps 3 --warmup 1 --option pair_parts=3 || exit 1
    done
    run c5_p2 --config c5 --steps 2 --warmup 1 --option pair_parts=2 && run c5_p3 --config c5 --steps 2 --warmup 1 --option pair_parts=3 || exit 1
)

r4_prio() (
    # option pair_prio_groups (raised wave priority for the longest pair groups): 0 (default) vs -1 vs 512
    mkdir -p gpurun_out/r4/prio
    run() {  # name, args
      local n=$1; shift
      timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-north-star --no-cpu-baseline "$@" > gpurun_out/r4/prio/$n.json 2> gpurun_out/r4/prio/$n.err || { tail -20 gpurun_out/r4/prio/$n.err; return 1; }
      python -c "import json; d=json.loads(open('gpurun_out/r4/prio/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['kernel']['kernel_gcups'], d['kernel']['avg_ms'], d.get('topk_vs_reference'))"
    }
    for cfg in ref sprot c2; do
      for pr in 0 -1 512 0; do run ${cfg}_pr${pr}_$RANDOM --config $cfg --option pair_prio_groups=$pr || exit 1; done
    done
)

r4_medians() (
    # the verdict's measure: median of 5 x 20-step runs, sprot / ref / C2, final build
    mkdir -p gpurun_out/r4/medians
    for cfg in sprot ref c2; do
      for i in 1 2 3 4 5; do
        timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-north-star --no-cpu-baseline > gpurun_out/r4/medians/${cfg}_$i.json 2> gpurun_out/r4/medians/${cfg}_$i.err || { tail -20 gpurun_out/r4/medians/${cfg}_$i.err; exit 1; }
      done
      python -c "
import json, statistics as st
v=[json.loads(open('gpurun_out/r4/medians/${cfg}_%d.json' % i).read().strip().splitlines()[-1]) for i in range(1, 6)]
print('$cfg', 'e2e median', st.median(d['value'] for d in v), 'kernel median', st.median(d['kernel']['kernel_gcups'] for d in v), [round(d['value']) for d in v])"
    done
)

name=${1:?usage: tools/r4_runs.sh <name> [args]}; shift
declare -F "r4_$name" > /dev/null || { echo "unknown run: $name" >&2; exit 2; }
"r4_$name" "$@"
