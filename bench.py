#!/usr/bin/env python3
"""Benchmark: GCUPS of the SW int16 database search on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1]): Smith-Waterman, BLOSUM62, gaps -11/-1,
one 400-residue query against a synthetic 1 M-sequence protein DB (lengths
1+Gamma(2,175) clipped to [16,4096], BLOSUM62 background, planted homologs;
libssa_amd/synthetic.py), top-k = 10.  A step is one search: at N=1 the
public sw_align() call (DB already packed in HBM, as the reference times
sw_align with the DB pre-loaded, benchmark/src/benchmark_util.c:27-48); at
N>1 each rank searches its own 1 M-sequence shard of an N M-sequence DB
(weak scaling: global IDs rank*1M + i), returns its exact top-k insertion
log, the logs are gathered to rank 0 over RCCL and replayed there
(ssa_amd_replay), giving the bit-exact global result.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|ref] [--seqs S]

Launch: under torchrun (WORLD_SIZE set) every process is one rank.  Without
it, `--gpus N` with N > 1 makes this process a launcher that never imports
torch or touches a GPU: it starts N child processes of bench.py (RANK,
LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), waits for them,
prints rank 0's JSON line and exits non-zero when any rank fails (the
reference fans out and joins its workers inside one call,
src/util/thread_pool.c:76-86, src/algo/manager.c:141-145).  N larger than
the visible GPU count is refused, except as a gloo rehearsal
(SSA_DIST_BACKEND=gloo: several ranks share a GPU, the exchange goes over
gloo).  --launch-selftest runs only the launch (ranks, env, rendezvous,
failure propagation) without the library.

Other BASELINE.json configurations (parity/extra measurements; the default
line is C2): --config c3 = NW BLOSUM50 -10/-2, 1000-residue query, 1 M
sequences per GPU; c4 = SW BLOSUM62 -11/-1 (API width 8) over 10 M sequences
split across the ranks (strong scaling); c5 = SW DNA +5/-4, gaps -4/-2,
10 k-nt query vs 50 M reads of 150 nt split across the ranks (strong); ref =
the reference's published benchmark shape (P18080, 513 aa, BLOSUM50 -3/-1,
548,208 synthetic sequences).
--seqs overrides the per-GPU sequence count of any config.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


# VALU instructions per cell of each scoring kernel (all its launches of a
# search), from PMC SQ_INSTS_VALU x 64 lanes / cells over the C2 (SW) and C3
# (NW) searches: profiles/r01/pmc_c2_sw_np16 (strip16), pmc_c2_r01b and
# pmc_c3_r01b (32-row pair strips), pmc_c2_np24 / pmc_c3_np24 (48-row strips),
# pmc_c2_rel / pmc_c3_rel (48-row strips, diagonal-relative values),
# pmc_c2_r01d / pmc_c3_r01d (SW running maximum along anti-diagonals),
# pmc_c2_r01e / pmc_c3_r01e (+ first-strip boundary from memory),
# pmc_{c2,c3,c5,ref}_r01g (+ diagonal add as v_add_u32, long_kernel),
# profiles/r02/pmc_c2_s3 (48-row SW strips, the default, 24-bit LDS address),
# profiles/r02/pmc_c3_np40 (80-row NW strips, the default) and
# profiles/r03/pmc_c2 (round 3: strip parts, long16_kernel; 6.654e9 x 64 /
# 1.406e11 = 3.03) and profiles/r03/final/pmc_c2 / pmc_c3 (round 3: the
# pair-row stream; SW 6.444e9 x 64 / 1.406e11 = 2.93, NW 80-row 1.439e10 x
# 64 / 3.516e11 = 2.62).  Keyed by (kernel, pair strip rows): the instruction
# count per cell depends on the strip height.
VALU_INSTR_PER_CELL = {("strip16_sw", 0): 5.59, ("strip_f16m_sw", 0): 4.79, ("pair_f16_sw", 48): 2.93,
                       ("pair_f16_nw", 48): 2.74, ("pair_f16_nw", 80): 2.62}
# share of those that are full-rate v_add_u32 (2.5 cycles per wave64
# instruction per SIMD in isolation; the packed/VOP3 rest 4.17,
# profiles/r01/ubench_valu_rates4.txt); from the DP loop's ISA census
# (tools/hotloop.py: per 48-row column SW 48 of 140.8 with the tail strip,
# NW 49 of 128.8 in round 2; the 80-row NW column's share scaled by the
# census ratio at 48 rows)
VALU_FAST_SHARE = {("pair_f16_sw", 48): 0.341, ("pair_f16_nw", 48): 0.380, ("pair_f16_nw", 80): 0.387}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="c2", choices=list(CONFIGS))
    p.add_argument("--seqs", type=int, default=None,
                   help="DB sequences per GPU (weak configs) or each GPU's share of the fixed DB (C4/C5)")
    p.add_argument("--qlen", type=int, default=None)
    p.add_argument("--algo", default=None, choices=["sw", "nw"])
    p.add_argument("--matrix", default=None)
    p.add_argument("--gap-open", type=int, default=None)
    p.add_argument("--gap-extend", type=int, default=None)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--long-tail", type=int, default=None,
                   help="replace N DB sequences by 5k-35k-residue ones (a UniProt-like length tail)")
    p.add_argument("--strip-np", type=int, default=16, help="int16/f16m strip kernels: packed rows per strip")
    p.add_argument("--pair-np", type=int, default=0,
                   help="pair kernel main strip of 2 x N rows: 0 auto (library's choice), 16, 24, 32, 36 (SW), 40")
    p.add_argument("--option", action="append", default=[], help="name=value passed to ssa_amd_set_option")
    p.add_argument("--alphabet", default=None, choices=["bg20", "sprot25", "uniform28"],
                   help="protein residue set: 20 standard (BLOSUM62 background), Swiss-Prot-like 25 "
                        "(+X,B,Z,U,O), the reference generator's uniform 28 (generate_db.c:117-118)")
    p.add_argument("--lengths", default="gamma", choices=["gamma", "uniform"],
                   help="protein lengths: 1+Gamma(2,175) in [16,4096], or uniform [16,1000) like generate_db.c")
    p.add_argument("--timeline", default=None,
                   help="N=1: after the timed steps, one more step with the wave timeline on, saved "
                        "to this .npy (tools/timeline.py analyses it)")
    p.add_argument("--torch-gather", action="store_true",
                   help="N>1: gather the shard logs with torch.distributed instead of ssa_amd_gather_logs")
    p.add_argument("--launch-selftest", action="store_true",
                   help="N>1 launcher check: the ranks verify their env and meet over gloo, no library/GPU")
    p.add_argument("--selftest-fail-rank", type=int, default=-1,
                   help="--launch-selftest: this rank exits with status 3 before the rendezvous")
    args = p.parse_args()
    cfg = CONFIGS[args.config]
    for key in ("qlen", "algo", "matrix", "gap_open", "gap_extend"):
        if getattr(args, key) is None:
            setattr(args, key, cfg[key])
    args.db = cfg["db"]
    if args.alphabet is None:
        args.alphabet = cfg.get("alphabet", "bg20")
    if args.long_tail is None:
        args.long_tail = cfg.get("long_tail", 0)
    args.width = cfg["width"]
    args.strong = cfg["total_seqs"] is not None
    return args


# BASELINE.json configs; "total_seqs" set = strong scaling (split across ranks)
CONFIGS = {
    "c2": dict(algo="sw", matrix="blosum62", gap_open=-11, gap_extend=-1, qlen=400, db="protein",
               seqs=1_000_000, total_seqs=None, width=16),
    "c3": dict(algo="nw", matrix="blosum50", gap_open=-10, gap_extend=-2, qlen=1000, db="protein",
               seqs=1_000_000, total_seqs=None, width=16),
    "c4": dict(algo="sw", matrix="blosum62", gap_open=-11, gap_extend=-1, qlen=400, db="protein",
               seqs=None, total_seqs=10_000_000, width=8),
    "c5": dict(algo="sw", matrix="const5_-4", gap_open=-4, gap_extend=-2, qlen=10_000, db="dna",
               seqs=None, total_seqs=50_000_000, width=16),
    # the shape of the reference's own published benchmark (BASELINE.md §1:
    # query P18080, 513 aa, BLOSUM50, gaps -3/-1, UniProtKB/Swiss-Prot
    # 2015_03 = 548,208 sequences; benchmark/src/benchmark_threads.c:36-46),
    # on a synthetic DB of that sequence count (no network for Swiss-Prot)
    "ref": dict(algo="sw", matrix="blosum50", gap_open=-3, gap_extend=-1, qlen=513, db="protein",
                seqs=548_208, total_seqs=None, width=16, query_file="tests/golden/data/P18080.fasta"),
    # the same in Swiss-Prot's form: its 25-symbol alphabet (+X, B, Z, U, O,
    # util_sequence.c:36-44) and a length tail of 300 entries of 5-35 k
    # residues (UniProt holds entries up to ~35 k); tests/golden/fullsize.json
    # "sprot" pins it to the reference's own search
    "sprot": dict(algo="sw", matrix="blosum50", gap_open=-3, gap_extend=-1, qlen=513, db="protein",
                  seqs=548_208, total_seqs=None, width=16, query_file="tests/golden/data/P18080.fasta",
                  alphabet="sprot25", long_tail=300),
}


def read_query_file(path):
    """First FASTA record as synthetic-alphabet codes (the product parses
    the same text itself through init_sequence_fasta)."""
    from libssa_amd import synthetic as syn
    lines = open(os.path.join(ROOT, path)).read().split("\n")
    seq = "".join(l.strip() for l in lines[1:] if not l.startswith(">")).upper()
    return np.array([syn.AA_ORDER.index(c) for c in seq], dtype=np.uint8)


def matrix_table(name):
    from oracle import pyoracle as po
    if name.startswith("const"):
        a, b = name[5:].split("_")
        return po.matrix_constant(int(a), int(b))
    tabs = np.load(os.path.join(ROOT, "tests", "golden", "tables.npz"))
    return tabs["matrices"][[str(x) for x in tabs["names"]].index(name)].copy()


def host_cpu():
    """(threads to use, description) of the host's CPU share: the affinity
    mask, capped by the cgroup CPU quota and OMP_NUM_THREADS when set (the GPU
    box exports the box's share there), plus the CPU model."""
    aff = len(os.sched_getaffinity(0))
    n, notes = aff, [f"affinity {aff}"]
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            qc = max(1, -(-int(quota) // int(period)))
            n = min(n, qc)
            notes.append(f"cgroup quota {qc}")
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
        notes.append(f"OMP_NUM_THREADS {omp}")
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, model, ", ".join(notes)


def cpu_baseline(codes, off, q, M, args):
    """The reference's own AVX2 int16 kernel (search_16_chunk ->
    search_16_avx2_sw, compiled from its sources into oracle/_ref) timed on
    the host's CPU share (every core of it) over a bounded sample, and on one
    thread; falls back to the int64 oracle port when the reference build is
    absent."""
    from oracle import pyoracle as po
    cores, model, share = host_cpu()
    algo = 0 if args.algo == "sw" else 1
    n = len(off) - 1
    if po.have_ref():
        cells_per_seq = float(off[-1]) / n * len(q)
        # the reference's search at the config's width: int16, or for width 8
        # its int8 kernel with the int16/int64 cascade (search_8.c:94-124)
        mode = po.MODE_SEARCH8_AVX2 if args.width == 8 else po.MODE_SEARCH16_AVX2
        kname = "AVX2 int8 search_8 cascade" if args.width == 8 else "AVX2 int16 search_16_chunk"

        def run(threads, seconds):
            # sample sized to ~seconds at a conservative 8 GCUPS per thread
            sample = int(min(n, max(1000, seconds * 8e9 * threads / cells_per_seq)))
            soff = off[:sample + 1]
            _, _, _, secs = po.ref_run(mode, algo, q, None, M, args.gap_open, args.gap_extend,
                                       k=args.k, threads=threads, repeat=2, db_off=(codes, soff))
            cells = float(soff[-1]) * len(q)
            return cells / secs / 1e9, sample, cells

        v, sample, cells = run(cores, args.cpu_seconds * 0.6)
        v1, sample1, _ = run(1, args.cpu_seconds * 0.3)
        return {"value": v, "unit": "GCUPS", "cores": cores, "kind": "reference",
                "one_thread_gcups": v1, "cpu_model": model, "host_share": share,
                "sample": f"first {sample} of {n} DB sequences ({cells:.3g} cells), reference {kname} "
                          f"on {cores} threads (best of 2), chunk 1000, k={args.k}; one thread: "
                          f"first {sample1} sequences"}
    po.build(quiet=True)
    sample = 2000
    soff = off[:sample + 1]
    t0 = time.perf_counter()
    po.scores(algo, q, codes[:int(soff[-1])], soff, M, args.gap_open, args.gap_extend, threads=cores)
    secs = time.perf_counter() - t0
    cells = float(soff[-1]) * len(q)
    return {"value": cells / secs / 1e9, "unit": "GCUPS", "cores": cores, "kind": "port", "cpu_model": model,
            "host_share": share, "sample": f"first {sample} DB sequences, oracle int64 scalar port on {cores} threads"}


def visible_gpus():
    """GPUs a child process would see, counted in a throwaway subprocess
    (torch.cuda.device_count() does not initialise HIP on this image, and the
    launcher itself never imports torch)."""
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=600)
        return int(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return 0


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch(args, argv):
    """Parent of an N-rank run started as `bench.py --gpus N` (no WORLD_SIZE):
    spawns the ranks, forwards their output, re-prints rank 0's JSON line,
    and propagates the first failure (the other ranks are stopped)."""
    import signal
    import threading
    N = args.gpus
    backend = os.environ.get("SSA_DIST_BACKEND", "nccl")
    ngpu = None
    if not args.launch_selftest:
        ngpu = visible_gpus()
        if N > ngpu and backend != "gloo":
            print(f"bench.py: --gpus {N} requested but {ngpu} GPU(s) visible; refusing to double ranks up "
                  f"(a gloo rehearsal on fewer GPUs: SSA_DIST_BACKEND=gloo)", file=sys.stderr)
            return 2
        if ngpu < 1:
            print("bench.py: no GPU visible", file=sys.stderr)
            return 2
    port = free_port()
    procs = []
    lines = []
    me = os.path.abspath(__file__)
    for r in range(N):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(N), LOCAL_WORLD_SIZE=str(N),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SSA_BENCH_LAUNCHER="bench.py --gpus")
        if ngpu is not None:
            env["SSA_BENCH_VISIBLE_GPUS"] = str(ngpu)
        procs.append(subprocess.Popen([sys.executable, "-u", me, *argv],
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), env=env))

    def pump():
        # rank 0's stdout: progress lines through, the JSON line held back
        for raw in procs[0].stdout:
            line = raw.decode(errors="replace").rstrip("\n")
            if line.startswith("{"):
                lines.append(line)
            else:
                print(line, flush=True)
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad and failed is None:
            failed = bad[0]
            print(f"bench.py: rank {failed[0]} exited with status {failed[1]}; stopping the other ranks",
                  file=sys.stderr, flush=True)
            deadline = time.time() + 10
            while time.time() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGTERM)
            deadline = time.time() + 10
            while time.time() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            for p in procs:
                p.wait()
            break
        if all(c is not None for c in codes):
            break
        time.sleep(0.2)
    th.join(10)
    if failed is not None:
        return failed[1] if failed[1] > 0 else 1
    if not lines:
        print("bench.py: rank 0 printed no result line", file=sys.stderr)
        return 1
    print(lines[-1], flush=True)
    return 0


def launch_selftest(args):
    """A rank of `bench.py --gpus N --launch-selftest`: checks the launch
    environment and meets the other ranks over gloo (no library, no GPU)."""
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ["LOCAL_RANK"])
    assert world == args.gpus and 0 <= rank < world and local == rank, (rank, local, world, args.gpus)
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
    if rank == args.selftest_fail_rank:
        print(f"rank {rank}: failing on purpose (--selftest-fail-rank)", file=sys.stderr, flush=True)
        sys.exit(3)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "local_rank": local, "pid": os.getpid(),
                                 "launcher": os.environ.get("SSA_BENCH_LAUNCHER")})
    dist.barrier()
    if rank == 0:
        print(json.dumps({"launch_selftest": "ok", "world": world, "ranks": got}), flush=True)
    dist.destroy_process_group()


def make_shard(args, cfg, rank, world):
    """This rank's contiguous ID slice of the config's synthetic DB, from the
    block-seeded generators (libssa_amd/synthetic.py: a slice is
    byte-identical to the same IDs of the whole DB).  Weak configs (C2/C3/ref):
    an N x seqs DB, ~1 M per rank; strong ones (C4/C5): the fixed 10 M / 50 M
    DB, so every N searches the same DB.  At N > 1 the ranks' ranges are cut
    so that their residue sums balance (ssa_amd_shard_bounds),
    not by sequence count.  At N = 1 C2 and C3 are exactly
    tests/golden/fullsize.json's c2/c3 DBs.
    --seqs: the per-rank sequence count of a weak config's DB, or the per-rank
    share of a strong config's fixed DB (then cut by count: the first share is
    the c4/c5 fixtures' DB).
    Returns (query, codes, offsets, first global ID, DB size, IDs the job searches)."""
    import libssa_amd as S
    from libssa_amd import synthetic as syn
    dna = args.db == "dna"
    if dna:
        q = syn.dna_query(args.qlen, 8)
    else:
        q = read_query_file(cfg["query_file"]) if cfg.get("query_file") else syn.protein_query(args.qlen, 7)
    hi = 4096 if args.lengths == "gamma" else 1000
    if cfg["total_seqs"] is None:
        per = args.seqs if args.seqs is not None else cfg["seqs"]
        total = job = per * world
        balanced = world > 1
    else:
        total = cfg["total_seqs"]
        per = args.seqs if args.seqs is not None else (total + world - 1) // world
        job = min(total, per * world)
        balanced = world > 1 and args.seqs is None
    if balanced and not dna:
        lens = syn.protein_lengths_range(total, 42, 0, job, query=q, lo=16, hi=hi, lengths=args.lengths)
        b = S.shard_bounds(lens, world)
        i0, i1 = b[rank], b[rank + 1]
    else:
        # equal-length reads (C5), or one GPU: cutting by count is balanced
        i0 = min(job, rank * per)
        i1 = min(job, i0 + per) if rank + 1 < world else job
    if dna:
        codes, off = syn.dna_reads_range(total, 43, i0, i1, 150, query=q)
        return q, codes, off, i0, total, job
    codes, off = syn.protein_db_range(total, 42, i0, i1, query=q, alphabet=args.alphabet, lengths=args.lengths,
                                      lo=16, hi=hi)
    return q, codes, off, i0, total, job


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the launcher: no torch, no GPU in this process
        sys.exit(launch(args, sys.argv[1:]))
    if args.launch_selftest:
        if "WORLD_SIZE" in os.environ:
            launch_selftest(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    backend = os.environ.get("SSA_DIST_BACKEND", "nccl")   # nccl == RCCL on ROCm; gloo for rehearsal
    dev = "cuda" if backend == "nccl" else "cpu"
    ranks_per_gpu = 1
    if world > 1:
        import torch
        import torch.distributed as dist
        ngpu = torch.cuda.device_count()
        if local >= ngpu:
            if backend != "gloo":
                raise SystemExit(f"bench.py rank {rank}: LOCAL_RANK {local} but only {ngpu} GPU(s) visible")
            # gloo rehearsal: several ranks share a GPU
            ranks_per_gpu = -(-world // max(1, ngpu))
            local = local % max(1, ngpu)
        torch.cuda.set_device(local)
        dist.init_process_group(backend)

    import libssa_amd as S
    from libssa_amd import synthetic as syn

    S.load()
    S.set_device(local)
    S.set_output_mode(S.OUTPUT_ERROR)
    S.set_option("strip_np", args.strip_np)
    S.set_option("pair_np", args.pair_np)
    for o in args.option:
        k, v = o.split("=")
        S.set_option(k, int(v))
    dna = args.db == "dna"
    S.init_symbol_translation(S.NUCLEOTIDE if dna else S.AMINOACID, S.FORWARD_STRAND, 1, 1)
    if args.matrix.startswith("const"):
        a, b = args.matrix[5:].split("_")
        S.init_constant_scores(int(a), int(b))
    else:
        S.init_score_matrix(S.MATRIX_BUILDIN, args.matrix)
    S.init_gap_penalties(args.gap_open, args.gap_extend)
    algo = S.SW if args.algo == "sw" else S.NW
    cfg = CONFIGS[args.config]

    # --- synthetic shard (untimed): generate, write FASTA, pack into HBM
    t0 = time.time()
    q, codes, off, id0, db_total, job_ids = make_shard(args, cfg, rank, world)
    args.qlen = len(q)
    args.seqs = len(off) - 1
    if not dna and args.long_tail > 0:
        # every (seqs / N)-th sequence becomes 5k-35k residues long (fresh
        # residues of the DB's alphabet); the others keep theirs
        codes, off = syn.with_long_tail(codes, off, args.long_tail, 77 + rank, args.alphabet)
    tmpdir = tempfile.mkdtemp(prefix=f"ssa_bench_{rank}_")
    path = os.path.join(tmpdir, "db.fas")
    syn.write_fasta(path, codes, off, nucleotide=dna)
    gen_s = time.time() - t0
    t1 = time.time()
    S.init_db(path)
    S.set_id_offset(id0)
    S.prepare_db()
    os.remove(path)
    os.rmdir(tmpdir)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q, nucleotide=dna))
    load_s = time.time() - t1
    setup_s = time.time() - t0
    cells_local = float(off[-1]) * args.qlen
    total_cells = cells_local
    if dist is not None:
        # the shards are cut by residues: sum the ranks' cells
        import torch
        tc = torch.tensor([cells_local], dtype=torch.float64, device=dev)
        dist.all_reduce(tc, op=dist.ReduceOp.SUM)
        total_cells = float(tc.item())

    # N > 1: the shards' insertion logs meet on rank 0 in the library's own
    # RCCL gather (ssa_amd_gather_logs); the RCCL unique id travels over the
    # torch process group once
    native = world > 1 and backend == "nccl" and not args.torch_gather
    gather_note = None
    rccl_ranks = None
    if native:
        import torch

        def agree(ok):
            # every rank takes the same path: MIN over the ranks' flags
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            return int(flag.item()) == 1
        # 1. local readiness (RCCL resolvable, device selectable) agreed on
        #    before anyone enters the collective ncclCommInitRank, so no rank
        #    waits there for a peer that gave up
        ready = S.dist_available()
        if not ready:
            gather_note = f"rank {rank}: RCCL not available to the library"
        if agree(ready):
            uid = None
            if rank == 0:
                try:
                    uid = S.dist_unique_id()
                except RuntimeError as e:
                    gather_note = str(e)
            obj = [uid]
            dist.broadcast_object_list(obj, src=0)
            ok = False
            if obj[0] is not None:
                try:
                    S.dist_init(rank, world, obj[0])
                    ok = True
                except RuntimeError as e:
                    gather_note = str(e)
            if not agree(ok):
                if ok:
                    S.dist_finalize()
                native = False
                gather_note = gather_note or "RCCL setup failed on another rank"
            else:
                rccl_ranks = S.dist_ranks()
        else:
            native = False
            gather_note = gather_note or "RCCL not available on another rank"

    def step():
        if world == 1:
            # the public sw_align / nw_align + free_alignment (libssa.h)
            return S.align_scores(qq, args.k, args.width, algo)
        log = S.search(qq, algo, args.k, args.width, S.LOG)
        if native:
            return S.gather_logs(log, args.k)
        from libssa_amd.dist import global_topk
        return global_topk(log, args.k, dist, rank, world, dev)

    def sync():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    gather_checked = None
    if native:
        # untimed: the RCCL gather must equal the torch.distributed gather of
        # the same logs -- this search's, and a synthetic rising log of 600
        # rows per rank at k = 600 (longer than the 512-row slot: the
        # exact-size ncclGather round).  Every rank joins every collective.
        # On any disagreement the timed steps use the torch gather.
        from libssa_amd.dist import global_topk
        log = S.search(qq, algo, args.k, args.width, S.LOG)
        long_log = [(1000 * (rank * 600 + i) + 7, 10 ** 6 * rank + i, 0, 0, 0) for i in range(600)]
        same = True
        for lg, kk in ((log, args.k), (long_log, 600)):
            a = S.gather_logs(lg, kk)
            b = global_topk(lg, kk, dist, rank, world, dev)
            if rank == 0:
                same = same and [tuple(map(int, x[:2])) for x in a] == [tuple(map(int, x[:2])) for x in b]
        import torch
        flag = torch.tensor([1 if same else 0], dtype=torch.int32, device=dev)
        dist.broadcast(flag, src=0)
        gather_checked = bool(int(flag.item()))
        if not gather_checked:
            S.dist_finalize()
            native = False
            gather_note = "RCCL gather disagreed with the torch.distributed gather: timed the torch gather"
    sync()
    kernel_ms, wide_ms, search_ms, d2h_ms, replay_ms, prep_ms, upload_ms, sync_ms = [], [], [], [], [], [], [], []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        res = step()
        st = S.stats()
        kernel_ms.append(st["kernel_ms"])
        wide_ms.append(st["wide_ms"])
        search_ms.append(st["search_ms"])
        prep_ms.append(st["prep_ms"])
        upload_ms.append(st["upload_ms"])
        sync_ms.append(st["sync_wait_ms"])
        d2h_ms.append(st["d2h_ms"])
        replay_ms.append(st["replay_ms"])
    sync()
    elapsed = time.perf_counter() - t_start
    if args.timeline and world == 1:
        # untimed: every DP wave's start/end on the s_memrealtime clock
        S.set_option("timeline", 1)
        step()
        np.save(args.timeline, S.timeline())
        S.set_option("timeline", 0)
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = S.stats()
    if native:
        S.dist_finalize()
    if rank != 0:
        dist.destroy_process_group()
        return
    ms_per_step = elapsed / args.steps * 1e3
    gcups = total_cells / (elapsed / args.steps) / 1e9
    kavg = float(np.mean(kernel_ms))
    # algorithmic bytes per launch: every residue once (1 B) + 4 B score per
    # sequence + the strip profile table
    alg_bytes = float(st["kernel_bytes"])
    achieved = alg_bytes / (kavg * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf):
        rec = json.load(open(tf)).get(f"{args.algo}_{args.seqs}_{args.qlen}_pair{st['strip_rows'] // 2}")
        if rec:
            traffic = rec["bytes_per_launch"]
    # VALU issue roofline: VOP3/VOP3P instructions issue at
    # 4.17 cycles per wave64 instruction per SIMD, v_add_u32 at 2.5 (measured
    # in isolation: profiles/r01/ubench_valu_rates4.txt); instructions per
    # cell from PMC SQ_INSTS_VALU (profiles/r01/pmc_{c2,c3,c5}_r01g).
    kkey = (st["kernel"], st["strip_rows"])
    instr_per_cell = VALU_INSTR_PER_CELL.get(kkey) if args.strip_np == 16 else None
    fast = VALU_FAST_SHARE.get(kkey, 0.0)
    issue_cycles = (1.0 - fast) * 4.17 + fast * 2.5
    valu_bound = (1024 * 2.4e9 / issue_cycles * 64 / instr_per_cell) if instr_per_cell else None
    out = {
        "metric": "GCUPS (SW int16, 400aa query vs synthetic DB) at 1/2/4/8 MI355X; top-k score bit-exact",
        "value": round(gcups, 2),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "i16",
        "data": "synthetic",
        "config": {"workload": f"{args.config.upper()}: {args.algo.upper()} {args.matrix} gaps {args.gap_open}/{args.gap_extend}, "
                               f"{args.qlen}-residue query vs {args.seqs} synthetic {args.db} seqs per GPU "
                               f"(mean len {float(off[-1]) / args.seqs:.1f}), top-{args.k}",
                   "db_seqs_per_gpu": args.seqs, "db_total_seqs": db_total, "query_len": args.qlen, "residues_per_gpu": int(off[-1]),
                   "cells_per_step": total_cells, "parallelism": f"db-shard x{world}", "job_seqs": job_ids, "pair_strip_rows": st["strip_rows"], "strip_np": args.strip_np,
                   "bit_width": args.width},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     # the resource that actually binds this integer DP
                     "binding": {"bound": "valu_issue",
                                 "achieved": round(cells_local / (kavg * 1e-3) / 1e9, 2),
                                 "peak": round(valu_bound / 1e9, 1) if valu_bound else None, "unit": "GCUPS",
                                 "frac": (cells_local / (kavg * 1e-3)) / valu_bound if valu_bound else None}},
        "kernel": {"name": st["kernel"], "avg_ms": round(kavg, 4),
                   "kernel_gcups": round(cells_local / (kavg * 1e-3) / 1e9, 2),
                   "wide_ms_avg": round(float(np.mean(wide_ms)), 4), "wide_count": int(st["wide_count"]),
                   "valu_issue_bound_gcups": round(valu_bound / 1e9, 1) if valu_bound else None,
                   "valu_issue_frac": (cells_local / (kavg * 1e-3)) / valu_bound if valu_bound else None,
                   "valu_instr_per_cell": instr_per_cell},
        "host_ms": {"search_call": round(float(np.mean(search_ms)), 3), "prep": round(float(np.mean(prep_ms)), 3),
                    "upload": round(float(np.mean(upload_ms)), 3), "sync_wait": round(float(np.mean(sync_ms)), 3), "d2h_filter": round(float(np.mean(d2h_ms)), 3),
                    "replay": round(float(np.mean(replay_ms)), 3)},
        "setup_s": round(setup_s, 1),
        "setup": {"generate_and_write_fasta_s": round(gen_s, 1), "init_db_and_pack_s": round(load_s, 1),
                  "pack_ms": round(st["pack_ms"], 1)},
        "top_hit": list(res[0]) if res else None,
        "gather": ("ssa_amd_gather_logs (RCCL)" if native else "torch.distributed") if world > 1 else None,
        "gather_equals_torch_gather": gather_checked,
        "rccl_ranks": rccl_ranks,
        "launcher": os.environ.get("SSA_BENCH_LAUNCHER", "torchrun" if world > 1 else None),
    }
    if ranks_per_gpu > 1:
        out["rehearsal"] = f"{world} ranks on {max(1, world // ranks_per_gpu)} GPU(s), exchange over {backend}"
    if gather_note:
        out["gather_note"] = gather_note
    # the same DB and query as a reference-pinned fixture: the step's top-k
    # against the reference's own (tests/golden/fullsize.json)
    fxs = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))

    def same_db(fx):
        return (fx.get("kind", "protein") == args.db and args.alphabet == fx.get("alphabet", "bg20")
                and args.lengths == fx.get("lengths", "gamma") and fx["n"] == db_total and fx["i1"] == job_ids
                and args.long_tail == fx.get("tail", 0) and fx.get("query_file") == cfg.get("query_file")
                and fx["qlen"] == args.qlen and fx["algo"] == args.algo and fx["gap_open"] == args.gap_open
                and fx["gap_extend"] == args.gap_extend and fx["matrix"] == args.matrix)
    # the fixture of this exact DB and search, if any (c2, c3, the c4 / c5
    # shares, c4full = the whole 10 M DB, c5share8 = one GPU's C5 share at
    # N = 8, c2x2/4/8 = C2's weak-scaling DBs): at N > 1 rank 0 holds the
    # gathered global top-k of the N shards
    fx = next((f for f in fxs.values() if same_db(f)), None)
    if fx and (args.long_tail == 0 or world == 1) and args.k in (1, 10, 64):
        out["topk_vs_reference"] = "match" if [list(x) for x in res] == fx[f"top{args.k}"] else "MISMATCH"
    if world == 1 and not args.no_cpu_baseline:
        from oracle import pyoracle as po
        M = matrix_table(args.matrix)
        try:
            out["cpu_baseline"] = cpu_baseline(codes, off, q, M, args)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
