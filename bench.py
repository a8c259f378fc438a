#!/usr/bin/env python3
"""Benchmark: GCUPS of the SW int16 database search on MI355X (BASELINE.json).

Headline workload (BASELINE.json configs[1]): Smith-Waterman, BLOSUM62, gaps
-11/-1, one 400-residue query against a synthetic 1 M-sequence protein DB
(lengths 1+Gamma(2,175) clipped to [16,4096], BLOSUM62 background, planted
homologs; libssa_amd/synthetic.py), top-k = 10.  A step is one search: at N=1
the public sw_align() call (DB already packed in HBM, as the reference times
sw_align with the DB pre-loaded, benchmark/src/benchmark_util.c:27-48); at
N>1 each rank searches its own ~1 M-sequence slice of an N M-sequence DB
(weak scaling, cut by residues), returns its exact top-k insertion log, the
logs are gathered to rank 0 over RCCL and replayed there (ssa_amd_replay),
giving the bit-exact global result.

The same JSON line carries a "north_star" record (BASELINE.json north_star):
SW int16, the same query against the FIXED 10 M-sequence DB (the c4full
fixture), cut into N residue-balanced ID slices -- the strong-scaling point
the driver's `--gpus 1/2/4/8` runs produce, top-k checked against the
reference's own search of that DB.  --no-north-star skips it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|ref|sprot|north_star] [--seqs S]

Launch: under torchrun (WORLD_SIZE set) every process is one rank.  Without
it, `--gpus N` with N > 1 makes this process a launcher that never imports
torch or touches a GPU: it starts N child processes of bench.py (RANK,
LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), waits for them,
prints rank 0's JSON line and exits non-zero when any rank fails (the
reference fans out and joins its workers inside one call,
src/util/thread_pool.c:76-86, src/algo/manager.c:141-145).  N larger than
the visible GPU count is refused, except as a gloo rehearsal
(SSA_DIST_BACKEND=gloo: several ranks share a GPU, the exchange goes over
gloo; the line then says "rehearsal" and n_gpus counts physical GPUs).
--launch-selftest runs only the launch (ranks, env, rendezvous, failure
propagation, the rank layout) without the library.

Other BASELINE.json configurations (libssa_amd/workloads.py; the default
line is C2): --config c3 = NW BLOSUM50 -10/-2, 1000-residue query, 1 M
sequences per GPU; c4 = SW BLOSUM62 -11/-1 (API width 8) over 10 M sequences
split across the ranks (strong scaling); c5 = SW DNA +5/-4, gaps -4/-2,
10 k-nt query vs 50 M reads of 150 nt split across the ranks (strong); ref =
the reference's published benchmark shape (P18080, 513 aa, BLOSUM50 -3/-1,
548,208 synthetic sequences); sprot = the same in Swiss-Prot's form.
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

from libssa_amd import workloads as W  # noqa: E402

CONFIGS = W.CONFIGS
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
PEAK_CLOCK_GHZ = 2.4           # MI355X_MICROARCH.md: the engine's peak clock (the VALU issue ceiling)


# The VALU issue roofline's measured input -- VALU lane-instructions per cell
# over a search's DP kernels (with the pass's own clock, reported beside) -- is
# a PMC measurement of the exact build and workload (tools/profile_pmc.sh -> tools/traffic_from_pmc.py
# -> profiles/traffic.json, filed under the workload key and the kernel-source
# hash, libssa_amd/workloads.py kernel_src_hash); a line whose build hashes
# differently reports it null with roofline.traffic_stale (rounds 1-5 kept it
# in a constant table here: profiles/r0*/pmc_*).
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
    p.add_argument("--no-north-star", action="store_true",
                   help="skip the north_star record (SW int16, q = 400 vs the fixed 10 M-sequence DB, strong)")
    p.add_argument("--north-star-steps", type=int, default=None, help="timed steps of the north_star record "
                   "(default: --steps, at most 10)")
    p.add_argument("--no-drop-in", action="store_true",
                   help="N>1: skip the drop_in record (the north-star DB through sw_align on all N devices of "
                        "rank 0's process, after the multi-process records)")
    p.add_argument("--drop-in-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--drop-in-seqs", type=int, default=None,
                   help="drop_in record: the first S IDs of the north-star DB instead of all 10 M")
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
    return args


def workload(args, name, overrides=True):
    """The config `name` with the command line's overrides (headline) or
    exactly as defined (north_star), as one namespace."""
    cfg = dict(CONFIGS[name])
    w = argparse.Namespace(config=name, cfg=cfg, db=cfg["db"], width=cfg["width"],
                           strong=cfg["total_seqs"] is not None, lengths="gamma", seqs=None,
                           alphabet=cfg.get("alphabet", "bg20"), long_tail=cfg.get("long_tail", 0))
    for key in ("qlen", "algo", "matrix", "gap_open", "gap_extend"):
        v = getattr(args, key) if overrides else None
        setattr(w, key, cfg[key] if v is None else v)
    w.k, w.cpu_seconds = args.k, args.cpu_seconds
    if overrides:
        w.seqs, w.lengths = args.seqs, args.lengths
        if args.alphabet is not None:
            w.alphabet = args.alphabet
        if args.long_tail is not None:
            w.long_tail = args.long_tail
    return w


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
    the host's CPU share (every core of it) and on one thread, each as the
    median of 5 runs after 1 warm-up run.  The all-core
    figure searches the whole DB unless one run would exceed --cpu-seconds/3
    (C2: the whole 1 M sequences, ~0.4 s a run on 16 threads); the one-thread
    figure the first sequences worth ~--cpu-seconds/7.5 per run.  Falls back to
    the int64 oracle port when the reference build is absent."""
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
            # sample sized to ~seconds per run at ~20 GCUPS per thread
            sample = int(min(n, max(1000, seconds * 20e9 * threads / cells_per_seq)))
            soff = off[:sample + 1]
            _, _, _, secs = po.ref_run(mode, algo, q, None, M, args.gap_open, args.gap_extend,
                                       k=args.k, threads=threads, repeat=6, db_off=(codes, soff), times=True)
            cells = float(soff[-1]) * len(q)
            return cells / float(np.median(secs[1:])) / 1e9, sample, cells, secs

        v, sample, cells, secs = run(cores, args.cpu_seconds / 3)
        v1, sample1, cells1, secs1 = run(1, args.cpu_seconds / 7.5)
        whole = "the whole DB" if sample == n else f"first {sample} of {n} DB sequences"
        return {"value": v, "unit": "GCUPS", "cores": cores, "kind": "reference",
                "one_thread_gcups": v1, "cpu_model": model, "host_share": share,
                "run_seconds": [round(x, 4) for x in secs], "one_thread_run_seconds": [round(x, 4) for x in secs1],
                "sample": f"{whole} ({cells:.3g} cells), reference {kname} on {cores} threads, median of 5 "
                          f"runs after 1 warm-up, chunk 1000, k={args.k}; one thread: first {sample1} of {n} "
                          f"sequences ({cells1:.3g} cells), median of 5 after 1 warm-up"}
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
                print(line, file=sys.stderr, flush=True)
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


def rehearsal_label(world, n_gpus, backend):
    return f"{world} ranks on {n_gpus} GPU(s), exchange over {backend}"


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
    # the rank layout main() would use, from the GPU count the launcher saw
    # (SSA_BENCH_VISIBLE_GPUS; absent in a selftest launch: one GPU assumed)
    ngpu = int(os.environ.get("SSA_BENCH_VISIBLE_GPUS", "1"))
    backend = os.environ.get("SSA_DIST_BACKEND", "nccl")
    layout = {}
    try:
        device, rpg, n_gpus = W.rank_layout(world, ngpu, local, backend)
        layout = {"device": device, "ranks_per_gpu": rpg, "n_gpus": n_gpus}
        if rpg > 1:
            layout["rehearsal"] = rehearsal_label(world, n_gpus, backend)
    except SystemExit as e:
        layout = {"refused": str(e)}
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "local_rank": local, "pid": os.getpid(),
                                 "launcher": os.environ.get("SSA_BENCH_LAUNCHER"), "layout": layout})
    dist.barrier()
    if rank == 0:
        print(json.dumps({"launch_selftest": "ok", "world": world, "ranks": got}), flush=True)
    dist.destroy_process_group()


class Job:
    """The rank's view of the job: process group, gather path, timing."""

    def __init__(self, rank, world, dist, dev, backend):
        self.rank, self.world, self.dist, self.dev, self.backend = rank, world, dist, dev, backend
        self.dev_index = 0           # this rank's GPU (ssa_amd_set_device)
        self.native = False          # ssa_amd_gather_logs over RCCL
        self.gather_note = None
        self.rccl_ranks = None
        self.gather_checked = None

    def reduce(self, x, op):
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def sum(self, x):
        return self.reduce(x, None if self.dist is None else self.dist.ReduceOp.SUM)

    def max(self, x):
        return self.reduce(x, None if self.dist is None else self.dist.ReduceOp.MAX)

    def min(self, x):
        return self.reduce(x, None if self.dist is None else self.dist.ReduceOp.MIN)

    def sync(self):
        if self.dist is not None:
            import torch
            self.dist.barrier()
            torch.cuda.synchronize()


def setup_native_gather(S, job):
    """N > 1: the shards' insertion logs meet on rank 0 in the library's own
    RCCL gather (ssa_amd_gather_logs); the RCCL unique id travels over the
    torch process group once."""
    import torch
    dist, rank, world = job.dist, job.rank, job.world

    def agree(ok):
        # every rank takes the same path: MIN over the ranks' flags
        return job.min(1.0 if ok else 0.0) == 1.0
    # 1. local readiness (RCCL resolvable, device selectable) agreed on
    #    before anyone enters the collective ncclCommInitRank, so no rank
    #    waits there for a peer that gave up
    ready = S.dist_available()
    if not ready:
        job.gather_note = f"rank {rank}: RCCL not available to the library"
    if not agree(ready):
        job.gather_note = job.gather_note or "RCCL not available on another rank"
        return
    uid = None
    if rank == 0:
        try:
            uid = S.dist_unique_id()
        except RuntimeError as e:
            job.gather_note = str(e)
    obj = [uid]
    dist.broadcast_object_list(obj, src=0)
    ok = False
    if obj[0] is not None:
        try:
            S.dist_init(rank, world, obj[0])
            ok = True
        except RuntimeError as e:
            job.gather_note = str(e)
    if not agree(ok):
        if ok:
            S.dist_finalize()
        job.gather_note = job.gather_note or "RCCL setup failed on another rank"
        return
    job.native = True
    job.rccl_ranks = S.dist_ranks()


def check_native_gather(S, job, qq, algo, k, width):
    """Untimed: the RCCL gather must equal the torch.distributed gather of
    the same logs -- this search's, and a synthetic rising log of 600 rows
    per rank at k = 600 (longer than the 512-row slot: the exact-size
    ncclGather round).  Every rank joins every collective.  On any
    disagreement the timed steps use the torch gather."""
    import torch
    from libssa_amd.dist import global_topk
    rank = job.rank
    log = S.search(qq, algo, k, width, S.LOG)
    long_log = [(1000 * (rank * 600 + i) + 7, 10 ** 6 * rank + i, 0, 0, 0) for i in range(600)]
    same = True
    for lg, kk in ((log, k), (long_log, 600)):
        a = S.gather_logs(lg, kk)
        b = global_topk(lg, kk, job.dist, rank, job.world, job.dev)
        if rank == 0:
            same = same and [tuple(map(int, x[:2])) for x in a] == [tuple(map(int, x[:2])) for x in b]
    flag = torch.tensor([1 if same else 0], dtype=torch.int32, device=job.dev)
    job.dist.broadcast(flag, src=0)
    job.gather_checked = bool(int(flag.item()))
    if not job.gather_checked:
        S.dist_finalize()
        job.native = False
        job.gather_note = "RCCL gather disagreed with the torch.distributed gather: timed the torch gather"


def configure(S, w):
    dna = w.db == "dna"
    S.init_symbol_translation(S.NUCLEOTIDE if dna else S.AMINOACID, S.FORWARD_STRAND, 1, 1)
    if w.matrix.startswith("const"):
        a, b = w.matrix[5:].split("_")
        S.init_constant_scores(int(a), int(b))
    else:
        S.init_score_matrix(S.MATRIX_BUILDIN, w.matrix)
    S.init_gap_penalties(w.gap_open, w.gap_extend)


def load_shard(S, w, job):
    """Untimed: this rank's contiguous ID slice of the workload's block-seeded
    DB (libssa_amd/workloads.py: the cut is the one the GPU tests search),
    written as FASTA, read through the plugin (init_db) and packed into HBM
    with its global ID offset.  Returns a namespace of the slice."""
    from libssa_amd import synthetic as syn
    configure(S, w)
    t0 = time.time()
    q = W.query(w.cfg, w.qlen)
    bounds, total, job_ids = W.cuts(w.cfg, job.world, q, w.seqs, w.lengths)
    i0, i1 = bounds[job.rank], bounds[job.rank + 1]
    codes, off = W.slice_db(w.cfg, q, total, i0, i1, w.alphabet, w.lengths)
    if w.db != "dna" and w.long_tail > 0:
        # every (seqs / N)-th sequence becomes 5k-35k residues long (fresh
        # residues of the DB's alphabet); the others keep theirs
        codes, off = syn.with_long_tail(codes, off, w.long_tail, 77 + job.rank, w.alphabet)
    tmpdir = tempfile.mkdtemp(prefix=f"ssa_bench_{job.rank}_")
    path = os.path.join(tmpdir, "db.fas")
    syn.write_fasta(path, codes, off, nucleotide=w.db == "dna")
    gen_s = time.time() - t0
    t1 = time.time()
    S.init_db(path)
    S.set_id_offset(i0)
    S.prepare_db()
    os.remove(path)
    os.rmdir(tmpdir)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q, nucleotide=w.db == "dna"))
    load_s = time.time() - t1
    cells_local = float(off[-1]) * len(q)
    return argparse.Namespace(q=q, qq=qq, codes=codes, off=off, id0=i0, total=total, job_ids=job_ids,
                              seqs=len(off) - 1, residues=int(off[-1]), qlen=len(q), cells_local=cells_local,
                              total_cells=job.sum(cells_local), gen_s=gen_s, load_s=load_s,
                              setup_s=time.time() - t0)


_OPTIONS = {}


def lean_events_on():
    """The library's lean_events option as this run set it (default 1)."""
    return _OPTIONS.get("lean_events", 1) != 0


def timed_steps(S, job, sh, w, steps, warmup, k):
    """W untimed warm-up steps, then exactly K steps between barrier +
    synchronize on both sides; the max over ranks of the elapsed time."""
    algo = S.SW if w.algo == "sw" else S.NW
    # N > 1: the host clock around each step's search and gather, on every
    # rank (two perf_counter reads per step; they add nothing measurable)
    split = {"search_s": [], "gather_s": []}

    def step(keep=True):
        if job.world == 1:
            # the public sw_align / nw_align + free_alignment (libssa.h).  The
            # timed loop calls them exactly as the reference's benchmark does,
            # free_alignment(sw_align(...)) with the hits unread
            # (benchmark/src/benchmark_util.c:27-48); the result is read from
            # one more, untimed search of the same query after the loop
            if not keep:
                S.align_free(sh.qq, k, w.width, algo)
                return None
            return S.align_scores(sh.qq, k, w.width, algo)
        t0 = time.perf_counter()
        log = S.search(sh.qq, algo, k, w.width, S.LOG)
        t1 = time.perf_counter()
        if job.native:
            res = S.gather_logs(log, k)
        else:
            from libssa_amd.dist import global_topk
            res = global_topk(log, k, job.dist, job.rank, job.world, job.dev)
        split["search_s"].append(t1 - t0)
        split["gather_s"].append(time.perf_counter() - t1)
        return res

    for _ in range(warmup):
        step()
    if job.native and job.gather_checked is None:
        check_native_gather(S, job, sh.qq, algo, k, w.width)
    split["search_s"].clear()
    split["gather_s"].clear()
    # the timed region holds only the searches (and at N > 1 the gather):
    # the library's running totals are read once on each side of it
    st0 = S.stats()
    job.sync()
    t_start = time.perf_counter()
    for _ in range(steps):
        res = step(keep=job.world > 1)
    job.sync()
    elapsed = job.max(time.perf_counter() - t_start)
    st = S.stats()
    if job.world == 1:
        res = step()
    n = st["total_searches"] - st0["total_searches"]
    if n > 0:
        avg = {"kernel_ms": (st["total_kernel_ms"] - st0["total_kernel_ms"]) / n,
               "search_ms": (st["total_search_ms"] - st0["total_search_ms"]) / n}
    else:
        # (a library build without the running totals: SSA_AMD_LIB A/B runs)
        avg = {"kernel_ms": st["kernel_ms"], "search_ms": st["search_ms"]}
    # (host-side breakdown: the last search's.  The timing markers around the
    # upload, the re-score tier and the filter are off by default (option
    # lean_events: they cost ~40 us a search), so one extra untimed local
    # search with them on fills in the breakdown)
    lean = lean_events_on()
    if lean:
        S.set_option("lean_events", 0)
        S.align_scores(sh.qq, k, w.width, algo)
        S.set_option("lean_events", 1)
    sb = S.stats() if lean else st
    for f in ("wide_ms", "prep_ms", "upload_ms", "sync_wait_ms", "d2h_ms", "replay_ms"):
        avg[f] = sb[f]
    ranks = rank_split(job, sh, avg, split, elapsed / steps) if job.world > 1 else None
    return argparse.Namespace(res=res, step=step, elapsed=elapsed, st=st, avg=avg, ranks=ranks)


def rank_split(job, sh, avg, split, step_s):
    """N > 1: where a step's time goes, rank by rank -- so a scaling run
    explains its own result (imbalance, host overhead or the collective).
    Every rank contributes (kernel ms, search ms, gather median / max ms,
    residues, cells) through one all-gather after the timed region; rank 0
    reports the lists and:
      kernel_balance_efficiency = (sum of rank cells / max rank kernel time)
                                  / sum of rank kernel rates  (1.0: no rank waits
                                  on the slowest kernel)
      residue_imbalance = max rank residues / mean rank residues
      step_split_ms: the slowest kernel, the search call's host overhead on that
                     rank, the gather (median and max over ranks and steps) and
                     the rest of the step (barrier skew between ranks)."""
    import torch
    g = np.array(split["gather_s"]) * 1e3
    s = np.array(split["search_s"]) * 1e3
    mine = torch.tensor([avg["kernel_ms"], avg["search_ms"], float(np.median(s)) if s.size else 0.0,
                         float(np.median(g)) if g.size else 0.0, float(g.max()) if g.size else 0.0,
                         float(sh.residues), float(sh.cells_local), float(sh.seqs)],
                        dtype=torch.float64, device=job.dev)
    rows = [torch.empty_like(mine) for _ in range(job.world)]
    job.dist.all_gather(rows, mine)
    R = np.array([r.cpu().numpy() for r in rows])
    kms, sms, step_search, gmed, gmax, res, cells, seqs = R.T
    rate = cells / (kms * 1e-3)
    slow = int(np.argmax(kms))
    return {
        "kernel_ms": [round(x, 4) for x in kms], "search_ms": [round(x, 4) for x in sms],
        "gather_ms_median": [round(x, 4) for x in gmed], "gather_ms_max": [round(x, 4) for x in gmax],
        "seqs": [int(x) for x in seqs], "residues": [int(x) for x in res],
        "kernel_gcups": [round(x / 1e9, 2) for x in rate],
        "kernel_ms_min": round(float(kms.min()), 4), "kernel_ms_max": round(float(kms.max()), 4),
        "kernel_ms_argmax": slow,
        "search_ms_min": round(float(sms.min()), 4), "search_ms_max": round(float(sms.max()), 4),
        "search_ms_argmax": int(np.argmax(sms)),
        "gather_ms": {"median": round(float(np.median(gmed)), 4), "max": round(float(gmax.max()), 4)},
        "kernel_balance_efficiency": round(float(cells.sum() / (kms.max() * 1e-3) / rate.sum()), 4),
        "residue_imbalance": round(float(res.max() / res.mean()), 5),
        "step_split_ms": {"step": round(step_s * 1e3, 4), "kernel_max": round(float(kms.max()), 4),
                          "search_host_overhead": round(float(sms[slow] - kms[slow]), 4),
                          "gather_median": round(float(np.median(gmed)), 4),
                          "rest": round(step_s * 1e3 - float(sms[slow]) - float(np.median(gmed)), 4)},
    }


def fixture_match(w, sh, res, k, world):
    """The step's top-k against the reference's own search of this exact DB
    (tests/golden/fullsize.json: c2, c3, the c4 / c5 shares, c4full = the
    whole 10 M DB, c5full / c5share8, c2x2/4/8 = C2's weak-scaling DBs); at
    N > 1 rank 0 holds the gathered global top-k of the N shards.  None when
    no fixture is this DB."""
    fxs = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))

    def same_db(fx):
        return (fx.get("kind", "protein") == w.db and w.alphabet == fx.get("alphabet", "bg20")
                and w.lengths == fx.get("lengths", "gamma") and fx["n"] == sh.total and fx["i1"] == sh.job_ids
                and w.long_tail == fx.get("tail", 0) and fx.get("query_file") == w.cfg.get("query_file")
                and fx["qlen"] == sh.qlen and fx["algo"] == w.algo and fx["gap_open"] == w.gap_open
                and fx["gap_extend"] == w.gap_extend and fx["matrix"] == w.matrix)
    fx = next((f for f in fxs.values() if same_db(f)), None)
    if res is None:
        return None      # ranks > 0 hold no gathered result
    if fx and (w.long_tail == 0 or world == 1) and k in (1, 10, 64):
        return "match" if [list(map(int, x[:2])) for x in res] == fx[f"top{k}"] else "MISMATCH"
    return None


def traffic_key(w, sh, st):
    """profiles/traffic.json key: the exact workload the PMC pass profiled."""
    return (f"{w.config}:{w.algo}:{w.matrix}:{w.alphabet}:{w.lengths}:tail{w.long_tail}:seqs{sh.seqs}:"
            f"q{sh.qlen}:rows{st['strip_rows']}")


def north_star(S, args, job):
    """BASELINE.json north_star as its own record: SW int16, BLOSUM62
    -11/-1, the 400-residue query (seed 7) against the FIXED 10 M-sequence
    DB of tests/golden/fullsize.json "c4full", cut into `world`
    residue-balanced ID slices -- strong scaling, like the reference's own
    thread-scaling benchmark (benchmark/src/benchmark_threads.c:34-60, timed
    as benchmark/src/benchmark_util.c:27-48).  Each rank generates and packs
    only its slice; the slices' logs meet through the same gather as the
    headline; the top-k is checked against c4full's (the 64-bit replay,
    width-independent)."""
    w = workload(args, "north_star", overrides=False)
    sh = load_shard(S, w, job)
    steps = args.north_star_steps if args.north_star_steps is not None else min(args.steps, 10)
    t = timed_steps(S, job, sh, w, steps, 1, args.k)
    kms = t.avg["kernel_ms"]
    kernel_gcups = sh.cells_local / (kms * 1e-3) / 1e9
    value = sh.total_cells / (t.elapsed / steps) / 1e9
    rec = {
        "workload": "SW int16 BLOSUM62 gaps -11/-1, 400-residue query (seed 7) vs the fixed 10 M-sequence "
                    "synthetic protein DB (tests/golden/fullsize.json c4full), residue-balanced ID slices per GPU",
        "scaling": "strong", "bit_width": 16, "n_gpus": args.n_gpus, "ranks": job.world, "steps": steps, "warmup": 1,
        "ms_per_step": round(t.elapsed / steps * 1e3, 3), "value": round(value, 2), "unit": "GCUPS",
        "target_gcups": 1000.0, "meets_target": value >= 1000.0,
        "db_total_seqs": sh.total, "db_total_residues": int(job.sum(sh.residues)),
        "cells_per_step": sh.total_cells,
        "rank0": {"seqs": sh.seqs, "residues": sh.residues, "kernel_ms": round(kms, 4),
                  "kernel_gcups": round(kernel_gcups, 2)},
        "kernel_ms_max_over_ranks": round(job.max(kms), 4),
        "kernel_gcups_min_over_ranks": round(job.min(kernel_gcups), 2),
        "search_ms_rank0": round(t.avg["search_ms"], 4),
        "hbm": {"algorithmic_bytes_rank0": float(t.st["kernel_bytes"]),
                "frac_of_peak": float(t.st["kernel_bytes"]) / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "setup_s": round(job.max(sh.setup_s), 1),
        "top_hit": list(map(int, t.res[0][:2])) if t.res else None,   # (rank 0: the gathered result)
        "gather": ("ssa_amd_gather_logs (RCCL)" if job.native else "torch.distributed") if job.world > 1 else None,
    }
    if t.ranks is not None:
        rec["ranks_split"] = t.ranks
    m = fixture_match(w, sh, t.res, args.k, job.world)
    if m is not None:
        rec["topk_vs_reference"] = m
    S.free_sequence(sh.qq)
    return rec


def drop_in_measure(S, args, torch_sync=None):
    """The drop_in record's measurement, run in a process of its own
    (bench.py --drop-in-child, started by drop_in below with SSA_AMD_DEVICES
    set): an UNCHANGED libssa caller -- no ssa_amd_set_device(s) call -- opens
    the north-star DB (the fixed 10 M sequences; --drop-in-seqs: its first S
    IDs) and the library, reading SSA_AMD_DEVICES at init_db, searches it on
    every listed device (include/libssa_amd.h: one persistent host thread per
    device slot inside sw_align, the DB cut into chunk-aligned residue-balanced
    record ranges, the slot logs merged on the host; the reference's own
    default is every core of the machine, src/util/thread_pool.c:39-47, its
    heaps merged in thread order, src/algo/manager.c:141-145).
    free_alignment(sw_align(...)) is timed exactly as the N = 1 headline."""
    w = workload(args, "north_star", overrides=False)
    from libssa_amd import synthetic as syn
    t0 = time.time()
    configure(S, w)
    q = W.query(w.cfg, w.qlen)
    _, total, job_ids = W.cuts(w.cfg, 1, q, args.drop_in_seqs, w.lengths)
    codes, off = W.slice_db(w.cfg, q, total, 0, job_ids, w.alphabet, w.lengths)
    tmpdir = tempfile.mkdtemp(prefix="ssa_dropin_")
    path = os.path.join(tmpdir, "db.fas")
    syn.write_fasta(path, codes, off)
    residues, seqs = int(off[-1]), len(off) - 1
    del codes, off
    S.init_db(path)
    devices = list(S.get_devices())
    S.set_id_offset(0)
    S.prepare_db()
    os.remove(path)
    os.rmdir(tmpdir)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    setup_s = time.time() - t0
    steps = args.north_star_steps if args.north_star_steps is not None else min(args.steps, 10)
    k = args.k
    S.align_free(qq, k, w.width, S.SW)                      # warm-up
    st0 = S.stats()
    if torch_sync:
        torch_sync()
    ts = time.perf_counter()
    for _ in range(steps):
        S.align_free(qq, k, w.width, S.SW)
    if torch_sync:
        torch_sync()
    elapsed = time.perf_counter() - ts
    st1 = S.stats()
    res = S.align_scores(qq, k, w.width, S.SW)             # untimed: the result and its per-slot split
    last = S.stats()
    S.free_sequence(qq)
    cells = float(residues) * len(q)
    step_ms = elapsed / steps * 1e3
    n = max(1, st1["total_searches"] - st0["total_searches"])
    skm, ssm = last["slot_kernel_ms"], last["slot_search_ms"]
    slow = int(np.argmax(ssm)) if ssm else 0
    rec = {
        "workload": "SW int16 BLOSUM62 gaps -11/-1, 400-residue query (seed 7) vs the north-star DB, one process, "
                    "an unchanged sw_align caller on every device SSA_AMD_DEVICES lists",
        "ssa_amd_devices": os.environ.get("SSA_AMD_DEVICES"),
        "devices": devices, "slots": int(last["slots"]), "bit_width": 16, "steps": steps, "warmup": 1,
        "db_seqs": seqs, "db_residues": residues, "cells_per_step": cells,
        "ms_per_step": round(step_ms, 3), "value": round(cells / (elapsed / steps) / 1e9, 2), "unit": "GCUPS",
        "kernel_ms_avg": round((st1["total_kernel_ms"] - st0["total_kernel_ms"]) / n, 4),
        "slot_device": list(last["slot_device"]), "slot_kernel_ms": [round(x, 4) for x in skm],
        "slot_search_ms": [round(x, 4) for x in ssm],
        # (the split of one search, the untimed one after the loop: its
        # slowest slot's kernel and host time, then the merge of the slot logs
        # and the rest of the call)
        "step_split_ms": {"step": round(step_ms, 4), "search": round(last["search_ms"], 4), "slowest_slot": slow,
                          "slot_kernel": round(skm[slow], 4) if skm else None,
                          "slot_host": round(ssm[slow] - skm[slow], 4) if skm else None,
                          "merge_and_rest": round(last["search_ms"] - ssm[slow], 4) if ssm else None},
        "setup_s": round(setup_s, 1),
        "top_hit": list(map(int, res[0][:2])) if res else None,
    }
    sh = argparse.Namespace(total=total, job_ids=job_ids, qlen=len(q))
    m = fixture_match(w, sh, res, k, 1)
    if m is not None:
        rec["topk_vs_reference"] = m
    return rec


def _run_child(cmd, env, timeout=900):
    """Runs the drop_in child; its last JSON line, or what went wrong."""
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"drop_in child exceeded {timeout} s"}
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"drop_in child exited with status {r.returncode}", "stderr_tail": r.stderr[-1500:]}
    return json.loads(lines[-1])


def drop_in(S, args, job, runner=None):
    """N > 1, after the multi-process records: the drop-in path, measured.
    Ranks != 0 release their device DBs (ssa_exit) and end (no collective
    follows); rank 0 releases its own and starts `bench.py --drop-in-child` with
    SSA_AMD_DEVICES listing one device slot per rank (a rehearsal's ranks
    share GPUs, so do its slots) -- a process of its own, so that whatever the
    single-process multi-GPU path does cannot take the multi-process line
    down with it (its failure becomes the record's "error").  Returns rank
    0's record (None elsewhere)."""
    if job.rank != 0:
        # (no barrier: a rank waiting in an RCCL barrier keeps a spinning
        # collective kernel on its GPU, which the child then shares)
        S.ssa_exit()
        return None
    S.ssa_exit()
    n_gpus = max(1, args.n_gpus)
    devices = [r % n_gpus for r in range(job.world)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")}
    env["SSA_AMD_DEVICES"] = ",".join(map(str, devices))
    cmd = [sys.executable, os.path.abspath(__file__), "--drop-in-child", "--k", str(args.k), "--steps", str(args.steps)]
    if args.north_star_steps is not None:
        cmd += ["--north-star-steps", str(args.north_star_steps)]
    if args.drop_in_seqs is not None:
        cmd += ["--drop-in-seqs", str(args.drop_in_seqs)]
    for o in getattr(args, "option", []):
        cmd += ["--option", o]
    t0 = time.time()
    rec = (runner or _run_child)(cmd, env)
    rec["child_wall_s"] = round(time.time() - t0, 1)
    rec["devices_requested"] = devices
    return rec


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the launcher: no torch, no GPU in this process
        sys.exit(launch(args, sys.argv[1:]))
    if args.launch_selftest:
        if "WORLD_SIZE" in os.environ:
            launch_selftest(args)
        return
    if args.drop_in_child:
        # (drop_in's child: no torch, no process group; the library reads
        # SSA_AMD_DEVICES at its first init_db -- this process never selects
        # a device itself)
        import libssa_amd as S
        S.load()
        S.set_output_mode(S.OUTPUT_ERROR)
        for o in args.option:
            k, v = o.split("=")
            S.set_option(k, int(v))
        print(json.dumps(drop_in_measure(S, args)), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    backend = os.environ.get("SSA_DIST_BACKEND", "nccl")   # nccl == RCCL on ROCm; gloo for rehearsal
    dev = "cuda" if backend == "nccl" else "cpu"
    ranks_per_gpu, args.n_gpus = 1, 1
    if world > 1:
        import torch
        import torch.distributed as dist
        # every rank derives the same layout from the world size and the
        # visible GPU count (a gloo rehearsal shares GPUs between ranks)
        local, ranks_per_gpu, args.n_gpus = W.rank_layout(world, torch.cuda.device_count(), local, backend)
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    job = Job(rank, world, dist, dev, backend)
    job.dev_index = local

    import libssa_amd as S

    S.load()
    S.set_device(local)
    S.set_output_mode(S.OUTPUT_ERROR)
    S.set_option("strip_np", args.strip_np)
    S.set_option("pair_np", args.pair_np)
    for o in args.option:
        k, v = o.split("=")
        S.set_option(k, int(v))
        _OPTIONS[k] = int(v)
    if world > 1 and backend == "nccl" and not args.torch_gather:
        setup_native_gather(S, job)

    # --- the headline workload (BASELINE.json metric; default C2)
    w = workload(args, args.config)
    sh = load_shard(S, w, job)
    t = timed_steps(S, job, sh, w, args.steps, args.warmup, args.k)
    res, st = t.res, t.st
    if args.timeline and world == 1:
        # untimed: every DP wave's start/end on the s_memrealtime clock
        S.set_option("timeline", 1)
        t.step()
        np.save(args.timeline, S.timeline())
        S.set_option("timeline", 0)
    S.free_sequence(sh.qq)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(sh.codes, sh.off, sh.q, matrix_table(w.matrix), w)
        except Exception as e:  # report, never hide
            cpu = {"value": None, "error": repr(e)}
    match = fixture_match(w, sh, res, args.k, world)
    codes_off = (sh.codes, sh.off)
    sh.codes = sh.off = None
    del codes_off

    # --- the north-star record (strong scaling of the fixed 10 M DB)
    ns = None if args.no_north_star else north_star(S, args, job)
    if job.native:
        S.dist_finalize()
    # --- the drop-in record (N > 1: one process on all N devices)
    di = None
    if world > 1 and not args.no_drop_in:
        di = drop_in(S, args, job)
        if di is not None and ns is not None and ns.get("value") and di.get("value"):
            di["vs_multi_process"] = round(di["value"] / ns["value"], 4)
    if rank != 0:
        dist.destroy_process_group()
        return

    steps = args.steps
    ms_per_step = t.elapsed / steps * 1e3
    gcups = sh.total_cells / (t.elapsed / steps) / 1e9
    kavg = t.avg["kernel_ms"]
    cells_local = sh.cells_local
    # algorithmic bytes per launch: every residue once (1 B) + 4 B score per
    # sequence + the strip profile table
    alg_bytes = float(st["kernel_bytes"])
    achieved = alg_bytes / (kavg * 1e-3) / 1e9
    tkey = traffic_key(w, sh, st)
    src_hash = W.kernel_src_hash()
    pf = W.profiled_figures(tkey, src_hash, os.path.join(ROOT, "profiles", "traffic.json"))
    traffic, tsrc = pf["traffic"], pf["source"]
    # VALU issue roofline: VOP3/VOP3P instructions issue at
    # 4.17 cycles per wave64 instruction per SIMD, v_add_u32 at 2.5 (measured
    # in isolation: profiles/r01/ubench_valu_rates4.txt); instructions per
    # cell from this build's PMC pass of this workload; the clock is the
    # engine's peak (a profiled pass runs slower, MI355X_MICROARCH.md: its
    # clock is reported beside, not used)
    kkey = (st["kernel"], st["strip_rows"])
    instr_per_cell = pf["valu_instr_per_cell"]
    if args.strip_np != 16:
        instr_per_cell = None
    fast = VALU_FAST_SHARE.get(kkey, 0.0)
    issue_cycles = (1.0 - fast) * 4.17 + fast * 2.5
    valu_bound = (1024 * PEAK_CLOCK_GHZ * 1e9 / issue_cycles * 64 / instr_per_cell) if instr_per_cell else None
    out = {
        "metric": "GCUPS (SW int16, 400aa query vs synthetic DB) at 1/2/4/8 MI355X; top-k score bit-exact",
        "value": round(gcups, 2),
        "unit": "GCUPS",
        "n_gpus": args.n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if w.strong else "weak",
        "vs_baseline": None,
        "dtype": "i16",
        "data": "synthetic",
        "config": {"workload": f"{w.config.upper()}: {w.algo.upper()} {w.matrix} gaps {w.gap_open}/{w.gap_extend}, "
                               f"{sh.qlen}-residue query vs {sh.seqs} synthetic {w.db} seqs per GPU "
                               f"(mean len {sh.residues / max(sh.seqs, 1):.1f}), top-{args.k}",
                   "db_seqs_per_gpu": sh.seqs, "db_total_seqs": sh.total, "query_len": sh.qlen,
                   "residues_per_gpu": sh.residues, "cells_per_step": sh.total_cells,
                   "parallelism": f"db-shard x{world}", "job_seqs": sh.job_ids, "pair_strip_rows": st["strip_rows"],
                   "strip_np": args.strip_np, "bit_width": w.width},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_key": tkey,
                     "traffic_source": tsrc, "kernel_src": src_hash, "traffic_stale": pf["stale"],
                     **({"traffic_stale_source": pf["stale_source"]} if pf.get("stale_source") else {}),
                     # the resource that actually binds this integer DP
                     "binding": {"bound": "valu_issue",
                                 "achieved": round(cells_local / (kavg * 1e-3) / 1e9, 2),
                                 "peak": round(valu_bound / 1e9, 1) if valu_bound else None, "unit": "GCUPS",
                                 "clock_ghz": PEAK_CLOCK_GHZ, "pmc_pass_clock_ghz": pf["clock_ghz"],
                                 "valu_instr_per_cell": instr_per_cell,
                                 "frac": (cells_local / (kavg * 1e-3)) / valu_bound if valu_bound else None}},
        "kernel": {"name": st["kernel"], "avg_ms": round(kavg, 4),
                   "kernel_gcups": round(cells_local / (kavg * 1e-3) / 1e9, 2),
                   "wide_ms_avg": round(t.avg["wide_ms"], 4), "wide_count": int(st["wide_count"]),
                   "valu_issue_bound_gcups": round(valu_bound / 1e9, 1) if valu_bound else None,
                   "valu_issue_frac": (cells_local / (kavg * 1e-3)) / valu_bound if valu_bound else None,
                   "valu_instr_per_cell": instr_per_cell},
        "host_ms": {"search_call": round(t.avg["search_ms"], 3), "prep": round(t.avg["prep_ms"], 3),
                    "upload": round(t.avg["upload_ms"], 3), "sync_wait": round(t.avg["sync_wait_ms"], 3),
                    "d2h_filter": round(t.avg["d2h_ms"], 3), "replay": round(t.avg["replay_ms"], 3)},
        "setup_s": round(sh.setup_s, 1),
        "setup": {"generate_and_write_fasta_s": round(sh.gen_s, 1), "init_db_and_pack_s": round(sh.load_s, 1),
                  "pack_ms": round(st["pack_ms"], 1)},
        "top_hit": list(map(int, res[0][:2])) if res else None,
        "gather": ("ssa_amd_gather_logs (RCCL)" if job.native else "torch.distributed") if world > 1 else None,
        "gather_equals_torch_gather": job.gather_checked,
        "rccl_ranks": job.rccl_ranks,
        "launcher": os.environ.get("SSA_BENCH_LAUNCHER", "torchrun" if world > 1 else None),
    }
    if t.ranks is not None:
        out["ranks_split"] = t.ranks
    if ranks_per_gpu > 1:
        out["ranks"] = world
        out["rehearsal"] = rehearsal_label(world, args.n_gpus, backend)
    if job.gather_note:
        out["gather_note"] = job.gather_note
    if match is not None:
        out["topk_vs_reference"] = match
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if ns is not None:
        out["north_star"] = ns
    if di is not None:
        out["drop_in"] = di
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
