"""Multi-process exchange of a sharded search on CPU (gloo, world size 2 and 3).

Each rank scores its contiguous ID shard with the oracle, builds the shard's
insertion log (what ssa_amd_search(..., SSA_AMD_LOG) returns on a GPU), and
the ranks run the production exchange (libssa_amd.dist: all_gather of log
lengths + one gather + ssa_amd_replay on rank 0).  Rank 0's result must equal
the single-process 64-bit reference top-k, tie IDs included.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from libssa_amd import synthetic as syn
from oracle import pyoracle as po
from tests.conftest import GOLDEN


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cuts, k, outdir, cap=None):
    import torch.distributed as dist
    import libssa_amd as S
    from libssa_amd.dist import global_topk
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    S.load()
    q = syn.protein_query(50, 1)
    codes, off = syn.protein_db(3000, 4, query=q, plant_every=200, lo=0, hi=150)
    tabs = np.load(os.path.join(GOLDEN, "tables.npz"))
    M = tabs["matrices"][2].copy()  # blosum62
    a, b = cuts[rank], cuts[rank + 1]
    sc = po.scores(0, q, codes, off, M, -11, -1)[a:b]
    lens = np.diff(off)[a:b]
    keep = np.nonzero(lens > 0)[0]
    log = po.topk_log(sc[keep], (keep + a).astype(np.uint64), k)
    res = global_topk([(s, i, 0, 0, 0) for s, i in log], k, dist, rank, world, "cpu",
                      **({} if cap is None else {"cap": cap}))
    if rank == 0:
        allsc = po.scores(0, q, codes, off, M, -11, -1)
        nz = np.nonzero(np.diff(off) > 0)[0]
        exp = po.topk(allsc[nz], nz.astype(np.uint64), k)
        with open(os.path.join(outdir, f"r{k}_{cap}.txt"), "w") as f:
            f.write("ok" if res == exp else f"mismatch {res[:5]} {exp[:5]}")
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cuts", [(2, [0, 1500, 3000]), (3, [0, 7, 2222, 3000])])
@pytest.mark.parametrize("k", [1, 10, 137])
def test_gloo_gather_replay_equals_single_process(tmp_path, world, cuts, k):
    mp.spawn(_worker, args=(world, _free_port(), cuts, k, str(tmp_path)), nprocs=world, join=True)
    assert open(tmp_path / f"r{k}_None.txt").read() == "ok"


@pytest.mark.parametrize("cap", [1, 40])
def test_gloo_log_longer_than_cap_falls_back(tmp_path, cap):
    """A shard log longer than the fixed exchange buffer takes the exact-size
    gather; the result is unchanged."""
    mp.spawn(_worker, args=(2, _free_port(), [0, 1500, 3000], 137, str(tmp_path), cap), nprocs=2, join=True)
    assert open(tmp_path / f"r137_{cap}.txt").read() == "ok"


def test_shard_log_property():
    """Every element accepted by the global heap is in its shard's log."""
    rng = np.random.default_rng(1)
    sc = rng.integers(0, 30, 4000)
    ids = np.arange(4000, dtype=np.uint64)
    for k in (1, 5, 64):
        glob = set(po.topk_log(sc, ids, k))
        shards = set()
        for a, b in ((0, 1000), (1000, 3333), (3333, 4000)):
            shards |= set(po.topk_log(sc[a:b], ids[a:b], k))
        assert glob <= shards


@pytest.mark.parametrize("cuts", [[0, 4000], [0, 1000, 3333, 4000], [0, 0, 17, 2500, 2500, 4000]])
@pytest.mark.parametrize("k", [1, 10, 300])
def test_native_merge_logs_equals_single_process(cuts, k):
    """ssa_amd_merge_logs -- rank 0's half of ssa_amd_gather_logs (csrc/dist.cpp)
    -- over shard logs in shard order equals the single-process reference
    heap, tie IDs included (tie-heavy scores, empty shards)."""
    import libssa_amd as S
    rng = np.random.default_rng(k)
    sc = rng.integers(0, 40, 4000)
    ids = np.arange(4000, dtype=np.uint64)
    logs = [[(s, i, 0, 0, 0) for s, i in po.topk_log(sc[a:b], ids[a:b], k)] for a, b in zip(cuts, cuts[1:])]
    assert S.merge_logs(logs, k) == po.topk(sc, ids, k)


@pytest.mark.gpu
def test_native_rccl_gather_world1(tmp_path):
    """ssa_amd_dist_init + ssa_amd_gather_logs over RCCL with one rank (the
    one-GPU box; the driver's 8-GPU run exercises N > 1): the ncclGather of
    fixed 513-row slots, for a log within the slot and one longer than it
    (rank 0's own rows beyond the slot are read from memory; with one rank no
    point-to-point remainder is sent -- that path runs over RCCL only at
    N > 1 and in-process in test_native_gather_fake_world), returns the
    replayed top-k."""
    import libssa_amd as S
    S.load()
    S.set_device(0)
    S.dist_init(0, 1, S.dist_unique_id())
    try:
        rng = np.random.default_rng(3)
        for n, k in ((300, 10), (5000, 2000)):
            sc = np.sort(rng.integers(0, 10 ** 6, n))       # rising: the log is the whole shard
            ids = np.arange(n, dtype=np.uint64)
            log = [(s, i, 0, 0, 0) for s, i in po.topk_log(sc, ids, k)]
            assert S.gather_logs(log, k) == po.topk(sc, ids, k)
    finally:
        S.dist_finalize()


def _fake_gather(logs, k, group):
    """Runs ssa_amd_gather_logs from len(logs) host threads, each the rank of
    an in-process group (ssa_amd_dist_init_fake); returns every rank's result
    and the ranks each saw."""
    import threading
    import libssa_amd as S
    W = len(logs)
    res, ranks, errs = [None] * W, [None] * W, []
    rounds = [None] * W

    def run(r):
        try:
            S.dist_init_fake(r, W, group)
            try:
                ranks[r] = S.dist_ranks()
                res[r] = S.gather_logs(logs[r], k)
                rounds[r] = S.stats()["gather_rounds"]
            finally:
                S.dist_finalize()
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not any(t.is_alive() for t in th), "fake collective did not drain"
    assert not errs, errs
    # one slot gather on every rank; the point-to-point remainder only on the
    # ranks whose log exceeds the 512-row slot and on rank 0 when any does
    long = [len(x) > 512 for x in logs]
    assert rounds[1:] == [2 if x else 1 for x in long[1:]], rounds
    assert rounds[0] == (2 if any(long[1:]) else 1), rounds
    return res, ranks


def _cuts(n, W, rng, empty):
    c = np.sort(rng.integers(0, n + 1, W - 1))
    if empty:
        c[: max(1, (W - 1) // 2)] = c[0]       # some ranks get no records
    return [0, *c.tolist(), n]


@pytest.mark.parametrize("W", [2, 3, 8])
@pytest.mark.parametrize("k", [1, 10, 300])
@pytest.mark.parametrize("kind", ["ties", "rising", "empty"])
def test_native_gather_fake_world(W, k, kind):
    """ssa_amd_gather_logs at W > 1 without hardware: W threads exchange
    through the library's in-process transport (the same slot layout, count
    rows and point-to-point remainder as over RCCL).  Rank 0 gets the
    single-process reference top-k (tie IDs included), the others nothing.
    "rising" scores make every shard log longer than the 512-row slot at
    k = 300, i.e. the point-to-point remainder; "empty" leaves ranks with no log."""
    rng = np.random.default_rng(W * 1000 + k)
    n = 6000
    if kind == "rising":
        sc = np.sort(rng.integers(0, 10 ** 6, n))
    else:
        sc = rng.integers(0, 40, n)
    ids = np.arange(n, dtype=np.uint64)
    cuts = _cuts(n, W, rng, kind == "empty")
    logs = [[(int(s), int(i), 0, 0, 0) for s, i in po.topk_log(sc[a:b], ids[a:b], k)] for a, b in zip(cuts, cuts[1:])]
    if kind == "rising" and k == 300:
        assert max(len(x) for x in logs) > 512
    res, ranks = _fake_gather(logs, k, group=W * 100 + k)
    assert ranks == [W] * W
    assert res[0] == po.topk(sc, ids, k)
    assert all(r == [] for r in res[1:])


def test_native_gather_fake_repeated_rounds():
    """Several gathers on one fake group, alternating one- and two-round
    exchanges (buffers grow and are reused): each equals the reference."""
    import threading
    import libssa_amd as S
    W, rng = 4, np.random.default_rng(5)
    cases = []
    for j, k in enumerate((10, 600, 1, 600, 64)):
        n = 4000
        sc = np.sort(rng.integers(0, 10 ** 5, n)) if k == 600 else rng.integers(0, 30, n)
        ids = np.arange(n, dtype=np.uint64)
        cuts = _cuts(n, W, rng, False)
        logs = [[(int(s), int(i), 0, 0, 0) for s, i in po.topk_log(sc[a:b], ids[a:b], k)]
                for a, b in zip(cuts, cuts[1:])]
        cases.append((logs, k, po.topk(sc, ids, k)))
    out = [[] for _ in range(W)]

    def run(r):
        S.dist_init_fake(r, W, 999)
        for logs, k, _ in cases:
            out[r].append(S.gather_logs(logs[r], k))
        S.dist_finalize()

    th = [threading.Thread(target=run, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not any(t.is_alive() for t in th)
    assert [x for x in out[0]] == [c[2] for c in cases]


def test_native_gather_fake_refusals():
    import libssa_amd as S
    S.load()
    assert S.dist_ranks() == 0
    with pytest.raises(RuntimeError):
        S.dist_init_fake(2, 2, 7)           # rank out of range
    S.dist_init_fake(0, 2, 8)
    with pytest.raises(RuntimeError):
        S.dist_init_fake(1, 2, 8)           # this thread already holds a rank
    S.dist_finalize()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("order", ["sorted", "reverse", "random"])
def test_shard_bounds_balance_residues(world, order):
    """ssa_amd_shard_bounds: contiguous ID ranges with residue sums within
    1 % of each other on a length-sorted DB (where cutting by sequence count
    would be off by ~10x), and at chunk-size multiples when asked."""
    import libssa_amd as S
    rng = np.random.default_rng(world)
    lens = np.clip(1 + rng.gamma(2.0, 175.0, 200_000).round(), 16, 4096).astype(np.uint64)
    if order == "sorted":
        lens = np.sort(lens)
    elif order == "reverse":
        lens = np.sort(lens)[::-1].copy()
    b = S.shard_bounds(lens, world)
    assert b[0] == 0 and b[-1] == len(lens) and all(x <= y for x, y in zip(b, b[1:]))
    res = [int(lens[x:y].sum()) for x, y in zip(b, b[1:])]
    assert max(res) / min(res) <= 1.01, res
    by_count = [int(lens[i * len(lens) // world:(i + 1) * len(lens) // world].sum()) for i in range(world)]
    if order != "random":
        assert max(by_count) / min(by_count) > 1.5
    b = S.shard_bounds(lens, world, align=1000)
    assert all(x % 1000 == 0 for x in b[:-1])
    res = [int(lens[x:y].sum()) for x, y in zip(b, b[1:])]
    assert max(res) / min(res) <= 1.1, res


def test_shard_bounds_edges():
    import libssa_amd as S
    assert S.shard_bounds([], 3) == [0, 0, 0, 0]
    assert S.shard_bounds([5], 1) == [0, 1]
    b = S.shard_bounds([0, 0, 10, 0, 10, 0], 2)
    assert b[0] == 0 and b[-1] == 6 and sum([0, 0, 10, 0, 10, 0][b[0]:b[1]]) == 10
    with pytest.raises(ValueError):
        S.shard_bounds([1, 2], 0)


# ---------------------------------------------------------------- bench.py launcher
BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")


def _bench(args, env_extra=None, timeout=300):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launcher_spawns_ranks(world):
    """`bench.py --gpus N` without a launcher starts N rank processes itself
    (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT), the ranks meet over
    gloo, and the parent prints rank 0's single JSON line."""
    import json
    r = _bench(["--gpus", str(world), "--launch-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["launch_selftest"] == "ok" and d["world"] == world
    assert [x["rank"] for x in d["ranks"]] == list(range(world))
    assert [x["local_rank"] for x in d["ranks"]] == list(range(world))
    assert len({x["pid"] for x in d["ranks"]}) == world
    assert all(x["launcher"] == "bench.py --gpus" for x in d["ranks"])


@pytest.mark.parametrize("world,visible,rehearsal", [(2, 1, True), (3, 1, True), (2, 8, False), (8, 8, False)])
def test_bench_rank_layout_labels_rehearsals(world, visible, rehearsal):
    """Every rank derives the same layout from the world size and the
    visible GPU count: a gloo run with more ranks than GPUs says
    "rehearsal" and counts physical GPUs in n_gpus (it never claims N GPUs
    for one GPU's work); one rank per GPU is not a rehearsal."""
    import json
    r = _bench(["--gpus", str(world), "--launch-selftest"],
               env_extra={"SSA_DIST_BACKEND": "gloo", "SSA_BENCH_VISIBLE_GPUS": str(visible)})
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    lay = [x["layout"] for x in d["ranks"]]
    assert all(x["n_gpus"] == min(world, visible) for x in lay)
    assert [x["device"] for x in lay] == [r % visible for r in range(world)]
    if rehearsal:
        assert all(x["ranks_per_gpu"] == -(-world // visible) for x in lay)
        assert all(x["rehearsal"] == f"{world} ranks on {visible} GPU(s), exchange over gloo" for x in lay)
    else:
        assert all(x["ranks_per_gpu"] == 1 and "rehearsal" not in x for x in lay)


def test_rank_layout_refuses_doubling_up_without_gloo():
    from libssa_amd import workloads as W
    assert W.rank_layout(1, 0, 0, "nccl") == (0, 1, 1)
    assert W.rank_layout(4, 8, 3, "nccl") == (3, 1, 4)
    assert W.rank_layout(4, 2, 3, "gloo") == (1, 2, 2)
    with pytest.raises(SystemExit):
        W.rank_layout(4, 2, 3, "nccl")


def test_workload_cuts_balance_and_cover():
    """The cut bench.py and the GPU tests share (libssa_amd/workloads.py):
    weak configs N x seqs IDs, strong ones the fixed DB; protein slices
    balanced by residues, contiguous, covering the job."""
    from libssa_amd import synthetic as syn
    from libssa_amd import workloads as W
    cfg = W.CONFIGS["north_star"]
    q = W.query(cfg)
    b, total, job = W.cuts(cfg, 4, q, seqs=None)
    assert total == job == 10_000_000 and b[0] == 0 and b[-1] == job and b == sorted(b)
    lens = syn.protein_lengths_range(total, 42, 0, job, query=q)
    res = [int(lens[x:y].sum()) for x, y in zip(b, b[1:])]
    assert max(res) / min(res) <= 1.001
    b2, total2, job2 = W.cuts(W.CONFIGS["c2"], 2, q, seqs=1000)
    assert (total2, job2) == (2000, 2000) and b2[0] == 0 and b2[-1] == 2000
    b5, total5, job5 = W.cuts(W.CONFIGS["c5"], 8, W.query(W.CONFIGS["c5"]))
    assert total5 == job5 == 50_000_000 and b5 == [r * 6_250_000 for r in range(9)]
    # a per-rank share of a strong config: cut by count (the c4 fixture's first share)
    b4, _, job4 = W.cuts(W.CONFIGS["c4"], 2, q, seqs=1_250_000)
    assert b4 == [0, 1_250_000, 2_500_000] and job4 == 2_500_000


def test_bench_launcher_propagates_failure():
    """A rank that dies takes the job down: the parent stops the others
    (which wait in the rendezvous for it) and exits with that rank's status."""
    import time
    t0 = time.time()
    r = _bench(["--gpus", "3", "--launch-selftest", "--selftest-fail-rank", "1"], timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with status 3" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert time.time() - t0 < 90


def test_bench_launcher_refuses_more_ranks_than_gpus():
    """N > visible GPUs fails loudly instead of doubling ranks up (this
    container has none)."""
    r = _bench(["--gpus", "2", "--no-cpu-baseline"], env_extra={"SSA_DIST_BACKEND": "nccl"})
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr


def _split_worker(rank, world, port, outdir):
    """One rank of the N > 1 bench line's per-rank split (bench.rank_split):
    synthetic per-rank times, the real all-gather over gloo."""
    import argparse
    import json
    import sys
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(BENCH))
    import bench
    job = bench.Job(rank, world, dist, "cpu", "gloo")
    # rank r: kernel (10 + r) ms over (1 + r / 10) x 1e9 residues of a 400-residue query
    res = int((1 + rank / 10) * 1e9)
    sh = argparse.Namespace(residues=res, cells_local=float(res) * 400, seqs=1000 + rank)
    avg = {"kernel_ms": 10.0 + rank, "search_ms": 10.2 + rank}
    split = {"search_s": [(10.2 + rank) / 1e3] * 5, "gather_s": [(0.05 + 0.01 * rank) / 1e3] * 4 + [1e-3]}
    out = bench.rank_split(job, sh, avg, split, (10.5 + world) / 1e3)
    if rank == 0:
        with open(os.path.join(outdir, "split.json"), "w") as f:
            json.dump(out, f)
    dist.destroy_process_group()


class _FakeLib:
    """The library calls bench.drop_in / drop_in_measure make, recorded (no
    GPU): init_db reads SSA_AMD_DEVICES as the library does; each search
    'runs' on every slot; slot s takes (1 + s) ms of kernel."""
    AMINOACID, NUCLEOTIDE, FORWARD_STRAND, MATRIX_BUILDIN, READ_FROM_STRING, SW = 0, 1, 1, 2, 1, 0

    def __init__(self, env=None):
        self.calls, self.devices, self.searches, self.records, self.env = [], [], 0, None, env or {}

    def __getattr__(self, name):        # configuration calls: recorded only
        return lambda *a: self.calls.append((name,) + a)

    def ssa_exit(self):
        self.calls.append(("ssa_exit",))

    def init_db(self, path):
        self.records = open(path).read().count(">")
        self.devices = [int(x) for x in self.env.get("SSA_AMD_DEVICES", "0").split(",")]
        self.calls.append(("init_db",))

    def get_devices(self):
        return list(self.devices)

    def align_free(self, q, k, width, algo):
        self.searches += 1

    def align_scores(self, q, k, width, algo):
        self.searches += 1
        return [(100 - i, 7 * i) for i in range(k)]

    def stats(self):
        n = len(self.devices)
        return {"total_searches": self.searches, "total_kernel_ms": float(n) * self.searches, "slots": n,
                "search_ms": 0.5 + n,
                "slot_device": list(self.devices), "slot_kernel_ms": [1.0 + s for s in range(n)],
                "slot_search_ms": [1.25 + s for s in range(n)]}


def _dropin_worker(rank, world, port, outdir):
    """One rank of bench.drop_in over gloo with the fake library; rank 0's
    child process is stood in for by drop_in_measure on a fake library that
    sees the child's environment."""
    import argparse
    import json
    import sys
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(BENCH))
    import bench
    job = bench.Job(rank, world, dist, "cpu", "gloo")
    job.dev_index = 0
    args = argparse.Namespace(n_gpus=1, steps=4, north_star_steps=None, k=10, drop_in_seqs=3000, cpu_seconds=1.0,
                              option=["graph=1"])
    lib = _FakeLib()
    child = {}

    def runner(cmd, env):
        child.update(cmd=cmd, env={k: env[k] for k in ("SSA_AMD_DEVICES",) if k in env},
                     ranked=[k for k in ("RANK", "WORLD_SIZE", "MASTER_PORT") if k in env])
        clib = _FakeLib(env)
        rec = bench.drop_in_measure(clib, args)
        child.update(calls=[c[0] for c in clib.calls], records=clib.records, searches=clib.searches)
        return rec
    rec = bench.drop_in(lib, args, job, runner=runner)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump({"rec": rec, "calls": [c[0] for c in lib.calls], "searches": lib.searches, "child": child}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_drop_in_record_on_gloo_rehearsal(tmp_path, world):
    """The N > 1 line's drop_in record (bench.drop_in): ranks != 0 release
    their device DBs and end; rank 0 releases its own and runs a child
    process (bench.py --drop-in-child) with SSA_AMD_DEVICES naming one device
    slot per rank -- a rehearsal on one GPU puts them all on device 0 -- and
    no rank variables; the child, an unchanged caller (no device selection of
    its own), opens the north-star DB (its first 3000 IDs here), times
    free_alignment(sw_align(...)) and reports the per-slot kernel / search
    split."""
    import json
    mp.spawn(_dropin_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = json.load(open(tmp_path / "rank0.json"))
    d, ch = r0["rec"], r0["child"]
    assert "--drop-in-child" in ch["cmd"] and ["--option", "graph=1"] == ch["cmd"][-2:]
    assert ch["env"]["SSA_AMD_DEVICES"] == ",".join(["0"] * world) and ch["ranked"] == []
    assert "set_device" not in ch["calls"] and "set_devices" not in ch["calls"]
    assert d["devices"] == [0] * world and d["slots"] == world and d["devices_requested"] == [0] * world
    assert d["db_seqs"] == 3000 and ch["records"] == 3000 and d["steps"] == 4
    assert d["cells_per_step"] == d["db_residues"] * 400
    assert d["slot_kernel_ms"] == [1.0 + s for s in range(world)]
    assert d["slot_search_ms"] == [1.25 + s for s in range(world)]
    sp = d["step_split_ms"]
    assert sp["slowest_slot"] == world - 1 and sp["slot_kernel"] == world and sp["slot_host"] == 0.25
    assert sp["search"] == 0.5 + world and sp["merge_and_rest"] == 0.25
    assert abs(sp["step"] - d["ms_per_step"]) < 1e-3 and d["value"] > 0
    assert d["top_hit"] == [100, 0] and "topk_vs_reference" not in d      # (a 3000-ID slice: no fixture)
    assert ch["searches"] == 4 + 2                                            # warm-up, 4 timed, the result
    assert r0["calls"] == ["ssa_exit"] and r0["searches"] == 0
    for r in range(1, world):
        rr = json.load(open(tmp_path / f"rank{r}.json"))
        assert rr["rec"] is None and rr["calls"] == ["ssa_exit"] and rr["searches"] == 0 and rr["child"] == {}


def test_bench_drop_in_child_failure_is_reported():
    """A failing child becomes the record's error, never the line's end."""
    import sys
    sys.path.insert(0, os.path.dirname(BENCH))
    import bench
    rec = bench._run_child([sys.executable, "-c", "import sys; sys.stderr.write('boom'); sys.exit(3)"], dict(os.environ))
    assert rec["error"].endswith("status 3") and rec["stderr_tail"] == "boom"
    rec = bench._run_child([sys.executable, "-c", "print('{\"value\": 5}')"], dict(os.environ))
    assert rec == {"value": 5}


@pytest.mark.parametrize("world", [2, 4])
def test_bench_rank_split_explains_the_step(tmp_path, world):
    """The N > 1 bench line explains its own result (what the driver's first
    8-GPU run reports): per-rank kernel and search ms (min / max / rank of
    max), the gather's own time (median and max over ranks and steps), the
    kernel balance efficiency, the residue imbalance of the cut and the step
    split, all gathered from every rank over the process group."""
    import json
    mp.spawn(_split_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d = json.load(open(tmp_path / "split.json"))
    assert d["kernel_ms"] == [10.0 + r for r in range(world)]
    assert d["search_ms"] == [round(10.2 + r, 4) for r in range(world)]
    assert d["kernel_ms_max"] == 10.0 + world - 1 and d["kernel_ms_argmax"] == world - 1
    assert d["search_ms_min"] == 10.2 and d["search_ms_argmax"] == world - 1
    assert d["gather_ms"]["max"] == 1.0
    assert d["gather_ms_median"] == [round(0.05 + 0.01 * r, 4) for r in range(world)]
    assert d["seqs"] == [1000 + r for r in range(world)]
    res = np.array([(1 + r / 10) * 1e9 for r in range(world)])
    kms = np.array([10.0 + r for r in range(world)])
    eff = (res * 400).sum() / (kms.max() * 1e-3) / ((res * 400) / (kms * 1e-3)).sum()
    assert abs(d["kernel_balance_efficiency"] - eff) < 1e-4 and d["kernel_balance_efficiency"] < 1
    assert abs(d["residue_imbalance"] - res.max() / res.mean()) < 1e-5
    sp = d["step_split_ms"]
    assert sp["kernel_max"] == kms.max() and abs(sp["search_host_overhead"] - 0.2) < 1e-6
    assert abs(sp["step"] - (sp["search_host_overhead"] + sp["kernel_max"] + sp["gather_median"] + sp["rest"])) < 1e-3
