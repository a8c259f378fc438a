"""bench.py's workloads (BASELINE.json configs) and how a job cuts them into
rank slices -- one module, so the GPU tests search exactly the slices the
driver's `bench.py --gpus N` runs.

A workload's DB is block-seeded (synthetic.protein_db_range /
dna_reads_range): any ID slice is byte-identical to the same IDs of the whole
DB, so a rank generates only its own slice.  Weak configs (total_seqs None)
search an N x seqs DB at N ranks; strong ones search one fixed DB at every N.
At N > 1 protein jobs are cut so that the ranks' residue sums balance
(ssa_amd_shard_bounds, the unit boundary nearest each ideal share), DNA reads
(equal lengths) by count.
"""
from __future__ import annotations

import os

import numpy as np

from . import synthetic as syn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

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
    # BASELINE.json north_star: SW int16, a 400-residue query against a
    # 10 M-sequence synthetic protein DB, strong scaling over 1..8 GPUs --
    # C4's DB (tests/golden/fullsize.json "c4full") at API width 16
    "north_star": dict(algo="sw", matrix="blosum62", gap_open=-11, gap_extend=-1, qlen=400, db="protein",
                       seqs=None, total_seqs=10_000_000, width=16),
}

DB_SEED = {"protein": 42, "dna": 43}
QUERY_SEED = {"protein": 7, "dna": 8}


def read_query_file(path: str) -> np.ndarray:
    """First FASTA record as synthetic-alphabet codes (the product parses
    the same text itself through init_sequence_fasta)."""
    lines = open(os.path.join(ROOT, path)).read().split("\n")
    seq = "".join(x.strip() for x in lines[1:] if not x.startswith(">")).upper()
    return np.array([syn.AA_ORDER.index(c) for c in seq], dtype=np.uint8)


def query(cfg: dict, qlen: int | None = None) -> np.ndarray:
    if cfg["db"] == "dna":
        return syn.dna_query(qlen or cfg["qlen"], QUERY_SEED["dna"])
    if cfg.get("query_file"):
        return read_query_file(cfg["query_file"])
    return syn.protein_query(qlen or cfg["qlen"], QUERY_SEED["protein"])


def cuts(cfg: dict, world: int, q: np.ndarray, seqs: int | None = None, lengths: str = "gamma"):
    """(bounds[world + 1], DB size, IDs the job searches): rank r searches
    IDs [bounds[r], bounds[r + 1]).  seqs: a weak config's per-rank sequence
    count, or a strong config's per-rank share (then cut by count: the first
    share is the c4/c5 fixtures' DB)."""
    if cfg["total_seqs"] is None:
        per = seqs if seqs is not None else cfg["seqs"]
        total = job = per * world
        balanced = world > 1
    else:
        total = cfg["total_seqs"]
        per = seqs if seqs is not None else (total + world - 1) // world
        job = min(total, per * world)
        balanced = world > 1 and seqs is None
    if balanced and cfg["db"] == "protein":
        from . import shard_bounds
        hi = 4096 if lengths == "gamma" else 1000
        lens = syn.protein_lengths_range(total, DB_SEED["protein"], 0, job, query=q, lo=16, hi=hi, lengths=lengths)
        return [int(x) for x in shard_bounds(lens, world)], total, job
    b = [min(job, r * per) for r in range(world)] + [job]
    return b, total, job


def slice_db(cfg: dict, q: np.ndarray, total: int, i0: int, i1: int, alphabet: str = "bg20",
             lengths: str = "gamma"):
    """(codes, offsets) of IDs [i0, i1) of the workload's DB."""
    if cfg["db"] == "dna":
        return syn.dna_reads_range(total, DB_SEED["dna"], i0, i1, 150, query=q)
    hi = 4096 if lengths == "gamma" else 1000
    return syn.protein_db_range(total, DB_SEED["protein"], i0, i1, query=q, alphabet=alphabet, lengths=lengths,
                                lo=16, hi=hi)


def rank_layout(world: int, ngpu: int, local: int, backend: str):
    """(device for this rank, ranks per GPU, physical GPUs the job uses).
    Every rank computes the same answer from the world size and the visible
    GPU count; more ranks than GPUs only as a gloo rehearsal (several ranks
    share a GPU, so the job's rate is that of min(world, ngpu) GPUs)."""
    ngpu = max(0, int(ngpu))
    if world <= max(ngpu, 1):
        return local, 1, world
    if backend != "gloo":
        raise SystemExit(f"{world} ranks but only {ngpu} GPU(s) visible (a rehearsal needs SSA_DIST_BACKEND=gloo)")
    n = max(1, ngpu)
    return local % n, -(-world // n), n


# The DP kernels' sources: a PMC-derived figure (HBM traffic, VALU
# instructions per cell, clock) describes the build it was measured on, so
# profiles/traffic.json files each record under this hash and bench.py reports
# it only while the sources still hash the same (roofline.traffic_stale).
KERNEL_SOURCES = ("libssa_amd/csrc/pair_kernel.h", "libssa_amd/csrc/kernels.hip", "libssa_amd/csrc/dp_common.h",
                  "libssa_amd/csrc/kernels.h", "libssa_amd/csrc/pair_sw.hip", "libssa_amd/csrc/pair_nw.hip")


def kernel_src_hash(root: str = ROOT) -> str:
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def profiled_figures(key: str, src_hash: str, path: str) -> dict:
    """The PMC figures profiles/traffic.json holds for workload `key`, if
    they were measured on kernel sources hashing to `src_hash`:
    {"traffic", "source", "valu_instr_per_cell", "clock_ghz", "stale"} --
    stale True (and every figure None) when the record belongs to another
    build, None when there is no record for the workload."""
    import json
    out = {"traffic": None, "source": None, "valu_instr_per_cell": None, "clock_ghz": None, "stale": None}
    if not os.path.exists(path):
        return out
    rec = json.load(open(path)).get(key)
    if not rec:
        return out
    if rec.get("kernel_src") != src_hash:
        out["stale"] = True
        out["stale_source"] = rec.get("source")
        return out
    out.update(traffic=rec["bytes_per_launch"], source=rec["source"], stale=False,
               valu_instr_per_cell=rec.get("valu_instr_per_cell"), clock_ghz=rec.get("clock_ghz"))
    return out
