#!/usr/bin/env python3
"""Per-call latency of searches on tiny DBs (benchmark_pairwise.c's regime:
one DB entry, one query, many calls), with the automatic long-entry routing
and with every group forced onto the long-entry kernels.

usage (on the GPU box): python tools/pairwise_probe.py [out file] [--one: P18080 / Q3ZAI3 only]
Prints per (DB, query, algorithm, routing) the mean time of one
align_free call, the device kernel time and the kernels that ran."""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import libssa_amd as S  # noqa: E402
from libssa_amd import synthetic as syn  # noqa: E402

S.load()
S.init_score_matrix(S.MATRIX_BUILDIN, "blosum50")
S.init_gap_penalties(-3, -1)
S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 3, 3)
S.set_thread_count(1)

ONE = "--one" in sys.argv        # the P18080 / Q3ZAI3 pair only (benchmark_pairwise.c's)
args = [a for a in sys.argv[1:] if not a.startswith("--")]
out = open(args[0], "w") if args else None


def say(s):
    print(s, flush=True)
    if out:
        out.write(s + "\n")
        out.flush()


def db(tmp, name, lens, seed):
    rng = np.random.default_rng(seed)
    lens = np.asarray(lens, np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    path = os.path.join(tmp, name + ".fasta")
    syn.write_fasta(path, codes, off)
    return path


with tempfile.TemporaryDirectory() as tmp:
    rng = np.random.default_rng(3)
    dbs = [("P18080 (1 x 513)", os.path.join(ROOT, "tests", "golden", "data", "P18080.fasta"), 1),
           ("64 x 1-700", db(tmp, "d64", rng.integers(1, 700, 64), 1), 64),
           ("1000 x 1-700", db(tmp, "d1k", rng.integers(1, 700, 1000), 2), 1000),
           ("8000 x 1-700", db(tmp, "d8k", rng.integers(1, 700, 8000), 3), 8000)]
    queries = [("Q3ZAI3 390", S.init_sequence_fasta(S.READ_FROM_FILE,
                                                    os.path.join(ROOT, "tests", "golden", "data", "Q3ZAI3.fasta")))]
    if ONE:
        dbs = dbs[:1]
    for n in (() if ONE else (24, 1000, 5000)):
        queries.append((f"synthetic {n}", S.init_sequence_fasta(S.READ_FROM_STRING,
                                                                syn.query_string(syn.protein_query(n, 900 + n)))))
    for dname, path, nent in dbs:
        S.init_db(path)
        ngroups = (nent + 63) // 64
        for qname, q in queries:
            for algo, an in ((S.SW, "SW"), (S.NW, "NW")):
                row = []
                ref = None
                for lg in (-1, ngroups):
                    S.set_option("long_groups", lg)
                    hits = (S.sw_align if algo == S.SW else S.nw_align)(q, 10, 16)
                    sc = [(h["score"], h["id"]) for h in hits]
                    if ref is None:
                        ref = sc
                    assert sc == ref, (dname, qname, an, lg)
                    n = 20
                    t0 = time.perf_counter()
                    for _ in range(n):
                        S.align_free(q, 10, 16, algo)
                    dt = (time.perf_counter() - t0) / n
                    st = S.stats()
                    row.append(f"{'auto' if lg < 0 else 'all long':8s} {dt * 1e6:9.1f} us (kernel {st['kernel_ms'] * 1e3:8.1f})"
                               f" {st['kernel']}/{st.get('long_kernel', '') if st.get('long_entries', 0) else '-'}")
                say(f"{dname:18s} {qname:16s} {an}: " + " | ".join(row))
    S.set_option("long_groups", -1)
