#!/usr/bin/env python3
"""Batched vs one-by-one searches (ssa_amd_search_batch):
nq protein queries of length qlen against the C2-style 1 M-sequence DB.

    python tools/batch_bench.py [--qlen 30] [--nq 16] [--seqs 1000000] [--k 10]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libssa_amd as S  # noqa: E402
from libssa_amd import synthetic as syn  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--qlen", type=int, nargs="+", default=[30, 100, 400])
    p.add_argument("--nq", type=int, default=16)
    p.add_argument("--seqs", type=int, default=1_000_000)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--algo", default="sw", choices=["sw", "nw"])
    p.add_argument("--option", action="append", default=[], help="name=value passed to ssa_amd_set_option")
    args = p.parse_args()
    S.load()
    for o in args.option:
        k, v = o.split("=")
        S.set_option(k, int(v))
    S.set_output_mode(S.OUTPUT_ERROR)
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
    nw = args.algo == "nw"
    algo = S.NW if nw else S.SW
    S.init_score_matrix(S.MATRIX_BUILDIN, "blosum50" if nw else "blosum62")
    S.init_gap_penalties(-10 if nw else -11, -2 if nw else -1)
    codes, off = syn.protein_db(args.seqs, 42, plant_every=10000, sampler="lut")
    path = os.path.join(tempfile.mkdtemp(), "db.fas")
    syn.write_fasta(path, codes, off)
    S.init_db(path)
    S.prepare_db()
    os.remove(path)
    for qlen in args.qlen:
        qs = [S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(syn.protein_query(qlen, 1000 + i)))
              for i in range(args.nq)]
        S.search_batch(qs, algo, args.k)
        t_one, t_batch, t_unf = [], [], []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            one = [S.align_scores(q, args.k, 16, algo) for q in qs]
            t_one.append(time.perf_counter() - t0)
            S.set_option("batch_fuse", 0)
            t0 = time.perf_counter()
            unf = S.search_batch(qs, algo, args.k)
            t_unf.append(time.perf_counter() - t0)
            S.set_option("batch_fuse", 1)
            t0 = time.perf_counter()
            bat = S.search_batch(qs, algo, args.k)
            t_batch.append(time.perf_counter() - t0)
            launches = S.stats()["kernel_launches"]
        assert bat == unf == [[(s, i) for s, i in x] for x in one]
        cells = float(off[-1]) * qlen * args.nq
        print(json.dumps({"algo": args.algo, "qlen": qlen, "nq": args.nq, "options": args.option,
                          "one_by_one_gcups": round(cells / min(t_one) / 1e9, 1),
                          "batch_unfused_gcups": round(cells / min(t_unf) / 1e9, 1),
                          "batch_fused_gcups": round(cells / min(t_batch) / 1e9, 1),
                          "fused_pair_launches": launches,
                          "one_by_one_ms_per_query": round(min(t_one) / args.nq * 1e3, 3),
                          "batch_fused_ms_per_query": round(min(t_batch) / args.nq * 1e3, 3)}), flush=True)
        for q in qs:
            S.free_sequence(q)


if __name__ == "__main__":
    main()
