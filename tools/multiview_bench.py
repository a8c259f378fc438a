#!/usr/bin/env python3
"""Times multi-view searches (several query views per search: NUCLEOTIDE with
both strands, TRANS_QUERY's six frames) and reports where the time goes.

    python tools/multiview_bench.py [--mode both|transq] [--seqs N] [--qlen L]

both:   DNA, constant 5/-4, gaps -4/-2, q = qlen nt vs N reads of 150 nt,
        BOTH_STRANDS (2 views).
transq: protein DB of N sequences (BLOSUM62 -11/-1), nucleotide query of
        qlen nt translated in 6 frames (TRANS_QUERY, BOTH_STRANDS).
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libssa_amd as S  # noqa: E402
from libssa_amd import synthetic as syn  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="both", choices=["both", "transq"])
    p.add_argument("--seqs", type=int, default=1_000_000)
    p.add_argument("--qlen", type=int, default=None)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--steps", type=int, default=5)
    args = p.parse_args()
    S.load()
    S.set_output_mode(S.OUTPUT_ERROR)
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "db.fas")
    if args.mode == "both":
        qlen = args.qlen or 2000
        q = syn.dna_query(qlen, 8)
        codes, off = syn.dna_reads(args.seqs, 150, 43, query=q, plant_every=100000)
        syn.write_fasta(path, codes, off, nucleotide=True)
        S.init_symbol_translation(S.NUCLEOTIDE, S.BOTH_STRANDS, 1, 1)
        S.init_constant_scores(5, -4)
        S.init_gap_penalties(-4, -2)
        qs = syn.query_string(q, nucleotide=True)
    else:
        qlen = args.qlen or 1200
        q = syn.dna_query(qlen, 8)
        codes, off = syn.protein_db(args.seqs, 42, plant_every=0, sampler="lut")
        syn.write_fasta(path, codes, off)
        S.init_symbol_translation(S.TRANS_QUERY, S.BOTH_STRANDS, 1, 1)
        S.init_score_matrix(S.MATRIX_BUILDIN, "blosum62")
        S.init_gap_penalties(-11, -1)
        qs = syn.query_string(q, nucleotide=True)
    S.init_db(path)
    S.prepare_db()
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, qs)
    S.sw_align(qq, args.k, 16)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = S.sw_align(qq, args.k, 16)
    dt = (time.perf_counter() - t0) / args.steps
    st = S.stats()
    out = {"mode": args.mode, "seqs": args.seqs, "qlen": qlen, "views": st["kernel_launches"],
           "ms_per_search": round(dt * 1e3, 3), "gcups": round(st["cells"] / dt / 1e9, 1),
           "kernel_ms": round(st["kernel_ms"], 3), "kernel_gcups": round(st["cells"] / st["kernel_ms"] / 1e6, 1),
           "host_ms": {k: round(st[k], 3) for k in ("search_ms", "prep_ms", "upload_ms", "sync_wait_ms", "d2h_ms",
                                                       "replay_ms")},
           "top": [(h["score"], h["id"]) for h in res[:3]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
