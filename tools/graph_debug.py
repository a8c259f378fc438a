"""Searches with option graph on and off and SSA_AMD_TRACE=1: the search
graph's capture steps, its timing nodes and kernel_ms against the direct
path, for SW and NW with long-entry kernels (a debugging aid)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SSA_AMD_TRACE"] = "1"
import numpy as np  # noqa: E402
import libssa_amd as S  # noqa: E402
from libssa_amd import synthetic as syn  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

S.load()
S.set_output_mode(S.OUTPUT_ERROR)
S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
S.init_score_matrix(S.MATRIX_BUILDIN, S.BLOSUM62)
S.init_gap_penalties(-11, -1)
rng = np.random.default_rng(41)
codes, off = syn.protein_db(20000, 42, lo=1, hi=1200)
seqs = [codes[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
for i in range(0, 300, 3):
    seqs[i] = rng.choice(syn.AA_CODES, int(rng.integers(3000, 6000))).astype(np.uint8)
db, doff = po.pack_db(seqs)
S.set_option("long_groups", int(sys.argv[1]) if len(sys.argv) > 1 else 2)
with tempfile.TemporaryDirectory() as tmp:
    path = os.path.join(tmp, "db.fas")
    syn.write_fasta(path, db, doff)
    S.init_db(path)
    for n, fn, name in ((400, S.sw_align, "sw"), (250, S.nw_align, "nw")):
        q = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(syn.protein_query(n, 900 + n)))
        for g in (1, 0, 1):
            S.set_option("graph", g)
            for i in range(4):
                hits = fn(q, 10, 16)
                st = S.stats()
                print(name, "graph opt", g, "search", i, "mode", st["graph"], "kernel_ms", round(st["kernel_ms"], 4),
                      hits[0]["score"], flush=True)
