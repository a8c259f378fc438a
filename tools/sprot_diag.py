"""One sprot-shape search with and without the rare merge: stats per search.
(Historical: option "rare_merge_ppm" was removed with the feature, DESIGN.md §3.1;
this produced profiles/r04/rare_merge/diag.txt.)"""
import json, os, sys, tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import libssa_amd as S
from libssa_amd import synthetic as syn, workloads as W

cfg = W.CONFIGS["sprot"]
q = W.query(cfg)
codes, off = W.slice_db(cfg, q, 548208, 0, 548208, "sprot25")
codes, off = syn.with_long_tail(codes, off, 300, 77, "sprot25")
S.load()
S.set_output_mode(S.OUTPUT_ERROR)
S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
S.init_score_matrix(S.MATRIX_BUILDIN, "blosum50")
S.init_gap_penalties(-3, -1)
with tempfile.TemporaryDirectory() as tmp:
    p = os.path.join(tmp, "db.fas")
    syn.write_fasta(p, codes, off)
    S.init_db(p)
    S.prepare_db()
qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
for ppm in [int(x) for x in sys.argv[1:]] or [5000, 0]:
    S.set_option("rare_merge_ppm", ppm)
    for _ in range(4):
        S.sw_align(qq, 10, 16)
        st = S.stats()
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()
                      if k in ("search_ms", "kernel_ms", "wide_ms", "d2h_ms", "replay_ms", "prep_ms", "sync_wait_ms",
                               "wide_count", "rare_merged", "rare_rescored", "strip_rows", "long_kernel",
                               "long_entries")} | {"ppm": ppm}), flush=True)
