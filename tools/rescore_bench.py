"""Times the exact re-score tiers on a DB where many lanes overflow 16 bits
(constant 127/-1, near-copies of the query; the int16 strip kernel): the int32
tier (long_kernel over the overflow list) against the int64 wide_kernel."""
import os, sys, tempfile, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import libssa_amd as S
from libssa_amd import synthetic as syn

def main():
    rng = np.random.default_rng(17)
    q = rng.choice(syn.AA_CODES, size=int(sys.argv[1]) if len(sys.argv) > 1 else 700).astype(np.uint8)
    n = 12000
    lens = rng.integers(20, 600, n)
    seqs = [rng.choice(syn.AA_CODES, size=int(x)).astype(np.uint8) for x in lens]
    for i in range(0, n, 8):
        a = int(rng.integers(0, 60))
        s = q[a:].copy()
        seqs[i] = s
    codes = np.concatenate(seqs)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    S.load()
    S.set_output_mode(S.OUTPUT_ERROR)
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
    S.init_constant_scores(127, -1)
    S.init_gap_penalties(-1, -1)
    with tempfile.TemporaryDirectory() as tmp:
        p = os.path.join(tmp, "db.fas")
        syn.write_fasta(p, codes, off)
        S.init_db(p)
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        S.set_option("sw_kernel", 1)
        S.set_option("long_groups", 0)
        for algo in (S.SW, S.NW):
            for r32 in (1, 0, 1, 0):
                S.set_option("rescore32", r32)
                t = []
                for _ in range(3):
                    S.sw_align(qq, 10, 16) if algo == S.SW else S.nw_align(qq, 10, 16)
                    st = S.stats()
                    t.append(st["wide_ms"])
                print(f"algo {algo} rescore32 {r32}: {st['wide_count']} lanes re-scored, wide_ms {min(t):.3f} "
                      f"(kernel {st['kernel_ms']:.3f} {st['kernel']})", flush=True)

main()
