#!/usr/bin/env python3
"""Generates the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container (needs /root/reference and
``make -C oracle ref``).  The reference sources are compiled in place into
oracle/_ref/ref_harness; this script feeds it inputs and stores inputs and
outputs as data:

  tests/golden/tables.npz      the 8 built-in matrices + both residue maps as
                               parsed by the reference (matrices.c, util_sequence.c)
  tests/golden/kat.json        known-answer cases of the reference's own tests
                                with the full top-k the reference's
                               64-bit and AVX2 16-bit searches return
  tests/golden/translate.npz   random nucleotide sequences (IUPAC codes
                               included) translated by the reference's
                               us_translate_sequence for every valid genetic
                               code, both sides, strands and frames
  tests/golden/align.json      COMPUTE_ALIGNMENT regions + CIGARs of the
                               reference's align_sequences (align.c, cigar.c)
                               on seeded pairs: SW and NW, NT constant scoring,
                               BLOSUM62, an asymmetric matrix
  tests/golden/random_*.npz    seeded synthetic DBs (regenerated from their
                               parameters by libssa_amd.synthetic) with the
                               reference's full int64 score vector (full_sw /
                               full_nw) and its 64-bit top-k for several k
  tests/golden/overflow.npz    the reference's own 8- and 16-bit overflow
                               flags of every sequence of seeded random cases
                               (chunk size 1: one count per sequence), SW and
                               NW, ordinary and pathological gap penalties
  tests/golden/fullsize.json   BASELINE.json's configurations at full (C2, C3:
                               1 M sequences) or share (C4: the first 1.25 M of
                               the 10 M DB, C5: the first 1 M of the 50 M
                               reads) size, plus the 25- and 28-symbol
                               alphabets: SHA-256 of the reference's full
                               score vector, its histogram, the top-k, and
                               the reference's overflow counters
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from libssa_amd import synthetic as syn  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
D = os.path.join(G, "data")
NAMES = ["blosum45", "blosum50", "blosum62", "blosum80", "blosum90", "pam30", "pam70", "pam250"]

# query of tests/algo/8/test_8_simd_avx2_sw.c:106-113 (one C string literal)
OVF534_QUERY = ("MVQRWLYSTNAKDIAVLYFMLAIFSGMAGTAMSLIIRLELAAPGSQYLHGNSQLFNVLVVGHAVLMIFFLVMPALIGGFG"
                "NYLLPLMIGATDTAFPRINNIAFWVLPMGLVCLVTSTLVESGAGTGWTVYPPLSSIQAHSGPSVDLAIFALHLTSISSLL"
                "GAINFIVTTLNMRTNGMTMHKLPLFVWSIFITAFLLLLSLPVLSAGITMLLLDRNFNTSFFEVSGGGDPILYEHLFWFFG"
                "HPEVYILIIPGFGIISHVVSTYSKKPVFGEISMVYAMASIGLLGFLVWSHHMYIVGLDADTRAYFTSATMIIAIPTGIKI"
                "FSWLATIHGGSIRLATPMLYAIAFLFLFTMGGLTGVALANASLDVAFHDTYYVVGHFHYVLSMGAIFSLFAGYYYWSPQI"
                "LGLNYNEKLAQIQFWLIFIGANVIFFPMHFLGINGMPRRIPDYPDAFAGWNYVASIGSFIATLSLFLFIYILYDQLVNGL"
                "NNKVNNKSVIYNKAPDFVESNTIFNLNTVKSSSIEFLLTSPPAVHSFNTPAVQS")

# (name, db file, nucleotide, query (file: or str:), scoring, gapO, gapE, k, chunk)
KATS = [
    ("libssa_const5_4", "AF091148.fas", True, "file:one_seq.fas", ("const", 5, -4), -4, -2, 5, 1000),
    ("bigger_AF091148", "AF091148.fas", True, "file:one_seq.fas", ("const", 2, -2), -4, -2, 10, 1000),
    ("searcher_simple", "short_db.fas", True, "str:AT", ("const", 1, -1), -1, -1, 1, 1),
    ("searcher_multi", "short_nuc_db.fas", True, "str:ATGCAAATTT", ("const", 1, -1), -1, -1, 8, 8),
    ("search64_test_fas", "test.fas", True,
     "str:ATGCCCAAGCTGAATAGCGTAGAGGGGTTTTCATCATTTGAGGACGATGTATAA", ("const", 1, -1), -1, -1, 5, 5),
    ("searcher_AA_const", "short_AA.fas", False,
     "str:HPEVYILIIPGFGIISHVVSTYSKKPVFGEISMVYAMASIGLLGFLVWSHHMYIVGLDADTRAYFTSATMIIAIPTGIKI",
     ("const", 1, -1), -1, -1, 1, 1),
    ("searcher_AA_blosum62", "short_AA.fas", False,
     "str:HPEVYILIIPGFGIISHVVSTYSKKPVFGEISMVYAMASIGLLGFLVWSHHMYIVGLDADTRAYFTSATMIIAIPTGIKI",
     ("builtin", "blosum62"), -1, -1, 1, 1),
    ("overflow_127", "NP_009305.1.fas", False, "file:NP_009305.1.fas", ("const", 127, -1), -1, -1, 1, 1),
    ("tmp_fas_8bit", "tmp.fas", True, "str:ATGCAAA", ("const", 1, -1), -1, -1, 1, 1),
    # tests/algo/8/test_8_simd_avx2_sw.c:104-124: 534, one 8-bit overflow
    ("sw_overflow_534", "NP_009305.1.fas", False, "str:" + OVF534_QUERY, ("const", 1, -1), -1, -1, 1, 1),
    ("config1_Q3ZAI3", "AF091148.fas", False, "file:Q3ZAI3.fasta", ("builtin", "blosum62"), -11, -1, 10, 1000),
    ("config1_Q3ZAI3_k300", "AF091148.fas", False, "file:Q3ZAI3.fasta", ("builtin", "blosum62"), -11, -1, 300, 1000),
    ("nt_file_matrix", "AF091148.fas", True, "file:one_seq.fas", ("file", "nuc_scoring_matrix.txt"), -3, -1, 20, 1000),
    ("blosum90_file", "AF091148_selection.fas", False, "file:P18080.fasta", ("file", "blosum90.txt"), -10, -1, 15, 1000),
]


def matrix_for(spec, tables):
    if spec[0] == "const":
        return po.matrix_constant(spec[1], spec[2])
    if spec[0] == "builtin":
        return tables[NAMES.index(spec[1])].copy()
    return po.matrix_parse(open(os.path.join(D, spec[1]), "rb").read())


def query_for(q, nt):
    if q.startswith("file:"):
        return po.map_query(po.read_query_fasta(os.path.join(D, q[5:])), nt)
    return po.map_query(q[4:].encode(), nt)


def main():
    if not po.have_ref():
        po.build(quiet=False)
    mats, maps = po.ref_run(po.MODE_TABLES)
    np.savez(os.path.join(G, "tables.npz"), matrices=mats, maps=maps, names=np.array(NAMES))
    print("tables: ok")

    kats = []
    for name, dbf, nt, q, spec, go, ge, k, chunk in KATS:
        M = matrix_for(spec, mats)
        qc = query_for(q, nt)
        seqs = [po.map_db(s, nt) for s in po.read_fasta(os.path.join(D, dbf))]
        case = {"name": name, "db": dbf, "nucleotide": nt, "query": q, "scoring": list(spec),
                "gap_open": go, "gap_extend": ge, "k": k, "chunk": chunk}
        for algo, an in ((0, "sw"), (1, "nw")):
            hits64, _, ns, _ = po.ref_run(po.MODE_SEARCH64, algo, qc, seqs, M, go, ge, k=k, chunk=chunk)
            hits16, ovf16, _, _ = po.ref_run(po.MODE_SEARCH16_AVX2, algo, qc, seqs, M, go, ge, k=k, chunk=chunk)
            _, ovf8, _, _ = po.ref_run(po.MODE_SEARCH8_AVX2, algo, qc, seqs, M, go, ge, k=k, chunk=chunk)
            case[an + "_64"] = hits64
            case[an + "_16_avx2"] = hits16
            case[an + "_16_overflow"] = int(ovf16)
            case[an + "_8_overflow"] = [int(x) for x in ovf8]
            case["nseq_nonempty"] = int(ns)
        kats.append(case)
        print(name, "sw", case["sw_64"][:3], "nw", case["nw_64"][:3])
    with open(os.path.join(G, "kat.json"), "w") as f:
        json.dump(kats, f, indent=1)

    # random synthetic cases: (tag, n, seed, qlen, qseed, matrix, gapO, gapE, plant_every)
    rnd = [
        ("small_b62", 3000, 11, 120, 3, "blosum62", -11, -1, 500),
        ("small_b50", 2500, 12, 333, 4, "blosum50", -10, -2, 700),
        ("medium_b62", 20000, 42, 400, 7, "blosum62", -11, -1, 2000),
    ]
    for tag, n, seed, qlen, qseed, mname, go, ge, plant in rnd:
        q = syn.protein_query(qlen, qseed)
        codes, off = syn.protein_db(n, seed, query=q, plant_every=plant, lo=0 if n < 10000 else 16, hi=1200)
        M = mats[NAMES.index(mname)].copy()
        out = {"n": n, "seed": seed, "qlen": qlen, "qseed": qseed, "matrix": mname,
               "gap_open": go, "gap_extend": ge, "plant_every": plant,
               "lo": 0 if n < 10000 else 16, "hi": 1200}
        arrays = {}
        for algo, an in ((0, "sw"), (1, "nw")):
            sc = po.ref_run(po.MODE_SCORES, algo, q, None, M, go, ge, db_off=(codes, off))
            arrays[an + "_scores"] = sc
            out[an + "_sha256"] = hashlib.sha256(sc.astype("<i8").tobytes()).hexdigest()
            for k in (1, 10, 100, 1000):
                hits, _, _, _ = po.ref_run(po.MODE_SEARCH64, algo, q, None, M, go, ge, k=k,
                                           db_off=(codes, off))
                out[f"{an}_top{k}"] = hits
        np.savez(os.path.join(G, f"random_{tag}.npz"), meta=np.array(json.dumps(out)), **arrays)
        print(tag, "ok", out["sw_top10"][:3])


VALID_GENCODES = [1, 2, 3, 4, 5, 6, 9, 10, 11, 12, 13, 14, 15, 16, 21, 22, 23]


def gen_translate():
    """Reference translations (util_sequence.c:332-382) of seeded random NT
    code sequences: query table = code g, DB table = the next valid code."""
    rng = np.random.default_rng(2024)
    arrays = {}
    for gi, g in enumerate(VALID_GENCODES):
        d = VALID_GENCODES[(gi + 1) % len(VALID_GENCODES)]
        lens = [2, 3, 4, 5, 6, 7, 8, 9] + list(rng.integers(10, 90, 24))
        seqs = []
        for n in lens:
            # mostly concrete bases (A C G T = 1 2 4 8), some IUPAC ambiguity codes
            conc = rng.choice(np.array([1, 2, 4, 8], np.uint8), n)
            amb = rng.integers(1, 16, n).astype(np.uint8)
            seqs.append(np.where(rng.random(n) < 0.15, amb, conc).astype(np.uint8))
        res = po.ref_run(po.MODE_TRANSLATE, k=g, chunk=d, seqs=seqs)
        db, off = po.pack_db(seqs)
        outs, ooff = [], [0]
        for per in res:
            for side in range(2):
                for strand in range(2):
                    for frame in range(3):
                        b = np.frombuffer(per[(side, strand, frame)], np.uint8)
                        outs.append(b)
                        ooff.append(ooff[-1] + len(b))
        arrays[f"g{g}_d{d}_db"] = db
        arrays[f"g{g}_d{d}_off"] = off
        arrays[f"g{g}_d{d}_out"] = np.concatenate(outs) if outs else np.zeros(0, np.uint8)
        arrays[f"g{g}_d{d}_outoff"] = np.array(ooff, np.uint64)
    np.savez_compressed(os.path.join(G, "translate.npz"), **arrays)
    print("translate ok", len(arrays) // 4, "code pairs")


def _mutate(rng, seq, alphabet, ident):
    out = []
    for c in seq:
        r = rng.random()
        if r < (1 - ident) * 0.7:
            out.append(rng.choice(alphabet))
        elif r < (1 - ident) * 0.85:
            continue
        elif r < (1 - ident):
            out += [c, rng.choice(alphabet)]
        else:
            out.append(c)
    return np.array(out if out else [alphabet[0]], np.uint8)


def gen_align():
    """Reference traceback (align_sequences) on seeded (query, DB) pairs."""
    rng = np.random.default_rng(77)
    mats = po.ref_run(po.MODE_TABLES)[0]
    nt = np.array([1, 2, 4, 8], np.uint8)
    asym = np.full(1024, -1, np.int64)
    for x in syn.AA_CODES:
        for y in syn.AA_CODES:
            asym[(int(x) << 5) + int(y)] = int(rng.integers(-6, 9))
    cases = [("nt_const5_4", nt, po.matrix_constant(5, -4), -4, -2),
             ("aa_blosum62", syn.AA_CODES, mats[NAMES.index("blosum62")], -11, -1),
             ("aa_asym", syn.AA_CODES, asym, -5, -2)]
    out = []
    for name, alpha, M, go, ge in cases:
        for t in range(4):
            q = rng.choice(alpha, int(rng.integers(5, 120))).astype(np.uint8)
            seqs = []
            for i in range(40):
                if i % 3 == 0:
                    seqs.append(_mutate(rng, q, alpha, rng.uniform(0.5, 0.95)))
                else:
                    seqs.append(rng.choice(alpha, int(rng.integers(1, 150))).astype(np.uint8))
            sw = po.scores(0, q, *po.pack_db(seqs), M, go, ge)
            keep = [s for s, v in zip(seqs, sw) if v > 0]   # score-0 SW regions are UB in the reference
            for algo in (0, 1):
                res = po.ref_run(po.MODE_ALIGN, algo, q, keep, M, go, ge)
                for s, (reg, cig) in zip(keep, res):
                    out.append({"case": name, "algo": algo, "gap_open": go, "gap_extend": ge,
                                "matrix": name, "query": q.tolist(), "db": s.tolist(),
                                "region": list(reg), "cigar": cig})
    mats_used = {name: [int(x) for x in M] for name, _, M, _, _ in cases}
    json.dump({"matrices": mats_used, "pairs": out}, open(os.path.join(G, "align.json"), "w"))
    print("align ok", len(out), "pairs")


def gen_overflow():
    """Per-sequence 8/16-bit overflow flags from the reference (the
    harness with chunk size 1 reports one overflow count per sequence)."""
    rng = np.random.default_rng(31)
    mats = po.ref_run(po.MODE_TABLES)[0]
    arrays, cases = {}, []
    for t in range(40):
        algo = t % 2
        mname = ["blosum62", "blosum50", "pam30", "const"][(t // 2) % 4]
        if mname == "const":
            match, mismatch = int(rng.integers(1, 128)), int(rng.integers(-20, 0))
            M = po.matrix_constant(match, mismatch)
        else:
            match = mismatch = 0
            M = mats[NAMES.index(mname)].copy()
        # ordinary penalties mostly; a few whose int8 sum wraps or is positive
        go = int(rng.choice([-1, -3, -5, -11, -11, -40, -100, 0, 5]))
        ge = int(rng.choice([-1, -1, -2, -4, -10, -50, 0, 3]))
        qlen = int(rng.choice([1, 2, 5, 17, 60, 130, 300, 700]))
        q = rng.choice(syn.AA_CODES, qlen).astype(np.uint8)
        lens = rng.integers(1, 400, 300)
        seqs = [rng.choice(syn.AA_CODES, int(n)).astype(np.uint8) for n in lens]
        for i in range(0, 300, 7):
            seqs[i] = q[: max(1, qlen - int(rng.integers(0, 5)))].copy()
        _, _, _, _, per8 = po.ref_run(po.MODE_SEARCH8_AVX2, algo, q, seqs, M, go, ge, k=5, chunk=1, threads=8,
                                      chunk_counts=True)
        _, _, _, _, per16 = po.ref_run(po.MODE_SEARCH16_AVX2, algo, q, seqs, M, go, ge, k=5, chunk=1, threads=8,
                                       chunk_counts=True)
        db, off = po.pack_db(seqs)
        arrays[f"c{t}_q"] = q
        arrays[f"c{t}_db"] = db
        arrays[f"c{t}_off"] = off
        arrays[f"c{t}_flags"] = (per8[:, 0].astype(np.uint8) | (per16[:, 1].astype(np.uint8) << 1))
        cases.append({"id": t, "algo": algo, "matrix": mname, "match": match, "mismatch": mismatch,
                      "gap_open": go, "gap_extend": ge})
        print("overflow case", t, algo, mname, go, ge, qlen, int(per8[:, 0].sum()), int(per16[:, 1].sum()))
    np.savez_compressed(os.path.join(G, "overflow.npz"), meta=np.array(json.dumps(cases)), **arrays)


# BASELINE.json configurations for the full-size fixtures (bench.py builds the
# same DBs from the same parameters): the block-seeded generators of
# libssa_amd.synthetic, so a share is the first IDs of the whole DB
FULLSIZE = {
    "c2": dict(kind="protein", n=1_000_000, i1=1_000_000, seed=42, qlen=400, qseed=7, matrix="blosum62",
               gap_open=-11, gap_extend=-1, algo="sw", width=16, alphabet="bg20"),
    "c3": dict(kind="protein", n=1_000_000, i1=1_000_000, seed=42, qlen=1000, qseed=7, matrix="blosum50",
               gap_open=-10, gap_extend=-2, algo="nw", width=16, alphabet="bg20"),
    "c4": dict(kind="protein", n=10_000_000, i1=1_250_000, seed=42, qlen=400, qseed=7, matrix="blosum62",
               gap_open=-11, gap_extend=-1, algo="sw", width=8, alphabet="bg20"),
    # the whole 10 M C4 DB on one GPU (top-k and counters pinned; the GPU
    # test does not pull the 10 M-entry log through Python)
    "c4full": dict(kind="protein", n=10_000_000, i1=10_000_000, seed=42, qlen=400, qseed=7, matrix="blosum62",
                   gap_open=-11, gap_extend=-1, algo="sw", width=8, alphabet="bg20"),
    "c5": dict(kind="dna", n=50_000_000, i1=1_000_000, seed=43, qlen=10_000, qseed=8, matrix="const5_-4",
               gap_open=-4, gap_extend=-2, algo="sw", width=16),
    # C2's weak-scaling DBs at N = 2, 4, 8 (N x 1 M sequences; rank r
    # searches IDs [r M, (r+1) M)): the global top-k bench.py gathers at N > 1
    **{f"c2x{w}": dict(kind="protein", n=w * 1_000_000, i1=w * 1_000_000, seed=42, qlen=400, qseed=7,
                       matrix="blosum62", gap_open=-11, gap_extend=-1, algo="sw", width=16, alphabet="bg20")
       for w in (2, 4, 8)},
    # one GPU's share of C5 at N = 8 (the first 6.25 M of the 50 M reads)
    "c5share8": dict(kind="dna", n=50_000_000, i1=6_250_000, seed=43, qlen=10_000, qseed=8, matrix="const5_-4",
                     gap_open=-4, gap_extend=-2, algo="sw", width=16),
    # the whole 50 M-read C5 DB (7.5e9 residues, 7.5e13 cells) on one GPU
    "c5full": dict(kind="dna", n=50_000_000, i1=50_000_000, seed=43, qlen=10_000, qseed=8, matrix="const5_-4",
                   gap_open=-4, gap_extend=-2, algo="sw", width=16),
    "sp25": dict(kind="protein", n=500_000, i1=500_000, seed=44, qlen=400, qseed=7, matrix="blosum62",
                 gap_open=-11, gap_extend=-1, algo="sw", width=16, alphabet="sprot25"),
    "u28": dict(kind="protein", n=200_000, i1=200_000, seed=45, qlen=400, qseed=7, matrix="blosum62",
                gap_open=-11, gap_extend=-1, algo="sw", width=16, alphabet="uniform28", lengths="uniform",
                lo=16, hi=1000),
    "u28nw": dict(kind="protein", n=200_000, i1=200_000, seed=45, qlen=400, qseed=7, matrix="blosum62",
                  gap_open=-11, gap_extend=-1, algo="nw", width=16, alphabet="uniform28", lengths="uniform",
                  lo=16, hi=1000),
    # the reference's own benchmark workload in Swiss-Prot's form (bench.py
    # --config sprot): P18080 vs 548 208 sequences of the 25-symbol alphabet,
    # BLOSUM50 -3/-1, 300 entries replaced by 5-35 k-residue ones
    "sprot": dict(kind="protein", n=548_208, i1=548_208, seed=42, qlen=513, query_file="tests/golden/data/P18080.fasta",
                  matrix="blosum50", gap_open=-3, gap_extend=-1, algo="sw", width=16, alphabet="sprot25",
                  tail=300, tail_seed=77),
    # round 6: the two bench_all shapes that had no fixture -- the reference's
    # benchmark shape in 20 letters (bench.py --config ref: P18080 vs 548 208
    # sequences, BLOSUM50 -3/-1) and C2's DB in the reference generator's
    # uniform 28 symbols at its full 1 M (bench.py --alphabet uniform28)
    "ref": dict(kind="protein", n=548_208, i1=548_208, seed=42, qlen=513, query_file="tests/golden/data/P18080.fasta",
                matrix="blosum50", gap_open=-3, gap_extend=-1, algo="sw", width=16, alphabet="bg20"),
    "u28c2": dict(kind="protein", n=1_000_000, i1=1_000_000, seed=42, qlen=400, qseed=7, matrix="blosum62",
                  gap_open=-11, gap_extend=-1, algo="sw", width=16, alphabet="uniform28"),
}


def fullsize_db(c):
    """(query codes, DB codes, offsets) of a FULLSIZE entry."""
    if c["kind"] == "dna":
        q = syn.dna_query(c["qlen"], c["qseed"])
        codes, off = syn.dna_reads_range(c["n"], c["seed"], 0, c["i1"], 150, query=q)
        return q, codes, off
    if c.get("query_file"):
        # the first record of the file, as bench.py reads it
        lines = open(os.path.join(ROOT, c["query_file"])).read().split("\n")
        seq = "".join(l.strip() for l in lines[1:] if not l.startswith(">")).upper()
        q = np.array([syn.AA_ORDER.index(ch) for ch in seq], dtype=np.uint8)
        assert len(q) == c["qlen"]
    else:
        q = syn.protein_query(c["qlen"], c["qseed"])
    codes, off = syn.protein_db_range(c["n"], c["seed"], 0, c["i1"], query=q, alphabet=c.get("alphabet", "bg20"),
                                      lengths=c.get("lengths", "gamma"), lo=c.get("lo", 16), hi=c.get("hi", 4096))
    if c.get("tail"):
        codes, off = syn.with_long_tail(codes, off, c["tail"], c["tail_seed"], c.get("alphabet", "bg20"))
    return q, codes, off


def gen_fullsize(names=None):
    mats = po.ref_run(po.MODE_TABLES)[0]
    path = os.path.join(G, "fullsize.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name, c in FULLSIZE.items():
        if names and name not in names:
            continue
        q, codes, off = fullsize_db(c)
        if c["matrix"].startswith("const"):
            a, b = c["matrix"][5:].split("_")
            M = po.matrix_constant(int(a), int(b))
        else:
            M = mats[NAMES.index(c["matrix"])].copy()
        n = len(off) - 1
        algo = 0 if c["algo"] == "sw" else 1
        mode = po.MODE_SEARCH8_AVX2 if c["width"] == 8 else po.MODE_SEARCH16_AVX2
        import time
        t0 = time.time()
        # k = n: every (score, id) stays in the reference's heap
        hits, ovf, ns, secs = po.ref_run(mode, algo, q, None, M, c["gap_open"], c["gap_extend"], k=n, threads=8,
                                         db_off=(codes, off), raw_hits=True)
        del codes
        assert ns == n == len(hits)
        arr = hits
        order = np.argsort(arr[:, 1], kind="stable")
        ids, sc = arr[order, 1], arr[order, 0]
        assert (ids == np.arange(n)).all()
        vals, counts = np.unique(sc, return_counts=True)
        rec = dict(c)
        rec.update({"nonempty": int(ns), "residues": int(off[-1]),
                    "sha256": hashlib.sha256(sc.astype("<i8").tobytes()).hexdigest(),
                    "hist_values": vals.tolist(), "hist_counts": counts.tolist(),
                    "overflow": list(ovf) if c["width"] == 8 else [0, int(ovf)],
                    "ref_seconds": round(secs, 2)})
        # the 64-bit single-thread result = the reference heap fed in ID order
        # (the oracle heap is pinned by tests/test_oracle.py)
        for k in (1, 10, 64):
            rec[f"top{k}"] = po.topk(sc, ids.astype(np.uint64), k)
        out[name] = rec
        print(name, "ok", round(time.time() - t0, 1), "s", rec["top10"][:3], rec["overflow"])
        json.dump(out, open(path, "w"), indent=1)


def _matrix_of(c, mats):
    if c["matrix"].startswith("const"):
        a, b = c["matrix"][5:].split("_")
        return po.matrix_constant(int(a), int(b))
    return mats[NAMES.index(c["matrix"])].copy()


# tie-heavy fixtures whose top-64 the reference's own 64-bit search pins
# (round 5): the top-64 boundary of each falls inside a band of equal scores
REF64 = {
    "u28": None, "u28nw": None, "sp25": None,
    # the first 100 k reads of C5's DB (q = 10 k, 1.5e11 cells): one planted
    # read, every other top-64 score is a random read's, ties throughout
    "c5s100k": dict(FULLSIZE["c5"], i1=100_000),
}


def gen_ref64(names=None):
    """The reference's 1-thread search_64 (search_64.c:44-79 -> minheap_add,
    minheap.c:75-91; ref_harness mode 1, one thread, chunk 1000: the heap is
    fed in ID order exactly as sw_align with one thread does) on tie-heavy
    fixtures -> tests/golden/ref64.json: the fixture's parameters and the
    reference heap's top-64, so the tie band at scale is pinned by the
    reference's heap, not by the oracle's replay.  Runs every fixture in its
    own process (one thread each)."""
    from concurrent.futures import ProcessPoolExecutor
    path = os.path.join(G, "ref64.json")
    todo = [n for n in REF64 if not names or n in names]
    with ProcessPoolExecutor(len(todo)) as ex:
        res = dict(zip(todo, ex.map(_ref64_one, todo)))
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name, (rec, hits, secs, oracle_top) in res.items():
        rec["top64"] = hits
        rec["ref_seconds"] = round(secs, 1)
        rec["oracle_heap_agrees"] = hits == oracle_top
        out[name] = rec
        print(name, "ref64", round(secs, 1), "s", "oracle heap agrees:", hits == oracle_top, hits[-4:])
    json.dump(out, open(path, "w"), indent=1)


def _ref64_one(name):
    c = REF64[name] or FULLSIZE[name]
    mats = po.ref_run(po.MODE_TABLES)[0]
    q, codes, off = fullsize_db(c)
    M = _matrix_of(c, mats)
    algo = 0 if c["algo"] == "sw" else 1
    hits, _, ns, secs = po.ref_run(po.MODE_SEARCH64, algo, q, None, M, c["gap_open"], c["gap_extend"], k=64,
                                   threads=1, db_off=(codes, off))
    rec = dict(c)
    rec.update({"nonempty": int(ns), "residues": int(off[-1])})
    # the oracle's heap replay over the exact scores, for the report only
    sc = po.scores(algo, q, codes, off, M, c["gap_open"], c["gap_extend"])
    lens = np.diff(off)
    keep = np.nonzero(lens > 0)[0]
    oracle_top = [list(x) for x in po.topk(sc[keep], keep.astype(np.uint64), 64)]
    return rec, [list(h) for h in hits], secs, oracle_top


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "ref64":
        gen_ref64(sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "overflow":
        gen_overflow()
    elif len(sys.argv) > 1 and sys.argv[1] == "fullsize":
        gen_fullsize(sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "translate":
        gen_translate()
    elif len(sys.argv) > 1 and sys.argv[1] == "align":
        gen_align()
    else:
        main()
        gen_translate()
        gen_align()
        gen_overflow()
        gen_fullsize()
