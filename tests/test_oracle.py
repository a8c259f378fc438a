"""The CPU restatement (oracle/ssa_oracle.c) pinned against the reference.

Two independent anchors:
  * the known-answer vectors written in the reference's own tests
    (expected values transcribed below with their file:line),
  * fixtures produced by the reference's own sources (tools/gen_golden.py ->
    tests/golden/*), checked list-for-list, including tie IDs.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as po
from libssa_amd import synthetic as syn
from tests.conftest import DATA, GOLDEN

TABLES = np.load(os.path.join(GOLDEN, "tables.npz"))
NAMES = [str(x) for x in TABLES["names"]]
KATS = json.load(open(os.path.join(GOLDEN, "kat.json")))


def kat_inputs(case):
    nt = case["nucleotide"]
    spec = case["scoring"]
    if spec[0] == "const":
        M = po.matrix_constant(spec[1], spec[2])
    elif spec[0] == "builtin":
        M = TABLES["matrices"][NAMES.index(spec[1])].copy()
    else:
        M = po.matrix_parse(open(os.path.join(DATA, spec[1]), "rb").read())
    q = case["query"]
    if q.startswith("file:"):
        qc = po.map_query(po.read_query_fasta(os.path.join(DATA, q[5:])), nt)
    else:
        qc = po.map_query(q[4:].encode(), nt)
    seqs = [po.map_db(s, nt) for s in po.read_fasta(os.path.join(DATA, case["db"]))]
    return qc, seqs, M


def test_maps_match_reference():
    assert (TABLES["maps"][0] == po.build_map(False)).all()
    assert (TABLES["maps"][1] == po.build_map(True)).all()


def test_builtin_matrices_parse_like_reference():
    # BLOSUM62 spot checks (matrices.c text; row/col 0 default -1)
    M = TABLES["matrices"][NAMES.index("blosum62")]
    A, W, star = 1, 20, 25
    assert M[(A << 5) + A] == 4 and M[(W << 5) + W] == 11 and M[(star << 5) + star] == 1
    assert M[0] == -1 and M[(A << 5)] == -1 and M[(28 << 5) + 28] == -1


def test_file_matrix_parser_matches_reference():
    ref = po.matrix_parse(open(os.path.join(DATA, "blosum90.txt"), "rb").read())
    assert (ref == TABLES["matrices"][NAMES.index("blosum90")]).all()


def test_constant_scoring_layout():
    M = po.matrix_constant(5, -4)
    assert M[(1 << 5) + 1] == 5 and M[(1 << 5) + 2] == -4
    assert M[0] == -1 and M[(3 << 5)] == -1   # code 0 row/col stays -1 (matrices.c:453-457)
    assert M[(15 << 5) + 15] == 5            # N == N is a match under constant scoring


# Expected lists as written in the reference's tests.
REF_TEST_VECTORS = {
    # tests/test_libssa.c:57-92 (5,-4 / -4,-2 / k=5 / 64-bit / 1 thread)
    ("libssa_const5_4", "sw"): [(91, 877), (91, 847), (91, 753), (91, 565), (91, 398)],
    ("libssa_const5_4", "nw"): [(33, 1050), (28, 908), (24, 938), (21, 378), (12, 75)],
    # tests/test_bigger_databases.c:76-81
    ("bigger_AF091148", "nw"): [(-88, 908), (-92, 1050), (-94, 938), (-98, 378), (-102, 75), (-104, 23),
                                (-106, 1229), (-110, 1148), (-110, 612), (-112, 1016)],
    ("bigger_AF091148", "sw"): [(20, 1177), (18, 384), (18, 277), (18, 215), (18, 214), (18, 210),
                                (18, 151), (18, 126), (18, 114), (18, 101)],
    # tests/algo/test_searcher.c:83-101 / 146-160
    ("searcher_simple", "sw"): [(2, 0)],
    ("searcher_simple", "nw"): [(-2, 0)],
    ("searcher_multi", "nw"): [(-1, 0), (-3, 3), (-4, 7), (-4, 6), (-4, 4), (-5, 2), (-6, 5), (-6, 1)],
    ("searcher_multi", "sw"): [(4, 3), (4, 1), (4, 0), (3, 7), (3, 5), (3, 4), (3, 2), (2, 6)],
    # tests/algo/test_searcher.c:407-505
    ("searcher_AA_const", "nw"): [(-87, 0)],
    ("searcher_AA_const", "sw"): [(3, 0)],
    ("searcher_AA_blosum62", "sw"): [(103, 0)],
    ("searcher_AA_blosum62", "nw"): [(82, 0)],
    # tests/algo/test_searcher.c:507-536
    ("overflow_127", "sw"): [(67818, 0)],
    ("overflow_127", "nw"): [(67818, 0)],
    # tests/algo/8/test_8_simd_avx2_sw.c:95-99
    ("tmp_fas_8bit", "sw"): [(4, 0)],
}
# tests/algo/64/test_search_64.c:68-112 assert scores + top ID only
REF_SCORES_TOP = {("search64_test_fas", "sw"): ([8, 8, 8, 8, 8], 4),
                  ("search64_test_fas", "nw"): ([-43, -50, -52, -52, -147], 4)}


@pytest.mark.parametrize("case", KATS, ids=[c["name"] for c in KATS])
@pytest.mark.parametrize("algo", ["sw", "nw"])
def test_oracle_matches_reference_kat(case, algo):
    qc, seqs, M = kat_inputs(case)
    got = po.search(0 if algo == "sw" else 1, qc, seqs, M, case["gap_open"], case["gap_extend"], case["k"])
    assert got == [tuple(x) for x in case[algo + "_64"]]
    # the reference's own 16-bit path always agrees on the score list
    assert [s for s, _ in got] == [s for s, _ in case[algo + "_16_avx2"]]
    key = (case["name"], algo)
    if key in REF_TEST_VECTORS:
        assert got == REF_TEST_VECTORS[key]
    if key in REF_SCORES_TOP:
        sc, top = REF_SCORES_TOP[key]
        assert [s for s, _ in got] == sc and got[0][1] == top


def _random_cases():
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("random_"))


@pytest.mark.parametrize("fname", _random_cases())
def test_oracle_matches_reference_random(fname):
    z = np.load(os.path.join(GOLDEN, fname))
    meta = json.loads(str(z["meta"]))
    q = syn.protein_query(meta["qlen"], meta["qseed"])
    codes, off = syn.protein_db(meta["n"], meta["seed"], query=q, plant_every=meta["plant_every"],
                                lo=meta["lo"], hi=meta["hi"])
    M = TABLES["matrices"][NAMES.index(meta["matrix"])].copy()
    for algo, an in ((0, "sw"), (1, "nw")):
        sc = po.scores(algo, q, codes, off, M, meta["gap_open"], meta["gap_extend"])
        assert (sc == z[an + "_scores"]).all()
        assert hashlib.sha256(sc.astype("<i8").tobytes()).hexdigest() == meta[an + "_sha256"]
        lens = np.diff(off)
        keep = np.nonzero(lens > 0)[0]
        for k in (1, 10, 100, 1000):
            got = po.topk(sc[keep], keep.astype(np.uint64), k)
            assert got == [tuple(x) for x in meta[f"{an}_top{k}"]]


def test_heap_tie_semantics_small():
    # strict '>' replacement: equal scores arriving later are dropped
    assert po.topk(np.array([5, 5, 5]), np.array([0, 1, 2]), 2) == [(5, 1), (5, 0)]
    # order: score desc, then id desc
    assert po.topk(np.array([1, 3, 3, 2]), np.array([0, 1, 2, 3]), 3) == [(3, 2), (3, 1), (2, 3)]


# ------------------------------------------------------------ overflow counters
OVF = np.load(os.path.join(GOLDEN, "overflow.npz"))
OVF_CASES = json.loads(str(OVF["meta"]))


def _ovf_matrix(c):
    if c["matrix"] == "const":
        return po.matrix_constant(c["match"], c["mismatch"])
    return TABLES["matrices"][NAMES.index(c["matrix"])].copy()


@pytest.mark.parametrize("case", OVF_CASES, ids=[f"c{c['id']}" for c in OVF_CASES])
def test_overflow_flags_match_reference(case):
    """Per-sequence 8/16-bit overflow flags of the reference's SIMD kernels
    (harness with chunk size 1, tools/gen_golden.py gen_overflow) equal the
    oracle's saturated replays -- ordinary penalties and ones whose int8 sum
    wraps or is positive (search_simd_sw.c / search_simd_nw.c)."""
    t = case["id"]
    q, db, off = OVF[f"c{t}_q"], OVF[f"c{t}_db"], OVF[f"c{t}_off"]
    got = po.overflow_flags(case["algo"], q, db, off, _ovf_matrix(case), case["gap_open"], case["gap_extend"])
    exp = OVF[f"c{t}_flags"]
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


@pytest.mark.parametrize("case", KATS, ids=[c["name"] for c in KATS])
def test_kat_overflow_counters(case):
    """m_run's counters (manager.c:157-160) for every KAT at widths 8 and 16,
    from the oracle's flags, equal the reference's (incl. the KATs written in
    its tests: overflow_127 1/1, sw_overflow_534 1/0, test.fas NW int8 4/0)."""
    qc, seqs, M = kat_inputs(case)
    db, off = po.pack_db(seqs)
    keep = np.diff(off) > 0
    for algo, an in ((0, "sw"), (1, "nw")):
        f = po.overflow_flags(algo, qc, db, off, M, case["gap_open"], case["gap_extend"])[keep]
        assert po.overflow_counts(8, f) == tuple(case[an + "_8_overflow"]), an
        assert po.overflow_counts(16, f)[1] == case[an + "_16_overflow"], an
    fixed = {"overflow_127": ((1, 1), (1, 1)), "sw_overflow_534": ((1, 0), None),
             "search64_test_fas": (None, (4, 0))}
    if case["name"] in fixed:
        for algo, exp in enumerate(fixed[case["name"]]):
            if exp is not None:
                assert tuple(case[("sw", "nw")[algo] + "_8_overflow"]) == exp
