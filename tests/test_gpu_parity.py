"""GPU parity: the HIP path through the C ABI against the oracle.

Everything here calls libssa_amd.so (sw_align / nw_align / ssa_amd_search),
which scores on the MI355X; the expected values come from the reference's own
fixtures (tests/golden) or from the oracle (oracle/ssa_oracle.c) on the same
seeded inputs.  Integer work: the bar is bit-exact scores AND the same IDs
among equal scores as the reference's 64-bit single-thread run.
"""
import hashlib
import json
import os
import tempfile

import numpy as np
import pytest

import libssa_amd as S
from libssa_amd import synthetic as syn
from oracle import pyoracle as po
from tests.conftest import DATA, GOLDEN, ROOT

pytestmark = pytest.mark.gpu

KATS = json.load(open(os.path.join(GOLDEN, "kat.json")))
TABLES = np.load(os.path.join(GOLDEN, "tables.npz"))
NAMES = [str(x) for x in TABLES["names"]]


@pytest.fixture(autouse=True)
def _counters_always():
    """Most tests run at OUTPUT_ERROR and still assert the overflow counters:
    ask for them explicitly (option "counters" 1; by default they are computed
    only at OUTPUT_INFO, where m_run prints them)."""
    S.set_option("counters", 1)
    # (the tests of pair-kernel plumbing use DBs small enough for long_plan's
    # latency rule to route every group away from it: off here, on in its
    # own test)
    S.set_option("long_latency", 0)
    yield
    S.set_option("counters", 1)
    S.set_option("long_latency", 1)     # (the default)


def configure(nucleotide, spec, go, ge, chunk=1000, strands=S.FORWARD_STRAND):
    S.set_output_mode(S.OUTPUT_ERROR)
    S.init_symbol_translation(S.NUCLEOTIDE if nucleotide else S.AMINOACID, strands, 1, 1)
    if spec[0] == "const":
        S.init_constant_scores(spec[1], spec[2])
    elif spec[0] == "builtin":
        S.init_score_matrix(S.MATRIX_BUILDIN, spec[1])
    else:
        S.init_score_matrix(S.READ_FROM_FILE, os.path.join(DATA, spec[1]))
    S.init_gap_penalties(go, ge)
    S.set_chunk_size(chunk)


def make_query(q):
    if q.startswith("file:"):
        return S.init_sequence_fasta(S.READ_FROM_FILE, os.path.join(DATA, q[5:]))
    return S.init_sequence_fasta(S.READ_FROM_STRING, q[4:])


# public-API runnable KATs (NUCLEOTIDE needs constant scoring, libssa.c:214-216)
API_KATS = [c for c in KATS if not (c["nucleotide"] and c["scoring"][0] != "const")]


@pytest.mark.parametrize("case", API_KATS, ids=[c["name"] for c in API_KATS])
@pytest.mark.parametrize("width", [S.BIT_WIDTH_16, S.BIT_WIDTH_8, S.BIT_WIDTH_64])
def test_kat_public_api(case, width):
    configure(case["nucleotide"], case["scoring"], case["gap_open"], case["gap_extend"], case["chunk"])
    # the default counter policy: computed because the output mode is INFO,
    # as m_run prints them there (manager.c:157-160)
    S.set_option("counters", -1)
    S.set_output_mode(S.OUTPUT_INFO)
    S.init_db(os.path.join(DATA, case["db"]))
    q = make_query(case["query"])
    for algo, fn in (("sw", S.sw_align), ("nw", S.nw_align)):
        got = [(h["score"], h["id"]) for h in fn(q, case["k"], width)]
        assert got == [tuple(x) for x in case[algo + "_64"]], (algo, got[:5])
        # m_run's overflow counters (manager.c:157-160) as the reference's own
        # 8/16-bit runs report them (tests/golden/kat.json from the harness;
        # incl. overflow_127 1/1, sw_overflow_534 1/0, test.fas NW int8 4/0)
        st = S.stats()
        exp = {S.BIT_WIDTH_8: tuple(case[algo + "_8_overflow"]), S.BIT_WIDTH_16: (0, case[algo + "_16_overflow"]),
               S.BIT_WIDTH_64: (0, 0)}[width]
        assert (st["overflow_8"], st["overflow_16"]) == exp, (algo, width)
        assert st["counters"] == 1
    S.free_sequence(q)


@pytest.mark.parametrize("nw", [0, 1])
def test_counters_skipped_when_unobserved(nw, tmp_path):
    """At OUTPUT_ERROR with the default policy the counter kernels do not run
    (stats counters = 0, overflow_8/16 read 0); the hits are unchanged, and
    at OUTPUT_INFO the same search reports the reference's counts."""
    case = next(c for c in API_KATS if c["name"] == "overflow_127")
    configure(case["nucleotide"], case["scoring"], case["gap_open"], case["gap_extend"], case["chunk"])
    S.set_option("counters", -1)
    S.init_db(os.path.join(DATA, case["db"]))
    q = make_query(case["query"])
    fn = S.nw_align if nw else S.sw_align
    algo = "nw" if nw else "sw"
    quiet = [(h["score"], h["id"]) for h in fn(q, case["k"], S.BIT_WIDTH_8)]
    st = S.stats()
    assert (st["counters"], st["overflow_8"], st["overflow_16"]) == (0, 0, 0)
    S.set_output_mode(S.OUTPUT_INFO)
    loud = [(h["score"], h["id"]) for h in fn(q, case["k"], S.BIT_WIDTH_8)]
    st = S.stats()
    assert quiet == loud == [tuple(x) for x in case[algo + "_64"]]
    assert st["counters"] == 1 and (st["overflow_8"], st["overflow_16"]) == tuple(case[algo + "_8_overflow"])
    S.set_output_mode(S.OUTPUT_ERROR)
    S.free_sequence(q)


OVF = np.load(os.path.join(GOLDEN, "overflow.npz"))
OVF_CASES = json.loads(str(OVF["meta"]))


@pytest.mark.parametrize("case", OVF_CASES, ids=[f"c{c['id']}" for c in OVF_CASES])
def test_overflow_counters_vs_reference_flags(case, tmp_path):
    """The reference's per-sequence 8/16-bit overflow flags (its own SIMD
    kernels, tools/gen_golden.py gen_overflow) summed the way m_run does
    equal ssa_amd_get_stats' counters at widths 8 and 16 -- ordinary and
    pathological (wrapping, zero, positive) gap penalties, SW and NW; the
    scores are checked against the oracle at every width too."""
    t = case["id"]
    q, db, off = OVF[f"c{t}_q"], OVF[f"c{t}_db"], OVF[f"c{t}_off"]
    flags = OVF[f"c{t}_flags"]
    if case["matrix"] == "const":
        spec = ("const", case["match"], case["mismatch"])
        M = po.matrix_constant(case["match"], case["mismatch"])
    else:
        spec = ("builtin", case["matrix"])
        M = TABLES["matrices"][NAMES.index(case["matrix"])].copy()
    configure(False, spec, case["gap_open"], case["gap_extend"])
    S.init_db(_write_db(str(tmp_path), db, off))
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    seqs = [db[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    exp_hits = po.search(case["algo"], q, seqs, M, case["gap_open"], case["gap_extend"], 5)
    fn = S.nw_align if case["algo"] else S.sw_align
    for width in (S.BIT_WIDTH_8, S.BIT_WIDTH_16):
        got = [(h["score"], h["id"]) for h in fn(qq, 5, width)]
        assert got == exp_hits, width
        st = S.stats()
        o8, o16 = po.overflow_counts(width, flags)
        assert (st["overflow_8"], st["overflow_16"]) == (o8 if width == 8 else 0, o16), width
    S.free_sequence(qq)


@pytest.mark.parametrize("algo", [0, 1])
def test_overflow_counters_two_views(algo, tmp_path):
    """NUCLEOTIDE with both strands: 2 query views x 2 DB strands per record.
    Width 8's 16-bit count is sum_e a8(e) * a16(e) -- the 8-bit overflow
    chunk holds an entry once per overflowing view and search_16_chunk re-runs
    every copy for every view (search_8.c:94-124) -- against the oracle's
    replays of the reference's saturated kernels (oracle_overflow_counts)."""
    rng = np.random.default_rng(5 + algo)
    q = syn.dna_query(1500, 3)
    seqs = []
    for i in range(80):
        n = int(rng.integers(20, 700))
        if i % 5 == 0:
            st0 = int(rng.integers(0, len(q) - n + 1))
            seqs.append(q[st0:st0 + n].copy())
        else:
            seqs.append(rng.choice(syn.NT_ACGT, n).astype(np.uint8))
    db, off = po.pack_db(seqs)
    configure(True, ("const", 127, -1), -1, -1, strands=S.BOTH_STRANDS)
    S.init_db(_write_db(str(tmp_path), db, off, nucleotide=True))
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q, nucleotide=True))
    views = [np.frombuffer(v[0], np.uint8) for v in S.query_views(qq)]
    assert len(views) == 2
    comp = np.zeros(32, np.uint8)
    comp[views[0]] = views[1][::-1]
    entries = []
    for x in seqs:
        entries += [x, comp[x[::-1]]]
    edb, eoff = po.pack_db(entries)
    M = po.matrix_constant(127, -1)
    flags = np.stack([po.overflow_flags(algo, v, edb, eoff, M, -1, -1) for v in views])
    fn = S.nw_align if algo else S.sw_align
    for width in (S.BIT_WIDTH_8, S.BIT_WIDTH_16):
        fn(qq, 5, width)
        st = S.stats()
        o8, o16 = po.overflow_counts(width, flags)
        assert (st["overflow_8"], st["overflow_16"]) == (o8 if width == 8 else 0, o16), width
    assert po.overflow_counts(8, flags)[1] > 0        # the product term is exercised
    S.free_sequence(qq)


@pytest.mark.parametrize("np_", [8, 16, 32])
def test_strip_heights_agree(np_):
    case = next(c for c in KATS if c["name"] == "config1_Q3ZAI3_k300")
    configure(False, case["scoring"], -11, -1)
    S.init_db(os.path.join(DATA, case["db"]))
    q = make_query(case["query"])
    S.set_option("strip_np", np_)
    try:
        for algo, fn in (("sw", S.sw_align), ("nw", S.nw_align)):
            got = [(h["score"], h["id"]) for h in fn(q, 300, 16)]
            assert got == [tuple(x) for x in case[algo + "_64"]]
    finally:
        S.set_option("strip_np", 16)
    S.free_sequence(q)


def _write_db(tmp, codes, off, nucleotide=False):
    path = os.path.join(tmp, "db.fas")
    syn.write_fasta(path, codes, off, nucleotide)
    return path


def _full_scores(q, algo, n_entries):
    """Every entry's exact score, via the insertion log with k >= #entries."""
    log = S.search(q, algo, n_entries, 16, S.LOG, cap=n_entries + 8)
    log.sort(key=lambda h: h[1])
    return np.array([h[0] for h in log], dtype=np.int64), np.array([h[1] for h in log], dtype=np.uint64)


@pytest.mark.parametrize("fname", sorted(f for f in os.listdir(GOLDEN) if f.startswith("random_")))
def test_random_golden_full_score_vectors(fname):
    z = np.load(os.path.join(GOLDEN, fname))
    meta = json.loads(str(z["meta"]))
    q = syn.protein_query(meta["qlen"], meta["qseed"])
    codes, off = syn.protein_db(meta["n"], meta["seed"], query=q, plant_every=meta["plant_every"],
                                lo=meta["lo"], hi=meta["hi"])
    lens = np.diff(off)
    keep = np.nonzero(lens > 0)[0]
    configure(False, ("builtin", meta["matrix"]), meta["gap_open"], meta["gap_extend"])
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        for algo, an in ((S.SW, "sw"), (S.NW, "nw")):
            sc, ids = _full_scores(qq, algo, len(keep))
            assert (ids == keep).all()
            assert (sc == z[an + "_scores"][keep]).all(), np.nonzero(sc != z[an + "_scores"][keep])[0][:10]
            for k in (1, 10, 100, 1000):
                fn = S.sw_align if algo == S.SW else S.nw_align
                got = [(h["score"], h["id"]) for h in fn(qq, k, 16)]
                assert got == [tuple(x) for x in meta[f"{an}_top{k}"]]
        S.free_sequence(qq)


@pytest.mark.parametrize("qlen", [1, 2, 8, 9, 15, 16, 17, 24, 25, 31, 32, 33, 40, 41, 47, 48, 49, 63, 64, 65, 72, 73,
                                  80, 81, 88, 89, 90, 95, 96, 97, 100, 113, 121])
@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_query_length_edges_vs_oracle(qlen, algo):
    rng = np.random.default_rng(qlen)
    q = syn.protein_query(qlen, 100 + qlen)
    # lengths straddling the 16-column blocks, plus empty records
    lens = np.array([0, 1, 2, 3, 15, 16, 17, 31, 32, 33, 47, 48, 49, 64, 65, 200, 0, 511, 512, 513]
                    + list(rng.integers(1, 300, 300)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    keep = np.nonzero(lens > 0)[0]
    exp = po.scores(algo, q, codes, off, M, -11, -1)[keep]
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        for swk in (0, 1):
            S.set_option("sw_kernel", swk)
            for np_ in (8, 16, 32):
                S.set_option("strip_np", np_)
                for pnp in ((16, 24, 32, 36, 40, 0) if swk == 0 and np_ == 16 else (0,)):
                    S.set_option("pair_np", pnp)
                    sc, ids = _full_scores(qq, algo, len(keep))
                    assert (ids == keep).all()
                    assert (sc == exp).all(), (swk, np_, pnp, np.nonzero(sc != exp)[0][:10])
                    # the sparse (device-filtered) path with the same plan
                    for k in (1, 10):
                        fn = S.sw_align if algo == S.SW else S.nw_align
                        got = [(h["score"], h["id"]) for h in fn(qq, k, 16)]
                        assert got == po.topk(exp, keep.astype(np.uint64), k)
        S.set_option("pair_np", 0)
        S.set_option("strip_np", 16)
        S.set_option("sw_kernel", 0)
        S.free_sequence(qq)


def _long_entry_case(qlen, algo, gaps, waves, huge, share4=None, long16=0, kernel=None):
    rng = np.random.default_rng(1000 + qlen)
    q = syn.protein_query(qlen, 200 + qlen)
    head = [3000, 1, 0, 2500, 17, 64, 4100, qlen + 7] + ([35000, 22000, 20001] if huge else [])
    lens = np.array(head + list(rng.integers(1, 400, 248)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    codes[int(off[7]) + 3:int(off[7]) + 3 + qlen] = q           # high-scoring entry
    codes[int(off[6]) + 100:int(off[6]) + 100 + qlen] = q       # inside a long one
    if huge:
        codes[int(off[8]) + 30000:int(off[8]) + 30000 + qlen] = q
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    keep = np.nonzero(lens > 0)[0]
    exp = po.scores(algo, q, codes, off, M, gaps[0], gaps[1])[keep]
    configure(False, ("builtin", "blosum62"), gaps[0], gaps[1])
    fn = S.sw_align if algo == S.SW else S.nw_align
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        S.set_option("long_waves", waves)
        S.set_option("long16", long16)
        if share4 is not None:
            S.set_option("long4_share_pct", share4)
        try:
            for lg in (1, 3, 0):
                S.set_option("long_groups", lg)
                sc, ids = _full_scores(qq, algo, len(keep))
                assert (ids == keep).all()
                assert (sc == exp).all(), (lg, np.nonzero(sc != exp)[0][:10])
                st = S.stats()
                if st["kernel"].startswith("pair"):
                    assert st["long_entries"] == 64 * lg
                    if lg:
                        packed = long16 and algo == S.SW
                        assert st["long_kernel"].startswith("long16" if packed else "long32"), st["long_kernel"]
                        assert kernel is None or st["long_kernel"] == kernel, (st["long_kernel"], kernel)
                got = [(h["score"], h["id"]) for h in fn(qq, 10, 16)]
                assert got == po.topk(exp, keep.astype(np.uint64), 10)
        finally:
            S.set_option("long_groups", -1)
            S.set_option("long_waves", 0)
            S.set_option("long16", 1)
            S.set_option("long4_share_pct", 1500)   # (the default)
        S.free_sequence(qq)


@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_tiny_db_routes_every_group_to_long_kernels(algo):
    """A DB too small to fill the chip (benchmark_pairwise.c's one entry; a few
    groups of ragged lengths): with a query of two strips or more the
    automatic plan sends every group to the long-entry kernels (long_plan's
    latency rule), with a one-strip query none; every score and the top hits
    equal the oracle's either way, at one and several long passes."""
    rng = np.random.default_rng(71)
    S.set_option("long_latency", 1)
    M = TABLES["matrices"][NAMES.index("blosum50")].copy()
    configure(False, ("builtin", "blosum50"), -3, -1)
    dbs = [np.array([513]), np.array([700, 0, 1] + list(rng.integers(1, 700, 150)))]
    for lens in dbs:
        lens = lens.astype(np.int64)
        off = np.zeros(len(lens) + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
        keep = np.nonzero(lens > 0)[0]
        with tempfile.TemporaryDirectory() as tmp:
            S.init_db(_write_db(tmp, codes, off))
            for qlen in (30, 390, 1100):
                q = syn.protein_query(qlen, 300 + qlen)
                exp = po.scores(algo, q, codes, off, M, -3, -1)[keep]
                qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
                sc, ids = _full_scores(qq, algo, len(keep))
                assert (ids == keep).all()
                assert (sc == exp).all(), (len(lens), qlen, np.nonzero(sc != exp)[0][:10])
                st = S.stats()
                assert st["kernel"].startswith("pair"), st["kernel"]
                if qlen == 30:
                    assert st["long_entries"] == 0
                else:
                    # (every group: 64 lanes each, covering every entry)
                    assert st["long_entries"] % 64 == 0 and st["long_entries"] >= len(keep), (qlen, st["long_entries"])
                fn = S.sw_align if algo == S.SW else S.nw_align
                got = [(h["score"], h["id"]) for h in fn(qq, 10, 16)]
                assert got == po.topk(exp, keep.astype(np.uint64), 10)
                S.free_sequence(qq)


def test_wave_timeline_and_priority_keep_scores():
    """Options that only change scheduling -- the wave timeline (one row per
    long_kernel lane and pair_kernel group, ssa_amd_get_timeline) and the raised
    priority of the longest pair groups -- leave every score as the oracle's;
    the timeline has a well-formed row for every group and long entry."""
    rng = np.random.default_rng(5)
    q = syn.protein_query(300, 55)
    lens = np.array([3000, 2800, 2600] + list(rng.integers(1, 500, 2000)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    exp = po.scores(S.SW, q, codes, off, M, -11, -1)
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        try:
            for lg, prio in ((1, -1), (0, 0), (2, 5)):
                S.set_option("long_groups", lg)
                S.set_option("pair_prio_groups", prio)
                S.set_option("timeline", 1)
                sc, ids = _full_scores(qq, S.SW, len(lens))
                assert (sc == exp).all(), (lg, prio, np.nonzero(sc != exp)[0][:10])
                # pair_np auto: 48-row SW strips, 80-row NW strips
                assert S.stats()["strip_rows"] == 48
                S.nw_align(qq, 5, 16)
                assert S.stats()["strip_rows"] == 80
                t = S.timeline()
                ngroups = (len(lens) + 63) // 64
                assert t.shape == (lg * 64 + ngroups - lg, 4)
                lng, pr = t[:lg * 64], t[lg * 64:]
                assert (pr[:, 0] == np.arange(lg, ngroups)).all()
                assert ((lng[:, 0] & 0x7fffffff) == np.arange(lg * 64)).all() and (lng[:, 0] >> 31 == 1).all()
                dur = (t[:, 2].astype(np.int64) - t[:, 1].astype(np.int64)) % (1 << 32)
                assert (dur < 100_000_000).all()          # under a second of the 100 MHz clock
        finally:
            S.set_option("timeline", 0)
            S.set_option("long_groups", -1)
            S.set_option("pair_prio_groups", 0)
        S.free_sequence(qq)


@pytest.mark.parametrize("algo,qlen", [(S.SW, 300), (S.SW, 49), (S.NW, 1000), (S.NW, 90)])
def test_strip_parts_keep_scores(algo, qlen):
    """pair_kernel with each group's strips split into dependent work units
    (option "pair_parts": all groups' first parts, then the second, ...; the
    strip boundary rows and SW running maxima cross workgroups): every score
    equals the oracle's with two and three parts (more are clamped to three;
    each part keeps its boundaries in a row buffer of its own), with and
    without long_kernel groups and start-order tickets."""
    rng = np.random.default_rng(qlen)
    q = syn.protein_query(qlen, 77 + qlen)
    lens = np.array([3000, 2800, 2600, 0, 1] + list(rng.integers(1, 500, 3000)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    codes[int(off[10]):int(off[10]) + min(qlen, int(lens[10]))] = q[:min(qlen, int(lens[10]))]
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    keep = np.nonzero(lens > 0)[0]
    exp = po.scores(algo, q, codes, off, M, -11, -1)[keep]
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        try:
            for parts, lg, ticket in ((2, -1, 1), (2, 0, 1), (3, -1, 1), (3, 0, 1), (50, 1, 1), (2, 2, 0),
                                      (3, 2, 0), (1, -1, 1)):
                S.set_option("pair_parts", parts)
                S.set_option("long_groups", lg)
                S.set_option("pair_ticket", ticket)
                sc, ids = _full_scores(qq, algo, len(keep))
                assert (ids == keep).all()
                assert (sc == exp).all(), (parts, lg, ticket, np.nonzero(sc != exp)[0][:10])
                assert S.stats()["kernel"].startswith("pair_f16")
                fn = S.sw_align if algo == S.SW else S.nw_align
                assert [(h["score"], h["id"]) for h in fn(qq, 10, 16)] == po.topk(exp, keep.astype(np.uint64), 10)
        finally:
            S.set_option("pair_parts", 0)
            S.set_option("long_groups", -1)
            S.set_option("pair_ticket", 1)
        S.free_sequence(qq)


@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_strip_part_wait_timeout_reruns_without_parts(algo):
    """A strip part whose wait for its group's first part runs into its
    bound (option "part_wait_us"; 0 here, so practically every second part
    times out) is not fatal: the search runs again without parts, the
    scores and top-k stay exact, and stats count the retry -- single
    queries and a fused batch (one pair_kernel launch for several queries)."""
    rng = np.random.default_rng(31)
    q = syn.protein_query(300, 5)
    lens = np.array([2000, 1500, 0] + list(rng.integers(1, 500, 6000)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    keep = np.nonzero(lens > 0)[0]
    exp = po.scores(algo, q, codes, off, M, -11, -1)[keep]
    configure(False, ("builtin", "blosum62"), -11, -1)
    fn = S.sw_align if algo == S.SW else S.nw_align
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        qs = [S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q[:n])) for n in (300, 290, 299)]
        try:
            S.set_option("part_wait_us", 0)
            for parts in (3, 2):
                S.set_option("pair_parts", parts)
                sc, ids = _full_scores(qq, algo, len(keep))
                assert (ids == keep).all() and (sc == exp).all(), (parts, np.nonzero(sc != exp)[0][:10])
                assert S.stats()["part_retries"] == 1, parts
            top = [(h["score"], h["id"]) for h in fn(qq, 10, 16)]
            assert top == po.topk(exp, keep.astype(np.uint64), 10)
            batch = S.search_batch(qs, algo, 10)
            assert S.stats()["part_retries"] >= 1
            S.set_option("part_wait_us", 2_000_000)
            single = [[tuple(map(int, h[:2])) for h in S.search(x, algo, 10)] for x in qs]
            assert [[tuple(map(int, h[:2])) for h in b] for b in batch] == single
            assert S.stats()["part_retries"] == 0
        finally:
            S.set_option("pair_parts", 0)
            S.set_option("part_wait_us", 2_000_000)
        for x in qs + [qq]:
            S.free_sequence(x)


LONG_QLENS = [1, 5, 63, 64, 65, 255, 256, 257, 384, 385, 400, 512, 513, 640, 641, 768, 769, 1024, 1025, 1500, 2049]


@pytest.mark.parametrize("qlen", LONG_QLENS)
@pytest.mark.parametrize("algo", [S.SW, S.NW])
@pytest.mark.parametrize("waves", [4, 1])
def test_long_entry_kernel_vs_oracle(qlen, algo, waves):
    """long_kernel (int32; an entry's query rows over the lanes of 4 waves or
    of one, passes of up to 1024 rows) on the leading (longest) groups --
    forced to 1 and 3 of the groups, and to none -- gives every entry the
    oracle's score; the DB has entries of 1..4100 residues, empty records and
    planted copies of the query; with 4 waves also entries of 20-35 k
    residues (UniProt's longest)."""
    _long_entry_case(qlen, algo, (-11, -1), waves, huge=waves == 4 and qlen in (5, 400, 513, 1025, 2049))


@pytest.mark.parametrize("qlen", LONG_QLENS)
def test_long16_kernel_vs_oracle(qlen):
    """long16_kernel (SW on packed 16-bit patterns, two rows per register,
    one wave per entry, rows per lane 4..16, passes of 1024 rows beyond) on the
    same DBs: every score the oracle's, with the 20-35 k-residue entries for
    the query lengths the benchmark configurations use."""
    _long_entry_case(qlen, S.SW, (-11, -1), 1, huge=qlen in (5, 400, 513, 1025, 2049), long16=1)



@pytest.mark.parametrize("gate", [0, 1])
def test_long_entries_without_the_gate(gate):
    """Option long_gate 0: the pair kernel does not wait for the long-entry
    workgroups to start (they are issued after the tables kernel, on the
    highest-priority streams) -- the scheduling changes, the scores do not."""
    S.set_option("long_gate", gate)
    try:
        _long_entry_case(400, S.SW, (-11, -1), 1, huge=True, long16=1)
        _long_entry_case(513, S.NW, (-11, -1), 0, huge=True)
    finally:
        S.set_option("long_gate", 1)


@pytest.mark.parametrize("qlen", [1025, 1032, 1500, 2056, 262, 513])
@pytest.mark.parametrize("rows", [1, 0, 2])
def test_long16_row_scan(qlen, rows):
    """long16_kernel beyond 1 024 query rows (long16_plan): whole passes plus
    1-8 query rows scored one row at a time by a prefix maximum over 64 columns
    per step (q = 1025 / 1032: one RL 16 pass + 1 / 8 rows, 2056: two + 8),
    two RL 12 passes for q = 1500, and the same lengths without the plan
    (option long16_rows 0: RL 16 passes) -- every score the oracle's, with
    the 20-35 k-residue entries."""
    # (option 2: the cost model below 1 024 rows too -- q = 262: RL 4 + 6, 513: RL 8 + 1)
    plan = {1025: ("long16_rl16+1", "long16_rl16", "long16_rl16+1"),
            1032: ("long16_rl16+8", "long16_rl16", "long16_rl16+8"),
            1500: ("long16_rl12", "long16_rl16", "long16_rl12"),
            2056: ("long16_rl16+8", "long16_rl16", "long16_rl16+8"),
            262: ("long16_rl6", "long16_rl6", "long16_rl4+6"),
            513: ("long16_rl10", "long16_rl10", "long16_rl8+1")}[qlen]
    S.set_option("long16_rows", rows)
    try:
        _long_entry_case(qlen, S.SW, (-11, -1), 1, huge=True, long16=1, kernel=plan[{1: 0, 0: 1, 2: 2}[rows]])
    finally:
        S.set_option("long16_rows", 1)


@pytest.mark.parametrize("qlen", [5, 400, 1025])
@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_long_entry_kernel_split_launches(qlen, algo):
    """Automatic split: the 35 k-residue entry's group at 4 waves per entry
    (stream 1), the other long groups at one wave per entry (stream 2), both
    beside the pair kernel."""
    _long_entry_case(qlen, algo, (-11, -1), 0, huge=True, share4=50000)


@pytest.mark.parametrize("algo,pnp,qlens", [
    (S.SW, 24, (49, 50, 53, 54, 57, 61, 66, 70, 74, 78, 82, 86, 90, 94, 95, 97, 101, 141, 513)),
    (S.NW, 40, (81, 82, 85, 89, 93, 97, 101, 105, 117, 121, 125, 133, 153, 157, 161, 165, 513)),
    (S.NW, 32, (65, 66, 69, 73, 77, 90, 94, 126))])
def test_tail_strip_four_row_granularity(algo, pnp, qlens):
    """Option tail_rows4 (default): after at least one main strip, the pair
    kernel's last strip is 4*k rows, not 8*k -- tails of 2 mod 4 packed rows
    (a two-dword LDS reload for their last rows, a padded global table pitch,
    2-row anti-diagonal groups).  Every remainder class against the oracle,
    with the option on and off."""
    rng = np.random.default_rng(pnp)
    lens = np.array([0, 1, 2, 15, 16, 17, 47, 48, 49, 513] + list(rng.integers(1, 300, 200)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    keep = np.nonzero(lens > 0)[0]
    configure(False, ("builtin", "blosum62"), -11, -1)
    fn = S.sw_align if algo == S.SW else S.nw_align
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        S.set_option("pair_np", pnp)
        try:
            for qlen in qlens:
                q = syn.protein_query(qlen, 300 + qlen)
                exp = po.scores(algo, q, codes, off, M, -11, -1)[keep]
                qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
                for t4 in (1, 0):
                    S.set_option("tail_rows4", t4)
                    sc, ids = _full_scores(qq, algo, len(keep))
                    assert (ids == keep).all()
                    assert (sc == exp).all(), (qlen, t4, np.nonzero(sc != exp)[0][:10])
                    assert S.stats()["kernel"].startswith("pair")
                    assert [(h["score"], h["id"]) for h in fn(qq, 10, 16)] == po.topk(exp, keep.astype(np.uint64), 10)
                S.free_sequence(qq)
        finally:
            S.set_option("pair_np", 0)
            S.set_option("tail_rows4", 1)


@pytest.mark.parametrize("gaps", [(0, 0), (-1, -4), (-5, -5), (-20, -7)])
@pytest.mark.parametrize("qlen", [64, 513])
@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_long_entry_kernel_gap_penalties(gaps, qlen, algo):
    """long_kernel's SW clamps E and F at 0 (exact for R <= 0) and its NW is
    the plain recurrence, as long16_kernel's SW clamps at the score-0 pattern:
    zero, steep and unequal gap penalties against the oracle."""
    _long_entry_case(qlen, algo, gaps, 4, huge=False)
    if algo == S.SW:
        _long_entry_case(qlen, algo, gaps, 1, huge=False, long16=1)


@pytest.mark.parametrize("match", [60, 102, 103, 120])
def test_long16_score_bound(match):
    """long16_kernel's exactness bound, base16 + min(m, n) maxM + maxM <=
    0x7BFF (engine.cpp long16_plan): a 300-residue query on a constant
    matrix with copies of itself planted in 2-5 k-residue entries scores
    300 x match; match 102 still fits (base16 0x0404), 103 and up the int32
    kernel takes the long groups -- every score exact either way."""
    rng = np.random.default_rng(match)
    q = rng.choice(syn.AA_CODES, size=300).astype(np.uint8)
    lens = np.array([5000, 4200, 3000, 2500] + list(rng.integers(1, 400, 700)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    for e, at in ((0, 4000), (2, 17), (3, 2200)):
        codes[int(off[e]) + at:int(off[e]) + at + 300] = q
    M = po.matrix_constant(match, -1)
    exp = po.scores(S.SW, q, codes, off, M, -3, -1)
    assert exp.max() == 300 * match
    configure(False, ("const", match, -1), -3, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        try:
            S.set_option("long_groups", 1)
            sc, _ = _full_scores(qq, S.SW, len(lens))
            assert (sc == exp).all(), np.nonzero(sc != exp)[0][:10]
            st = S.stats()
            if st["long_entries"]:
                assert st["long_kernel"].startswith("long16" if match <= 102 else "long32"), st["long_kernel"]
        finally:
            S.set_option("long_groups", -1)
        S.free_sequence(qq)


@pytest.mark.parametrize("match", [40, 55, 127])
def test_sw_f16_pattern_limit(match):
    """Scores around the f16-pattern kernel's exact range (29695) and the
    int16 range (65534): every score still exact (re-routed lanes)."""
    rng = np.random.default_rng(match)
    base = rng.choice(syn.AA_CODES, size=1200).astype(np.uint8)
    seqs = [base[:n] for n in (200, 500, 540, 560, 600, 700, 1200)] + [rng.choice(syn.AA_CODES, 300).astype(np.uint8)]
    codes = np.concatenate(seqs)
    off = np.zeros(len(seqs) + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    M = po.matrix_constant(match, -1)
    exp = po.scores(0, base, codes, off, M, -3, -1)
    configure(False, ("const", match, -1), -3, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(base))
        for swk in (0, 1):
            S.set_option("sw_kernel", swk)
            sc, _ = _full_scores(qq, S.SW, len(seqs))
            assert (sc == exp).all(), (swk, sc, exp)
        S.set_option("sw_kernel", 0)
        S.free_sequence(qq)


@pytest.mark.parametrize("n_long", [5, 200])
def test_nw_f16_length_bound(n_long):
    """NW on f16 patterns admits entries up to a length bound derived from the
    query, matrix and gaps (engine.cpp nw_f16_limit): with R=-30 and a
    100-residue query it is 874, the int16 bound 984.  Lengths straddle both;
    by default the groups holding entries beyond the bound go to long_kernel
    (exact int32, nothing left for the int64 re-score); without it a few long
    entries are re-scored exactly, many long ones switch the whole search to
    the int16 kernel -- every score stays exact either way."""
    rng = np.random.default_rng(n_long)
    q = syn.protein_query(100, 11)
    lens = np.concatenate([np.arange(860, 890), [980, 984, 985, 990, 1200],
                           rng.integers(860, 1000, n_long), rng.integers(1, 400, 300)]).astype(np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    exp = po.scores(S.NW, q, codes, off, M, -40, -30)
    configure(False, ("builtin", "blosum62"), -40, -30)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        try:
            for swk, lg in ((0, -1), (0, 0), (1, -1)):
                S.set_option("sw_kernel", swk)
                S.set_option("long_groups", lg)
                sc, _ = _full_scores(qq, S.NW, len(lens))
                assert (sc == exp).all(), (swk, lg, np.nonzero(sc != exp)[0][:10])
                if (swk, lg) == (0, -1):
                    assert S.stats()["kernel"] == "pair_f16_nw" and S.stats()["wide_count"] == 0
                else:
                    assert S.stats()["wide_count"] >= 2
        finally:
            S.set_option("sw_kernel", 0)
            S.set_option("long_groups", -1)
        S.free_sequence(qq)


def test_sw_large_matrix_values_fall_back(tmp_path):
    """|score| > 1024 is outside the f16-pattern kernel's contract: the
    engine must pick the int16 kernel (or int64) and stay exact."""
    txt = "   A  R  N\nA 2000 -5 -1500\nR -5 7 -1\nN -1500 -1 6\n"
    mpath = tmp_path / "big.txt"
    mpath.write_text(txt)
    M = po.matrix_parse(txt)
    rng = np.random.default_rng(7)
    alpha = np.array([1, 16, 13], np.uint8)   # A R N codes
    q = rng.choice(alpha, 90).astype(np.uint8)
    seqs = [rng.choice(alpha, n).astype(np.uint8) for n in rng.integers(1, 120, 200)]
    codes = np.concatenate(seqs)
    off = np.zeros(len(seqs) + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    for algo in (S.SW, S.NW):
        exp = po.scores(algo, q, codes, off, M, -4, -2)
        configure(False, ("file", str(mpath)), -4, -2)
        S.init_db(_write_db(str(tmp_path), codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        sc, _ = _full_scores(qq, algo, len(seqs))
        assert (sc == exp).all()
        S.free_sequence(qq)


@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_wide_kernel_matches_oracle(algo):
    """Every entry forced through the exact int64 re-score kernel."""
    q = syn.protein_query(77, 5)
    codes, off = syn.protein_db(700, 9, query=q, plant_every=100, lo=1, hi=400)
    M = TABLES["matrices"][NAMES.index("blosum50")].copy()
    exp = po.scores(algo, q, codes, off, M, -10, -2)
    configure(False, ("builtin", "blosum50"), -10, -2)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        S.set_option("force_wide", 1)
        try:
            sc, _ = _full_scores(qq, algo, 700)
        finally:
            S.set_option("force_wide", 0)
        assert (sc == exp).all()
        assert S.stats()["wide_count"] == 700
        S.free_sequence(qq)


@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_int16_overflow_reroute(algo):
    """Scores beyond int16 (SW >= 65535, NW beyond the proven bound) come
    back exact through the overflow list (reference test_searcher.c:507-536
    shape: constant 127/-1 self-alignment)."""
    rng = np.random.default_rng(3)
    base = rng.choice(syn.AA_CODES, size=900).astype(np.uint8)
    seqs = [base, base[:600], rng.choice(syn.AA_CODES, size=300).astype(np.uint8), base[100:]]
    codes = np.concatenate(seqs)
    off = np.zeros(len(seqs) + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    M = po.matrix_constant(127, -1)
    exp = po.scores(algo, base, codes, off, M, -1, -1)
    assert exp.max() > 65535
    configure(False, ("const", 127, -1), -1, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(base))
        try:
            # by default the entries beyond the f16 bound go to long_kernel
            # (int32); without it through the overflow list
            for lg in (-1, 0):
                S.set_option("long_groups", lg)
                sc, _ = _full_scores(qq, algo, 4)
                assert (sc == exp).all(), lg
                if lg == 0:
                    assert S.stats()["wide_count"] >= 1
                # through the device filter (k <= 64): the int32 tier after the
                # result's copy when the header reports overflowed lanes
                # (option tier_defer, default) or before the filter
                fn = S.sw_align if algo == S.SW else S.nw_align
                ids = np.arange(4, dtype=np.uint64)
                for td in (1, 0):
                    S.set_option("tier_defer", td)
                    for k in (1, 3):
                        assert [(h["score"], h["id"]) for h in fn(qq, k, 16)] == po.topk(exp, ids, k), (lg, td, k)
        finally:
            S.set_option("long_groups", -1)
            S.set_option("tier_defer", 1)
        S.free_sequence(qq)


@pytest.mark.parametrize("qlen,n", [(700, 12000), (1300, 3000)])
@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_int32_rescore_tier_vs_oracle(algo, qlen, n):
    """Overflowed lanes (here: the int16 strip kernel, constant 127/-1, where
    >= 10 % of the entries -- copies of the query -- score beyond 16 bits)
    are re-scored by the exact int32 tier (long_kernel over the overflow
    list, one wave per entry) instead of the int64 one-thread-per-entry
    kernel: every score equals the oracle's full_sw / full_nw, the same
    lanes are re-scored, and the tier is far faster (reference: the
    re-score cascade of src/algo/16/search_16.c:101-109).  q = 1300 takes
    the tier's multi-pass route (more than 1024 query rows: each wave's
    scratch row reused across the list entries it loops over)."""
    rng = np.random.default_rng(17 + qlen)
    q = rng.choice(syn.AA_CODES, size=qlen).astype(np.uint8)
    lens = rng.integers(20, 600, n)
    seqs = [rng.choice(syn.AA_CODES, size=int(x)).astype(np.uint8) for x in lens]
    for i in range(0, n, 8):                 # 1 in 8: a near-copy of the query
        a = int(rng.integers(0, 60))
        s = q[a:].copy()
        s[rng.random(len(s)) < 0.02] = syn.AA_CODES[0]
        seqs[i] = s
    codes = np.concatenate(seqs)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    M = po.matrix_constant(127, -1)
    exp = po.scores(algo, q, codes, off, M, -1, -1)
    configure(False, ("const", 127, -1), -1, -1)
    S.set_option("counters", 0)          # (timed below: no overflow-counter replays in wide_ms)
    S.set_option("lean_events", 0)       # (wide_ms needs the tier's markers)
    ms = {}
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        try:
            S.set_option("sw_kernel", 1)
            S.set_option("long_groups", 0)
            for r32 in (1, 0):
                S.set_option("rescore32", r32)
                sc, ids = _full_scores(qq, algo, n)
                assert (sc == exp).all(), (r32, np.nonzero(sc != exp)[0][:10])
                st = S.stats()
                assert st["wide_count"] >= n // 10, st["wide_count"]
                fn = S.sw_align if algo == S.SW else S.nw_align
                best = []
                for _ in range(3):
                    assert [(h["score"], h["id"]) for h in fn(qq, 10, 16)] == po.topk(exp, ids, 10)
                    best.append(S.stats()["wide_ms"])
                ms[r32] = min(best)
        finally:
            S.set_option("sw_kernel", 0)
            S.set_option("long_groups", -1)
            S.set_option("rescore32", 1)
            S.set_option("lean_events", 1)
        S.free_sequence(qq)
    # the speed ratio is reported, not asserted (tools/rescore_bench.py
    # measures it; a shared box must not fail an exact test on timing)
    print(f"re-score of {st['wide_count']} lanes: int32 tier {ms[1]:.3f} ms, int64 kernel {ms[0]:.3f} ms")
    assert ms[0] > 0 and ms[1] > 0, ms


def test_filter_host_with_side_tier_overflow():
    """Options filter_host 1/2/3 (the filter's result in pinned memory) with
    side_tier 1 (the int32 re-score tier beside the filter) on a DB whose
    pair-kernel lanes overflow (SW maxima <= |R| are re-scored exactly: half
    the entries share no residue with the query): the host must wait for
    the tier before it reads the exact scores -- every combination equals
    the oracle, and the timing read at the end never fails."""
    rng = np.random.default_rng(23)
    a, b = syn.AA_CODES[:10], syn.AA_CODES[10:]
    q = rng.choice(a, size=300).astype(np.uint8)
    n = 3000
    lens = rng.integers(20, 400, n)
    seqs = [rng.choice(b if i % 2 else syn.AA_CODES, size=int(x)).astype(np.uint8) for i, x in enumerate(lens)]
    codes = np.concatenate(seqs)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    exp = po.scores(S.SW, q, codes, off, po.matrix_constant(5, -4), -3, -20)
    ids = np.arange(n, dtype=np.uint64)
    configure(False, ("const", 5, -4), -3, -20)
    S.set_option("counters", 0)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        try:
            for side in (1, 0):
                S.set_option("side_tier", side)
                for fh in (1, 2, 3, 0):
                    S.set_option("filter_host", fh)
                    for k in (1, 10, 64):
                        got = [(h["score"], h["id"]) for h in S.sw_align(qq, k, 16)]
                        assert got == po.topk(exp, ids, k), (side, fh, k)
                        st = S.stats()
                        assert st["kernel"] == "pair_f16_sw" and st["wide_count"] >= n // 3, (side, fh, st["wide_count"])
        finally:
            S.set_option("side_tier", 0)
            S.set_option("filter_host", 0)
            S.set_option("counters", -1)
        S.free_sequence(qq)


def test_search_graph_replays_exactly():
    """Option graph 1 (default 0): the usual search's stream operations --
    upload, tables, long-entry kernels on their own streams, the pair kernel
    with strip parts, the filter, the result's copy -- are captured once per
    launch plan into a HIP graph and replayed with the changed arguments (gate
    target, strip-part epoch, copy length) set on their nodes.  Results equal
    the call-by-call path and the oracle over alternating plans (query
    lengths, SW/NW, k), repeated queries replay the cached graph (stats graph
    2), a new plan is captured (1), and kernel_ms, read from the graph's own
    event nodes, stays that of the direct path."""
    rng = np.random.default_rng(41)
    codes, off = syn.protein_db(20000, 42, lo=1, hi=1200)
    # a few long entries: the long-entry streams join the graph
    lens = np.diff(off).astype(np.int64)
    seqs = [codes[int(off[i]):int(off[i + 1])] for i in range(len(lens))]
    for i in range(0, 300, 3):
        seqs[i] = rng.choice(syn.AA_CODES, int(rng.integers(3000, 6000))).astype(np.uint8)
    db, doff = po.pack_db(seqs)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    ids = np.arange(len(seqs), dtype=np.uint64)
    configure(False, ("builtin", "blosum62"), -11, -1)
    S.set_option("counters", 0)          # (counted searches run call by call)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, db, doff))
        qs = {n: syn.protein_query(n, 900 + n) for n in (60, 250, 400)}
        qq = {n: S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q)) for n, q in qs.items()}
        exp = {(n, a): po.scores(a, q, db, doff, M, -11, -1) for n, q in qs.items() for a in (S.SW, S.NW)}
        # each plan three times (a plan's first search may also build its
        # pair-row stream, a one-time operation: its shape is the plan's from
        # the second search on), then each again after the others (four plans
        # cached), then k = 1 (the same kernels as k = 10, other arguments)
        order = ([(400, S.SW, 10)] * 3 + [(60, S.SW, 10)] * 3 + [(250, S.NW, 64)] * 3
                 + [(400, S.SW, 10), (60, S.SW, 10), (250, S.NW, 64), (400, S.SW, 1), (60, S.NW, 10)])
        try:
            S.set_option("long_groups", 2)
            got = {}
            for g in (1, 0):
                S.set_option("graph", g)
                got[g] = []
                for n, a, k in order:
                    fn = S.sw_align if a == S.SW else S.nw_align
                    hits = [(h["score"], h["id"]) for h in fn(qq[n], k, 16)]
                    st = S.stats()
                    got[g].append((hits, st["graph"], st["kernel_ms"]))
                    assert hits == po.topk(exp[(n, a)], ids, k), (g, n, a, k)
            assert [x[0] for x in got[1]] == [x[0] for x in got[0]]
            modes = [x[1] for x in got[1]]
            assert all(m == 0 for _, m, _ in got[0]), [x[1] for x in got[0]]
            print("graph modes", modes, "kernel ms", [round(x[2], 3) for x in got[1]], [round(x[2], 3) for x in got[0]])
            assert modes[0] == 1 and min(modes) >= 1, str(modes)
            assert [modes[i] for i in (2, 5, 8, 10, 11, 12)] == [2] * 6, str(modes)
            # (a capturing search's kernel_ms also holds the capture, which
            # runs between its two timing records)
            for (h1, m1, k1), (h0, m0, k0) in zip(got[1], got[0]):
                if m1 == 2:
                    assert 0 < k1 and 0.75 * k0 < k1 < 1.33 * k0 + 0.05, (k1, k0)
        finally:
            S.set_option("graph", 0)
            S.set_option("long_groups", -1)
        for q in qq.values():
            S.free_sequence(q)


def test_shard_logs_replay_to_global_result():
    """The insertion logs of consecutive ID shards, concatenated in shard
    order and replayed, equal the single-DB top-k including tie IDs."""
    q = syn.protein_query(60, 1)
    codes, off = syn.protein_db(4000, 2, query=q, plant_every=300, lo=10, hi=200)
    n = 4000
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        qs = syn.query_string(q)
        full = {}
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, qs)
        for k in (1, 7, 50, 333):
            full[k] = [(h["score"], h["id"]) for h in S.sw_align(qq, k, 16)]
        cuts = [0, 1000, 1700, 3100, n]
        for k in (1, 7, 50, 333):
            log = []
            for r in range(len(cuts) - 1):
                a, b = cuts[r], cuts[r + 1]
                sub_off = off[a:b + 1] - off[a]
                path = os.path.join(tmp, f"shard{r}.fas")
                syn.write_fasta(path, codes[int(off[a]):int(off[b])], sub_off)
                S.init_db(path)
                S.set_id_offset(a)
                log += S.search(qq, S.SW, k, 16, S.LOG)
            S.set_id_offset(0)
            assert S.replay(log, k) == full[k]
        S.free_sequence(qq)


def test_nucleotide_both_strands_and_multi_query():
    """NUCLEOTIDE with both strands: 2 query strands x 2 DB strands, heap
    order chunk by chunk (search_64.c:44-56); checked against a CPU replay
    of the same insertion order built from oracle scores."""
    seqs = po.read_fasta(os.path.join(DATA, "AF091148.fas"))[:300]
    dbc = [po.map_db(s, True) for s in seqs]
    qraw = po.read_query_fasta(os.path.join(DATA, "one_seq.fas"))
    qf = po.map_query(qraw, True)
    comp = np.array([0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15], np.uint8)
    qr = comp[qf[::-1]]
    M = po.matrix_constant(2, -3)
    entries = []
    for i, d in enumerate(dbc):
        if len(d):
            entries.append((i, 0, d))
            entries.append((i, 1, comp[d[::-1]]))
    db, off = po.pack_db([e[2] for e in entries])
    for algo in (0, 1):
        sq = [po.scores(algo, qv, db, off, M, -5, -2) for qv in (qf, qr)]
        chunk = 37
        order_s, order_i = [], []
        e0 = 0
        while e0 < len(entries):
            cend = (entries[e0][0] // chunk + 1) * chunk
            e1 = e0
            while e1 < len(entries) and entries[e1][0] < cend:
                e1 += 1
            for v in range(2):
                for e in range(e0, e1):
                    order_s.append(sq[v][e])
                    order_i.append(entries[e][0])
            e0 = e1
        exp = po.topk(np.array(order_s), np.array(order_i, np.uint64), 25)
        configure(True, ("const", 2, -3), -5, -2, chunk=chunk, strands=S.BOTH_STRANDS)
        with tempfile.TemporaryDirectory() as tmp:
            path = os.path.join(tmp, "db.fas")
            with open(path, "wb") as f:
                for s in seqs:
                    f.write(b">x\n" + s + b"\n")
            S.init_db(path)
            qq = S.init_sequence_fasta(S.READ_FROM_STRING, qraw.decode())
            fn = S.sw_align if algo == 0 else S.nw_align
            got = [(h["score"], h["id"]) for h in fn(qq, 25, 16)]
            S.free_sequence(qq)
        assert [s for s, _ in got] == [s for s, _ in exp]
        assert got == exp
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
    S.set_chunk_size(1000)


def _insertion_order(entries, views_scores, chunk):
    """Reference 64-bit insertion order (search_64.c:44-56): DB IDs in chunks
    of `chunk`; within a chunk every query view (outer) over the chunk's
    entries in adapter order (inner)."""
    order = []
    e0 = 0
    while e0 < len(entries):
        cend = (entries[e0][0] // chunk + 1) * chunk
        e1 = e0
        while e1 < len(entries) and entries[e1][0] < cend:
            e1 += 1
        for v, sc in enumerate(views_scores):
            for e in range(e0, e1):
                order.append((int(sc[e]), entries[e][0], v, entries[e][1], entries[e][2]))
        e0 = e1
    return order


@pytest.mark.parametrize("mode", ["TRANS_DB", "TRANS_QUERY", "TRANS_BOTH"])
@pytest.mark.parametrize("strands", [S.FORWARD_STRAND, S.BOTH_STRANDS, S.COMPLEMENTARY_STRAND])
def test_translated_search_vs_oracle(mode, strands):
    """Translated searches: query views x DB entries (strand/frame) in the
    reference's insertion order; frames translated by the reference-pinned
    translation (tests/test_translate.py), scores by the oracle."""
    rng = np.random.default_rng(strands * 7 + len(mode))
    t = getattr(S, mode)
    chunk = 23
    comp = np.array([0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15], np.uint8)
    # DNA records (lengths >= 2: the reference's (len - frame) / 3 underflows
    # for shorter ones), a few empty records, IUPAC codes now and then
    nrec = 160
    lens = rng.integers(2, 400, nrec)
    lens[[5, 77]] = 0
    dna = []
    for n in lens:
        c = rng.choice(np.array([1, 2, 4, 8], np.uint8), n)
        dna.append(np.where(rng.random(n) < 0.05, rng.integers(1, 16, n), c).astype(np.uint8))
    nt_text = b"-ACMGRSVTWYHKDBN"
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    S.set_output_mode(S.OUTPUT_ERROR)
    S.init_symbol_translation(t, strands, 1, 1)
    S.init_score_matrix(S.MATRIX_BUILDIN, "blosum62")
    S.init_gap_penalties(-11, -1)
    sel = [s for s in range(2) if (s + 1) & strands]
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "db.fas")
        if t == S.TRANS_QUERY:
            prot = [rng.choice(syn.AA_CODES, int(n) // 3).astype(np.uint8) for n in lens]
            qdna = dna[3][:240] if len(dna[3]) >= 240 else rng.choice(np.array([1, 2, 4, 8], np.uint8), 240)
            # plant translated query frames in the DB
            for i, (s, f) in enumerate([(0, 0), (1, 2), (0, 1)]):
                prot[20 + 40 * i] = np.frombuffer(S.translate(0, qdna.tobytes(), s, f), np.uint8).copy()
            syn.write_fasta(path, np.concatenate(prot), np.concatenate([[0], np.cumsum([len(p) for p in prot])]).astype(np.uint64))
            entries = [(i, 0, p) for i, p in enumerate(prot) if len(p)]
            qviews = [np.frombuffer(S.translate(0, qdna.tobytes(), s, f), np.uint8) for s in sel for f in range(3)]
            qtext = bytes(nt_text[c] for c in qdna).decode()
        else:
            with open(path, "wb") as f:
                for d in dna:
                    f.write(b">r\n" + bytes(nt_text[c] for c in d) + b"\n")
            entries = []
            for i, d in enumerate(dna):
                if len(d) == 0:
                    continue
                for s in sel:
                    for fr in range(3):
                        e = np.frombuffer(S.translate(1, d.tobytes(), s, fr), np.uint8)
                        entries.append((i, s if strands == S.BOTH_STRANDS else strands, fr, e))
            entries = [(e[0], e[1], e[2], e[3]) for e in entries]
            if t == S.TRANS_DB:
                qprot = np.frombuffer(S.translate(1, dna[9].tobytes(), 0, 1), np.uint8)[:90]
                qviews = [qprot]
                qtext = syn.query_string(qprot)
            else:
                qdna = dna[9][:300]
                qviews = [np.frombuffer(S.translate(0, qdna.tobytes(), s, f), np.uint8) for s in sel for f in range(3)]
                qtext = bytes(nt_text[c] for c in qdna).decode()
        if t == S.TRANS_QUERY:
            ent = [(e[0], 0, 0) for e in entries]
            seqs = [e[2] for e in entries]
        else:
            ent = [(e[0], e[1], e[2]) for e in entries]
            seqs = [e[3] for e in entries]
        db, off = po.pack_db(seqs)
        S.init_db(path)
        S.set_chunk_size(chunk)
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, qtext)
        assert len(S.query_views(qq)) == len(qviews)
        for algo in (S.SW, S.NW):
            vs = [po.scores(algo, qv, db, off, M, -11, -1) for qv in qviews]
            order = _insertion_order(ent, vs, chunk)
            for k in (1, 17, 200):
                exp = po.topk(np.array([o[0] for o in order], np.int64),
                              np.array([o[1] for o in order], np.uint64), k)
                fn = S.sw_align if algo == S.SW else S.nw_align
                got = [(h["score"], h["id"]) for h in fn(qq, k, 16)]
                assert got == exp, (mode, strands, algo, k, got[:5], exp[:5])
        S.free_sequence(qq)
        S.set_chunk_size(1000)
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)


# reference tests/test_libssa.c:48-93 (COMPUTE_ALIGNMENT, 64-bit, 1 thread)
ALIGN_KAT = {
    "sw": [(877, 91, "2MD2MIM2I3MD3MD4M2D8M5I3M5IM3I7MI7M3I5MI3M"),
           (847, 91, "2MD2MIM2I3MD3MD4M2D8M5I3M5IM3I7MI7M3I4MI4M"),
           (753, 91, "2MD2MIM2I3MD3MD3M2D9M5I3M5IM3I7MI7M3I5MI3M"),
           (565, 91, "2MD2MIM2I3MD3MD4M2D8M5I3M5IM3I7MI7M3I5MI3M"),
           (398, 91, "2MD2MIM2I3MD3MD3M2D9M5I3M5IM3I7MI7M3I5MI3M")],
    "nw": [(1050, 33, "2MI2MI6M3I6MD3M19I4M3IMI3M5I3M5IM3I7MI7M4IMIMI4MI2M7I"),
           (908, 28, "2MI2MI6M3I6MD3M5IM2I2M3I2M5IMI9MD2M3I3M9I2M3I2M4I2M2IMI4MI2M7I"),
           (938, 24, "2MI2MI6M3I6MD3M5IM2I2M3I2M5IMI9MD2M3I3M9I2M3I2M4IM3IMIMIM2I5M10I"),
           (378, 21, "2MI2MI6M3I5M9I2M7IM6IMI3M3I6M5I3M5IM3I7MI7M4IMIMI4MI2M7I"),
           (75, 12, "2MI2MI6M3I5M9I2M7IM6IMI3M3I6M5I3M5IM3I7MI7M4IMIMI4MI2M7I")],
}


@pytest.mark.parametrize("width", [S.BIT_WIDTH_64, S.BIT_WIDTH_16, S.BIT_WIDTH_8])
def test_compute_alignment_kat(width):
    S.set_output_mode(S.OUTPUT_ERROR)
    S.init_constant_scores(5, -4)
    S.init_gap_penalties(-4, -2)
    S.init_symbol_translation(S.NUCLEOTIDE, S.FORWARD_STRAND, 3, 3)
    S.set_thread_count(1)
    S.init_db(os.path.join(DATA, "AF091148.fas"))
    q = S.init_sequence_fasta(S.READ_FROM_FILE, os.path.join(DATA, "one_seq.fas"))
    for name, fn in (("sw", S.sw_align), ("nw", S.nw_align)):
        got = [(h["id"], h["score"], h["alignment"]) for h in fn(q, 5, width, S.COMPUTE_ALIGNMENT)]
        assert got == ALIGN_KAT[name], (name, got)
    # COMPUTE_SCORE leaves the alignment fields empty
    assert all(h["alignment"] is None for h in S.sw_align(q, 5, width, S.COMPUTE_SCORE))
    S.free_sequence(q)
    S.set_thread_count(0)


@pytest.mark.parametrize("pattern", ["ties", "rising", "random"])
def test_device_topk_filter_matches_full_scan(pattern):
    """The device candidate filter (kernels.hip filter_*) must give exactly
    the host full-scan result: heavy ties, scores rising with the ID (most
    entries are candidates: exercises the > 64 K candidate path), random."""
    rng = np.random.default_rng(len(pattern))
    q = syn.protein_query(50, 3)
    n = 90000
    if pattern == "ties":
        seqs = [q[:30].copy() for _ in range(n)]
    elif pattern == "rising":
        seqs = [np.concatenate([q[: 1 + (i * 49) // n], rng.choice(syn.AA_CODES, 5)]).astype(np.uint8)
                for i in range(n)]
    else:
        seqs = [rng.choice(syn.AA_CODES, int(rng.integers(5, 80))).astype(np.uint8) for _ in range(n)]
    codes = np.concatenate(seqs)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        for algo, fn in ((S.SW, S.sw_align), (S.NW, S.nw_align)):
            for k in (1, 2, 10, 64):
                for width in (8, 16):
                    S.set_option("no_filter", 1)
                    full = [(h["score"], h["id"]) for h in fn(qq, k, width)]
                    st_full = S.stats()
                    S.set_option("no_filter", 0)
                    got = [(h["score"], h["id"]) for h in fn(qq, k, width)]
                    st = S.stats()
                    assert got == full, (pattern, algo, k)
                    assert (st["overflow_8"], st["overflow_16"]) == (st_full["overflow_8"], st_full["overflow_16"])
                    log_full = None
            S.set_option("no_filter", 1)
            log_full = S.search(qq, algo, 7, 16, S.LOG)
            S.set_option("no_filter", 0)
            assert S.search(qq, algo, 7, 16, S.LOG) == log_full
        S.free_sequence(qq)


def _filter_candidates(sc, k):
    """numpy restatement of the device filter's bound (kernels.hip,
    filter_block): entry e of mini m (64 entries) of block b (4096) is
    forwarded iff its score beats both the k-th largest value of the earlier
    minis of b and the k-th largest value of all minis of the blocks before b
    (INT32_MIN while fewer than k), where a mini's value is its maximum --
    except the DB's first mini, which gives its k largest entries."""
    lo = np.iinfo(np.int32).min
    n = len(sc)
    nm, nb = -(-n // 64), -(-n // 4096)
    pad = np.full(nb * 4096, lo, np.int64)
    pad[:n] = sc
    mm = pad.reshape(nb * 64, 64).max(1).reshape(nb, 64)
    vals = [[np.sort(pad[:64])[::-1][:k]] + [mm[0, m:m + 1] for m in range(1, 64)]]
    vals += [[mm[b, m:m + 1] for m in range(64)] for b in range(1, nb)]

    def kth(v):
        v = np.concatenate(v) if len(v) else np.zeros(0, np.int64)
        return lo if len(v) < k else int(np.sort(v)[::-1][k - 1])
    t_block = np.array([kth([x for bb in vals[:b] for x in bb]) for b in range(nb)], np.int64)
    t_local = np.array([[kth(vals[b][:m]) for m in range(64)] for b in range(nb)], np.int64).ravel()[:nm]
    e = np.arange(n)
    return int(np.count_nonzero(sc > np.maximum(t_block[e // 4096], t_local[e // 64])))


@pytest.mark.parametrize("n,pattern", [(100, "random"), (4097, "rising"), (90000, "random"), (90000, "rising"),
                                       (700000, "random"), (700000, "falling")])
def test_device_filter_candidate_count_is_exact(n, pattern):
    """The filter's lane moves (DPP, v_permlane16/32_swap) and its
    cross-wave scan of the block summaries must give exactly the bounds the
    definition gives: stats filter_candidates equals the count of the numpy
    restatement on the oracle's scores (700 k entries: 171 blocks, all 16
    scan waves busy), and the top-k equals the oracle's."""
    rng = np.random.default_rng(n + len(pattern))
    q = syn.protein_query(24, 5)
    lens = rng.integers(4, 20, n)
    if pattern == "rising":          # scores climb with the ID: most entries forwarded
        seqs = [np.concatenate([q[: 1 + (i * 23) // n], rng.choice(syn.AA_CODES, 3)]) for i in range(n)]
    elif pattern == "falling":       # best entries first: the bounds rise early
        seqs = [np.concatenate([q[: 1 + ((n - 1 - i) * 23) // n], rng.choice(syn.AA_CODES, 3)]) for i in range(n)]
    else:
        seqs = None
    if seqs is None:
        off = np.zeros(n + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        codes = rng.choice(syn.AA_CODES, int(off[-1])).astype(np.uint8)
    else:
        codes = np.concatenate(seqs).astype(np.uint8)
        off = np.zeros(n + 1, np.uint64)
        np.cumsum([len(s) for s in seqs], out=off[1:])
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    exp = po.scores(S.SW, q, codes, off, M, -11, -1)
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        ids = np.arange(n, dtype=np.uint64)
        try:
            # option filter_host: the result written into pinned host memory
            # by the last filter block (with a system-scope release, or with
            # system-scope stores) instead of the D2H copy -- incl. more
            # candidates than the pinned buffer holds ("rising"); the filter
            # as one launch (decoupled look-back, the default) and as three
            for one in (1, 0):
                S.set_option("filter_onepass", one)
                for fh in (0, 1, 2, 3):
                    S.set_option("filter_host", fh)
                    for k in (1, 10, 64):
                        got = [(h["score"], h["id"]) for h in S.sw_align(qq, k, 16)]
                        assert got == po.topk(exp, ids, k), (pattern, k, fh, one)
                        assert S.stats()["filter_candidates"] == _filter_candidates(exp, k), (pattern, k, fh, one)
            # the block scan at every list width (filter_prefix_r<16/32/64>,
            # k on both sides of 16 and 32) and the general scan; the
            # one-pass look-back's merges at every width
            S.set_option("filter_host", 0)
            for one, regs in ((0, 1), (0, 0), (1, 1)):
                S.set_option("filter_onepass", one)
                S.set_option("filter_prefix_regs", regs)
                for k in (1, 10, 16, 17, 32, 33, 64):
                    got = [(h["score"], h["id"]) for h in S.sw_align(qq, k, 16)]
                    assert got == po.topk(exp, ids, k), (pattern, k, regs, one)
                    assert S.stats()["filter_candidates"] == _filter_candidates(exp, k), (pattern, k, regs, one)
        finally:
            S.set_option("filter_host", 0)
            S.set_option("filter_prefix_regs", 1)
            S.set_option("filter_onepass", 1)
        S.free_sequence(qq)


@pytest.mark.parametrize("mode", ["both_strands", "trans_query"])
def test_multiview_device_filter_matches_full_scan(mode):
    """Multi-view searches (NUCLEOTIDE both strands: 2 query views;
    TRANS_QUERY both strands: 6 frames) run every view back to back and one
    device filter over all (view, entry) scores in the chunk-interleaved
    insertion order; it must equal the host scan of every score (no_filter),
    ties, overflow counters and insertion logs included."""
    rng = np.random.default_rng(3)
    if mode == "both_strands":
        q = syn.dna_query(120, 4)
        n = 20000
        # short reads, many exact repeats of query pieces: heavy ties on both strands
        seqs = [q[int(s):int(s) + 25].copy() if i % 3 else rng.choice(syn.NT_ACGT, 40).astype(np.uint8)
                for i, s in enumerate(rng.integers(0, 90, n))]
        codes = np.concatenate(seqs)
        off = np.zeros(n + 1, np.uint64)
        np.cumsum([len(c) for c in seqs], out=off[1:])
        S.set_output_mode(S.OUTPUT_ERROR)
        S.init_symbol_translation(S.NUCLEOTIDE, S.BOTH_STRANDS, 1, 1)
        S.init_constant_scores(2, -3)
        S.init_gap_penalties(-5, -2)
        qstr = syn.query_string(q, nucleotide=True)
        nucleotide = True
    else:
        q = syn.dna_query(150, 5)
        n = 15000
        seqs = [rng.choice(syn.AA_CODES, int(rng.integers(5, 120))).astype(np.uint8) for _ in range(n)]
        codes = np.concatenate(seqs)
        off = np.zeros(n + 1, np.uint64)
        np.cumsum([len(c) for c in seqs], out=off[1:])
        S.set_output_mode(S.OUTPUT_ERROR)
        S.init_symbol_translation(S.TRANS_QUERY, S.BOTH_STRANDS, 1, 1)
        S.init_score_matrix(S.MATRIX_BUILDIN, "blosum62")
        S.init_gap_penalties(-11, -1)
        qstr = syn.query_string(q, nucleotide=True)
        nucleotide = False
    try:
        for chunk in (1000, 37):
            S.set_chunk_size(chunk)
            with tempfile.TemporaryDirectory() as tmp:
                path = os.path.join(tmp, "db.fas")
                syn.write_fasta(path, codes, off, nucleotide=nucleotide)
                S.init_db(path)
                qq = S.init_sequence_fasta(S.READ_FROM_STRING, qstr)
                for algo, fn in ((S.SW, S.sw_align), (S.NW, S.nw_align)):
                    for k in (1, 10, 64):
                        for width in (8, 16):
                            S.set_option("no_filter", 1)
                            full = [(h["score"], h["id"]) for h in fn(qq, k, width)]
                            st_full = S.stats()
                            S.set_option("no_filter", 0)
                            got = [(h["score"], h["id"]) for h in fn(qq, k, width)]
                            st = S.stats()
                            assert got == full, (mode, chunk, algo, k, width, got[:4], full[:4])
                            assert (st["overflow_8"], st["overflow_16"]) == \
                                (st_full["overflow_8"], st_full["overflow_16"])
                    S.set_option("no_filter", 1)
                    log_full = S.search(qq, algo, 9, 16, S.LOG)
                    S.set_option("no_filter", 0)
                    assert S.search(qq, algo, 9, 16, S.LOG) == log_full
                    # the filter's bounds over the chunk-interleaved order (its
                    # d_order indirection): with k >= all (view, entry) pairs the
                    # insertion log is every score in insertion order
                    total = S.stats()["entries"] * len(S.query_views(qq))
                    order_sc = np.array([h[0] for h in S.search(qq, algo, total, 16, S.LOG, cap=total + 8)],
                                        np.int64)
                    assert len(order_sc) == total
                    for k in (1, 10, 64):
                        for one in (1, 0):            # the filter as one launch and as three
                            S.set_option("filter_onepass", one)
                            fn(qq, k, 16)
                            assert S.stats()["filter_candidates"] == _filter_candidates(order_sc, k), \
                                (mode, chunk, k, one)
                        S.set_option("filter_onepass", 1)
                S.free_sequence(qq)
    finally:
        S.set_option("no_filter", 0)
        S.set_option("filter_onepass", 1)
        S.set_chunk_size(1000)
        S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)


def test_packed_db_save_load_roundtrip(tmp_path):
    """ssa_amd_save_db / ssa_amd_load_db: a reloaded packed DB gives the same
    results as packing from the plugin (protein, and NUCLEOTIDE with both
    strands = two entries per record), and a file packed under other
    settings is refused."""
    q = syn.protein_query(120, 4)
    codes, off = syn.protein_db(5000, 8, query=q, plant_every=500, lo=1, hi=600)
    configure(False, ("builtin", "blosum62"), -11, -1)
    path = _write_db(str(tmp_path), codes, off)
    S.init_db(path)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    ref = {k: [(h["score"], h["id"]) for h in S.sw_align(qq, k, 16)] for k in (5, 100)}
    ref_nw = [(h["score"], h["id"]) for h in S.nw_align(qq, 50, 16)]
    pk = str(tmp_path / "db.ssapack")
    assert S.save_db(pk) == 0
    S.init_db(path)                 # new generation: would repack from the plugin
    assert S.load_db(pk) == 0
    for k in (5, 100):
        assert [(h["score"], h["id"]) for h in S.sw_align(qq, k, 16)] == ref[k]
    assert [(h["score"], h["id"]) for h in S.nw_align(qq, 50, 16)] == ref_nw
    S.free_sequence(qq)
    # refused: other symbol type
    S.init_symbol_translation(S.NUCLEOTIDE, S.BOTH_STRANDS, 1, 1)
    S.init_db(path)
    assert S.load_db(pk) != 0
    # NUCLEOTIDE both strands round trip
    seqs = po.read_fasta(os.path.join(DATA, "AF091148.fas"))[:400]
    configure(True, ("const", 2, -3), -5, -2, strands=S.BOTH_STRANDS)
    S.init_db(os.path.join(DATA, "AF091148.fas"))
    qn = S.init_sequence_fasta(S.READ_FROM_FILE, os.path.join(DATA, "one_seq.fas"))
    ref = [(h["score"], h["id"], h["db_strand"]) for h in S.sw_align(qn, 40, 16)]
    pk2 = str(tmp_path / "nt.ssapack")
    assert S.save_db(pk2) == 0
    S.init_db(os.path.join(DATA, "AF091148.fas"))
    assert S.load_db(pk2) == 0
    assert [(h["score"], h["id"], h["db_strand"]) for h in S.sw_align(qn, 40, 16)] == ref
    S.free_sequence(qn)
    del seqs
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)


@pytest.mark.parametrize("nslots", [2, 3])
def test_multi_device_slots_match_single_device(nslots):
    """ssa_amd_set_devices: the DB split over several device slots (here all
    on the one GPU of the box, which exercises the same split, per-slot
    packing, threads and log merge) returns exactly the single-device
    results -- protein (one view) and NUCLEOTIDE both strands (two views,
    chunk-interleaved insertion order)."""
    q = syn.protein_query(90, 12)
    codes, off = syn.protein_db(6000, 13, query=q, plant_every=700, lo=1, hi=500)
    with tempfile.TemporaryDirectory() as tmp:
        configure(False, ("builtin", "blosum62"), -11, -1, chunk=97)
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        runs = []
        for devs in ([], [0] * nslots):
            assert S.set_devices(devs) == 0
            runs.append([[(h["score"], h["id"]) for h in fn(qq, k, 16)]
                         for fn in (S.sw_align, S.nw_align) for k in (1, 10, 64, 500)]
                        + [S.search(qq, S.SW, 25, 16, S.LOG)])
        assert runs[0] == runs[1]
        S.free_sequence(qq)
        configure(True, ("const", 2, -3), -5, -2, chunk=37, strands=S.BOTH_STRANDS)
        S.init_db(os.path.join(DATA, "AF091148.fas"))
        qn = S.init_sequence_fasta(S.READ_FROM_FILE, os.path.join(DATA, "one_seq.fas"))
        runs = []
        for devs in ([], [0] * nslots):
            assert S.set_devices(devs) == 0
            runs.append([[(h["score"], h["id"], h["db_strand"]) for h in fn(qn, k, 16)]
                         for fn in (S.sw_align, S.nw_align) for k in (3, 50)])
        assert runs[0] == runs[1]
        S.free_sequence(qn)
    S.set_devices([])
    S.set_chunk_size(1000)
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_full_size_config_properties(cfg, tmp_path):
    """BASELINE.json sizes (1 M sequences; C2 SW q=400 BLOSUM62 -11/-1, C3 NW
    q=1000 BLOSUM50 -10/-2), checked through size-independent properties:
    the default f16 pair kernel and the independent int16 strip kernel agree
    on all 1 M scores; the oracle's int64 scores agree on a seeded sample of
    500 entries and on every top-100 hit; the top-k lists from the device
    filter equal a host replay of the full score vector."""
    algo, mname, go, ge, qlen = (S.SW, "blosum62", -11, -1, 400) if cfg == "c2" else (S.NW, "blosum50", -10, -2, 1000)
    q = syn.protein_query(qlen, 7)
    codes, off = syn.protein_db(1_000_000, 42, query=q, plant_every=10000, sampler="lut")
    configure(False, ("builtin", mname), go, ge)
    path = str(tmp_path / "big.fas")
    syn.write_fasta(path, codes, off)
    S.init_db(path)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    n = len(off) - 1
    vecs = {}
    for swk in (0, 1):
        S.set_option("sw_kernel", swk)
        log = S.search(qq, algo, n + 1, 16, S.LOG, cap=n + 8)
        assert len(log) == n
        vecs[swk] = np.array([h[0] for h in log], np.int64)
        assert S.stats()["kernel"] == (("pair_f16_" if swk == 0 else "strip16_") + ("sw" if algo == S.SW else "nw"))
    S.set_option("sw_kernel", 0)
    assert (vecs[0] == vecs[1]).all(), np.nonzero(vecs[0] != vecs[1])[0][:10]
    sc = vecs[0]
    M = TABLES["matrices"][NAMES.index(mname)].copy()
    rng = np.random.default_rng(99)
    top = np.argsort(-sc, kind="stable")[:100]
    sample = np.unique(np.concatenate([rng.choice(n, 500, replace=False), top]))
    seqs = [codes[int(off[i]):int(off[i + 1])] for i in sample]
    db, soff = po.pack_db(seqs)
    exp = po.scores(algo, q, db, soff, M, go, ge)
    assert (exp == sc[sample]).all()
    ids = np.arange(n, dtype=np.uint64)
    fn = S.sw_align if algo == S.SW else S.nw_align
    for k in (1, 10, 64):
        assert [(h["score"], h["id"]) for h in fn(qq, k, 16)] == po.topk(sc, ids, k)
    S.free_sequence(qq)


@pytest.mark.parametrize("cfg", ["c5", "ref"])
def test_other_config_properties(cfg, tmp_path):
    """The other bench shapes, scaled to a few seconds: C5 (DNA reads of 150
    nt, constant +5/-4, gaps -4/-2; a 2000-nt query instead of 10 k, 200 k
    reads instead of 50 M) and the reference's published benchmark shape
    (P18080, BLOSUM50, gaps -3/-1; 100 k synthetic sequences).  Same
    properties as above: default kernel == int16 strip kernel on every score,
    oracle int64 on a sample + the top hits, device top-k == host replay."""
    if cfg == "c5":
        algo, go, ge, nuc = S.SW, -4, -2, True
        q = syn.dna_query(2000, 8)
        codes, off = syn.dna_reads(200_000, 150, 43, query=q, plant_every=10000)
        configure(True, ("const", 5, -4), go, ge)
        M = po.matrix_constant(5, -4)
    else:
        algo, go, ge, nuc = S.SW, -3, -1, False
        text = open(os.path.join(DATA, "P18080.fasta")).read().split("\n")
        seq = "".join(l.strip() for l in text[1:] if not l.startswith(">")).upper()
        q = np.array([syn.AA_ORDER.index(c) for c in seq], dtype=np.uint8)
        codes, off = syn.protein_db(100_000, 44, query=q, plant_every=5000, sampler="lut")
        configure(False, ("builtin", "blosum50"), go, ge)
        M = TABLES["matrices"][NAMES.index("blosum50")].copy()
    path = str(tmp_path / "db.fas")
    syn.write_fasta(path, codes, off, nucleotide=nuc)
    S.init_db(path)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q, nucleotide=nuc))
    n = len(off) - 1
    vecs = {}
    for swk in (0, 1):
        S.set_option("sw_kernel", swk)
        log = S.search(qq, algo, n + 1, 16, S.LOG, cap=n + 8)
        assert len(log) == n
        vecs[swk] = np.array([h[0] for h in log], np.int64)
        if swk == 1:
            assert S.stats()["kernel"] == "strip16_sw"
        elif cfg == "c5":
            assert S.stats()["kernel"] == "pair_f16_sw"
    S.set_option("sw_kernel", 0)
    assert (vecs[0] == vecs[1]).all(), np.nonzero(vecs[0] != vecs[1])[0][:10]
    sc = vecs[0]
    rng = np.random.default_rng(98)
    top = np.argsort(-sc, kind="stable")[:50]
    sample = np.unique(np.concatenate([rng.choice(n, 300, replace=False), top]))
    seqs = [codes[int(off[i]):int(off[i + 1])] for i in sample]
    db, soff = po.pack_db(seqs)
    assert (po.scores(algo, q, db, soff, M, go, ge) == sc[sample]).all()
    ids = np.arange(n, dtype=np.uint64)
    for k in (1, 10, 64):
        assert [(h["score"], h["id"]) for h in S.sw_align(qq, k, 16)] == po.topk(sc, ids, k)
    S.free_sequence(qq)


def test_search_batch_matches_single_queries():
    """ssa_amd_search_batch returns each query's sw_align/nw_align result."""
    codes, off = syn.protein_db(3000, 21, lo=1, hi=500)
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qs = [S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(syn.protein_query(n, n)))
              for n in (5, 30, 64, 200, 401)]
        for algo, fn in ((S.SW, S.sw_align), (S.NW, S.nw_align)):
            for k in (1, 20, 100):
                assert S.search_batch(qs, algo, k) == [[(h["score"], h["id"]) for h in fn(q, k, 16)] for q in qs]
        for q in qs:
            S.free_sequence(q)


@pytest.mark.parametrize("upload", [1, 0])
def test_upload_kernel_new_query_every_search(upload):
    """Option upload_kernel: the per-search upload block (matrix, boundary,
    query) read from the pinned staging buffer by a kernel with system-scope
    loads.  The buffer is rewritten for every search, so consecutive searches
    with different queries, matrices and gaps must each see their own block."""
    codes, off = syn.protein_db(3000, 31, lo=1, hi=500)
    ids = np.arange(len(off) - 1, dtype=np.uint64)
    S.set_option("upload_kernel", upload)
    try:
        with tempfile.TemporaryDirectory() as tmp:
            for rnd, (mname, go, ge) in enumerate([("blosum62", -11, -1), ("blosum50", -10, -2), ("blosum62", -3, -1)]):
                configure(False, ("builtin", mname), go, ge)
                if rnd == 0:
                    S.init_db(_write_db(tmp, codes, off))
                M = TABLES["matrices"][NAMES.index(mname)].copy()
                for n in (40, 333, 100, 401):
                    q = syn.protein_query(n, 500 + n + rnd)
                    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
                    for algo, fn in ((S.SW, S.sw_align), (S.NW, S.nw_align)):
                        exp = po.scores(algo, q, codes, off, M, go, ge)
                        assert [(h["score"], h["id"]) for h in fn(qq, 10, 16)] == po.topk(exp, ids, 10), (upload, mname, n, algo)
                    S.free_sequence(qq)
    finally:
        S.set_option("upload_kernel", 1)


def test_search_batch_pipelined_sub_batches():
    """Batches beyond one pipelined sub-batch (16 queries), every k up to the
    device filter's 64, a lone last query, and overflowing queries (int64
    re-score inside a pipelined batch) -- each equal to its single search."""
    codes, off = syn.protein_db(4000, 22, lo=1, hi=700)
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        lens = (3, 17, 30, 48, 49, 96, 100, 150, 233, 400, 401, 7, 64, 300, 20, 55, 90)
        qs = [S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(syn.protein_query(n, 100 + n)))
              for n in lens]
        for algo, fn in ((S.SW, S.sw_align), (S.NW, S.nw_align)):
            for k in (1, 7, 64):
                for sub in (qs, qs[:9], qs[:2]):
                    exp = [[(h["score"], h["id"]) for h in fn(q, k, 16)] for q in sub]
                    t0 = S.stats()
                    assert S.search_batch(sub, algo, k) == exp, (algo, k, len(sub))
                    # the running totals count every query of the batch once
                    # (17 = one sub-batch plus a lone query through run_search)
                    t1 = S.stats()
                    assert t1["total_searches"] - t0["total_searches"] == len(sub), (algo, k, len(sub))
                    dk = t1["total_kernel_ms"] - t0["total_kernel_ms"]
                    assert abs(dk - t1["kernel_ms"]) <= 1e-6 * max(1.0, dk), (dk, t1["kernel_ms"])
                    assert t1["total_search_ms"] - t0["total_search_ms"] <= t1["search_ms"] + 1e-6
        for q in qs:
            S.free_sequence(q)
    # scores beyond the 16-bit range: re-scored by the int64 kernel per query
    configure(False, ("const", 127, -1), -1, -1)
    S.init_db(os.path.join(DATA, "NP_009305.1.fas"))
    qa = S.init_sequence_fasta(S.READ_FROM_FILE, os.path.join(DATA, "NP_009305.1.fas"))
    qb = S.init_sequence_fasta(S.READ_FROM_STRING, "MKTAYIAKQRQISFVKSHFSRQ")
    for algo, fn in ((S.SW, S.sw_align), (S.NW, S.nw_align)):
        exp = [[(h["score"], h["id"]) for h in fn(q, 1, 16)] for q in (qa, qb, qa)]
        assert exp[0] == [(67818, 0)]
        assert S.search_batch([qa, qb, qa], algo, 1) == exp
    S.free_sequence(qa)
    S.free_sequence(qb)


@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_search_batch_fused_launch(algo):
    """A sub-batch whose queries share one pair-kernel plan (strip heights and
    counts) is scored by ONE pair_kernel launch over all of them (stats
    kernel_launches = 1 per sub-batch): one-strip queries (no row buffer),
    multi-strip ones (a row buffer per query), with strip parts, with the
    longest group on long_kernel per query, k = 1..64.  Every query's result
    equals its own sw_align / nw_align and the unfused batch's."""
    rng = np.random.default_rng(31 + algo)
    codes, off = syn.protein_db(6000, 23 + algo, lo=1, hi=900)
    lens = np.diff(off).astype(np.int64)
    configure(False, ("builtin", "blosum62"), -11, -1)
    fn = S.sw_align if algo == S.SW else S.nw_align
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        try:
            for qlens, opts in (([30] * 8, {}), ([97, 104, 100, 99, 101, 98, 103, 102], {}),
                                ([97, 104, 100, 99, 101, 98, 103, 102], {"pair_parts": 2}),
                                ([97, 104, 100, 99, 101, 98, 103, 102], {"pair_parts": 3}),
                                ([30, 29, 31, 28, 27, 26, 30, 25], {"long_groups": 1}),
                                ([5] * 3, {})):
                qs = [S.init_sequence_fasta(S.READ_FROM_STRING,
                                            syn.query_string(syn.protein_query(n, int(rng.integers(1 << 30)))))
                      for n in qlens]
                for k, v in opts.items():
                    S.set_option(k, v)
                for k in (1, 10, 64):
                    exp, ncand = [], 0
                    for q in qs:
                        exp.append([(h["score"], h["id"]) for h in fn(q, k, 16)])
                        ncand += S.stats()["filter_candidates"]
                    S.set_option("batch_fuse", 0)
                    assert S.search_batch(qs, algo, k) == exp, (qlens, opts, k, "unfused")
                    assert S.stats()["kernel_launches"] == len(qs)
                    S.set_option("batch_fuse", 1)
                    got = S.search_batch(qs, algo, k)
                    assert got == exp, (qlens, opts, k)
                    # (the three-launch filter over the fused batch's queries)
                    S.set_option("filter_onepass", 0)
                    assert S.search_batch(qs, algo, k) == exp, (qlens, opts, k, "three-launch filter")
                    S.set_option("filter_onepass", 1)
                    # every query's own filter pass: the same candidates as alone
                    assert S.stats()["filter_candidates"] == ncand, (qlens, opts, k)
                    # NW with long_kernel groups and counters keeps one launch per query
                    unfusable = algo == S.NW and "long_groups" in opts
                    assert S.stats()["kernel_launches"] == (len(qs) if unfusable else 1), (qlens, opts)
                S.set_option("pair_parts", 0)
                S.set_option("long_groups", -1)
                for q in qs:
                    S.free_sequence(q)
        finally:
            S.set_option("batch_fuse", 1)
            S.set_option("pair_parts", 0)
            S.set_option("long_groups", -1)
            S.set_option("filter_onepass", 1)
    assert lens.max() > 0


CLI = os.path.join(os.path.dirname(po.__file__), "_ref", "libssa_example_amd")


@pytest.mark.skipif(not os.path.exists(CLI), reason="reference CLI not built (make -C oracle ref)")
@pytest.mark.parametrize("algo", ["SW", "NW"])
@pytest.mark.parametrize("bits", [8, 16, 64])
def test_reference_cli_links_and_matches(algo, bits):
    """The reference's own caller, src/libssa_example.c, compiled unchanged
    against include/libssa.h and linked to libssa_amd.so (oracle/Makefile),
    searches on the GPU and prints the reference's 64-bit top-300 list for
    the C1-style query (Q3ZAI3, BLOSUM62, gaps -11/-1, AF091148 as protein)."""
    import re
    import subprocess
    case = next(c for c in KATS if c["name"] == "config1_Q3ZAI3_k300")
    r = subprocess.run([CLI, "-N", "4", "-O", "-11", "-E", "-1", "-M", "BLOSUM62", "-i", os.path.join(DATA, "Q3ZAI3.fasta"),
                        "-d", os.path.join(DATA, case["db"]), "-c", "300", "-t", algo, "-b", str(bits), "-s", "AVX2"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Nr of alignments: 300" in r.stdout
    line = r.stdout.split("(Score, DB-ID), ")[1].splitlines()[0]
    got = [(int(a), int(b)) for a, b in re.findall(r"\((-?\d+), (\d+)\)", line)]
    assert got == [tuple(x) for x in case[algo.lower() + "_64"]]


def _cli(db, query, algo, bits, k, devices, threads=4):
    import subprocess
    env = dict(os.environ, SSA_AMD_DEVICES=devices)
    r = subprocess.run([CLI, "-N", str(threads), "-O", "-11", "-E", "-1", "-M", "BLOSUM62", "-i", query, "-d", db,
                        "-c", str(k), "-t", algo, "-b", str(bits), "-s", "AVX2"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, (devices, r.stderr[-2000:])
    return r.stdout


@pytest.mark.skipif(not os.path.exists(CLI), reason="reference CLI not built (make -C oracle ref)")
@pytest.mark.parametrize("algo", ["SW", "NW"])
def test_reference_cli_on_several_devices_via_env(algo, tmp_path):
    """An unchanged libssa caller on several GPUs: the reference's CLI
    (src/libssa_example.c, compiled unchanged) with SSA_AMD_DEVICES=0,0,0
    runs three device slots (here all on the box's one GPU: the same split,
    per-slot packing, persistent slot threads and log merge as on three
    GPUs) and prints exactly the single-device output -- every line but
    m_run's per-worker bookkeeping lines, of which the reference too prints
    one per worker thread (src/algo/manager.c:147-148).  Two DBs: AF091148
    (1403 records, 2 chunks of the CLI's 1000: one slot is empty) and 5000
    synthetic proteins (5 chunks)."""
    codes, off = syn.protein_db(5000, 71, lo=1, hi=900)
    big = _write_db(str(tmp_path), codes, off)
    query = os.path.join(DATA, "Q3ZAI3.fasta")
    for db, k in ((os.path.join(DATA, "AF091148.fas"), 300), (big, 500)):
        for bits in (8, 16):
            one = _cli(db, query, algo, bits, k, "current")
            three = _cli(db, query, algo, bits, k, "0,0,0")

            def split(out):
                book = [ln for ln in out.splitlines() if "Processed chunks" in ln]
                return [ln for ln in out.splitlines() if "Processed chunks" not in ln], book
            body1, book1 = split(one)
            body3, book3 = split(three)
            assert body1 == body3, (db, bits)
            assert f"Nr of alignments: {k}" in one
            assert len(book1) == 1 and len(book3) == 3, (book1, book3)
            seqs = [int(ln.rsplit(" ", 1)[1]) for ln in book3]
            assert sum(seqs) == int(book1[0].rsplit(" ", 1)[1]), (book1, book3)
    # the CLI's -N (set_thread_count, the reference's number of search
    # workers) caps the listed devices: -N 2 of 0,0,0 runs two slots
    two = _cli(big, query, algo, 16, 500, "0,0,0", threads=2)
    assert [ln for ln in two.splitlines() if "Processed chunks" not in ln] == \
        [ln for ln in _cli(big, query, algo, 16, 500, "current").splitlines() if "Processed chunks" not in ln]
    assert sum("Processed chunks" in ln for ln in two.splitlines()) == 2


BENCH_THREADS = os.path.join(os.path.dirname(po.__file__), "_ref", "benchmark_threads_amd")


@pytest.mark.skipif(not os.path.exists(BENCH_THREADS), reason="reference benchmark not built (make -C oracle ref)")
def test_reference_thread_sweep_becomes_device_slot_sweep(tmp_path):
    """The reference's own thread-sweep benchmark (benchmark/src/
    benchmark_threads.c + benchmark_util.c, compiled unchanged) on six listed
    device slots: its set_thread_count(2, 3, 5, 6, 0, 0) sweep runs 2, 3, 5,
    6, 6, 6 slots (0 = every listed device), each of its 360 searches (SW/NW x
    8/16/64 bit x 10) completes, and it logs its 36 timing rows to
    results/ as on the CPU.  Its DB and query paths are fixed
    (data/uniprot_sprot.fasta, data/P18080): a 20000-entry synthetic protein
    DB and the Q3ZAI3 query stand in (the reference's data/ files are not on
    the GPU box)."""
    import shutil
    import subprocess
    os.makedirs(tmp_path / "data")
    os.makedirs(tmp_path / "results")
    codes, off = syn.protein_db(20_000, 91, lo=8, hi=1200)
    syn.write_fasta(str(tmp_path / "data" / "uniprot_sprot.fasta"), codes, off, False)
    shutil.copy(os.path.join(DATA, "Q3ZAI3.fasta"), tmp_path / "data" / "P18080")
    env = dict(os.environ, SSA_AMD_DEVICES="0,0,0,0,0,0", SSA_AMD_TRACE="1")
    r = subprocess.run([BENCH_THREADS], cwd=str(tmp_path), capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [ln for ln in r.stdout.splitlines() if ln.startswith("P18080,")]
    assert len(rows) == 36, r.stdout[-2000:]
    expect = []
    for t in (2, 3, 5, 6, 0, 0):
        for algo in ("SW", "NW"):
            for b in (8, 16, 64):
                simd = "NO_SIMD" if b == 64 else "AVX2"
                expect.append(f"P18080,{simd},{algo},{b}_bit,{t}_t")
    assert [",".join(ln.split(",")[:5]) for ln in rows] == expect
    for ln in rows:
        times = [float(x) for x in ln.split(",")[5:]]
        assert len(times) == 10 and all(0.0 < x < 30.0 for x in times), ln
    slots = [int(ln.split(" on ")[1].split()[0]) for ln in r.stderr.splitlines()
             if ln.startswith("trace: run_search on ")]
    assert slots == [n for n in (2, 3, 5, 6, 6, 6) for _ in range(60)], slots[:80]
    logs = os.listdir(tmp_path / "results")
    assert len(logs) == 1 and logs[0].endswith("_threads")
    with open(tmp_path / "results" / logs[0]) as f:
        assert f.read().count("\n") == 36


@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_plan_cache_follows_scoring_and_options(algo, tmp_path):
    """The per-DB plan cache (engine.cpp cached_plan) reuses a plan only for
    the same query under unchanged settings: one query searched under
    BLOSUM62 -11/-1, then gaps -3/-1, then BLOSUM50, then an option change
    (strip height), then the first setting again -- every full score vector
    equals the oracle's for the setting in force."""
    rng = np.random.default_rng(41)
    lens = np.array([2600] + list(rng.integers(1, 500, 299)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    q = syn.protein_query(150, 77)
    codes[int(off[5]) + 2:int(off[5]) + 2 + 150] = q
    configure(False, ("builtin", "blosum62"), -11, -1)
    S.init_db(_write_db(str(tmp_path), codes, off))
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    steps = [("blosum62", -11, -1, None), ("blosum62", -3, -1, None), ("blosum50", -3, -1, None),
             ("blosum50", -3, -1, 16), ("blosum62", -11, -1, 0)]
    try:
        for name, go, ge, pnp in steps:
            S.init_score_matrix(S.MATRIX_BUILDIN, name)
            S.init_gap_penalties(go, ge)
            if pnp is not None:
                S.set_option("pair_np", pnp)
            exp = po.scores(algo, q, codes, off, TABLES["matrices"][NAMES.index(name)].copy(), go, ge)
            for _ in range(2):                   # the second search takes the cached plan
                sc, ids = _full_scores(qq, algo, len(lens))
                assert (ids == np.arange(len(lens))).all()
                assert (sc == exp).all(), (name, go, ge, pnp, np.nonzero(sc != exp)[0][:10])
            if pnp == 16 and S.stats()["kernel"].startswith("pair"):
                assert S.stats()["strip_rows"] == 32
    finally:
        S.set_option("pair_np", 0)


def test_ssa_exit_releases_device_memory(tmp_path):
    """ssa_exit (libssa.c:266-271 frees the reference's state and ends its
    thread pool) also releases the device copies of the DB -- what bench.py's
    drop_in record relies on before its child packs the north-star DB."""
    import torch
    codes, off = syn.protein_db(200_000, 77, lo=16, hi=2000)
    configure(False, ("builtin", "blosum62"), -11, -1)
    S.init_db(_write_db(str(tmp_path), codes, off))
    free0 = torch.cuda.mem_get_info(0)[0]
    S.prepare_db()
    free1 = torch.cuda.mem_get_info(0)[0]
    S.ssa_exit()
    free2 = torch.cuda.mem_get_info(0)[0]
    packed = free0 - free1
    assert packed > int(off[-1]) * 4, (free0, free1)          # row buffer alone: 4 B per residue slot
    # (the runtime may keep part of what was freed for its own reuse)
    assert free2 - free1 > 0.5 * packed, (free0, free1, free2)
    # packing the same DB again takes no more than the first time: nothing leaked
    configure(False, ("builtin", "blosum62"), -11, -1)
    S.init_db(_write_db(str(tmp_path), codes, off))
    S.prepare_db()
    free3 = torch.cuda.mem_get_info(0)[0]
    assert free3 > free1 - 0.05 * packed, (free0, free1, free2, free3)
    S.ssa_exit()
    # the library works again after it
    configure(False, ("builtin", "blosum62"), -11, -1)
    S.init_db(_write_db(str(tmp_path), codes[:int(off[1000])], off[:1001]))
    q = syn.protein_query(50, 3)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    exp = po.scores(S.SW, q, codes[:int(off[1000])], off[:1001], M, -11, -1)
    assert [(h["score"], h["id"]) for h in S.sw_align(qq, 5, 16)] == po.topk(exp, np.arange(1000, dtype=np.uint64), 5)
    S.free_sequence(qq)


def test_device_env_selects_slots(tmp_path):
    """SSA_AMD_DEVICES, read at the first init_db unless the caller chose
    devices: all / unset / empty = every visible device, current = the
    current one, a list (repeats allowed), invalid lists fall back to the
    current device with an error; set_thread_count(n) caps the list at its
    first n; an explicit ssa_amd_set_device(s) wins over both."""
    import subprocess
    import sys
    db = os.path.join(DATA, "test.fas")
    prog = ("import sys; sys.path.insert(0, %r); import libssa_amd as S; S.load(); "
            "S.set_output_mode(S.OUTPUT_ERROR); " % ROOT)
    n = S.device_count()

    def devs(env, pre=""):
        e = dict(os.environ)
        e.pop("SSA_AMD_DEVICES", None)
        if env is not None:
            e["SSA_AMD_DEVICES"] = env
        r = subprocess.run([sys.executable, "-c", prog + pre + f"S.init_db({db!r}); print(S.get_devices())"],
                           capture_output=True, text=True, timeout=300, env=e)
        assert r.returncode == 0, r.stderr[-2000:]
        return eval(r.stdout.strip().splitlines()[-1]), r.stdout
    allv = list(range(n)) if n > 1 else [0]
    assert devs(None)[0] == allv
    assert devs("")[0] == allv
    assert devs("all")[0] == allv
    assert devs("current")[0] == [0]
    assert devs("0,0,0")[0] == [0, 0, 0]
    assert devs("0")[0] == [0]
    for bad in ("0,99", "x", "0;1", "-1"):
        got, out = devs(bad)
        assert got == [0] and "SSA_AMD_DEVICES" in out, (bad, got, out)
    assert devs("0,0", pre="S.set_device(0); ")[0] == [0]
    assert devs("current", pre="S.set_devices([0, 0]); ")[0] == [0, 0]
    # set_thread_count caps the listed devices, before or after init_db
    assert devs("0,0,0", pre="S.set_thread_count(2); ")[0] == [0, 0]
    assert devs("0,0,0", pre="S.set_thread_count(1); ")[0] == [0]
    assert devs("0,0,0", pre="S.set_thread_count(7); ")[0] == [0, 0, 0]
    got, _ = devs("0,0,0", pre="S.set_thread_count(2); S.init_db(%r); S.set_thread_count(0); " % db)
    assert got == [0, 0, 0]
    # ... but never an explicit choice
    assert devs("0,0,0", pre="S.set_devices([0, 0, 0, 0]); S.set_thread_count(2); ")[0] == [0, 0, 0, 0]


@pytest.mark.parametrize("gaps", [(0, 0), (-5, 0), (0, -1), (-1, -3), (-20, -7)])
@pytest.mark.parametrize("algo", [S.SW, S.NW])
def test_gap_penalty_edges_vs_oracle(gaps, algo):
    """Zero gap-open/extension and steep gaps: the diagonal-relative frame's
    offsets and floors (|R| = 0 makes every floor equal) stay exact."""
    rng = np.random.default_rng(5)
    q = syn.protein_query(57, 11)
    lens = np.array([0, 1, 5, 17, 48, 49, 130] + list(rng.integers(1, 200, 150)), dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    keep = np.nonzero(lens > 0)[0]
    exp = po.scores(algo, q, codes, off, M, gaps[0], gaps[1])[keep]
    configure(False, ("builtin", "blosum62"), gaps[0], gaps[1])
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        for pnp in (16, 24, 32, 36, 40, 0):
            S.set_option("pair_np", pnp)
            sc, ids = _full_scores(qq, algo, len(keep))
            assert (sc == exp).all(), (pnp, np.nonzero(sc != exp)[0][:10])
        S.set_option("pair_np", 0)
        S.free_sequence(qq)


# ------------------------------------------------ full-size reference pins
FULL = json.load(open(os.path.join(GOLDEN, "fullsize.json")))


def _fullsize_inputs(c):
    """The FULLSIZE DBs of tools/gen_golden.py, regenerated from the same
    block-seeded generators (a share = the first IDs of the whole DB)."""
    if c["kind"] == "dna":
        q = syn.dna_query(c["qlen"], c["qseed"])
        codes, off = syn.dna_reads_range(c["n"], c["seed"], 0, c["i1"], 150, query=q)
        return q, codes, off
    q = _fullsize_query(c)
    codes, off = syn.protein_db_range(c["n"], c["seed"], 0, c["i1"], query=q, alphabet=c.get("alphabet", "bg20"),
                                      lengths=c.get("lengths", "gamma"), lo=c.get("lo", 16), hi=c.get("hi", 4096))
    if c.get("tail"):
        # a UniProt-like length tail (the "sprot" fixture: bench.py --config sprot)
        codes, off = syn.with_long_tail(codes, off, c["tail"], c["tail_seed"], c.get("alphabet", "bg20"))
    return q, codes, off


def _fullsize_query(c):
    if c.get("query_file"):
        lines = open(os.path.join(ROOT, c["query_file"])).read().split("\n")
        seq = "".join(x.strip() for x in lines[1:] if not x.startswith(">")).upper()
        return np.array([syn.AA_ORDER.index(ch) for ch in seq], dtype=np.uint8)
    return syn.protein_query(c["qlen"], c["qseed"])


# fixtures pinned by top-k and counters only (the GPU test does not pull their
# multi-million-entry logs through Python)
LARGE = ("c4full", "c5share8", "c5full")


@pytest.mark.parametrize("name", sorted(k for k in FULL if k not in LARGE and not k.startswith("c2x")))
def test_fullsize_matches_reference_hash(name, tmp_path):
    """BASELINE.json's configurations at full size (C2, C3: 1 M sequences) or
    one GPU's share (C4: the first 1.25 M of the 10 M DB at width 8; C5: the
    first 1 M of the 50 M reads, q = 10 000 nt), plus 25- and 28-symbol
    alphabets: the SHA-256 of the full int64 score vector in ID order, the
    score histogram, the top-1/10/64 and m_run's overflow counters equal the
    reference's own 16/8-bit AVX2 search of the same DB
    (tests/golden/fullsize.json, tools/gen_golden.py fullsize)."""
    c = FULL[name]
    q, codes, off = _fullsize_inputs(c)
    n = len(off) - 1
    dna = c["kind"] == "dna"
    if c["matrix"].startswith("const"):
        a, b = c["matrix"][5:].split("_")
        spec = ("const", int(a), int(b))
    else:
        spec = ("builtin", c["matrix"])
    configure(dna, spec, c["gap_open"], c["gap_extend"])
    path = os.path.join(str(tmp_path), "db.fas")
    syn.write_fasta(path, codes, off, dna)
    del codes
    S.init_db(path)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q, nucleotide=dna))
    algo = S.SW if c["algo"] == "sw" else S.NW
    # k = n: every entry is inserted, so the log is the full score vector
    log = S.search(qq, algo, n, c["width"], S.LOG, cap=n + 8)
    st = S.stats()
    assert [st["overflow_8"], st["overflow_16"]] == c["overflow"]
    assert len(log) == n
    arr = np.array([(h[1], h[0]) for h in log], dtype=np.int64)
    arr = arr[np.argsort(arr[:, 0], kind="stable")]
    assert (arr[:, 0] == np.arange(n)).all()
    sc = arr[:, 1]
    vals, counts = np.unique(sc, return_counts=True)
    assert vals.tolist() == c["hist_values"] and counts.tolist() == c["hist_counts"]
    assert hashlib.sha256(sc.astype("<i8").tobytes()).hexdigest() == c["sha256"]
    fn = S.sw_align if algo == S.SW else S.nw_align
    for k in (1, 10, 64):
        got = [[h["score"], h["id"]] for h in fn(qq, k, c["width"])]
        assert got == c[f"top{k}"], k
        st = S.stats()
        assert [st["overflow_8"], st["overflow_16"]] == c["overflow"], k
    # without the counters (the benchmark's OUTPUT_ERROR), with the rare-code
    # merge allowed (it runs on Swiss-Prot's 25 symbols) -- same top-k
    S.set_option("counters", 0)
    S.set_option("rare_merge", 1)
    try:
        for k in (1, 10, 64):
            got = [[h["score"], h["id"]] for h in fn(qq, k, c["width"])]
            assert got == c[f"top{k}"], ("no counters", k)
            if c.get("alphabet") == "sprot25" and c["algo"] == "sw":
                assert S.stats()["rare_merged"] > 0
    finally:
        S.set_option("counters", 1)
        S.set_option("rare_merge", 0)
    S.free_sequence(qq)


REF64 = json.load(open(os.path.join(GOLDEN, "ref64.json")))


@pytest.mark.parametrize("name", sorted(REF64))
def test_tie_band_matches_reference_search64(name, tmp_path):
    """The tie band at scale, pinned by the reference's OWN 64-bit search:
    tests/golden/ref64.json holds the top-64 of the reference's one-thread
    search_64 (src/algo/64/search_64.c:44-79 -> minheap_add,
    src/util/minheap.c:50-91; tools/gen_golden.py ref64) on tie-heavy DBs --
    the 28-symbol SW and NW fixtures, the 25-symbol one and the first 100 k
    reads of C5's DB (q = 10 000 nt) -- whose 64th score lies inside a band
    of equal scores.  sw_align / nw_align's top-64 (score and ID) equals that
    list, at API widths 16 and 8."""
    c = REF64[name]
    q, codes, off = _fullsize_inputs(c)
    assert len(off) - 1 == c["nonempty"] and int(off[-1]) == c["residues"]
    dna = c["kind"] == "dna"
    if c["matrix"].startswith("const"):
        a, b = c["matrix"][5:].split("_")
        spec = ("const", int(a), int(b))
    else:
        spec = ("builtin", c["matrix"])
    configure(dna, spec, c["gap_open"], c["gap_extend"])
    path = os.path.join(str(tmp_path), "db.fas")
    syn.write_fasta(path, codes, off, dna)
    del codes
    S.init_db(path)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q, nucleotide=dna))
    fn = S.sw_align if c["algo"] == "sw" else S.nw_align
    top = c["top64"]
    assert top[-1][0] == top[-2][0], "the fixture's 64th score is inside a tie band"
    for width in (16, 8):
        for counters in (1, 0):      # (0, with option rare_merge: the merge may run, sp25)
            S.set_option("counters", counters)
            S.set_option("rare_merge", 1 - counters)
            got = [[h["score"], h["id"]] for h in fn(qq, 64, width)]
            assert got == top, (width, counters, [x for x in zip(got, top) if x[0] != x[1]][:5])
    S.set_option("counters", 1)
    S.set_option("rare_merge", 0)
    S.free_sequence(qq)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", [k for k in LARGE if k in FULL])
def test_large_db_matches_reference(name, tmp_path):
    """BASELINE.json's largest single-GPU workloads at their stated size: C4's
    whole 10 M-sequence DB (3.5e9 residues) at API width 8, C5's whole 50 M
    reads (7.5e9 residues, q = 10 000 nt: 7.5e13 cells per search) and one
    GPU's share of C5 at N = 8 (the first 6.25 M reads):
    sw_align's top-1/10/64 and m_run's overflow counters equal the
    reference's own AVX2 search of the same DB (tests/golden/fullsize.json;
    the full score vectors' hashes are pinned on the 1.25 M / 1 M shares)."""
    c = FULL[name]
    q, codes, off = _fullsize_inputs(c)
    assert len(off) - 1 == c["nonempty"] and int(off[-1]) == c["residues"]
    dna = c["kind"] == "dna"
    if c["matrix"].startswith("const"):
        a, b = c["matrix"][5:].split("_")
        spec = ("const", int(a), int(b))
    else:
        spec = ("builtin", c["matrix"])
    configure(dna, spec, c["gap_open"], c["gap_extend"])
    path = os.path.join(str(tmp_path), "db.fas")
    syn.write_fasta(path, codes, off, dna)
    del codes, off
    S.init_db(path)
    os.remove(path)
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q, nucleotide=dna))
    for k in (1, 10, 64):
        got = [[h["score"], h["id"]] for h in S.sw_align(qq, k, c["width"])]
        assert got == c[f"top{k}"], k
        st = S.stats()
        assert [st["overflow_8"], st["overflow_16"]] == c["overflow"], k
    S.free_sequence(qq)


@pytest.mark.parametrize("name,world,balanced", [("c2x2", 2, False), ("c2x2", 3, True), ("c4full", 4, True)])
def test_sharded_db_logs_merge_to_reference_topk(name, world, balanced, tmp_path):
    """bench.py's multi-GPU path at full size, on one GPU: a fixture's DB
    searched as `world` contiguous ID shards (each packed with its global ID
    offset, ssa_amd_set_id_offset), their insertion logs merged by the native
    shard merge (ssa_amd_merge_logs, what ssa_amd_gather_logs runs on rank 0):
    top-1/10/64 equal the reference's own search of the whole DB
    (tests/golden/fullsize.json).  C2's 2 M-sequence weak-scaling DB cut by
    count (bench.py's weak shards at N = 2) and by residues into 3; C4's
    whole 10 M DB cut by residues into 4 (ssa_amd_shard_bounds, bench.py's
    strong shards at N = 4)."""
    c = FULL[name]
    q = _fullsize_query(c)
    configure(False, ("builtin", c["matrix"]), c["gap_open"], c["gap_extend"])
    if balanced:
        lens = syn.protein_lengths_range(c["n"], c["seed"], 0, c["i1"], query=q)
        cuts = S.shard_bounds(lens, world)
        res = [int(lens[a:b].sum()) for a, b in zip(cuts, cuts[1:])]
        assert max(res) / min(res) <= 1.01
        del lens
    else:
        cuts = [r * c["i1"] // world for r in range(world + 1)]
    logs = []
    try:
        for r in range(world):
            i0, i1 = cuts[r], cuts[r + 1]
            codes, off = syn.protein_db_range(c["n"], c["seed"], i0, i1, query=q, alphabet=c.get("alphabet", "bg20"),
                                              lo=16, hi=4096)
            path = os.path.join(str(tmp_path), f"db{r}.fas")
            syn.write_fasta(path, codes, off, False)
            del codes, off
            S.init_db(path)
            S.set_id_offset(i0)
            S.prepare_db()
            os.remove(path)
            qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
            logs.append(S.search(qq, S.SW, 64, c["width"], S.LOG))
            S.free_sequence(qq)
    finally:
        S.set_id_offset(0)
    for k in (1, 10, 64):
        got = [[int(a), int(b)] for a, b in S.merge_logs([[h for h in L] for L in logs], k)]
        assert got == c[f"top{k}"], k


def _gather_from_threads(logs, k, group):
    """ssa_amd_gather_logs from len(logs) host threads, each one rank of the
    library's in-process transport (ssa_amd_dist_init_fake: the slot layout,
    count rows and exact-size round of the RCCL path); rank 0's result."""
    import threading
    world = len(logs)
    res, errs = [None] * world, []

    def run(r):
        try:
            S.dist_init_fake(r, world, group)
            try:
                res[r] = S.gather_logs(logs[r], k)
            finally:
                S.dist_finalize()
        except Exception as e:  # reported below
            errs.append(repr(e))
    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    assert all(x == [] for x in res[1:])
    return [[int(a), int(b)] for a, b in res[0]]


@pytest.mark.parametrize("config,world,fixture", [("c2", 4, "c2x4"), ("c2", 8, "c2x8"), ("north_star", 8, "c4full")])
def test_driver_cuts_gather_to_reference_topk(config, world, fixture, tmp_path):
    """Exactly what the driver's `bench.py --gpus N` searches, on one GPU:
    the workload cut into N rank slices by libssa_amd/workloads.py (the cut
    bench.py imports: C2's weak-scaling N M-sequence DB, and the north-star
    10 M-sequence DB, both residue-balanced), each slice packed with its
    global ID offset and searched at API width 16, and the real shard logs
    gathered by ssa_amd_gather_logs from N threads over the in-process
    transport: rank 0's top-1/10/64 equal the reference's own search of the
    whole DB (tests/golden/fullsize.json; reference: the thread heaps merged
    in thread order, src/algo/manager.c:141-145)."""
    from libssa_amd import workloads as W
    cfg = W.CONFIGS[config]
    fx = FULL[fixture]
    q = W.query(cfg)
    bounds, total, job = W.cuts(cfg, world, q)
    assert (total, job) == (fx["n"], fx["i1"])
    configure(False, ("builtin", cfg["matrix"]), cfg["gap_open"], cfg["gap_extend"])
    logs = []
    try:
        for r in range(world):
            codes, off = W.slice_db(cfg, q, total, bounds[r], bounds[r + 1])
            path = os.path.join(str(tmp_path), f"db{r}.fas")
            syn.write_fasta(path, codes, off, False)
            del codes, off
            S.init_db(path)
            S.set_id_offset(bounds[r])
            S.prepare_db()
            os.remove(path)
            qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
            logs.append(S.search(qq, S.SW, 64, 16, S.LOG))
            S.free_sequence(qq)
    finally:
        S.set_id_offset(0)
    for k in (1, 10, 64):
        assert _gather_from_threads(logs, k, group=7000 + 10 * world + k) == fx[f"top{k}"], k


@pytest.mark.parametrize("gaps", [(-11, 2), (3, -1)])
def test_every_lane_rescored_exactly(gaps, tmp_path):
    """SW with a positive gap increment sends every lane to the exact int64
    kernel (no cap on the overflow list: more entries than the pinned
    mirror holds); scores and top-k equal the oracle's full_sw, which runs
    the reference recurrence with the same penalties."""
    q = syn.protein_query(60, 11)
    codes, off = syn.protein_db(6000, 9, query=q, plant_every=700, lo=5, hi=120)
    configure(False, ("builtin", "blosum62"), gaps[0], gaps[1])
    S.init_db(_write_db(str(tmp_path), codes, off))
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    exp = po.scores(0, q, codes, off, M, gaps[0], gaps[1])
    got, ids = _full_scores(qq, S.SW, len(off) - 1)
    assert (got == exp).all()
    seqs = [codes[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    assert [(h["score"], h["id"]) for h in S.sw_align(qq, 20, 16)] == po.search(0, q, seqs, M, gaps[0], gaps[1], 20)
    assert S.stats()["wide_count"] == len(off) - 1
    S.free_sequence(qq)


def test_residue_classes_follow_the_query(tmp_path):
    """28-symbol DB (the reference generator's alphabet): per-query residue
    classes (codes whose matrix rows agree on the query's residues share one
    code on the device) change with the query -- a standard-residue query, one
    holding X and '*', one holding U and O -- and every full score vector and
    top-k equals the oracle's, SW and NW, queries alternating so the cached
    class-coded residues are rebuilt and reused."""
    codes, off = syn.protein_db_range(20000, 5, alphabet="uniform28", lengths="uniform", lo=16, hi=600)
    configure(False, ("builtin", "blosum62"), -11, -1)
    S.init_db(_write_db(str(tmp_path), codes, off))
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    base = syn.protein_query(300, 3)
    qs = [base.copy(), base.copy(), base.copy()]
    qs[1][::17] = syn.AA_ORDER.index("X")
    qs[1][5::23] = syn.AA_ORDER.index("*")
    qs[2][::19] = syn.AA_ORDER.index("U")
    qs[2][7::29] = syn.AA_ORDER.index("O")
    seqs = [codes[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    for q in qs + qs[::-1]:
        qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
        for algo in (S.SW, S.NW):
            got, _ = _full_scores(qq, algo, len(off) - 1)
            assert (got == po.scores(algo, q, codes, off, M, -11, -1)).all(), algo
            fn = S.sw_align if algo == S.SW else S.nw_align
            assert [(h["score"], h["id"]) for h in fn(qq, 10, 16)] == po.search(algo, q, seqs, M, -11, -1, 10)
            assert S.stats()["kernel"].startswith("pair"), S.stats()["kernel"]
        S.free_sequence(qq)


@pytest.mark.parametrize("qlen", [50, 300, 700])
@pytest.mark.parametrize("waves", [0, 1])
def test_overflow_counters_long_nw_entries(qlen, waves, tmp_path):
    """NW with -10/-2 gaps: entries of 15-20 k residues cross the 16-bit flag
    threshold along the top boundary (the device replays those row by row and
    stops in the first row), shorter ones are decided from bounds or replayed
    column by column; widths 8 and 16 against the oracle's column-major
    replay of the reference's saturated kernels."""
    rng = np.random.default_rng(qlen)
    q = syn.protein_query(qlen, 5)
    lens = [10, 60, 61, 200, 1000, 15000, 16300, 16390, 16400, 17000, 20000] + list(rng.integers(1, 3000, 30))
    seqs = [rng.choice(syn.AA_CODES, int(n)).astype(np.uint8) for n in lens]
    db, off = po.pack_db(seqs)
    configure(False, ("builtin", "blosum62"), -10, -2)
    S.init_db(_write_db(str(tmp_path), db, off))
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    flags = po.overflow_flags(1, q, db, off, M, -10, -2)
    exp_hits = po.search(1, q, seqs, M, -10, -2, 5)
    S.set_option("long_waves", waves)
    try:
        for width in (S.BIT_WIDTH_8, S.BIT_WIDTH_16):
            assert [(h["score"], h["id"]) for h in S.nw_align(qq, 5, width)] == exp_hits
            st = S.stats()
            o8, o16 = po.overflow_counts(width, flags)
            assert (st["overflow_8"], st["overflow_16"]) == (o8 if width == 8 else 0, o16), width
    finally:
        S.set_option("long_waves", 0)
    S.free_sequence(qq)


@pytest.mark.parametrize("waves", [0, 1])
def test_overflow_counters_nw_matrix_maximum(waves, tmp_path):
    """NW whose matrix maximum reaches the 16-bit ceiling: a 2000-residue query
    with constant scores +20/-5 against copies of itself (identity 60-100 %,
    trimmed and extended) and random entries; the 16-bit flag then turns on
    H == I_MAX somewhere inside the matrix, which the device takes from the
    long kernel's exact extremes (the pair kernel's lanes cannot reach it);
    widths 8 and 16 against the oracle's replays."""
    rng = np.random.default_rng(77)
    q = syn.protein_query(2000, 9)
    seqs = []
    for i in range(120):
        if i % 6 == 0:
            x = q.copy()
            mut = rng.random(len(x)) < rng.uniform(0.0, 0.4)
            x[mut] = rng.choice(syn.AA_CODES, int(mut.sum()))
            a, b = int(rng.integers(0, 300)), int(rng.integers(1700, 2001))
            x = np.concatenate([x[a:b], rng.choice(syn.AA_CODES, int(rng.integers(0, 800)))]).astype(np.uint8)
            seqs.append(x)
        else:
            seqs.append(rng.choice(syn.AA_CODES, int(rng.integers(10, 3000))).astype(np.uint8))
    db, off = po.pack_db(seqs)
    configure(False, ("const", 20, -5), -10, -2)
    S.init_db(_write_db(str(tmp_path), db, off))
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    M = po.matrix_constant(20, -5)
    flags = po.overflow_flags(1, q, db, off, M, -10, -2)
    assert ((flags >> 1) & 1).sum() > 0                # the 16-bit flag occurs
    exp_hits = po.search(1, q, seqs, M, -10, -2, 5)
    S.set_option("long_waves", waves)
    try:
        for width in (S.BIT_WIDTH_8, S.BIT_WIDTH_16):
            assert [(h["score"], h["id"]) for h in S.nw_align(qq, 5, width)] == exp_hits
            st = S.stats()
            o8, o16 = po.overflow_counts(width, flags)
            assert (st["overflow_8"], st["overflow_16"]) == (o8 if width == 8 else 0, o16), width
    finally:
        S.set_option("long_waves", 0)
    S.free_sequence(qq)


@pytest.mark.gpu
def test_pair_row_stream_follows_the_plan():
    """The pair kernel's per-column pair-row offsets (pair_addr_kernel) are
    cached per DB and rebuilt when the table they address changes: row width
    (48-, 32- and 80-row strips, tail-only queries at their own width) and
    the per-query class map (queries with X / U, O on a 28-symbol DB).
    Queries alternate back and forth so every rebuild is followed by reuse;
    every full score vector equals the oracle's, SW and NW."""
    codes, off = syn.protein_db_range(6000, 9, alphabet="uniform28", lengths="uniform", lo=1, hi=500)
    configure(False, ("builtin", "blosum62"), -11, -1)
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    qs = []
    for m, seed in ((400, 1), (20, 2), (60, 3), (130, 4), (7, 5)):
        qs.append(syn.protein_query(m, seed))
    qx = syn.protein_query(300, 6)
    qx[::13] = syn.AA_ORDER.index("X")
    qu = syn.protein_query(45, 7)
    qu[::5] = syn.AA_ORDER.index("U")
    qu[2::7] = syn.AA_ORDER.index("O")
    order = [qs[0], qs[1], qx, qs[2], qu, qs[0], qs[3], qs[4], qx, qs[1], qu, qs[3]]
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        n = len(off) - 1
        keep = np.nonzero(np.diff(off.astype(np.int64)) > 0)[0]
        for i, q in enumerate(order):
            qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
            for algo in (S.SW, S.NW):
                exp = po.scores(algo, q, codes, off, M, -11, -1)
                sc, ids = _full_scores(qq, algo, len(keep))
                assert (ids == keep).all(), (i, algo)
                assert (sc == exp[keep]).all(), (i, algo, len(q), np.nonzero(sc != exp[keep])[0][:10])
                assert S.stats()["kernel"].startswith("pair"), S.stats()["kernel"]
            S.free_sequence(qq)
        assert n == len(off) - 1


@pytest.mark.gpu
def test_short_sw_queries_take_32_row_strips():
    """Short SW queries whose rows fill 32-row strips better (q <= 32 and
    48 < q <= 64) run the pair kernel's 32-row strips at four waves per SIMD
    (engine.cpp pair_strip_np); every score stays the oracle's, and the other
    lengths keep 48-row strips; NW queries of up to 48 rows take 48-row
    strips instead of 80-row ones."""
    rng = np.random.default_rng(11)
    lens = np.array(list(rng.integers(1, 700, 3000)) + [0, 1, 15, 16, 17], dtype=np.int64)
    off = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = rng.choice(syn.AA_CODES, size=int(off[-1])).astype(np.uint8)
    keep = np.nonzero(lens > 0)[0]
    M = TABLES["matrices"][NAMES.index("blosum62")].copy()
    configure(False, ("builtin", "blosum62"), -11, -1)
    with tempfile.TemporaryDirectory() as tmp:
        S.init_db(_write_db(tmp, codes, off))
        for m, rows in ((1, 32), (17, 32), (30, 32), (32, 32), (33, 48), (48, 48), (49, 32), (64, 32), (65, 48)):
            q = syn.protein_query(m, 100 + m)
            exp = po.scores(S.SW, q, codes, off, M, -11, -1)
            qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
            sc, ids = _full_scores(qq, S.SW, len(keep))
            assert (ids == keep).all(), m
            assert (sc == exp[keep]).all(), (m, np.nonzero(sc != exp[keep])[0][:10])
            assert S.stats()["strip_rows"] == rows, m
            if m in (30, 48, 49, 65):
                # NW: 48-row strips up to 48 query rows, then 80-row ones
                exp_nw = po.scores(S.NW, q, codes, off, M, -11, -1)
                sc, ids = _full_scores(qq, S.NW, len(keep))
                assert (sc == exp_nw[keep]).all(), (m, np.nonzero(sc != exp_nw[keep])[0][:10])
                assert S.stats()["strip_rows"] == (48 if m <= 48 else 80), m
            S.free_sequence(qq)



@pytest.mark.parametrize("algo,gaps,matrix", [(S.SW, (-11, -1), "blosum62"), (S.SW, (-3, -1), "blosum50"),
                                              (S.NW, (-10, -2), "blosum50")])
def test_rare_code_merge_exact(algo, gaps, matrix, tmp_path):
    """Swiss-Prot's rare letters (X, B, Z, U, O) in ~8 % of the entries: the
    query's residue classes leave a 25-code pair table (two workgroups per
    CU), so the rarest classes are scored through ONE upper-bound class (the
    maximum of their rows) and every forwarded entry holding one is
    re-scored exactly (engine.cpp plan_view, option rare_merge).  Near-copies
    of the query carry rare letters, so upper bounds reach the top-k and the
    exact re-score decides it: sw_align / nw_align's top-1/10/64 equal the
    oracle's (the reference's 64-bit search order), with the merge on and
    off, and the merge reports what it merged and re-scored."""
    rng = np.random.default_rng(71 + algo)
    q = syn.protein_query(300, 13)
    codes, off = syn.protein_db_range(30000, 91, alphabet="bg20", lengths="uniform", lo=16, hi=700, query=q,
                                      plant_every=700)
    codes = codes.copy()
    rare = np.array([syn.AA_ORDER.index(c) for c in "XBZUO"], np.uint8)
    lens = np.diff(off).astype(np.int64)
    n = len(lens)
    # ~8 % of the entries get 1-3 rare letters; every planted homolog too
    # (the merge declines when more than a quarter of the entries hold one)
    hit = rng.random(n) < 0.08
    hit[np.arange(350, n, 700)] = True
    for i in np.nonzero(hit)[0]:
        for _ in range(int(rng.integers(1, 4))):
            codes[int(off[i]) + int(rng.integers(0, lens[i]))] = rare[int(rng.integers(0, 5))]
    M = TABLES["matrices"][NAMES.index(matrix)].copy()
    keep = np.nonzero(lens > 0)[0]
    exp_sc = po.scores(algo, q, codes, off, M, gaps[0], gaps[1])
    configure(False, ("builtin", matrix), gaps[0], gaps[1])
    S.init_db(_write_db(str(tmp_path), codes, off))
    qq = S.init_sequence_fasta(S.READ_FROM_STRING, syn.query_string(q))
    fn = S.sw_align if algo == S.SW else S.nw_align
    # (the overflow counters decide from exact scores: a search that computes
    # them never merges -- off here, as at the benchmark's OUTPUT_ERROR)
    S.set_option("counters", 0)
    try:
        for rm in (1, 0):
            S.set_option("rare_merge", rm)
            for k in (1, 10, 64):
                got = [(h["score"], h["id"]) for h in fn(qq, k, 16)]
                assert got == po.topk(exp_sc[keep], keep.astype(np.uint64), k), (rm, k)
                st = S.stats()
                if rm:
                    assert st["rare_merged"] >= 4 and st["rare_rescored"] > 0, st
                else:
                    assert st["rare_merged"] == 0 and st["rare_rescored"] == 0
        # the log (k = n: no device filter) never merges; its scores are exact
        S.set_option("rare_merge", 1)
        sc, ids = _full_scores(qq, algo, n)
        assert (sc == exp_sc[ids.astype(np.int64)]).all()
        assert S.stats()["rare_merged"] == 0
        # counters on: no merge, same result
        S.set_option("counters", 1)
        got = [(h["score"], h["id"]) for h in fn(qq, 10, 16)]
        assert got == po.topk(exp_sc[keep], keep.astype(np.uint64), 10)
        assert S.stats()["rare_merged"] == 0
    finally:
        S.set_option("rare_merge", 0)
        S.set_option("counters", 1)
    S.free_sequence(qq)
