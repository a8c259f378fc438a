"""Translated modes (TRANS_QUERY / TRANS_DB / TRANS_BOTH) -- host side, no GPU.

The six-frame translation (reference util_sequence.c:201-288, 332-382) is
pinned two ways: the reference's own known-answer strings
(tests/test_util_sequence.c:104-234, test_db_adapter.c:172-220) and
tests/golden/translate.npz, the reference's us_translate_sequence output for
every valid genetic code on seeded random nucleotide sequences with IUPAC
ambiguity codes (tools/gen_golden.py gen_translate).  The query buffers a
search uses (searcher.c:42-90, query.c:131-160) are read back through
ssa_amd_query_views.
"""
import os

import numpy as np
import pytest

import libssa_amd as S
from oracle import pyoracle as po
from tests.conftest import GOLDEN

DNA = b"ATGCCCAAGCTGAATAGCGTAGAGGGGTTTTCATCATTTGAGGACGATGTATAA"
RNA = DNA.replace(b"T", b"U")
# reference test_util_sequence.c:128-182 (query table = genetic code 3)
FRAMES = {
    (0, 0): "MPKTNSVEGFSSFEDDV*", (0, 1): "CPSWMA*RGFHHLRTMY", (0, 2): "AQAE*RRGVFIIWGRCM",
    (1, 0): "LYIVTKWWKPTYAIQTGH", (1, 1): "YTSSSNDENPSTTFSLG", (1, 2): "MHRPQMMKTPTRYSAWA",
}


def aa_codes(s: str) -> bytes:
    return po.map_query(s.encode(), False).tobytes()


def nt_codes(s: bytes) -> bytes:
    return po.map_db(s, True).tobytes()


@pytest.fixture(autouse=True)
def _quiet():
    S.set_output_mode(S.OUTPUT_ERROR)
    yield
    S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)


def test_reference_translation_kats():
    S.init_symbol_translation(S.TRANS_QUERY, S.BOTH_STRANDS, 1, 3)   # (type, strands, db, query)
    for (strand, frame), exp in FRAMES.items():
        assert S.translate(0, nt_codes(DNA), strand, frame) == aa_codes(exp), (strand, frame)
    # RNA: U maps to T (test_translate_query_RNA)
    assert S.translate(0, nt_codes(RNA), 0, 0) == aa_codes(FRAMES[(0, 0)])
    # DB side uses the DB table (test_translate_db: us_init_translation(1, 3))
    S.init_symbol_translation(S.TRANS_DB, S.FORWARD_STRAND, 3, 1)
    assert S.translate(1, nt_codes(DNA), 0, 0) == aa_codes(FRAMES[(0, 0)])


def test_short_sequences_translate_to_empty():
    S.init_symbol_translation(S.TRANS_BOTH, S.BOTH_STRANDS, 1, 1)
    for n in range(0, 3):
        for f in range(3):
            assert S.translate(1, b"\x01" * n, 0, f) == b""
            assert S.translate(0, b"\x01" * n, 1, f) == b""


def test_translation_matches_reference_for_every_genetic_code():
    z = np.load(os.path.join(GOLDEN, "translate.npz"))
    pairs = sorted({k.rsplit("_", 1)[0] for k in z.files})
    assert len(pairs) == 17
    for p in pairs:
        g, d = (int(x[1:]) for x in p.split("_"))
        db, off = z[p + "_db"], z[p + "_off"]
        out, ooff = z[p + "_out"], z[p + "_outoff"]
        S.init_symbol_translation(S.TRANS_BOTH, S.BOTH_STRANDS, d, g)
        idx = 0
        for i in range(len(off) - 1):
            seq = db[int(off[i]):int(off[i + 1])].tobytes()
            for side in range(2):
                for strand in range(2):
                    for frame in range(3):
                        exp = out[int(ooff[idx]):int(ooff[idx + 1])].tobytes()
                        idx += 1
                        assert S.translate(side, seq, strand, frame) == exp, (p, i, side, strand, frame)


@pytest.mark.parametrize("strands", [S.FORWARD_STRAND, S.COMPLEMENTARY_STRAND, S.BOTH_STRANDS])
def test_translated_query_views(strands):
    """TRANS_QUERY / TRANS_BOTH search 3 frames per selected strand, in the
    order strand 0 then 1, frame 0..2 (query.c:145-156, searcher.c:52-70)."""
    for t in (S.TRANS_QUERY, S.TRANS_BOTH):
        S.init_symbol_translation(t, strands, 1, 3)
        q = S.init_sequence_fasta(S.READ_FROM_STRING, DNA.decode())
        views = S.query_views(q)
        want = [(s, f) for s in range(2) if (s + 1) & strands for f in range(3)]
        assert [(v[1], v[2]) for v in views] == want
        for codes, s, f in views:
            assert codes == aa_codes(FRAMES[(s, f)])
        S.free_sequence(q)


def test_untranslated_query_views():
    S.init_symbol_translation(S.TRANS_DB, S.BOTH_STRANDS, 1, 1)
    q = S.init_sequence_fasta(S.READ_FROM_STRING, "MPKTNSV")
    assert S.query_views(q) == [(aa_codes("MPKTNSV"), 0, 0)]
    S.free_sequence(q)
    S.init_symbol_translation(S.NUCLEOTIDE, S.BOTH_STRANDS, 1, 1)
    q = S.init_sequence_fasta(S.READ_FROM_STRING, "ACGTN")
    v = S.query_views(q)
    assert [(x[1], x[2]) for x in v] == [(0, 0), (1, 0)]
    assert v[0][0] == nt_codes(b"ACGTN")
    comp = {1: 8, 2: 4, 4: 2, 8: 1, 15: 15}
    assert v[1][0] == bytes(comp[c] for c in reversed(nt_codes(b"ACGTN")))
    S.free_sequence(q)
