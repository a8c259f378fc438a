"""COMPUTE_ALIGNMENT traceback (host side, no GPU): region + CIGAR of
ssa_amd_align_pair -- the routine sw_align/nw_align run on their hits --
against tests/golden/align.json, the reference's own align_sequences
(align.c:39-182, cigar.c:48-346) on 960 seeded pairs (SW and NW; constant
NT scoring, BLOSUM62, an asymmetric matrix that exposes the reference's
M[query][db] vs M[db][query] mix).  The reference's KAT CIGARs
(tests/test_libssa.c:48-93) are checked end to end on the GPU in
tests/test_gpu_parity.py::test_compute_alignment_kat."""
import json
import os

import pytest

import libssa_amd as S
from tests.conftest import GOLDEN

AA_LETTERS = "-ABCDEFGHIKLMNPQRSTVWXYZU*OJ"
G = json.load(open(os.path.join(GOLDEN, "align.json")))


def matrix_text(m):
    """Matrix file text for a 32x32 table over the amino-acid letters."""
    codes = sorted({i >> 5 for i, v in enumerate(m) if v != -1 and 0 < (i >> 5) < 28})
    lines = ["   " + " ".join(AA_LETTERS[c] for c in codes)]
    for x in codes:
        lines.append(AA_LETTERS[x] + " " + " ".join(str(m[(x << 5) + y]) for y in codes))
    return "\n".join(lines) + "\n"


def configure(case):
    S.set_output_mode(S.OUTPUT_ERROR)
    if case == "nt_const5_4":
        S.init_symbol_translation(S.NUCLEOTIDE, S.FORWARD_STRAND, 1, 1)
        S.init_constant_scores(5, -4)
    elif case == "aa_blosum62":
        S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
        S.init_score_matrix(S.MATRIX_BUILDIN, "blosum62")
    else:
        S.init_symbol_translation(S.AMINOACID, S.FORWARD_STRAND, 1, 1)
        S.init_score_matrix(S.READ_FROM_STRING, matrix_text(G["matrices"][case]))


@pytest.mark.parametrize("case", ["nt_const5_4", "aa_blosum62", "aa_asym"])
def test_traceback_matches_reference(case):
    configure(case)
    pairs = [p for p in G["pairs"] if p["case"] == case]
    assert len(pairs) > 100
    S.init_gap_penalties(pairs[0]["gap_open"], pairs[0]["gap_extend"])
    for p in pairs:
        reg, cig = S.align_pair(S.SW if p["algo"] == 0 else S.NW, bytes(p["query"]), bytes(p["db"]))
        assert (list(reg), cig) == (p["region"], p["cigar"]), (case, p["algo"], p["query"][:8])


def test_zero_score_local_alignment_is_empty():
    """The reference leaves the region uninitialised when no cell scores > 0
    (align.c:39-85, undefined behaviour); here it is all zeros, CIGAR ''."""
    configure("aa_blosum62")
    S.init_gap_penalties(-11, -1)
    w = AA_LETTERS.index("W")
    c = AA_LETTERS.index("C")
    # W vs C scores -2 in BLOSUM62: no positive cell
    assert S.align_pair(S.SW, bytes([w, w]), bytes([c])) == ((0, 0, 0, 0), "")
