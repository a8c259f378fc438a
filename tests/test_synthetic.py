"""The block-seeded synthetic DB generators (libssa_amd/synthetic.py): any ID
slice is byte-identical to the same IDs of the whole DB, so a strong-scaling
run at N = 1/2/4/8 ranks (bench.py make_shard) searches one and the same DB,
and the full-size fixtures' DBs (tests/golden/fullsize.json) are regenerated
exactly on the GPU box."""
import numpy as np
import pytest

from libssa_amd import synthetic as syn


def _slices(fn, n, cuts, **kw):
    parts = [fn(n, 42, a, b, **kw) for a, b in zip(cuts, cuts[1:])]
    codes = np.concatenate([p[0] for p in parts])
    lens = np.concatenate([np.diff(p[1].astype(np.int64)) for p in parts])
    return codes, lens


@pytest.mark.parametrize("alphabet,lengths", [("bg20", "gamma"), ("sprot25", "gamma"), ("uniform28", "uniform")])
def test_protein_slices_equal_whole(alphabet, lengths):
    n = 3 * syn.BLOCK + 1234
    q = syn.protein_query(200, 7)
    whole, off = syn.protein_db_range(n, 42, query=q, alphabet=alphabet, lengths=lengths, plant_every=5000)
    for cuts in ([0, n], [0, n // 2, n], [0, 17, syn.BLOCK, syn.BLOCK + 1, 2 * syn.BLOCK + 5, n], list(range(0, n + 1, n // 8))[:8] + [n]):
        codes, lens = _slices(syn.protein_db_range, n, cuts, query=q, alphabet=alphabet, lengths=lengths,
                              plant_every=5000)
        assert (lens == np.diff(off.astype(np.int64))).all()
        assert (codes == whole).all()


def test_dna_slices_equal_whole():
    n = 2 * syn.BLOCK + 999
    q = syn.dna_query(2000, 8)
    whole, off = syn.dna_reads_range(n, 43, 0, n, 150, query=q, plant_every=10000)
    for cuts in ([0, n], [0, 1, syn.BLOCK - 1, n], list(range(0, n + 1, n // 4))[:4] + [n]):
        parts = [syn.dna_reads_range(n, 43, a, b, 150, query=q, plant_every=10000) for a, b in zip(cuts, cuts[1:])]
        assert (np.concatenate([p[0] for p in parts]) == whole).all()
        assert sum(len(p[1]) - 1 for p in parts) == n


def test_alphabets():
    """sprot25 holds the 20 standard residues plus X, B, Z, U, O; uniform28 all
    28 codes of the reference generator (generate_db.c:117-118)."""
    c25, _ = syn.alphabet_table("sprot25")
    c28, p28 = syn.alphabet_table("uniform28")
    assert len(set(c25.tolist())) == 25 and len(c28) == 28 and np.allclose(p28, 1 / 28)
    codes, _ = syn.protein_db_range(200000, 3, alphabet="uniform28", lengths="uniform", lo=16, hi=1000)
    assert len(np.unique(codes)) == 28
