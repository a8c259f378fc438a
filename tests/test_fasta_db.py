"""libssa_fasta_db.so -- the DB plugin (reference contract
src/libssa_extern_db.h, tests/test_libssa_extern_db.c:12-55): record index
== ID, residues without whitespace, empty records kept, NULL past the end.
The parallel mmap parser must agree byte for byte with a plain sequential
reading of the file, including files large enough to be split across
threads (> 8 MiB) with cut points inside multi-line records."""
import ctypes
import os

import numpy as np

from libssa_amd import DB_LIB_PATH


class SeqInfo(ctypes.Structure):
    _fields_ = [("ID", ctypes.c_size_t), ("seqlen", ctypes.c_size_t), ("seq", ctypes.c_void_p)]


def _lib():
    L = ctypes.CDLL(DB_LIB_PATH)
    L.ssa_db_init.argtypes = [ctypes.c_char_p]
    L.ssa_db_init.restype = ctypes.c_int
    L.ssa_db_get_sequence_count.restype = ctypes.c_size_t
    L.ssa_db_get_sequence.argtypes = [ctypes.c_size_t]
    L.ssa_db_get_sequence.restype = ctypes.POINTER(SeqInfo)
    return L


def _expected(data: bytes):
    recs, cur = [], None
    for line in data.split(b"\n"):
        if line.startswith(b">"):
            cur = []
            recs.append(cur)
        elif cur is not None:
            cur.append(bytes(c for c in line if c not in b" \t\r\v\f"))
    return [b"".join(r) for r in recs]


def _check(tmp_path, data: bytes):
    p = tmp_path / "db.fas"
    p.write_bytes(data)
    L = _lib()
    assert L.ssa_db_init(str(p).encode()) == 0
    exp = _expected(data)
    n = L.ssa_db_get_sequence_count()
    assert n == len(exp)
    for i in [j for j in list(range(min(n, 2000))) + list(range(max(0, n - 2000), n)) + [n // 2, n // 3] if j < n]:
        r = L.ssa_db_get_sequence(i).contents
        assert r.ID == i
        assert ctypes.string_at(r.seq, r.seqlen) == exp[i], i
    assert not L.ssa_db_get_sequence(n)
    L.ssa_db_close()


def test_small_edge_cases(tmp_path):
    data = (b"junk before\n>a\nAC GT\r\nTT\n>empty\n>b desc\n\n  A\tC\n>c\nGG" )
    _check(tmp_path, data)
    _check(tmp_path, b"")
    _check(tmp_path, b">only\n")


def test_large_file_parallel_parse(tmp_path):
    rng = np.random.default_rng(5)
    parts = []
    letters = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    for i in range(120000):
        n = int(rng.integers(0, 300))
        s = letters[rng.integers(0, 20, n)].tobytes()
        if i % 7 == 0:   # multi-line record
            s = b"\n".join(s[j:j + 60] for j in range(0, len(s), 60))
        if i % 11 == 0:
            s = s.replace(b"A", b" A")
        parts.append(b">r%d\n%s\n" % (i, s))
    data = b"".join(parts)
    assert len(data) > (8 << 20)
    _check(tmp_path, data)


def test_bulk_allocated_arena(tmp_path):
    """A residue arena above the 32 MiB threshold of csrc/bulk_alloc.h (an
    anonymous mapping on transparent huge pages, grown without zeroing)
    parses byte for byte like the sequential reading, as do the small
    files on the ordinary allocator above."""
    rng = np.random.default_rng(9)
    letters = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    lens = rng.integers(150, 350, 200000)
    res = letters[rng.integers(0, 20, int(lens.sum()))].tobytes()
    parts, at = [], 0
    for i, n in enumerate(lens):
        s = res[at:at + n]
        at += n
        if i % 5 == 0:   # multi-line record
            s = b"\n".join(s[j:j + 80] for j in range(0, len(s), 80))
        parts.append(b">r%d\n%s\n" % (i, s))
    data = b"".join(parts)
    assert lens.sum() > (32 << 20)
    _check(tmp_path, data)
