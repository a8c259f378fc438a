"""Python side of the oracle -- TEST INFRASTRUCTURE ONLY.

Loads ``oracle/libssa_oracle.so`` (the C restatement in ``ssa_oracle.c``) and,
when built, drives ``oracle/_ref/ref_harness`` (the reference's own sources).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
import this module, and only as the checker.

FASTA handling here is an independent re-implementation of the DB-provider
contract the reference's tests pin (``tests/test_libssa_extern_db.c:12-55``):
record index = ID, multi-line records joined, whitespace dropped, empty
records kept with length 0.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libssa_oracle.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")

SW, NW = 0, 1

_lib = None


def build(quiet: bool = True) -> None:
    """Compile the C restatement (and the reference harness when the
    reference sources are present)."""
    out = subprocess.DEVNULL if quiet else None
    subprocess.check_call(["make", "-C", HERE, "libssa_oracle.so"], stdout=out)
    if os.path.isdir("/root/reference/src"):
        subprocess.check_call(["make", "-C", HERE, "-j8", "ref"], stdout=out)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_scores.argtypes = [ctypes.c_int, P, P, ctypes.c_size_t, P, ctypes.c_size_t, P,
                                    ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.oracle_topk.argtypes = [P, P, ctypes.c_size_t, ctypes.c_size_t, P, P]
        L.oracle_topk.restype = ctypes.c_size_t
        L.oracle_topk_log.argtypes = [P, P, ctypes.c_size_t, ctypes.c_size_t, P, P]
        L.oracle_topk_log.restype = ctypes.c_size_t
        L.oracle_map_db.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, P]
        L.oracle_map_db.restype = ctypes.c_size_t
        L.oracle_map_query.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, P]
        L.oracle_map_query.restype = ctypes.c_size_t
        L.oracle_matrix_parse.argtypes = [ctypes.c_char_p, P]
        L.oracle_matrix_constant.argtypes = [ctypes.c_int, ctypes.c_int, P]
        L.oracle_build_map.argtypes = [ctypes.c_int, P]
        L.oracle_nw_overflow.argtypes = [ctypes.c_int, P, ctypes.c_size_t, P, ctypes.c_size_t, P,
                                         ctypes.c_int, ctypes.c_int, P]
        L.oracle_nw_overflow.restype = ctypes.c_int
        L.oracle_overflow_flags.argtypes = [ctypes.c_int, P, P, ctypes.c_size_t, P, ctypes.c_size_t, P,
                                            ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.oracle_overflow_counts.argtypes = [ctypes.c_int, P, ctypes.c_size_t, ctypes.c_size_t, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------- FASTA / maps
def read_fasta(path: str) -> list[bytes]:
    """Records in file order; sequence lines joined, whitespace removed."""
    seqs: list[bytes] = []
    cur: list[bytes] | None = None
    with open(path, "rb") as f:
        for line in f:
            if line.startswith(b">"):
                if cur is not None:
                    seqs.append(b"".join(cur))
                cur = []
            elif cur is not None:
                cur.append(b"".join(line.split()))
    if cur is not None:
        seqs.append(b"".join(cur))
    return seqs


def build_map(nucleotide: bool) -> np.ndarray:
    m = np.zeros(256, dtype=np.int8)
    lib().oracle_build_map(int(nucleotide), _ptr(m))
    return m


def map_db(seq: bytes, nucleotide: bool) -> np.ndarray:
    out = np.zeros(max(len(seq), 1), dtype=np.uint8)
    lib().oracle_map_db(int(nucleotide), seq, len(seq), _ptr(out))
    return out[: len(seq)]


def map_query(seq: bytes, nucleotide: bool) -> np.ndarray:
    out = np.zeros(max(len(seq), 1), dtype=np.uint8)
    n = lib().oracle_map_query(int(nucleotide), seq, len(seq), _ptr(out))
    return out[:n].copy()


def read_query_fasta(path: str) -> bytes:
    """First record only, header line skipped (query.c:187-264)."""
    recs = read_fasta(path)
    return recs[0] if recs else b""


# ------------------------------------------------------------------- matrices
def matrix_constant(match: int, mismatch: int) -> np.ndarray:
    m = np.zeros(1024, dtype=np.int64)
    lib().oracle_matrix_constant(match, mismatch, _ptr(m))
    return m


def matrix_parse(text: str | bytes) -> np.ndarray:
    if isinstance(text, str):
        text = text.encode()
    m = np.zeros(1024, dtype=np.int64)
    lib().oracle_matrix_parse(text, _ptr(m))
    return m


# --------------------------------------------------------------------- scoring
def pack_db(seqs: list[np.ndarray]) -> tuple[np.ndarray, np.ndarray]:
    lens = np.array([len(s) for s in seqs], dtype=np.uint64)
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    db = np.concatenate([np.asarray(s, dtype=np.uint8) for s in seqs]) if seqs else np.zeros(0, np.uint8)
    if db.size == 0:
        db = np.zeros(1, dtype=np.uint8)
    return np.ascontiguousarray(db), off


def scores(algo: int, query: np.ndarray, db: np.ndarray, off: np.ndarray, matrix: np.ndarray,
           gap_open: int, gap_extend: int, threads: int = 8) -> np.ndarray:
    """Exact int64 score of every DB sequence (full_sw / full_nw semantics)."""
    n = len(off) - 1
    out = np.zeros(max(n, 1), dtype=np.int64)
    q = np.ascontiguousarray(query, dtype=np.uint8)
    if q.size == 0:
        q = np.zeros(1, dtype=np.uint8)
        qlen = 0
    else:
        qlen = len(query)
    lib().oracle_scores(algo, _ptr(db), _ptr(off), n, _ptr(q), qlen, _ptr(matrix),
                        gap_open, gap_extend, _ptr(out), threads)
    return out[:n]


def overflow_flags(algo: int, query: np.ndarray, db: np.ndarray, off: np.ndarray, matrix: np.ndarray,
                   gap_open: int, gap_extend: int, threads: int = 8) -> np.ndarray:
    """Per DB sequence: bit 0 = the reference's 8-bit kernel overflows, bit 1
    = its 16-bit kernel does (SW: score rule; NW: saturated replay,
    oracle_nw_overflow).  Empty sequences / query: 0."""
    n = len(off) - 1
    out = np.zeros(max(n, 1), dtype=np.uint8)
    q = np.ascontiguousarray(query, dtype=np.uint8)
    qlen = len(q)
    if q.size == 0:
        q = np.zeros(1, dtype=np.uint8)
    lib().oracle_overflow_flags(algo, _ptr(db), _ptr(off), n, _ptr(q), qlen, _ptr(matrix),
                                gap_open, gap_extend, _ptr(out), threads)
    return out[:n]


def overflow_counts(width: int, flags: np.ndarray) -> tuple[int, int]:
    """(overflow_8, overflow_16) of a search from [views][seqs] flags."""
    f = np.ascontiguousarray(np.atleast_2d(flags), dtype=np.uint8)
    out = np.zeros(2, dtype=np.uint64)
    lib().oracle_overflow_counts(width, _ptr(f), f.shape[0], f.shape[1], _ptr(out))
    return int(out[0]), int(out[1])


def topk(sc: np.ndarray, ids: np.ndarray, k: int) -> list[tuple[int, int]]:
    """Reference min-heap replay in the given insertion order, sorted
    score desc / id desc."""
    sc = np.ascontiguousarray(sc, dtype=np.int64)
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    os_ = np.zeros(max(k, 1), dtype=np.int64)
    oi = np.zeros(max(k, 1), dtype=np.uint64)
    c = lib().oracle_topk(_ptr(sc), _ptr(ids), len(sc), k, _ptr(os_), _ptr(oi))
    return [(int(os_[i]), int(oi[i])) for i in range(c)]


def topk_log(sc: np.ndarray, ids: np.ndarray, k: int) -> list[tuple[int, int]]:
    """Elements the reference heap accepts, in insertion order."""
    sc = np.ascontiguousarray(sc, dtype=np.int64)
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    os_ = np.zeros(max(len(sc), 1), dtype=np.int64)
    oi = np.zeros(max(len(sc), 1), dtype=np.uint64)
    c = lib().oracle_topk_log(_ptr(sc), _ptr(ids), len(sc), k, _ptr(os_), _ptr(oi))
    return [(int(os_[i]), int(oi[i])) for i in range(c)]


def search(algo: int, query: np.ndarray, seqs: list[np.ndarray], matrix: np.ndarray,
           gap_open: int, gap_extend: int, k: int, threads: int = 8) -> list[tuple[int, int]]:
    """64-bit single-thread reference result: scores for every non-empty DB
    sequence, heap replay in ascending ID order."""
    db, off = pack_db(seqs)
    sc = scores(algo, query, db, off, matrix, gap_open, gap_extend, threads)
    lens = np.diff(off)
    keep = np.nonzero(lens > 0)[0]
    return topk(sc[keep], keep.astype(np.uint64), k)


# ------------------------------------------------------------ reference harness
def have_ref() -> bool:
    return os.path.exists(REF_HARNESS)


MODE_SCORES, MODE_SEARCH64, MODE_SEARCH16_AVX2, MODE_SEARCH16_SSE2, MODE_TABLES, MODE_TRANSLATE = 0, 1, 2, 3, 4, 5
MODE_ALIGN = 6
MODE_SEARCH8_AVX2 = 7


def ref_run(mode: int, algo: int = 0, query=None, seqs=None, matrix=None, gap_open: int = 0,
            gap_extend: int = 0, k: int = 10, chunk: int = 1000, threads: int = 1, repeat: int = 1,
            db_off=None, views=None, chunk_counts=False, raw_hits=False, times=False):
    """Runs the reference harness.  Returns raw per-seq scores (mode 0), the
    tables blob (mode 4), or (hits, overflow_count, nseq, seconds) for the
    searches -- overflow_count is the 16-bit count, or (o8, o16) for the
    8-bit mode 7; with chunk_counts the per-chunk [nchunks, 2] (o8, o16)
    array is appended.  views: a list of equal-length query views (searched
    as one multi-view query) instead of `query`.  raw_hits: the hits as an
    int64 [count, 2] (score, id) array instead of a list of tuples (the
    multi-million-hit full-size fixtures).  times: the searches return
    the seconds of every repeat (a list) in place of the best."""
    nviews = 0
    if views is not None:
        nviews = len(views)
        query = np.concatenate([np.asarray(v, np.uint8) for v in views])
    if query is None:
        query = np.zeros(0, np.uint8)
    if matrix is None:
        matrix = np.full(1024, -1, np.int64)
    if db_off is not None:
        db, off = db_off
    else:
        db, off = pack_db(seqs or [])
    nseq = len(off) - 1
    hdr = b"SSAR" + struct.pack("<IIIQQiiII", mode, algo, threads, k, chunk, gap_open, gap_extend,
                                repeat, nviews)
    with tempfile.TemporaryDirectory() as td:
        req = os.path.join(td, "req.bin")
        rsp = os.path.join(td, "rsp.bin")
        with open(req, "wb") as f:
            f.write(hdr)
            f.write(np.ascontiguousarray(matrix, dtype=np.int64).tobytes())
            q = np.ascontiguousarray(query, dtype=np.uint8)
            f.write(struct.pack("<Q", len(q)))
            f.write(q.tobytes())
            f.write(struct.pack("<Q", nseq))
            f.write(np.ascontiguousarray(off, dtype=np.uint64).tobytes())
            f.write(np.ascontiguousarray(db[: int(off[-1])], dtype=np.uint8).tobytes())
        subprocess.check_call([REF_HARNESS, req, rsp])
        data = open(rsp, "rb").read()
    if mode == MODE_SCORES:
        return np.frombuffer(data, dtype=np.int64).copy()
    if mode == MODE_ALIGN:
        # per sequence: (q_begin, q_end, d_begin, d_end), cigar
        out, pos = [], 0
        for _ in range(nseq):
            v = struct.unpack_from("<5Q", data, pos)
            out.append((v[:4], data[pos + 40: pos + 40 + v[4]].decode()))
            pos += 40 + v[4]
        return out
    if mode == MODE_TRANSLATE:
        # per sequence: side 0/1 x strand 0/1 x frame 0..2, each u64 len + codes
        out, pos = [], 0
        for _ in range(nseq):
            per = {}
            for side in range(2):
                for strand in range(2):
                    for frame in range(3):
                        n = struct.unpack_from("<Q", data, pos)[0]
                        per[(side, strand, frame)] = data[pos + 8: pos + 8 + n]
                        pos += 8 + n
            out.append(per)
        return out
    if mode == MODE_TABLES:
        mats = np.frombuffer(data[: 8 * 8 * 1024], dtype=np.int64).reshape(8, 1024).copy()
        maps = np.frombuffer(data[8 * 8 * 1024:], dtype=np.int8).reshape(2, 256).copy()
        return mats, maps
    cnt = struct.unpack_from("<Q", data, 0)[0]
    arr = np.frombuffer(data, dtype=np.int64, count=2 * cnt, offset=8).reshape(cnt, 2)
    hits = arr.copy() if raw_hits else [(int(a), int(b)) for a, b in arr]
    pos = 8 + 16 * cnt
    ovf, ns = struct.unpack_from("<QQ", data, pos)
    secs = struct.unpack_from("<d", data, pos + 16)[0]
    o8, nch = struct.unpack_from("<QQ", data, pos + 24)
    if mode == MODE_SEARCH8_AVX2:
        ovf = (o8, ovf)
    if times:
        tpos = pos + 40 + 16 * nch
        nrep = struct.unpack_from("<Q", data, tpos)[0]
        secs = list(struct.unpack_from(f"<{nrep}d", data, tpos + 8))
    if chunk_counts:
        per = np.frombuffer(data, dtype=np.uint64, count=2 * nch, offset=pos + 40).reshape(nch, 2).copy()
        return hits, ovf, ns, secs, per
    return hits, ovf, ns, secs
