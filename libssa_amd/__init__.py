"""libssa_amd -- MI355X-native optimal-alignment database search.

Python mirror of the C ABI in ``include/libssa.h`` / ``include/libssa_amd.h``
(the reference's public API, ``src/libssa.h:122-263``), loaded with ctypes
from the in-tree ``libssa_amd/lib/libssa_amd.so``.  Function names, argument
meaning and error behaviour are the reference's: configuration errors end the
process with status 1 (``fatal``), query-file errors return ``None``.

The library itself holds no Python: the scoring runs in the gfx950 kernels
of ``csrc/kernels.hip``; there is no CPU fallback, and loading fails loudly
when the shared library has not been built (``python -m libssa_amd.build``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_double, c_int, c_int8, c_long, c_size_t, c_uint8, \
    c_uint32, c_uint64, c_int64, c_int32, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
# SSA_AMD_LIB: an alternative build of the library (A/B measurements only)
LIB_PATH = os.environ.get("SSA_AMD_LIB") or os.path.join(LIB_DIR, "libssa_amd.so")
DB_LIB_PATH = os.path.join(LIB_DIR, "libssa_fasta_db.so")

# ---- constants (libssa.h) ---------------------------------------------------
BLOSUM45, BLOSUM50, BLOSUM62, BLOSUM80, BLOSUM90 = "blosum45", "blosum50", "blosum62", "blosum80", "blosum90"
PAM30, PAM70, PAM250 = "pam30", "pam70", "pam250"
NUCLEOTIDE, AMINOACID, TRANS_QUERY, TRANS_DB, TRANS_BOTH = 0, 1, 2, 3, 4
FORWARD_STRAND, COMPLEMENTARY_STRAND, BOTH_STRANDS = 1, 2, 3
BIT_WIDTH_8, BIT_WIDTH_16, BIT_WIDTH_64 = 8, 16, 64
OUTPUT_SILENT, OUTPUT_ERROR, OUTPUT_WARNING, OUTPUT_INFO = 0, 1, 2, 3
COMPUTE_SCORE, COMPUTE_ALIGNMENT = 0, 1
READ_FROM_FILE, READ_FROM_STRING, MATRIX_BUILDIN = 0, 1, 2
COMPUTE_ON_SSE2, COMPUTE_ON_SSE41, COMPUTE_ON_AVX2 = 0, 1, 2
SW, NW = 0, 1
TOPK, LOG = 0, 1


class db_seq_t(Structure):
    _fields_ = [("seq", c_void_p), ("len", c_size_t), ("ID", c_size_t), ("strand", c_int), ("frame", c_int)]


class q_seq_t(Structure):
    _fields_ = [("seq", c_void_p), ("len", c_size_t), ("strand", c_int), ("frame", c_int)]


class alignment_t(Structure):
    _fields_ = [("db_seq", db_seq_t), ("query", q_seq_t), ("alignment", c_char_p), ("alignment_len", c_size_t),
                ("score", c_long), ("align_q_start", c_size_t), ("align_q_end", c_size_t),
                ("align_d_start", c_size_t), ("align_d_end", c_size_t)]


class alignment_list_t(Structure):
    _fields_ = [("alignments", POINTER(POINTER(alignment_t))), ("len", c_size_t)]


class ssa_hit_t(Structure):
    _fields_ = [("score", c_int64), ("db_id", c_uint64), ("query_id", c_uint8), ("db_strand", c_uint8),
                ("db_frame", c_uint8), ("pad", c_uint8 * 5)]


class ssa_amd_stats_t(Structure):
    _fields_ = [("search_ms", c_double), ("kernel_ms", c_double), ("wide_ms", c_double), ("d2h_ms", c_double),
                ("replay_ms", c_double), ("pack_ms", c_double), ("cells", c_uint64), ("entries", c_uint64),
                ("overflow_8", c_uint64), ("overflow_16", c_uint64), ("wide_count", c_uint64),
                ("kernel_launches", c_uint32), ("device", c_int32), ("kernel_bytes", c_uint64),
                ("kernel", ctypes.c_char * 32), ("prep_ms", c_double), ("upload_ms", c_double),
                ("sync_wait_ms", c_double), ("strip_rows", c_uint32), ("counters", c_uint32),
                ("long_entries", c_uint32), ("long_kernel", ctypes.c_char * 24), ("part_retries", c_uint32),
                ("total_searches", c_uint64), ("total_kernel_ms", c_double), ("total_search_ms", c_double),
                ("filter_candidates", c_uint64), ("gather_ms", c_double), ("gather_rounds", c_uint32),
                ("rare_merged", c_uint32), ("rare_rescored", c_uint32), ("slots", c_uint32),
                ("slot_device", ctypes.c_int32 * 16), ("slot_kernel_ms", c_double * 16),
                ("slot_search_ms", c_double * 16), ("graph", c_uint32)]


assert ctypes.sizeof(db_seq_t) == 32 and ctypes.sizeof(q_seq_t) == 24
assert ctypes.sizeof(alignment_t) == 112 and ctypes.sizeof(alignment_list_t) == 16
assert ctypes.sizeof(ssa_hit_t) == 24

# every symbol include/*.h declares (checked by tests/test_abi.py)
EXPORTS = {
    "libssa_amd.so": ["set_output_mode", "set_simd_compute_mode", "set_chunk_size", "set_thread_count",
                      "init_score_matrix", "init_constant_scores", "init_gap_penalties", "init_symbol_translation",
                      "init_db", "init_sequence_fasta", "free_sequence", "sw_align", "nw_align", "free_alignment",
                      "ssa_exit", "ssa_amd_device_count", "ssa_amd_set_device", "ssa_amd_set_id_offset",
                      "ssa_amd_prepare_db", "ssa_amd_get_stats", "ssa_amd_set_option", "ssa_amd_search",
                      "ssa_amd_replay", "ssa_amd_query_views", "ssa_amd_translate", "ssa_amd_align_pair",
                      "ssa_amd_save_db", "ssa_amd_load_db", "ssa_amd_set_devices", "ssa_amd_search_batch",
                      "ssa_amd_dist_unique_id", "ssa_amd_dist_unique_id_bytes", "ssa_amd_dist_init",
                      "ssa_amd_dist_finalize", "ssa_amd_gather_logs", "ssa_amd_merge_logs", "ssa_amd_get_timeline",
                      "ssa_amd_dist_available", "ssa_amd_dist_init_fake", "ssa_amd_dist_ranks", "ssa_amd_shard_bounds",
                      "ssa_amd_get_devices"],
    "libssa_fasta_db.so": ["ssa_db_init", "ssa_db_get_sequence_count", "ssa_db_get_sequence", "ssa_db_close"],
}

_lib = None


def load():
    """Loads the in-tree shared library (fails loudly if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libssa_amd native library not built: {LIB_PATH} missing "
                           "(run `python -m libssa_amd.build`)")
    ctypes.CDLL(DB_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P = c_void_p
    sig = {
        "set_output_mode": ([c_int], None), "set_simd_compute_mode": ([c_int], None),
        "set_chunk_size": ([c_size_t], None), "set_thread_count": ([c_size_t], None),
        "init_score_matrix": ([c_int, c_char_p], None), "init_constant_scores": ([c_int8, c_int8], None),
        "init_gap_penalties": ([c_int8, c_int8], None), "init_symbol_translation": ([c_int] * 4, None),
        "init_db": ([c_char_p], None), "init_sequence_fasta": ([c_int, c_char_p], P),
        "free_sequence": ([P], None),
        "sw_align": ([P, c_size_t, c_int, c_int], POINTER(alignment_list_t)),
        "nw_align": ([P, c_size_t, c_int, c_int], POINTER(alignment_list_t)),
        "free_alignment": ([POINTER(alignment_list_t)], None), "ssa_exit": ([], None),
        "ssa_amd_device_count": ([], c_int), "ssa_amd_set_device": ([c_int], None),
        "ssa_amd_set_id_offset": ([c_size_t], None), "ssa_amd_prepare_db": ([], c_int),
        "ssa_amd_get_stats": ([POINTER(ssa_amd_stats_t)], None), "ssa_amd_set_option": ([c_char_p, c_long], None),
        "ssa_amd_search": ([P, c_int, c_size_t, c_int, c_int, POINTER(ssa_hit_t), c_size_t], c_size_t),
        "ssa_amd_replay": ([POINTER(ssa_hit_t), c_size_t, c_size_t, POINTER(ssa_hit_t)], c_size_t),
        "ssa_amd_query_views": ([P, POINTER(q_seq_t), c_size_t], c_size_t),
        "ssa_amd_save_db": ([c_char_p], c_int), "ssa_amd_load_db": ([c_char_p], c_int),
        "ssa_amd_set_devices": ([POINTER(c_int), c_int], c_int),
        "ssa_amd_get_devices": ([POINTER(c_int), c_int], c_int),
        "ssa_amd_search_batch": ([POINTER(c_void_p), c_size_t, c_int, c_size_t, c_int, POINTER(ssa_hit_t),
                                  POINTER(c_size_t)], c_size_t),
        "ssa_amd_align_pair": ([c_int, c_char_p, c_size_t, c_char_p, c_size_t, POINTER(c_size_t), c_char_p, c_size_t],
                               c_size_t),
        "ssa_amd_translate": ([c_int, c_char_p, c_size_t, c_int, c_int, c_char_p, c_size_t], c_size_t),
        "ssa_amd_dist_unique_id": ([c_char_p], c_int), "ssa_amd_dist_unique_id_bytes": ([], c_size_t),
        "ssa_amd_dist_init": ([c_int, c_int, c_char_p], c_int), "ssa_amd_dist_finalize": ([], None),
        "ssa_amd_gather_logs": ([POINTER(ssa_hit_t), c_size_t, c_size_t, POINTER(ssa_hit_t)], c_size_t),
        "ssa_amd_merge_logs": ([POINTER(ssa_hit_t), POINTER(c_size_t), c_size_t, c_size_t, c_size_t,
                                POINTER(ssa_hit_t)], c_size_t),
        "ssa_amd_get_timeline": ([c_void_p, c_size_t], c_size_t),
        "ssa_amd_dist_available": ([], c_int), "ssa_amd_dist_init_fake": ([c_int, c_int, c_int], c_int),
        "ssa_amd_dist_ranks": ([], c_int),
        "ssa_amd_shard_bounds": ([c_void_p, c_size_t, c_size_t, c_size_t, POINTER(c_size_t)], c_int),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("SSA_AMD_LIB") and not hasattr(L, name):
            continue            # an older build under A/B measurement
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _b(s):
    return s.encode() if isinstance(s, str) else s


# ---- thin Pythonic layer (same names as the C API) ---------------------------
def set_output_mode(mode): load().set_output_mode(mode)
def set_simd_compute_mode(mode): load().set_simd_compute_mode(mode)
def set_chunk_size(size): load().set_chunk_size(size)
def set_thread_count(n): load().set_thread_count(n)
def init_score_matrix(mode, matrix): load().init_score_matrix(mode, _b(matrix))
def init_constant_scores(match, mismatch): load().init_constant_scores(match, mismatch)
def init_gap_penalties(gap_open, gap_extend): load().init_gap_penalties(gap_open, gap_extend)
def init_symbol_translation(t, strands, db_gencode, q_gencode):
    load().init_symbol_translation(t, strands, db_gencode, q_gencode)
def init_db(path): load().init_db(_b(path))
def init_sequence_fasta(mode, s): return load().init_sequence_fasta(mode, _b(s))
def free_sequence(q): load().free_sequence(q)
def ssa_exit(): load().ssa_exit()


def _unpack(alist):
    if not alist:
        return []
    a = alist.contents
    out = []
    for i in range(a.len):
        x = a.alignments[i].contents
        out.append({"score": int(x.score), "id": int(x.db_seq.ID), "db_len": int(x.db_seq.len),
                    "db_strand": x.db_seq.strand, "db_frame": x.db_seq.frame,
                    "q_len": int(x.query.len), "q_strand": x.query.strand, "q_frame": x.query.frame,
                    "db_seq": ctypes.string_at(x.db_seq.seq, x.db_seq.len) if x.db_seq.seq else b"",
                    "alignment": x.alignment.decode() if x.alignment else None,
                    "region": (int(x.align_q_start), int(x.align_q_end), int(x.align_d_start), int(x.align_d_end))})
    return out


def sw_align(q, hitcount, bit_width=BIT_WIDTH_16, align_type=COMPUTE_SCORE):
    """Returns the reference's alignment list as a list of dicts (freed)."""
    L = load()
    al = L.sw_align(q, hitcount, bit_width, align_type)
    res = _unpack(al)
    L.free_alignment(al)
    return res


def align_scores(q, hitcount, bit_width=BIT_WIDTH_16, algo=SW):
    """sw_align / nw_align (COMPUTE_SCORE) + free_alignment, exactly the
    public calls the reference's benchmark times (benchmark_util.c:27-48),
    returning only [(score, db_id)] -- reading two fields per hit keeps the
    Python side to a few microseconds (bench.py's timed step)."""
    L = load()
    al = (L.sw_align if algo == SW else L.nw_align)(q, hitcount, bit_width, COMPUTE_SCORE)
    out = []
    if al:
        a = al.contents
        arr = a.alignments
        for i in range(a.len):
            x = arr[i].contents
            out.append((x.score, x.db_seq.ID))
    L.free_alignment(al)
    return out


def align_free(q, hitcount, bit_width=BIT_WIDTH_16, algo=SW):
    """free_alignment(sw_align(...)) / free_alignment(nw_align(...)) with the
    hits unread: the call the reference's benchmark times
    (benchmark/src/benchmark_util.c:27-48)."""
    L = load()
    L.free_alignment((L.sw_align if algo == SW else L.nw_align)(q, hitcount, bit_width, COMPUTE_SCORE))


def nw_align(q, hitcount, bit_width=BIT_WIDTH_16, align_type=COMPUTE_SCORE):
    L = load()
    al = L.nw_align(q, hitcount, bit_width, align_type)
    res = _unpack(al)
    L.free_alignment(al)
    return res


def device_count():
    return load().ssa_amd_device_count()


def set_device(dev): load().ssa_amd_set_device(dev)


def set_devices(devs):
    """ssa_amd_set_devices: search on all of `devs` from this process ([] = single device)."""
    arr = (c_int * max(len(devs), 1))(*devs)
    return load().ssa_amd_set_devices(arr, len(devs))


def get_devices():
    """ssa_amd_get_devices: the device slots the next search uses (after
    SSA_AMD_DEVICES, read at the first init_db unless set_device(s) ran)."""
    arr = (c_int * 16)()
    n = load().ssa_amd_get_devices(arr, 16)
    return [arr[i] for i in range(min(n, 16))]


def set_id_offset(off): load().ssa_amd_set_id_offset(off)
def prepare_db(): return load().ssa_amd_prepare_db()
def set_option(name, value): load().ssa_amd_set_option(_b(name), value)
def save_db(path): return load().ssa_amd_save_db(_b(path))
def load_db(path): return load().ssa_amd_load_db(_b(path))




def stats():
    s = ssa_amd_stats_t()          # (per call: threads of a fake dist group read their own)
    load().ssa_amd_get_stats(ctypes.byref(s))
    d = {f: getattr(s, f) for f, _ in ssa_amd_stats_t._fields_}
    d["kernel"] = d["kernel"].decode()
    d["long_kernel"] = d["long_kernel"].decode()
    n = d["slots"]
    for f in ("slot_device", "slot_kernel_ms", "slot_search_ms"):
        d[f] = list(d[f])[:n]
    return d


def timeline():
    """ssa_amd_get_timeline: the last search's DP wave rows (option
    "timeline") as a uint32 array [rows, 4]: (group or 0x80000000 | lane,
    start, end, place), s_memrealtime ticks (100 MHz)."""
    import numpy as np
    L = load()
    n = L.ssa_amd_get_timeline(None, 0)
    out = np.zeros((n, 4), np.uint32)
    if n:
        L.ssa_amd_get_timeline(out.ctypes.data, n)
    return out


_hitbuf = [None, 0]     # reused output array (a fresh 64 Ki-entry ctypes array per call costs ~0.2 ms)


def _hits(cap):
    if _hitbuf[1] < cap:
        _hitbuf[0], _hitbuf[1] = (ssa_hit_t * cap)(), cap
    return _hitbuf[0]


def search(q, algo, hitcount, bit_width=BIT_WIDTH_16, mode=TOPK, cap=None):
    """ssa_amd_search: sorted top-k (mode=TOPK) or the shard insertion log
    (mode=LOG) as a list of (score, global_id, query_id, strand, frame)."""
    L = load()
    explicit = cap is not None
    if cap is None:
        cap = max(hitcount, 1) if mode == TOPK else max(4 * hitcount + 4096, 65536)
    while True:
        buf = _hits(cap)
        n = L.ssa_amd_search(q, algo, hitcount, bit_width, mode, buf, cap)
        if n < cap or explicit or mode == TOPK:
            break
        cap *= 4            # a log filled the buffer: search again with room
    return [(buf[i].score, buf[i].db_id, buf[i].query_id, buf[i].db_strand, buf[i].db_frame) for i in range(n)]


def replay(log, hitcount):
    """ssa_amd_replay over a (concatenated) insertion log."""
    L = load()
    n = len(log)
    arr = (ssa_hit_t * max(n, 1))()
    for i, h in enumerate(log):
        arr[i].score, arr[i].db_id = int(h[0]), int(h[1])
        if len(h) > 2:
            arr[i].query_id, arr[i].db_strand, arr[i].db_frame = int(h[2]), int(h[3]), int(h[4])
    out = (ssa_hit_t * max(hitcount, 1))()
    c = L.ssa_amd_replay(arr, n, hitcount, out)
    return [(out[i].score, out[i].db_id) for i in range(c)]


def query_views(q):
    """ssa_amd_query_views: [(codes: bytes, strand, frame)] of the search's query buffers."""
    L = load()
    buf = (q_seq_t * 8)()
    n = L.ssa_amd_query_views(q, buf, 8)
    return [(ctypes.string_at(buf[i].seq, buf[i].len), buf[i].strand, buf[i].frame) for i in range(min(n, 8))]


def translate(db_side, nt_codes, strand, frame):
    """ssa_amd_translate on mapped nucleotide codes; returns amino-acid codes (bytes)."""
    L = load()
    src = bytes(nt_codes)
    out = ctypes.create_string_buffer(len(src) // 3 + 1)
    n = L.ssa_amd_translate(db_side, src, len(src), strand, frame, out, len(out))
    return out.raw[:n]


def align_pair(algo, query_codes, db_codes):
    """ssa_amd_align_pair: ((q_begin, q_end, d_begin, d_end), cigar) of one pair."""
    L = load()
    q, d = bytes(query_codes), bytes(db_codes)
    reg = (c_size_t * 4)()
    n = L.ssa_amd_align_pair(algo, q, len(q), d, len(d), reg, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    L.ssa_amd_align_pair(algo, q, len(q), d, len(d), reg, buf, n + 1)
    return tuple(reg), buf.value.decode()


def search_batch(queries, algo, hitcount, bit_width=BIT_WIDTH_16):
    """ssa_amd_search_batch: per query, the sorted top-k [(score, id), ...]."""
    L = load()
    nq = len(queries)
    qs = (c_void_p * max(nq, 1))(*queries)
    out = (ssa_hit_t * max(nq * hitcount, 1))()
    counts = (c_size_t * max(nq, 1))()
    L.ssa_amd_search_batch(qs, nq, algo, hitcount, bit_width, out, counts)
    return [[(out[i * hitcount + j].score, out[i * hitcount + j].db_id) for j in range(counts[i])] for i in range(nq)]


# ---- multi-process gather over RCCL (libssa_amd.h ssa_amd_dist_*) ------------
def dist_unique_id():
    """Rank 0: the RCCL unique id (bytes) to hand to every rank."""
    L = load()
    buf = ctypes.create_string_buffer(L.ssa_amd_dist_unique_id_bytes())
    if L.ssa_amd_dist_unique_id(buf) != 0:
        raise RuntimeError("ssa_amd_dist_unique_id failed")
    return buf.raw


def dist_available():
    """ssa_amd_dist_available: True when this rank could enter ssa_amd_dist_init."""
    return load().ssa_amd_dist_available() == 0


def dist_init(rank, world, uid):
    if load().ssa_amd_dist_init(rank, world, uid) != 0:
        raise RuntimeError(f"ssa_amd_dist_init({rank}, {world}) failed")


def dist_init_fake(rank, world, group=0):
    """ssa_amd_dist_init_fake: the calling thread becomes rank `rank` of an
    in-process group of `world` threads (test support)."""
    if load().ssa_amd_dist_init_fake(rank, world, group) != 0:
        raise RuntimeError(f"ssa_amd_dist_init_fake({rank}, {world}, {group}) failed")


def dist_ranks():
    """ssa_amd_dist_ranks: ranks of the communicator (ncclCommCount)."""
    return load().ssa_amd_dist_ranks()


def dist_finalize(): load().ssa_amd_dist_finalize()


def shard_bounds(lengths, world, align=1):
    """ssa_amd_shard_bounds: world + 1 record bounds of residue-balanced
    contiguous shards (cuts at multiples of `align`)."""
    import numpy as np
    lens = np.ascontiguousarray(lengths, dtype=np.uint64)
    out = (c_size_t * (world + 1))()
    if load().ssa_amd_shard_bounds(lens.ctypes.data, len(lens), world, align, out) != 0:
        raise ValueError("ssa_amd_shard_bounds: world must be >= 1")
    return [int(x) for x in out]


def _hit_array(log):
    arr = (ssa_hit_t * max(len(log), 1))()
    for i, h in enumerate(log):
        arr[i].score, arr[i].db_id = int(h[0]), int(h[1])
        if len(h) > 2:
            arr[i].query_id, arr[i].db_strand, arr[i].db_frame = int(h[2]), int(h[3]), int(h[4])
    return arr


def gather_logs(log, hitcount):
    """ssa_amd_gather_logs (collective): rank 0 gets the global sorted top-k
    [(score, db_id)], the other ranks []."""
    L = load()
    arr = _hit_array(log)
    out = (ssa_hit_t * max(hitcount, 1))()
    c = L.ssa_amd_gather_logs(arr, len(log), hitcount, out)
    return [(out[i].score, out[i].db_id) for i in range(c)]


def merge_logs(logs, hitcount):
    """ssa_amd_merge_logs: rank 0's merge of per-shard logs (in shard order)."""
    L = load()
    stride = max([len(x) for x in logs] + [1])
    rows = (ssa_hit_t * (stride * max(len(logs), 1)))()
    for r, lg in enumerate(logs):
        for i, h in enumerate(lg):
            rows[r * stride + i].score, rows[r * stride + i].db_id = int(h[0]), int(h[1])
            if len(h) > 2:
                rows[r * stride + i].query_id = int(h[2])
                rows[r * stride + i].db_strand, rows[r * stride + i].db_frame = int(h[3]), int(h[4])
    counts = (c_size_t * max(len(logs), 1))(*[len(x) for x in logs])
    out = (ssa_hit_t * max(hitcount, 1))()
    c = L.ssa_amd_merge_logs(rows, counts, len(logs), stride, hitcount, out)
    return [(out[i].score, out[i].db_id) for i in range(c)]
