"""Seeded synthetic databases and queries.

Protein DB: residues i.i.d. over the 20 standard amino acids with BLOSUM62
background frequencies; lengths ``1 + round(Gamma(k=2, theta=175))`` clipped
to [16, 4096] (mean ~350); one planted homolog per ``plant_every`` sequences
(a mutated copy of the query: 30-95 % identity, short indels) so the top-k is
not all ties and the int8 path sees scores >= 255.

DNA reads: i.i.d. ACGT, fixed length, with planted substrings of the query.

Everything is returned already mapped to the reference's residue codes
(AA: ``-ABCDEFGHIKLMNPQRSTVWXYZU*OJ`` = 0..27; NT: ``-ACMGRSVTWYHKDBN``), as a
concatenated ``uint8`` array plus ``uint64`` offsets, and can be written as
FASTA for the ``libssa_extern_db`` provider.
"""
from __future__ import annotations

import numpy as np

AA_ORDER = "-ABCDEFGHIKLMNPQRSTVWXYZU*OJ"
NT_ORDER = "-ACMGRSVTWYHKDBN"

# BLOSUM62 background frequencies (Henikoff & Henikoff 1992), standard 20.
_BG = {
    "A": 0.074, "R": 0.052, "N": 0.045, "D": 0.054, "C": 0.025, "Q": 0.034, "E": 0.054,
    "G": 0.074, "H": 0.026, "I": 0.068, "L": 0.099, "K": 0.058, "M": 0.025, "F": 0.047,
    "P": 0.039, "S": 0.057, "T": 0.051, "W": 0.013, "Y": 0.032, "V": 0.073,
}
AA_CODES = np.array([AA_ORDER.index(c) for c in _BG], dtype=np.uint8)
AA_PROBS = np.array(list(_BG.values()), dtype=np.float64)
AA_PROBS /= AA_PROBS.sum()
NT_ACGT = np.array([NT_ORDER.index(c) for c in "ACGT"], dtype=np.uint8)


def protein_query(length: int = 400, seed: int = 7) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.choice(AA_CODES, size=length, p=AA_PROBS).astype(np.uint8)


def _mutate(rng: np.random.Generator, q: np.ndarray) -> np.ndarray:
    ident = rng.uniform(0.30, 0.95)
    out = q.copy()
    sub = rng.random(len(out)) > ident
    out[sub] = rng.choice(AA_CODES, size=int(sub.sum()), p=AA_PROBS)
    # a few short indels
    for _ in range(int(rng.integers(0, 4))):
        pos = int(rng.integers(0, len(out)))
        if rng.random() < 0.5:
            ins = rng.choice(AA_CODES, size=int(rng.integers(1, 6)), p=AA_PROBS)
            out = np.concatenate([out[:pos], ins, out[pos:]])
        else:
            out = np.concatenate([out[:pos], out[pos + int(rng.integers(1, 6)):]])
    return out.astype(np.uint8)


def _aa_lut() -> np.ndarray:
    """65536-entry inverse-CDF table of the background frequencies."""
    cdf = np.cumsum(AA_PROBS)
    u = (np.arange(65536) + 0.5) / 65536.0
    return AA_CODES[np.minimum(np.searchsorted(cdf, u), len(AA_CODES) - 1)].astype(np.uint8)


def protein_db(n: int, seed: int = 42, query: np.ndarray | None = None, plant_every: int = 10000,
               lo: int = 16, hi: int = 4096, shape: float = 2.0, theta: float = 175.0, sampler: str = "choice"):
    """Returns (codes uint8[total], offsets uint64[n+1]).  sampler "lut"
    draws residues through a 16-bit inverse-CDF table (same distribution to
    1/65536, ~10x faster; used for the large bench DBs) instead of
    Generator.choice (kept for the committed golden fixtures)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = np.clip(1 + np.rint(rng.gamma(shape, theta, size=n)), lo, hi).astype(np.int64)
    plants = []
    if query is not None and plant_every > 0 and n > 0:
        for pos in range(int(rng.integers(0, plant_every)) if n > plant_every else 0, n, plant_every):
            hom = _mutate(rng, query)
            lens[pos] = len(hom)
            plants.append((pos, hom))
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    total = int(off[-1])
    if sampler == "lut":
        codes = _aa_lut()[rng.integers(0, 65536, size=total, dtype=np.uint16)]
    else:
        codes = rng.choice(AA_CODES, size=total, p=AA_PROBS).astype(np.uint8)
    for pos, hom in plants:
        codes[int(off[pos]):int(off[pos + 1])] = hom
    return codes, off


# --------------------------------------------------------------------------
# Block-seeded generators: sequence ID range [i0, i1) of an n-sequence DB,
# generated without the rest of it.  Block b (BLOCK consecutive IDs) draws
# from its own PCG64(SeedSequence([seed, b])) stream, so a rank's shard is
# byte-identical to the same slice of the whole DB: a strong-scaling run at
# N = 1/2/4/8 GPUs searches one and the same DB (bench.py c4/c5), and a test
# can regenerate any share of a 10 M-sequence DB in seconds.
# --------------------------------------------------------------------------
BLOCK = 1 << 16

# Residue sets (amino-acid codes of AA_ORDER) and their frequencies:
#   bg20      the 20 standard residues, BLOSUM62 background frequencies;
#   sprot25   + X, B, Z, U, O at roughly UniProtKB/Swiss-Prot's (tiny) rates,
#             i.e. the 25 symbols util_sequence.c:36-44 maps for a real DB;
#   uniform28 the reference's own DB generator: every one of the 28 symbols
#             of "-ABCDEFGHIKLMNPQRSTVWXYZU*OJ" equally likely
#             (benchmark/src/generate_db.c:117-120; '-' is unknown to the
#             provider and becomes code 0, util_sequence.c:303-309).
# (each at least two of the 65536 slots of the sampling table)
_RARE25 = {"X": 2e-4, "B": 5e-5, "Z": 5e-5, "U": 3.1e-5, "O": 3.1e-5}


def alphabet_table(alphabet: str) -> tuple[np.ndarray, np.ndarray]:
    if alphabet == "bg20":
        return AA_CODES, AA_PROBS
    if alphabet == "sprot25":
        codes = np.concatenate([AA_CODES, [AA_ORDER.index(c) for c in _RARE25]]).astype(np.uint8)
        probs = np.concatenate([AA_PROBS * (1.0 - sum(_RARE25.values())), list(_RARE25.values())])
        return codes, probs / probs.sum()
    if alphabet == "uniform28":
        return np.arange(28, dtype=np.uint8), np.full(28, 1.0 / 28)
    raise ValueError(f"unknown alphabet {alphabet}")


def _lut(codes: np.ndarray, probs: np.ndarray) -> np.ndarray:
    cdf = np.cumsum(probs)
    u = (np.arange(65536) + 0.5) / 65536.0
    return codes[np.minimum(np.searchsorted(cdf, u), len(codes) - 1)].astype(np.uint8)


def _protein_block(n: int, seed: int, b: int, query, plant_every: int, lo: int, hi: int, lengths: str):
    """Block b's lengths, planted homologs and residue stream (the caller
    draws the residues from the returned generator, after the lengths)."""
    b0, b1 = b * BLOCK, min(n, (b + 1) * BLOCK)
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, b])))
    if lengths == "gamma":
        lens = np.clip(1 + np.rint(rng.gamma(2.0, 175.0, size=b1 - b0)), lo, hi).astype(np.int64)
    else:
        lens = rng.integers(lo, hi, size=b1 - b0).astype(np.int64)
    plants = []
    if query is not None and plant_every > 0:
        prng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, b, 1])))
        first = b0 + ((plant_every // 2 - b0) % plant_every)
        for pos in range(first, b1, plant_every):
            hom = _mutate(prng, query)
            lens[pos - b0] = len(hom)
            plants.append((pos - b0, hom))
    return b0, b1, lens, plants, rng


def _blocks(i0: int, i1: int):
    return range(i0 // BLOCK, (i1 + BLOCK - 1) // BLOCK if i1 > i0 else i0 // BLOCK)


def protein_db_range(n: int, seed: int, i0: int = 0, i1: int | None = None, query: np.ndarray | None = None,
                     plant_every: int = 10000, lo: int = 16, hi: int = 4096, alphabet: str = "bg20",
                     lengths: str = "gamma"):
    """Sequences [i0, i1) of the block-seeded n-sequence protein DB:
    (codes uint8[total], offsets uint64[i1 - i0 + 1]).

    lengths "gamma": 1 + round(Gamma(2, 175)) clipped to [lo, hi] (SURVEY.md
    §8d); "uniform": uniform in [lo, hi) like generate_db.c:109-112.  A mutated
    copy of the query (30-95 % identity, short indels) replaces every
    sequence whose ID is plant_every/2 modulo plant_every."""
    i1 = n if i1 is None else min(i1, n)
    if not 0 <= i0 <= i1:
        raise ValueError("bad ID range")
    codes_a, probs_a = alphabet_table(alphabet)
    lut = _lut(codes_a, probs_a)
    parts, lens_all = [], []
    for b in _blocks(i0, i1):
        b0, b1, lens, plants, rng = _protein_block(n, seed, b, query, plant_every, lo, hi, lengths)
        off = np.zeros(b1 - b0 + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        codes = lut[rng.integers(0, 65536, size=int(off[-1]), dtype=np.uint16)]
        for pos, hom in plants:
            codes[off[pos]:off[pos + 1]] = hom
        s0, s1 = max(i0, b0) - b0, min(i1, b1) - b0
        parts.append(codes[off[s0]:off[s1]])
        lens_all.append(lens[s0:s1])
    lens = np.concatenate(lens_all) if lens_all else np.zeros(0, np.int64)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    codes = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return codes, off


def protein_lengths_range(n: int, seed: int, i0: int = 0, i1: int | None = None, query: np.ndarray | None = None,
                          plant_every: int = 10000, lo: int = 16, hi: int = 4096, lengths: str = "gamma"):
    """The lengths of sequences [i0, i1) of protein_db_range's DB, without
    drawing residues (cheap for a whole 10 M-sequence DB: bench.py's
    residue-balanced shard cuts)."""
    i1 = n if i1 is None else min(i1, n)
    out = []
    for b in _blocks(i0, i1):
        b0, b1, lens, _, _ = _protein_block(n, seed, b, query, plant_every, lo, hi, lengths)
        out.append(lens[max(i0, b0) - b0:min(i1, b1) - b0])
    return np.concatenate(out) if out else np.zeros(0, np.int64)


def with_long_tail(codes: np.ndarray, off: np.ndarray, count: int, seed: int, alphabet: str = "bg20",
                   lo: int = 5000, hi: int = 35000):
    """A UniProt-like length tail: sequences 0, n//count, 2 n//count, ...
    (count of them) are replaced by fresh i.i.d. residues of the alphabet with
    lengths uniform in [lo, hi]; every other sequence keeps its residues.
    Returns (codes, offsets)."""
    n = len(off) - 1
    if count <= 0 or n == 0:
        return codes, off
    rng = np.random.default_rng(seed)
    lens = np.diff(off).astype(np.int64)
    tail = np.zeros(n, bool)
    tail[np.arange(count) * (n // count)] = True
    lens[tail] = rng.integers(lo, hi + 1, int(tail.sum()))
    noff = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=noff[1:])
    seg = np.repeat(np.arange(n), lens)
    src = off[seg].astype(np.int64) + (np.arange(len(seg)) - noff[seg].astype(np.int64))
    ncodes = _lut(*alphabet_table(alphabet))[rng.integers(0, 65536, size=len(seg), dtype=np.uint16)]
    keep = ~tail[seg]
    ncodes[keep] = codes[src[keep]]
    return ncodes, noff


def dna_reads_range(n: int, seed: int, i0: int = 0, i1: int | None = None, length: int = 150,
                    query: np.ndarray | None = None, plant_every: int = 100000):
    """Reads [i0, i1) of the block-seeded n-read DNA DB (i.i.d. ACGT; every
    read whose ID is 0 modulo plant_every is a query substring with 0-10 %
    substitutions)."""
    i1 = n if i1 is None else min(i1, n)
    parts = []
    for b in _blocks(i0, i1):
        b0, b1 = b * BLOCK, min(n, (b + 1) * BLOCK)
        rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, b])))
        codes = NT_ACGT[rng.integers(0, 4, size=(b1 - b0) * length, dtype=np.uint8)]
        if query is not None and len(query) >= length and plant_every > 0:
            for pos in range(b0 + (-b0 % plant_every), b1, plant_every):
                start = int(rng.integers(0, len(query) - length + 1))
                read = query[start:start + length].copy()
                sub = rng.random(length) < rng.uniform(0.0, 0.10)
                read[sub] = NT_ACGT[rng.integers(0, 4, size=int(sub.sum()))]
                codes[(pos - b0) * length:(pos - b0 + 1) * length] = read
        s0, s1 = max(i0, b0) - b0, min(i1, b1) - b0
        parts.append(codes[s0 * length:s1 * length])
    codes = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    off = np.arange(max(i1 - i0, 0) + 1, dtype=np.uint64) * np.uint64(length)
    return codes, off


def dna_query(length: int = 10000, seed: int = 8) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.choice(NT_ACGT, size=length).astype(np.uint8)


def dna_reads(n: int, length: int = 150, seed: int = 43, query: np.ndarray | None = None,
              plant_every: int = 100000):
    rng = np.random.Generator(np.random.PCG64(seed))
    codes = rng.choice(NT_ACGT, size=n * length).astype(np.uint8)
    if query is not None and len(query) >= length:
        for pos in range(0, n, plant_every):
            start = int(rng.integers(0, len(query) - length + 1))
            read = query[start:start + length].copy()
            sub = rng.random(length) < rng.uniform(0.0, 0.10)
            read[sub] = rng.choice(NT_ACGT, size=int(sub.sum()))
            codes[pos * length:(pos + 1) * length] = read
    off = np.arange(n + 1, dtype=np.uint64) * np.uint64(length)
    return codes, off


def to_ascii(codes: np.ndarray, nucleotide: bool = False) -> np.ndarray:
    order = NT_ORDER if nucleotide else AA_ORDER
    table = np.frombuffer(order.encode(), dtype=np.uint8)
    return table[codes]


def write_fasta(path: str, codes: np.ndarray, off: np.ndarray, nucleotide: bool = False,
                line: int = 0) -> None:
    """Writes one record per sequence ('>i' header, sequence on one line).
    Vectorised per block of records: each block's residues are converted
    at once and the "\\n>i\\n" separators inserted at the record starts
    (np.insert), so a 10 M-sequence DB takes seconds, not minutes."""
    table = np.frombuffer((NT_ORDER if nucleotide else AA_ORDER).encode(), dtype=np.uint8)
    n = len(off) - 1
    off = np.asarray(off, dtype=np.int64)
    with open(path, "wb", buffering=1 << 24) as f:
        blk = 65536
        for b0 in range(0, n, blk):
            b1 = min(n, b0 + blk)
            heads = [b">%d\n" % i for i in range(b0, b1)]
            # record r's insert: the previous record's newline (r > b0), its header
            ilen = np.fromiter((len(h) + 1 for h in heads), dtype=np.int64, count=b1 - b0)
            ilen[0] -= 1
            r0, r1 = int(off[b0]), int(off[b1])
            out = np.insert(table[codes[r0:r1]], np.repeat(off[b0:b1] - r0, ilen),
                            np.frombuffer(b"\n".join(heads), dtype=np.uint8))
            f.write(out.tobytes())
            f.write(b"\n")


def query_string(codes: np.ndarray, nucleotide: bool = False) -> str:
    return to_ascii(codes, nucleotide).tobytes().decode()
