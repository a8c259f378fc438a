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
    """Writes one record per sequence ('>i' header, sequence on one line)."""
    asc = to_ascii(codes, nucleotide)
    n = len(off) - 1
    with open(path, "wb", buffering=1 << 24) as f:
        # build in blocks to bound memory
        blk = 65536
        for b0 in range(0, n, blk):
            b1 = min(n, b0 + blk)
            parts = []
            for i in range(b0, b1):
                parts.append(b">%d\n" % i)
                parts.append(asc[int(off[i]):int(off[i + 1])].tobytes())
                parts.append(b"\n")
            f.write(b"".join(parts))


def query_string(codes: np.ndarray, nucleotide: bool = False) -> str:
    return to_ascii(codes, nucleotide).tobytes().decode()
