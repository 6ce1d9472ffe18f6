"""Seeded synthetic DNA for benches and tests (SURVEY.md §8(d) config definitions).

Base composition from the reference samples (C .330, T .295, A .230, G .146).  Sequences
derive from a few random ancestors by substitutions (ts:tv = 2:1) and length-preserving
indel pairs (per-site delete + compensating insert), so alignments contain gaps and ties.
"""

from __future__ import annotations

import numpy as np

ALPHA = np.frombuffer(b"ACGT", dtype=np.uint8)
COMPOSITION = np.array([0.230, 0.330, 0.146, 0.295])
COMPOSITION = COMPOSITION / COMPOSITION.sum()
_TRANSITION = np.array([2, 3, 0, 1])           # A<->G, C<->T
_TRANSVERSIONS = np.array([[1, 3], [0, 2], [1, 3], [0, 2]])


def family_codes(n: int, length: int, seed: int, *, ancestors: int = 64, max_sub: float = 0.20,
                 indel_rate: float = 0.01) -> np.ndarray:
    """(n, length) uint8 base codes 0..3 (equal lengths)."""
    rng = np.random.default_rng(seed)
    anc = rng.choice(4, size=(ancestors, length), p=COMPOSITION).astype(np.uint8)
    fam = rng.integers(0, ancestors, size=n)
    seqs = anc[fam].copy()
    rates = rng.uniform(0.0, max_sub, size=n)
    sub = rng.random((n, length)) < rates[:, None]
    is_ts = rng.random((n, length)) < 2.0 / 3.0
    pick = rng.integers(0, 2, size=(n, length))
    ts = _TRANSITION[seqs]
    tv = _TRANSVERSIONS[seqs, pick]
    seqs = np.where(sub, np.where(is_ts, ts, tv), seqs).astype(np.uint8)
    nindel = rng.binomial(length, indel_rate, size=n)
    for k in np.nonzero(nindel)[0]:
        m = int(nindel[k])
        s = np.delete(seqs[k], rng.choice(length, size=m, replace=False))
        pos = np.sort(rng.integers(0, len(s) + 1, size=m))
        seqs[k] = np.insert(s, pos, rng.choice(4, size=m, p=COMPOSITION).astype(np.uint8))
    return seqs


def family_sequences(n: int, length: int, seed: int, **kw) -> list[str]:
    codes = family_codes(n, length, seed, **kw)
    raw = ALPHA[codes]
    return [row.tobytes().decode() for row in raw]


def family_packed(n: int, length: int, seed: int, **kw) -> tuple[np.ndarray, np.ndarray]:
    """Same sequences as ``family_sequences`` as (bytes, offsets) ready for Engine.upload_packed."""
    codes = family_codes(n, length, seed, **kw)
    buf = np.ascontiguousarray(ALPHA[codes]).reshape(-1)
    offs = np.arange(n + 1, dtype=np.int64) * length
    return np.concatenate([buf, np.zeros(1, np.uint8)]), offs


def random_sequences(n: int, lo: int, hi: int, seed: int, alphabet: str = "ACGT",
                     n_rate: float = 0.0) -> list[str]:
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(alphabet.encode(), dtype=np.uint8)
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        s = alpha[rng.integers(0, len(alpha), size=L)]
        if n_rate:
            s = np.where(rng.random(L) < n_rate, ord("N"), s).astype(np.uint8)
        out.append(s.tobytes().decode())
    return out


def mutate(seqs: list[str], seed: int, rate: float = 0.1, alphabet: str = "ACGTN") -> list[str]:
    rng = np.random.default_rng(seed)
    out = []
    for s in seqs:
        b = bytearray(s.encode())
        for k in range(len(b)):
            if rng.random() < rate:
                b[k] = ord(alphabet[int(rng.integers(0, len(alphabet)))])
        if len(b) > 4 and rng.random() < 0.5:
            d = int(rng.integers(0, len(b)))
            del b[d : d + int(rng.integers(1, 4))]
        out.append(b.decode())
    return out
