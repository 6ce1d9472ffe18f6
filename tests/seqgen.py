"""Seeded synthetic sequence generators shared by tests and bench.

Base composition from the reference samples (C .330, T .295, A .230, G .146); sequences are
derived from a few random ancestors by substitutions (ts:tv = 2:1) and length-preserving
indel pairs, so that alignments contain gaps and tied paths.
"""

from __future__ import annotations

import numpy as np

ALPHA = np.frombuffer(b"ACGT", dtype=np.uint8)
COMPOSITION = np.array([0.230, 0.330, 0.146, 0.295])
COMPOSITION = COMPOSITION / COMPOSITION.sum()
_TRANSITION = np.array([2, 3, 0, 1])  # A<->G, C<->T


def family_sequences(n: int, length: int, seed: int, *, ancestors: int = 64, max_sub: float = 0.20,
                     indel_rate: float = 0.01) -> list[str]:
    rng = np.random.default_rng(seed)
    anc = rng.choice(4, size=(ancestors, length), p=COMPOSITION)
    out = []
    fam = rng.integers(0, ancestors, size=n)
    rates = rng.uniform(0.0, max_sub, size=n)
    for k in range(n):
        s = anc[fam[k]].copy()
        sub = rng.random(length) < rates[k]
        nsub = int(sub.sum())
        if nsub:
            is_ts = rng.random(nsub) < 2.0 / 3.0
            cur = s[sub]
            tv = (cur + rng.choice([1, 3], size=nsub)) % 4
            tv = np.where(tv == _TRANSITION[cur], (tv + 1) % 4, tv)  # keep transversions transversions
            s[sub] = np.where(is_ts, _TRANSITION[cur], tv)
        nindel = rng.binomial(length, indel_rate)
        if nindel:
            lst = list(s)
            for _ in range(nindel):
                d = int(rng.integers(0, len(lst)))
                del lst[d]
                ins = int(rng.integers(0, len(lst) + 1))
                lst.insert(ins, int(rng.choice(4, p=COMPOSITION)))
            s = np.asarray(lst)
        out.append(ALPHA[s].tobytes().decode())
    return out


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
            r = rng.random()
            if r < rate:
                b[k] = ord(alphabet[int(rng.integers(0, len(alphabet)))])
        # random indel
        if len(b) > 4 and rng.random() < 0.5:
            d = int(rng.integers(0, len(b)))
            del b[d : d + int(rng.integers(1, 4))]
        out.append(b.decode())
    return out
