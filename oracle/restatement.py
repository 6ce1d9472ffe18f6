"""CPU restatement of the TaxI2 all-pairs distance hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product
(``taxi2_amd``) never does.  It is the readable, pure-Python statement of the
semantics that the C restatement (``oracle/taxi2_oracle.c``) and the HIP kernels
(``taxi2_amd/csrc``) must reproduce.

Parity anchors:
  * ``normalize``            <- ``src/itaxotools/taxi2/sequences.py:20-25``
  * ``align``                <- ``src/itaxotools/taxi2/align.py:72-157`` calling Biopython 1.85
    ``PairwiseAligner(**Scores).align(x, y)[0]`` (third-party C, absent here; restated from its
    published algorithm: ``_pairwisealigner.c`` NW/Gotoh global fill + first-path generator).
    Pinned by the 50 ``tests/test_align.py:49-163`` vectors (``tests/golden/align_tests.json``);
    tie order among equal-score paths is NOT pinned by any reference vector ("tie parity unpinned").
  * ``counts`` / metrics     <- ``src/itaxotools/taxi2/distances.py:282-348`` calling
    ``itaxotools.calculate_distances`` 0.1.1 (third-party Rust, absent); semantics inferred and
    pinned by ``tests/test_distances/metrics.tsv`` (26 rows x 4 metrics) and
    ``tests/test_distances.py:515-521`` (``tests/golden/metric_tests.json``).
  * ``ncd``                  <- ``src/itaxotools/taxi2/distances.py:351-358`` calling alfpy 1.0.6
    ``ncd.Distance(SeqRecords((0, 1), (x, y))).pairwise_distance(0, 1)`` (third-party, absent;
    restated: SeqRecords upper-cases, complexity = len(zlib.compress(s.encode())), default level).
    zlib itself is this interpreter's zlib 1.2.11 -- the same library alfpy calls.  No reference
    test pins an NCD value: parity for NCD is pinned to zlib 1.2.11's own output only.

Pure-Python loops: use it for small cases only (golden vectors, < ~300 bp pairs).
"""

from __future__ import annotations

import math
from typing import NamedTuple

NEG_INF = float("-inf")

# --------------------------------------------------------------------------- A1
_TR_NORMALIZE = str.maketrans("?", "N", "-")


def normalize(seq: str) -> str:
    """``Sequence.normalize`` (sequences.py:20-25): '?'->'N', delete '-', upper()."""
    return seq.translate(_TR_NORMALIZE).upper()


# --------------------------------------------------------------------------- A4
class Scores(NamedTuple):
    """``align.py:17-35`` defaults; field order = ``Scores.defaults`` key order."""

    match_score: int = 1
    mismatch_score: int = -1
    internal_open_gap_score: int = -8
    internal_extend_gap_score: int = -1
    end_open_gap_score: int = -1
    end_extend_gap_score: int = -1

    def is_linear(self) -> bool:
        """Biopython ``_get_algorithm``: NW/SW when every open == extend, else Gotoh."""
        return (
            self.internal_open_gap_score == self.internal_extend_gap_score
            and self.end_open_gap_score == self.end_extend_gap_score
        )


# --------------------------------------------------------------------------- A8
NUC = frozenset("ACGTacgt")
_BASE = {"A": 0, "C": 1, "G": 2, "T": 3, "a": 0, "c": 1, "g": 2, "t": 3}


class Counts(NamedTuple):
    valid: int
    ts: int
    tv: int
    gap: int

    @property
    def mism(self) -> int:
        return self.ts + self.tv


def nuc_span(s: str) -> tuple[int, int]:
    """(first, last) index of an ACGT letter; (len+1, -1) when there is none."""
    first = next((k for k, c in enumerate(s) if c in NUC), len(s) + 1)
    last = next((k for k in range(len(s) - 1, -1, -1) if s[k] in NUC), -1)
    return first, last


def counts(x: str, y: str) -> Counts:
    """Column counters of two aligned strings (calc ``seq_distances_*`` semantics, A8).

    Common range = [max(first Nuc of x, of y), min(last Nuc of x, of y)], zip-truncated to
    the shorter string.  Inside it: both Nuc -> valid (+ts for A<->G / C<->T, +tv otherwise
    when the bases differ); one '-' against a Nuc -> gap.  Everything else is ignored.
    """
    fx, lx = nuc_span(x)
    fy, ly = nuc_span(y)
    lo, hi = max(fx, fy), min(lx, ly, len(x) - 1, len(y) - 1)
    valid = ts = tv = gap = 0
    for k in range(lo, hi + 1):
        a, b = x[k], y[k]
        an, bn = a in NUC, b in NUC
        if an and bn:
            valid += 1
            d = _BASE[a] ^ _BASE[b]
            if d == 2:
                ts += 1
            elif d:
                tv += 1
        elif (a == "-" and bn) or (b == "-" and an):
            gap += 1
    return Counts(valid, ts, tv, gap)


def _div(a: float, b: float) -> float:
    return a / b if b else math.nan


def _log(v: float) -> float:
    if v > 0:
        return math.log(v)
    return -math.inf if v == 0 else math.nan


def metric_value(label: str, c: Counts) -> float:
    """f64 metric from counters; NaN/inf mean 'undefined' (wrapped to None, distances.py:291)."""
    if label == "p":
        return _div(c.mism, c.valid)
    if label == "p-gaps":
        return _div(c.mism + c.gap, c.valid + c.gap)
    if label == "jc":
        p = _div(c.mism, c.valid)
        if math.isnan(p):
            return p
        return -0.75 * _log(1.0 - (4.0 / 3.0) * p)
    if label == "k2p":
        if not c.valid:
            return math.nan
        P = c.ts / c.valid
        Q = c.tv / c.valid
        return -0.5 * _log(1.0 - 2.0 * P - Q) - 0.25 * _log(1.0 - 2.0 * Q)
    raise KeyError(label)


def metric(label: str, x: str, y: str) -> float | None:
    """``DistanceMetric.<label>.calculate(x, y).d`` for already aligned / raw strings."""
    v = metric_value(label, counts(x, y))
    return None if (math.isnan(v) or math.isinf(v)) else v


# --------------------------------------------------------------------------- A5-A7
M_, IX, IY = 1, 2, 4  # Biopython trace bits (M, Ix, Iy); NW uses D=M_, V=IX, H=IY


def _gotoh(x: str, y: str, sc: Scores, swapped: bool):
    nA, nB = len(x), len(y)
    o, e = sc.internal_open_gap_score, sc.internal_extend_gap_score
    eo, ee = sc.end_open_gap_score, sc.end_extend_gap_score
    M = [[NEG_INF] * (nB + 1) for _ in range(nA + 1)]
    X = [[NEG_INF] * (nB + 1) for _ in range(nA + 1)]
    Y = [[NEG_INF] * (nB + 1) for _ in range(nA + 1)]
    tM = [[0] * (nB + 1) for _ in range(nA + 1)]
    tX = [[0] * (nB + 1) for _ in range(nA + 1)]
    tY = [[0] * (nB + 1) for _ in range(nA + 1)]
    M[0][0] = 0
    for j in range(1, nB + 1):
        Y[0][j] = eo + ee * (j - 1)
        tY[0][j] = M_ if j == 1 else IY
    for i in range(1, nA + 1):
        X[i][0] = eo + ee * (i - 1)
        tX[i][0] = M_ if i == 1 else IX

    def sel(a, b, c):
        best = max(a, b, c)
        t = (M_ if a == best else 0) | (IX if b == best else 0) | (IY if c == best else 0)
        return best, t

    for i in range(1, nA + 1):
        for j in range(1, nB + 1):
            s = sc.match_score if x[i - 1] == y[j - 1] else sc.mismatch_score
            best, t = sel(M[i - 1][j - 1], X[i - 1][j - 1], Y[i - 1][j - 1])
            M[i][j], tM[i][j] = best + s, t
            ox, ex = (eo, ee) if j == nB else (o, e)
            X[i][j], tX[i][j] = sel(M[i - 1][j] + ox, X[i - 1][j] + ex, Y[i - 1][j] + ox)
            oy, ey = (eo, ee) if i == nA else (o, e)
            Y[i][j], tY[i][j] = sel(M[i][j - 1] + oy, X[i][j - 1] + oy, Y[i][j - 1] + ey)

    order = (M_, IY, IX) if swapped else (M_, IX, IY)
    best = max(M[nA][nB], X[nA][nB], Y[nA][nB])
    end = {M_: M[nA][nB], IX: X[nA][nB], IY: Y[nA][nB]}
    state = next(s for s in order if end[s] == best)
    # Traceback from (nA, nB): each step takes the first predecessor in priority order.
    cols = []
    i, j = nA, nB
    while i > 0 or j > 0:
        trace = {M_: tM, IX: tX, IY: tY}[state][i][j]
        if state == M_:
            cols.append((x[i - 1], y[j - 1]))
            i, j = i - 1, j - 1
        elif state == IX:
            cols.append((x[i - 1], "-"))
            i -= 1
        else:
            cols.append(("-", y[j - 1]))
            j -= 1
        if i == 0 and j == 0:
            break
        state = next(s for s in order if trace & s)
    cols.reverse()
    return "".join(c[0] for c in cols), "".join(c[1] for c in cols), best


def _nw(x: str, y: str, sc: Scores, swapped: bool):
    nA, nB = len(x), len(y)
    e, ee = sc.internal_extend_gap_score, sc.end_extend_gap_score
    S = [[0] * (nB + 1) for _ in range(nA + 1)]
    T = [[0] * (nB + 1) for _ in range(nA + 1)]
    D, V, H = M_, IX, IY
    for j in range(1, nB + 1):
        S[0][j], T[0][j] = j * ee, H
    for i in range(1, nA + 1):
        S[i][0], T[i][0] = i * ee, V
    for i in range(1, nA + 1):
        for j in range(1, nB + 1):
            s = sc.match_score if x[i - 1] == y[j - 1] else sc.mismatch_score
            d = S[i - 1][j - 1] + s
            v = S[i - 1][j] + (ee if j == nB else e)
            h = S[i][j - 1] + (ee if i == nA else e)
            best = max(d, v, h)
            S[i][j] = best
            T[i][j] = (D if d == best else 0) | (V if v == best else 0) | (H if h == best else 0)
    order = (V, H, D) if swapped else (H, V, D)
    cols = []
    i, j = nA, nB
    while i > 0 or j > 0:
        mv = next(s for s in order if T[i][j] & s)
        if mv == D:
            cols.append((x[i - 1], y[j - 1]))
            i, j = i - 1, j - 1
        elif mv == V:
            cols.append((x[i - 1], "-"))
            i -= 1
        else:
            cols.append(("-", y[j - 1]))
            j -= 1
    cols.reverse()
    return "".join(c[0] for c in cols), "".join(c[1] for c in cols), S[nA][nB]


def align(x: str, y: str, scores: Scores = Scores(), swapped: bool = False):
    """First global alignment of target ``x`` vs query ``y`` -> (aligned_x, aligned_y, score).

    ``swapped=True`` gives the (x, y) view of the alignment Biopython returns for target=y,
    query=x (fill identical with Ix<->Iy exchanged, so only the tie priority changes).
    """
    if scores.is_linear():
        return _nw(x, y, scores, swapped)
    return _gotoh(x, y, scores, swapped)


def aligned_counts(x: str, y: str, scores: Scores = Scores()) -> tuple[Counts, Counts, int]:
    """(counts of (x,y), counts of (y,x), score) through explicit traceback + ``counts``."""
    ax, ay, score = align(x, y, scores)
    bx, by, score_b = align(x, y, scores, swapped=True)
    assert score == score_b
    return counts(ax, ay), counts(by, bx), int(score)


METRICS = ("p", "p-gaps", "jc", "k2p")


# --------------------------------------------------------------------------- A9
def complexity(s: str) -> int:
    """alfpy ``ncd.complexity``: size of the zlib-compressed (default level) encoded string."""
    import zlib

    return len(zlib.compress(s.encode()))


def ncd(x: str, y: str) -> float:
    """alfpy ``ncd.Distance.pairwise_distance`` on ``SeqRecords`` (upper-cased) x, y."""
    X, Y = x.upper(), y.upper()
    c1, c2, c12 = float(complexity(X)), float(complexity(Y)), float(complexity(X + Y))
    return (c12 - min(c1, c2)) / max(c1, c2)


# --------------------------------------------------------------------------- A10
class Replicate(NamedTuple):
    query_id: str
    query_length: int
    included: tuple  # (id, length, distance)
    excluded: tuple


def dereplicate(items: list[tuple[str, int]], dist, similarity: float):
    """Dereplicate's greedy walk (``tasks/dereplicate.py:180-196, 289-337, 393-425``), restated as
    one explicit loop instead of the reference's lazily pulled generator chain.

    ``items`` = (id, unaligned length) of the sequences that passed the length filter, in input
    order; ``dist(i, j)`` = the (already x100-adjusted) distance of the ordered pair or None.
    The reference pulls pair k of the x-major product only after every earlier pair has been
    through ``find_replicates``, so each pair is tested against the exclusions made so far;
    groups are runs of consecutive pairs with equal x id.  Returns (summary lines, the surviving
    pairs in order, the final excluded set)."""
    excluded: set[str] = set()
    lines: list[Replicate] = []
    kept: list[tuple[int, int]] = []
    group = None  # [query id, query length, best (id, length, distance)]
    for i, (xi, lx) in enumerate(items):
        for j, (yj, ly) in enumerate(items):
            if xi == yj or xi in excluded or yj in excluded:
                continue
            kept.append((i, j))
            d = dist(i, j)
            if group is None or group[0] != xi:
                group = [xi, lx, (xi, lx, d)]  # the query, with its first pair's distance
            if d is None or not d <= similarity:
                continue
            best = group[2]
            if ly > best[1]:
                inc, exc = (yj, ly, d), best
                group[2] = inc
            else:
                inc, exc = best, (yj, ly, d)
            excluded.add(exc[0])
            lines.append(Replicate(group[0], group[1], inc, exc))
    return lines, kept, excluded


# --------------------------------------------------------------------------- A11
def subset_aggregates(ids: list[str], partition: dict, value, n_metrics: int) -> dict:
    """VersusAll's per-partition ``DistanceAggregator`` (``tasks/versus_all.py:57-96, 617-640``):
    over the ordered product x-major, key (partition.get(id_x), partition.get(id_y)) in first-seen
    order; per metric ``[sum, min, max, count]`` with min from +inf, max from 0.0, None skipped and
    the sum accumulated in visiting order.  ``value(i, j, k)`` -> float or None."""
    aggs: dict = {}
    n = len(ids)
    for i in range(n):
        for j in range(n):
            key = (partition.get(ids[i], None), partition.get(ids[j], None))
            acc = aggs.setdefault(key, [[0.0, math.inf, 0.0, 0] for _ in range(n_metrics)])
            for k in range(n_metrics):
                v = value(i, j, k)
                if v is None:
                    continue
                a = acc[k]
                a[0] += v
                if v < a[1]:
                    a[1] = v
                if v > a[2]:
                    a[2] = v
                a[3] += 1
    return aggs
