"""Distances and distance metrics (``src/itaxotools/taxi2/distances.py``), GPU-backed.

* ``DistanceMetric`` registry with the reference labels ``p``, ``p-gaps``, ``jc``, ``k2p``,
  ``ncd``, ``bbc(k)`` and ``fromLabel`` parsing (``distances.py:282-312``).
* ``calculate(x, y) -> Distance`` keeps the reference's per-pair signature
  (``distances.py:297-298``) and its None rule for NaN/inf (``distances.py:290-292``), but the
  value comes from the MI355X engine (a batch of one).  Bulk callers use
  :func:`calculate_many`, one engine call for any number of pairs.
* Writers ``DistanceHandler.Linear`` / ``Matrix`` / ``Linear.WithExtras`` reproduce the
  reference's tab-separated formats (``distances.py:34-279``, fixtures under tests/golden).
* NCD (``distances.py:351-358`` -> alfpy 1.0.6 ``ncd``) runs on the GPU with zlib-1.2.11-exact
  compressed lengths (``taxi2_ncd_pairs``); BBC is a label only (out of scope).
"""

from __future__ import annotations

import math
import re
from pathlib import Path
from typing import Iterable, NamedTuple

import numpy as np

from .handlers import FileHandler, Tabfile as _TabRows
from .sequences import Sequence
from .types import Container, Type


class Distance(NamedTuple):
    metric: "DistanceMetric"
    x: Sequence
    y: Sequence
    d: float | None


class Distances(Container[Distance]):
    @classmethod
    def fromPath(cls, path: Path, handler: type, *args, **kwargs) -> "Distances":
        return cls(handler, path, "r", *args, **kwargs)


# ============================================================================ metrics
class DistanceMetric(Type):
    """Metrics for calculating distances."""

    label: str

    def __str__(self) -> str:
        return self.label

    @staticmethod
    def _is_number(x) -> bool:
        return not (x is None or math.isnan(x) or math.isinf(x))

    def calculate(self, x: Sequence, y: Sequence) -> Distance:
        return Distance(self, x, y, self._calculate(x.seq, y.seq))

    def _calculate(self, x: str, y: str) -> float | None:
        vals = calculate_many([self], [x], [y])
        v = float(vals[0, 0])
        return v if self._is_number(v) else None

    @classmethod
    def fromLabel(cls, label: str):
        arg = None
        m = re.search(r"(\w+)\((\d+)\)", label)
        if m:
            label = m.group(1) + "({})"
            arg = m.group(2)
        for child in cls:
            if label == child.label:
                return child(int(arg)) if arg else child()
        return None


class Unknown(DistanceMetric):
    label = "?"

    def _calculate(self, x: str, y: str):
        raise NotImplementedError("unknown metric")


class Uncorrected(DistanceMetric):
    label = "p"


class UncorrectedWithGaps(DistanceMetric):
    label = "p-gaps"


class JukesCantor(DistanceMetric):
    label = "jc"


class Kimura2P(DistanceMetric):
    label = "k2p"


class NCD(DistanceMetric):
    """alfpy 1.0.6 ``ncd.Distance(SeqRecords((0, 1), (x, y))).pairwise_distance(0, 1)``
    (``distances.py:351-358``): (C(X+Y) - min(C(X), C(Y))) / max(C(X), C(Y)) with X, Y the
    upper-cased strings and C = len(zlib.compress(.)) -- computed by the engine."""

    label = "ncd"


class BBC(DistanceMetric):
    label = "bbc({})"

    def __init__(self, k: int = 10):
        self.k = k

    def __str__(self) -> str:
        return self.label.format(self.k)

    def __eq__(self, other) -> bool:
        return super().__eq__(other) and self.k == other.k

    def __hash__(self) -> int:
        return hash((type(self), self.k))

    def _calculate(self, x: str, y: str):
        raise NotImplementedError("BBC is out of scope for the MI355X engine (SURVEY.md §2 row 4)")


COUNTER_LABELS = ("p", "p-gaps", "jc", "k2p")  # alignment-column counters (one kernel pass)
ENGINE_LABELS = COUNTER_LABELS + ("ncd",)


def engine_metric(metric: DistanceMetric) -> bool:
    return str(metric) in ENGINE_LABELS


def check_ncd_strings(strings) -> None:
    """The reference compresses ``str.upper().encode()`` (UTF-8).  The engine stores one latin-1
    byte per character and compresses its UTF-8 upper case (``deflate_len.hpp upper_utf8``: "é" ->
    "É" as two bytes, "ß" -> "SS", "ÿ" -> "Ÿ"), which is the same for every character up to
    U+00FF; a character past latin-1 has no stored byte, so it is refused instead of silently
    differing."""
    for s in strings:
        if not s.isascii() and any(ord(c) > 0xFF for c in s):
            raise ValueError("NCD on the MI355X engine needs latin-1 sequences (characters up to U+00FF)")


def calculate_many(metrics: Iterable[DistanceMetric], xs: list[str], ys: list[str], *, engine=None) -> np.ndarray:
    """Pre-aligned distances for pairs (xs[k], ys[k]): (count, M) float64, NaN/inf = None.

    One engine call per kind of metric for the whole batch; replaces ``count x M`` Rust / alfpy
    calls (``distances.py:323-358``)."""
    from ._native import Engine

    metrics = list(metrics)
    for m in metrics:
        if not engine_metric(m):
            m._calculate("", "")  # raises the metric's NotImplementedError
    if len(xs) != len(ys):
        raise ValueError("xs and ys differ in length")
    eng = engine or Engine.default()
    n = len(xs)
    labels = [str(m) for m in metrics]
    out = np.empty((n, len(labels)))
    cidx = [k for k, lab in enumerate(labels) if lab != "ncd"]
    nidx = [k for k, lab in enumerate(labels) if lab == "ncd"]
    if nidx:
        check_ncd_strings(xs)
        check_ncd_strings(ys)
    s = eng.upload(list(xs) + list(ys), align=False)
    try:
        if cidx:
            out[:, cidx] = eng.list_pairs(s, s, np.arange(n), np.arange(n) + n, [labels[k] for k in cidx])
        if nidx:
            v = eng.ncd_pairs(s, s, np.arange(n), np.arange(n) + n, aligned=False, both=False)
            for k in nidx:
                out[:, k] = v
    finally:
        s.free()
    return out


def to_optional(v: float) -> float | None:
    return v if (v == v and v not in (math.inf, -math.inf)) else None


# ============================================================================ handlers
class DistanceHandler(FileHandler):
    def __init__(self, path: Path, mode: str = "r", missing: str = "NA", formatter: str = "{:f}", *args, **kwargs):
        self.missing = missing
        self.formatter = formatter
        super().__init__(path, mode, *args, **kwargs)

    def distanceFromText(self, text: str) -> float | None:
        return None if text == self.missing else float(text)

    def distanceToText(self, d: float | None) -> str:
        return self.missing if d is None else self.formatter.format(d)


class _LineWriter:
    """Groups consecutive distances into output lines (reference ``_assemble_line``)."""

    def _open_writer(self, *args, **kwargs):
        self._fh = open(self.path, "w")
        self._line: list[Distance] = []
        self._wrote_headers = False

    def _same_line(self, a: Distance, b: Distance) -> bool:
        raise NotImplementedError

    def _write_item(self, d: Distance) -> None:
        if self._line and not self._same_line(self._line[0], d):
            self._flush()
        self._line.append(d)

    def _flush(self) -> None:
        if not self._line:
            return
        if not self._wrote_headers:
            self._write_headers(self._line)
            self._wrote_headers = True
        self._write_scores(self._line)
        self._line = []

    def _close_writer(self) -> None:
        self._flush()
        self._fh.close()

    def _row(self, fields) -> None:
        self._fh.write("\t".join(fields) + "\n")


class Linear(_LineWriter, DistanceHandler):
    """``idx  idy  <metric>...`` one line per (x, y) (distances.py:59-123)."""

    def _read_items(self):
        rows = _TabRows(self.path, "r", has_headers=True)
        it = iter(rows)
        first = next(it, None)
        headers = rows.header_row
        if headers is None:
            return
        metrics = [DistanceMetric.fromLabel(h) for h in headers[2:]]
        for row in ([first] if first is not None else []) + list(it):
            for text, metric in zip(row[2:], metrics):
                yield Distance(metric, Sequence(row[0], None), Sequence(row[1], None), self.distanceFromText(text))

    def _same_line(self, a: Distance, b: Distance) -> bool:
        return a.x.id == b.x.id and a.y.id == b.y.id

    def _write_headers(self, line: list[Distance]) -> None:
        self._row(("idx", "idy", *[str(d.metric) for d in line]))

    def _write_scores(self, line: list[Distance]) -> None:
        self._row((line[0].x.id, line[0].y.id, *[self.distanceToText(d.d) for d in line]))


class Matrix(_LineWriter, DistanceHandler):
    """Square / rectangular matrix, one row per x (distances.py:126-186)."""

    def _read_items(self, metric: DistanceMetric = None):
        metric = metric or DistanceMetric.Unknown()
        rows = _TabRows(self.path, "r", has_headers=True)
        it = iter(rows)
        first = next(it, None)
        headers = rows.header_row
        if headers is None:
            return
        idys = headers[1:]
        for row in ([first] if first is not None else []) + list(it):
            sx = Sequence(row[0], None)
            for text, idy in zip(row[1:], idys):
                yield Distance(metric, sx, Sequence(idy, None), self.distanceFromText(text))

    def _same_line(self, a: Distance, b: Distance) -> bool:
        return a.x.id == b.x.id

    def _write_headers(self, line: list[Distance]) -> None:
        self._row(("", *[d.y.id for d in line]))

    def _write_scores(self, line: list[Distance]) -> None:
        self._row((line[0].x.id, *[self.distanceToText(d.d) for d in line]))


class WithExtras(Linear):
    """``seqid (query)  <extras x>  seqid (reference)  <extras y>  <metrics>``
    (distances.py:189-279)."""

    def __init__(self, path: Path, mode: str = "r", missing: str = "NA", formatter: str = "{:f}", *args, **kwargs):
        super().__init__(path, mode, missing, formatter, *args, **kwargs)

    def _open_writer(self, idxHeader: str = "seqid", idyHeader: str = "seqid", tagX: str = " (query)",
                     tagY: str = " (reference)"):
        super()._open_writer()
        self.idxHeader, self.idyHeader, self.tagX, self.tagY = idxHeader, idyHeader, tagX, tagY

    def _read_items(self, idxHeader: str = None, idyHeader: str = None, tagX: str = " (query)",
                    tagY: str = " (reference)", idxColumn: int = 0, idyColumn: int = 1):
        rows = _TabRows(self.path, "r", has_headers=True)
        it = iter(rows)
        first = next(it, None)
        headers = rows.header_row
        if headers is None:
            return
        if idxHeader and idyHeader:
            idxColumn = headers.index(idxHeader + tagX)
            idyColumn = headers.index(idyHeader + tagY)
        starts = [k for k, h in enumerate(headers) if DistanceMetric.fromLabel(h)]
        if not starts:
            raise Exception("No metrics found in the header line!")
        m0 = starts[0]
        sx, sy = slice(idxColumn + 1, idyColumn), slice(idyColumn + 1, m0)
        metrics = [DistanceMetric.fromLabel(h) for h in headers[m0:]]
        kx = [h.removesuffix(tagX) for h in headers[sx]]
        ky = [h.removesuffix(tagY) for h in headers[sy]]
        for row in ([first] if first is not None else []) + list(it):
            ex = dict(zip(kx, row[sx]))
            ey = dict(zip(ky, row[sy]))
            for text, metric in zip(row[m0:], metrics):
                yield Distance(metric, Sequence(row[idxColumn], None, ex), Sequence(row[idyColumn], None, ey),
                               self.distanceFromText(text))

    def _write_headers(self, line: list[Distance]) -> None:
        ex = [k + self.tagX for k in line[0].x.extras.keys()]
        ey = [k + self.tagY for k in line[0].y.extras.keys()]
        self._row((self.idxHeader + self.tagX, *ex, self.idyHeader + self.tagY, *ey, *[str(d.metric) for d in line]))

    def _write_scores(self, line: list[Distance]) -> None:
        ex = [v if v is not None else self.missing for v in line[0].x.extras.values()]
        ey = [v if v is not None else self.missing for v in line[0].y.extras.values()]
        self._row((line[0].x.id, *ex, line[0].y.id, *ey, *[self.distanceToText(d.d) for d in line]))
