"""Pairwise aligners (``src/itaxotools/taxi2/align.py``), GPU-backed.

``PairwiseAligner.Biopython`` keeps the reference's name and contract -- the first global
alignment Biopython 1.85 ``PairwiseAligner(**scores).align(x, y)[0]`` returns, as gapped
strings (``align.py:72-157``) -- but computes it with the MI355X engine (trace fill + walk,
``taxi2_amd/csrc/trace_kernel.hpp``).  ``align_pairs`` aligns a whole batch per engine call.
``PairwiseAligner.Rust`` (the unused calculate_distances aligner, ``align.py:54-69``) is out of
scope.
"""

from __future__ import annotations

from typing import Iterable, Iterator

import numpy as np

from .pairs import SequencePair, SequencePairs
from .sequences import Sequence
from .types import Type


class Scores(dict):
    """Can access keys like attributes (``align.py:17-35``)."""

    defaults = dict(
        match_score=1,
        mismatch_score=-1,
        internal_open_gap_score=-8,
        internal_extend_gap_score=-1,
        end_open_gap_score=-1,
        end_extend_gap_score=-1,
    )

    def __init__(self, **kwargs):
        super().__init__(self.defaults | kwargs)
        self.__dict__ = self

    def __repr__(self) -> str:
        return f"<{type(self).__name__}: " + ", ".join(f"{k}={v}" for k, v in self.items()) + ">"

    def as_tuple(self) -> tuple[int, ...]:
        return tuple(self[k] for k in self.defaults)


class PairwiseAligner(Type):
    def __init__(self, scores: Scores = None):
        self.scores = scores or Scores()

    def align(self, pair: SequencePair) -> SequencePair:
        raise NotImplementedError()

    def align_pairs(self, pairs: Iterable[SequencePair]) -> SequencePairs:
        return SequencePairs(self._align_stream(pairs))

    def align_product_rows(self, xs: list[Sequence], ys: list[Sequence], rows: range | None = None,
                           max_pairs: int = 1 << 16, sets: tuple | None = None) -> Iterator[list[SequencePair]]:
        """Row x of the x-major product xs x ys (``rows``: a range of x, default all), as the aligned
        pairs (x, y) for every y -- what ``align_many([SequencePair(x, y) for y in ys])`` gives per
        row, with both sides uploaded ONCE (not once per row; ``sets`` = (xs, ys) already uploaded
        by the caller with ``upload_sets``, kept) and up to ``max_pairs`` pairs per engine call."""
        rows = range(len(xs)) if rows is None else rows
        if not len(rows):
            return
        eng = self.engine
        own = sets is None
        sx, sy = self.upload_sets(xs, ys) if own else sets
        same = sx is sy
        sc = Scores(**self.scores).as_tuple()
        ny = len(ys)
        per = max(1, max_pairs // max(1, ny))
        try:
            for r0 in range(rows.start, rows.stop, per):
                r1 = min(rows.stop, r0 + per)
                xi = np.repeat(np.arange(r0, r1), ny)
                yi = np.tile(np.arange(ny), r1 - r0)
                strings = eng.align_strings(sx, sy, xi, yi, sc) if ny else []
                for i, x in enumerate(range(r0, r1)):
                    X = xs[x]
                    yield [SequencePair(Sequence(X.id, ax, X.extras), Sequence(Y.id, ay, Y.extras))
                           for Y, (ax, ay) in zip(ys, strings[i * ny:(i + 1) * ny])]
        finally:
            if own:
                sx.free()
                if not same:
                    sy.free()

    def upload_sets(self, xs: list[Sequence], ys: list[Sequence]) -> tuple:
        """The engine sets ``align_product_rows`` aligns from (one set when xs is ys)."""
        sx = self.engine.upload([s.seq for s in xs], align=True)
        return sx, (sx if xs is ys else self.engine.upload([s.seq for s in ys], align=True))

    def _align_stream(self, pairs: Iterable[SequencePair]) -> Iterator[SequencePair]:
        for pair in pairs:
            yield self.align(pair)


class Rust(PairwiseAligner):
    def __init__(self, scores: Scores = None):
        raise NotImplementedError("PairwiseAligner.Rust is out of scope for the MI355X engine")


class Biopython(PairwiseAligner):
    """First Biopython global alignment, computed on the GPU."""

    batch = 4096

    def __init__(self, scores: Scores = None, engine=None):
        super().__init__(scores)
        self._engine = engine

    @property
    def engine(self):
        from ._native import Engine

        if self._engine is None:
            self._engine = Engine.default()
        return self._engine

    def align(self, pair: SequencePair) -> SequencePair:
        return self.align_many([pair])[0]

    def align_many(self, pairs: list[SequencePair]) -> list[SequencePair]:
        if not pairs:
            return []
        eng = self.engine
        xs = [p.x.seq for p in pairs]
        ys = [p.y.seq for p in pairs]
        st = eng.upload(xs + ys, align=True)
        n = len(pairs)
        try:
            strings = eng.align_strings(st, st, np.arange(n), np.arange(n) + n, Scores(**self.scores).as_tuple())
        finally:
            st.free()
        return [
            SequencePair(Sequence(p.x.id, ax, p.x.extras), Sequence(p.y.id, ay, p.y.extras))
            for p, (ax, ay) in zip(pairs, strings)
        ]

    def _align_stream(self, pairs: Iterable[SequencePair]) -> Iterator[SequencePair]:
        buf: list[SequencePair] = []
        for pair in pairs:
            buf.append(pair)
            if len(buf) >= self.batch:
                yield from self.align_many(buf)
                buf = []
        if buf:
            yield from self.align_many(buf)
