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
