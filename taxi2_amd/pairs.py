"""Sequence pairs (``src/itaxotools/taxi2/pairs.py``), host side.

``SequencePairs.fromProduct`` defines the output order of versusAll / versusReference:
x outer, y inner (``pairs.py:23-25``, pinned by ``tests/test_pairs.py:92-112``).  The GPU
tasks never materialize the product; they use the same order when emitting results.
"""

from __future__ import annotations

from pathlib import Path
from typing import NamedTuple

from .handlers import FileHandler, Tabfile as _TabRows
from .sequences import Sequence, Sequences
from .types import Container


class SequencePair(NamedTuple):
    x: Sequence
    y: Sequence


class SequencePairs(Container[SequencePair]):
    @classmethod
    def fromPath(cls, path: Path, handler: type, *args, **kwargs) -> "SequencePairs":
        return cls(handler, path, "r", *args, **kwargs)

    @classmethod
    def fromProduct(cls, xs: Sequences, ys: Sequences) -> "SequencePairs":
        return cls(lambda: (SequencePair(x, y) for x in xs for y in ys))


class SequencePairHandler(FileHandler):
    pass


class Tabfile(SequencePairHandler):
    """``idx idy seqx seqy`` rows (pairs.py:32-48)."""

    def _read_items(self):
        rows = _TabRows(self.path, "r", has_headers=True)
        for idx, idy, sx, sy in rows:
            yield SequencePair(Sequence(idx, sx), Sequence(idy, sy))

    def _open_writer(self):
        self._fh = open(self.path, "w")
        self._fh.write("\t".join(("idx", "idy", "seqx", "seqy")) + "\n")

    def _write_item(self, pair: SequencePair) -> None:
        self._fh.write("\t".join((pair.x.id, pair.y.id, pair.x.seq, pair.y.seq)) + "\n")

    def _close_writer(self) -> None:
        self._fh.close()


def format_pattern(x: str, y: str) -> str:
    """Middle line of aligned_pairs.txt: '|' identical non-gap, '-' any gap, '.' otherwise
    (pairs.py:59-69)."""
    out = []
    for a, b in zip(x, y):
        if a == b and a != "-":
            out.append("|")
        elif a == "-" or b == "-":
            out.append("-")
        else:
            out.append(".")
    return "".join(out)


class Formatted(SequencePairHandler):
    """Blocks of ``idx / idy``, aligned x, pattern, aligned y, separated by blank lines
    (pairs.py:51-97)."""

    def _read_items(self):
        with open(self.path, "r") as fh:
            while True:
                lines = [fh.readline().strip() for _ in range(5)]
                if not any(lines):
                    return
                idx, idy = lines[0].split(" / ")
                yield SequencePair(Sequence(idx, lines[1]), Sequence(idy, lines[3]))

    def _open_writer(self):
        self._fh = open(self.path, "w")
        self._first = True

    def _write_item(self, pair: SequencePair) -> None:
        if not self._first:
            self._fh.write("\n")
        self._first = False
        self._fh.write(f"{pair.x.id} / {pair.y.id}\n{pair.x.seq}\n{format_pattern(pair.x.seq, pair.y.seq)}\n{pair.y.seq}\n")

    def _close_writer(self) -> None:
        self._fh.close()
