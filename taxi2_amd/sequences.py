"""Sequence model (``src/itaxotools/taxi2/sequences.py``), host side.

``Sequence.normalize`` (``sequences.py:20-25``) is part of the hot path's contract: it is what
the aligner sees when ``params.pairs.align`` is on (``versus_all.py:522-525``).  The GPU
engine consumes the normalized strings as bytes.
"""

from __future__ import annotations

from pathlib import Path
from typing import NamedTuple

from .handlers import FileHandler, Tabfile as _TabRows, sanitize
from .types import Container

_NORMALIZE = str.maketrans("?", "N", "-")


class Sequence(NamedTuple):
    id: str
    seq: str
    extras: dict[str, str] = dict()

    def normalize(self) -> "Sequence":
        """'?' -> 'N', delete '-', upper-case (sequences.py:22-25)."""
        return Sequence(self.id, self.seq.translate(_NORMALIZE).upper(), self.extras)

    def get_sanitized_id_with_extras(self) -> str:
        return sanitize("_".join([self.id] + list(self.extras.values())))


class Sequences(Container[Sequence]):
    @classmethod
    def fromPath(cls, path: Path, handler: type, *args, **kwargs) -> "Sequences":
        return cls(handler, path, "r", *args, **kwargs)

    def normalize(self) -> "Sequences":
        return Sequences(lambda: (s.normalize() for s in self))


class SequenceHandler(FileHandler):
    pass


class Tabfile(SequenceHandler):
    """TAB-separated sequences (``sequences.py:172-234``): id / sequence columns chosen by
    header (``idHeader``/``seqHeader``) or index; every other column becomes an ``extras``
    entry keyed by its sanitized header."""

    def _read_items(self, idHeader: str = None, seqHeader: str = None, hasHeader: bool = False,
                    idColumn: int = 0, seqColumn: int = 1):
        if idHeader and seqHeader:
            columns = (idHeader, seqHeader)
            hasHeader = True
        else:
            columns = (idColumn, seqColumn)
        rows = _TabRows(self.path, "r", columns=columns, has_headers=hasHeader, get_all_columns=True)
        try:
            it = iter(rows)
            first = next(it, None)
            headers = rows.headers if hasHeader else None
            keys = [sanitize(h) for h in headers[2:]] if headers is not None else None
            if first is None:
                return
            for row in _chain1(first, it):
                extras = dict(zip(keys, row[2:])) if keys is not None else dict()
                yield Sequence(row[0], row[1], extras)
        finally:
            rows.close()

    def _open_writer(self, idHeader: str = None, seqHeader: str = None, hasHeader: bool = False):
        self._fh = open(self.path, "w")
        self._hdr = (idHeader, seqHeader) if (idHeader and seqHeader) else None
        self._wrote = False

    def _write_item(self, s: Sequence) -> None:
        if self._hdr and not self._wrote:
            self._fh.write("\t".join((self._hdr[0], *s.extras.keys(), self._hdr[1])) + "\n")
        self._wrote = True
        self._fh.write("\t".join((s.id, *s.extras.values(), s.seq)) + "\n")

    def _close_writer(self) -> None:
        if self._hdr and not self._wrote:
            self._fh.write("\t".join(self._hdr) + "\n")
        self._fh.close()


class Fasta(SequenceHandler):
    """Plain FASTA (``sequences.py:47-134``, without the organism variants)."""

    def _read_items(self):
        with open(self.path, "r") as fh:
            title, parts = None, []
            for line in fh:
                if line.startswith(">"):
                    if title is not None:
                        yield Sequence(title, "".join(parts))
                    title, parts = line[1:].rstrip(), []
                elif title is not None:
                    parts.append(line.strip().replace(" ", "").replace("\r", ""))
            if title is not None:
                yield Sequence(title, "".join(parts))

    def _open_writer(self, line_width: int = 60):
        self._fh = open(self.path, "w")
        self._w = line_width

    def _write_item(self, s: Sequence) -> None:
        self._fh.write(">" + s.id + "\n")
        if self._w:
            for k in range(0, len(s.seq), self._w):
                self._fh.write(s.seq[k : k + self._w] + "\n")
            self._fh.write("\n")
        else:
            self._fh.write(s.seq + "\n")

    def _close_writer(self) -> None:
        self._fh.close()


def _chain1(first, it):
    yield first
    yield from it
