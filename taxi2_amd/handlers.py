"""Tab-separated file I/O in the reference's FileHandler shape (host side, not hot path).

Public behaviour mirrors ``src/itaxotools/taxi2/handlers.py``:
  * ``Handler(path, "r"|"w", **options)`` is a context manager; readers are iterable and have
    ``read()``; writers have ``write(item)``; ``close()`` flushes (``handlers.py:24-103``);
  * ``Tabular`` selects columns by index or header name, optionally appending every other
    column in ascending order (``get_all_columns``), and exposes ``headers``
    (``handlers.py:106-207``);
  * ``Tabfile`` rows: every line loses its LAST character (``line[:-1]``, so a final line
    without a newline loses a real character, exactly as the reference), empty lines are
    skipped, fields split on TAB (``handlers.py:211-217``); rows are written TAB-joined.
Excel input (openpyxl) is out of scope.

Implementation: readers are plain generators and writers small stateful objects; there is no
generator-coroutine priming protocol.
"""

from __future__ import annotations

import re
import unicodedata
from pathlib import Path
from typing import Iterator

from .types import Type

Row = tuple


class FileHandler(Type):
    """Base reader/writer.  Subclasses implement ``_read_items`` and/or ``_writer``."""

    def __init__(self, path: Path, mode: str = "r", *args, **kwargs):
        if mode not in ("r", "w"):
            raise ValueError('Mode must be "r" or "w"')
        self.path = Path(path)
        self.mode = mode
        self.closed = False
        if mode == "r":
            self._it = iter(self._read_items(*args, **kwargs))
        else:
            self._open_writer(*args, **kwargs)

    # -- protocol
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __iter__(self):
        assert self.readable()
        return self

    def __next__(self):
        assert self.readable()
        return next(self._it)

    def read(self):
        try:
            return next(self._it)
        except StopIteration:
            return None

    def write(self, item) -> None:
        assert self.writable()
        self._write_item(item)

    def close(self) -> None:
        if not self.closed:
            if self.mode == "w":
                self._close_writer()
            else:
                close = getattr(self._it, "close", None)
                if close:
                    close()
            self.closed = True

    def readable(self) -> bool:
        return self.mode == "r"

    def writable(self) -> bool:
        return self.mode == "w"

    # -- to implement
    def _read_items(self, *args, **kwargs) -> Iterator:
        raise NotImplementedError

    def _open_writer(self, *args, **kwargs) -> None:
        raise NotImplementedError

    def _write_item(self, item) -> None:
        raise NotImplementedError

    def _close_writer(self) -> None:
        pass


class Tabular(FileHandler):
    """Rows of fields with optional header row and column selection."""

    def _rows(self) -> Iterator[Row]:
        raise NotImplementedError

    def _read_items(self, columns=None, has_headers: bool = False, get_all_columns: bool = False):
        if columns is not None:
            columns = tuple(columns)
            if not columns:
                raise ValueError("Columns argument must contain at least one item")
            if isinstance(columns[0], str):
                has_headers = True
        self.has_headers = has_headers
        self.header_row = None
        self.column_order = None
        rows = self._rows()
        if has_headers:
            self.header_row = next(rows, None)
            if self.header_row is None:
                return
        if columns is None:
            yield from rows
            return
        if isinstance(columns[0], str):
            missing = set(columns) - set(self.header_row)
            if missing:
                raise ValueError(f"Column header(s) not found in file: {missing}")
            columns = tuple(self.header_row.index(c) for c in columns)
        if get_all_columns:
            if self.has_headers:
                width = len(self.header_row)
            else:
                first = next(rows, None)
                if first is None:
                    self.column_order = columns
                    return
                width = len(first)
                rows = _prepend(first, rows)
            columns = columns + tuple(sorted(set(range(width)) - set(columns)))
        self.column_order = columns
        for row in rows:
            yield tuple(row[c] for c in columns)

    def _prime_headers(self):
        # Headers are known once the first item is pulled; pull lazily and keep it.
        if not hasattr(self, "has_headers"):
            first = self.read()
            if first is not None:
                self._it = _prepend(first, self._it)

    @property
    def headers(self) -> Row | None:
        assert self.readable()
        self._prime_headers()
        if not self.has_headers:
            return None
        if self.header_row is None:
            return None
        if self.column_order:
            return tuple(self.header_row[c] for c in self.column_order)
        return self.header_row

    def _open_writer(self, columns=None):
        self._fh = open(self.path, "w")
        if columns is not None:
            columns = tuple(columns)
            if not columns:
                raise ValueError("Columns argument must contain at least one item")
            self._write_item(columns)

    def _write_item(self, row) -> None:
        self._fh.write("\t".join(row) + "\n")

    def _close_writer(self) -> None:
        self._fh.close()

    @classmethod
    def get_headers(cls, path: Path) -> Row:
        with cls(path) as handler:
            return handler.read()


class Tabfile(Tabular, FileHandler):
    def _rows(self) -> Iterator[Row]:
        with open(self.path, "r", encoding="utf-8", errors="surrogateescape") as fh:
            for line in fh:
                line = line[:-1]
                if line:
                    yield tuple(line.split("\t"))


def _prepend(first, it):
    yield first
    yield from it


# ----------------------------------------------------------------------------- sanitize
_MULTI = {
    "Ä": "Ae", "Ö": "Oe", "Ü": "Ue", "ä": "ae", "ö": "oe", "ü": "ue", "ß": "ss", "Æ": "Ae",
    "æ": "ae", "Œ": "OE", "œ": "oe", "Þ": "Th", "þ": "th",
}


def _ascii_fold(text: str) -> str:
    out = []
    for ch in text:
        if ch in _MULTI:
            out.append(_MULTI[ch])
            continue
        if ord(ch) < 128:
            out.append(ch)
            continue
        base = unicodedata.normalize("NFKD", ch)
        folded = "".join(c for c in base if not unicodedata.combining(c))
        out.append(folded if folded and all(ord(c) < 128 for c in folded) else ch)
    return "".join(out)


def sanitize(text: str) -> str:
    """``encoding.py:sanitize``: fold accented letters to ASCII, drop leading punctuation and
    replace remaining runs of non-word characters with '_'."""
    text = _ascii_fold(unicodedata.normalize("NFKC", text))
    text = re.sub(r"^[^\w ]+", "", text)
    return re.sub(r"[^\w ]+", "_", text)
