"""Partitions: individual -> subset maps (``src/itaxotools/taxi2/partitions.py``), the species /
genera inputs of VersusAll's summary and subset aggregation (``versus_all.py:272-275, 605-684``).

``Partition`` is a dict; ``Partition.fromPath(path, PartitionHandler.X, **kw)`` reads one with
  * ``Tabfile``: columns by header name (``idHeader`` + ``subHeader``, header row implied) or by
    index (``idColumn`` / ``subColumn``, ``hasHeader``) (``partitions.py:78-106``);
  * ``Fasta``: ``>individual<separator>subset`` titles, separator ``|`` by default; titles without
    the separator are skipped with a message (``partitions.py:125-157``);
and an optional ``filter(Classification) -> Classification | None`` applied to every row
(``subset_first_word`` keeps the subset's first word and drops single-word subsets,
``partitions.py:63-72``).  Spart (``itaxotools.spart_parser``) and Excel (openpyxl) need
libraries this image does not have: they raise.
"""

from __future__ import annotations

from pathlib import Path
from typing import Callable, Iterator, NamedTuple

from .handlers import FileHandler


class Classification(NamedTuple):
    individual: str
    subset: str


class Partition(dict):
    """Keys are individuals, values are subsets."""

    @classmethod
    def fromPath(cls, path: Path, handler: type, *args, **kwargs) -> "Partition":
        return handler.as_dict(path, *args, **kwargs)


def _fasta_titles(path: Path) -> Iterator[str]:
    """Titles of a FASTA file as Biopython's SimpleFastaParser yields them: text before the first
    '>' is ignored, a title is its line after '>' with trailing whitespace removed."""
    with open(path, "r") as fh:
        for line in fh:
            if line.startswith(">"):
                yield line[1:].rstrip()


class PartitionHandler:
    def __init__(self, path: Path, mode: str = "r", filter: Callable | None = None, *args, **kwargs):
        if mode != "r":
            raise NotImplementedError("partitions are read-only")
        self.path = Path(path)
        self.filter = filter
        self._args, self._kwargs = args, kwargs

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return None

    def __iter__(self) -> Iterator[Classification]:
        for c in self._classifications(*self._args, **self._kwargs):
            if self.filter:
                c = self.filter(c)
            if c is None:
                continue
            yield c

    def _classifications(self, *args, **kwargs) -> Iterator[Classification]:
        raise NotImplementedError

    @classmethod
    def as_dict(cls, path: Path, *args, **kwargs) -> Partition:
        part = Partition()
        for individual, subset in cls(path, "r", *args, **kwargs):
            part[individual] = subset
        return part

    @staticmethod
    def subset_first_word(c: Classification) -> Classification | None:
        parts = c.subset.split(" ", 1)
        if len(parts) < 2:
            print(f"Cannot split subset {c.subset} for individual {c.individual}")
            return None
        return Classification(c.individual, parts[0])


class Tabfile(PartitionHandler):
    def _classifications(self, idHeader: str = None, subHeader: str = None, hasHeader: bool = False,
                         idColumn: int = 0, subColumn: int = 1) -> Iterator[Classification]:
        if idHeader and subHeader:
            columns, hasHeader = (idHeader, subHeader), True
        else:
            columns = (idColumn, subColumn)
        with FileHandler.Tabfile(self.path, "r", columns=columns, has_headers=hasHeader) as rows:
            for individual, subset in rows:
                yield Classification(individual, subset)


class Fasta(PartitionHandler):
    def _classifications(self, separator: str = "|") -> Iterator[Classification]:
        for title in _fasta_titles(self.path):
            parts = title.split(separator, 1)
            if len(parts) < 2:
                print(f"Could not extract partition info from fasta line: {title}")
                continue
            yield Classification(parts[0], parts[1])

    @classmethod
    def has_subsets(cls, path: Path, separator: str = "|") -> bool:
        if not separator:
            return False
        for title in _fasta_titles(path):
            return len(title.split(separator, 1)) == 2
        return None

    @classmethod
    def guess_subset_separator(cls, path: Path) -> str | None:
        for title in _fasta_titles(path):
            for sep in "|.":
                if sep in title:
                    return sep
            return None
        return None


class _Unavailable(PartitionHandler):
    lib = ""

    def _classifications(self, *args, **kwargs):
        raise NotImplementedError(f"{type(self).__name__} partitions need {self.lib}, which is not installed")


class Spart(_Unavailable):
    lib = "itaxotools.spart_parser"


class Excel(_Unavailable):
    lib = "openpyxl"


PartitionHandler.Tabfile = Tabfile
PartitionHandler.Fasta = Fasta
PartitionHandler.Spart = Spart
PartitionHandler.Excel = Excel
