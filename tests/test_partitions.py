"""Partition readers against the reference's own fixtures and expected maps
(tests/test_partitions.py:29-113 of the reference; data files under tests/golden/partitions)."""

from __future__ import annotations

import pytest

from tests.conftest import GOLDEN

D = GOLDEN / "partitions"

SIMPLE = {"sample1": "speciesA", "sample2": "speciesA", "sample3": "speciesA", "sample4": "speciesA",
          "sample5": "speciesB", "sample6": "speciesB", "sample7": "speciesC"}
MISSING = {"sample3": "speciesA", "sample4": "speciesA", "sample6": "speciesB", "sample7": "speciesC"}
GENERA = {"sample1": "genusX", "sample2": "genusX", "sample3": "genusX", "sample4": "genusX",
          "sample5": "genusY", "sample6": "genusY", "sample7": "genusY"}


def cases():
    from taxi2_amd.partitions import Classification, PartitionHandler as H

    return [
        (SIMPLE, "simple.tsv", H.Tabfile, {}),
        (SIMPLE, "extras.tsv", H.Tabfile, dict(idHeader="seqid", subHeader="organism")),
        (GENERA, "genera.tsv", H.Tabfile, dict(filter=H.subset_first_word, idHeader="seqid", subHeader="organism")),
        (SIMPLE, "simple.fas", H.Fasta, {}),
        (SIMPLE, "simple.dot.fas", H.Fasta, dict(separator=".")),
        (MISSING, "missing.fas", H.Fasta, {}),
        (GENERA, "genera.fas", H.Fasta, dict(filter=H.subset_first_word)),
        (SIMPLE, "genera.fas", H.Fasta, dict(filter=lambda x: Classification(x.individual, x.subset.split(" ")[1]))),
    ]


@pytest.mark.parametrize("k", range(8))
def test_read_partition(k):
    from taxi2_amd.partitions import Partition

    want, name, handler, kw = cases()[k]
    got = Partition.fromPath(D / name, handler, **kw)
    assert got == want and isinstance(got, dict)


def test_unavailable_formats():
    from taxi2_amd.partitions import Partition, PartitionHandler

    with pytest.raises(NotImplementedError):
        Partition.fromPath(D / "simple.tsv", PartitionHandler.Spart)


def test_fasta_separator_guess():
    from taxi2_amd.partitions import PartitionHandler

    assert PartitionHandler.Fasta.guess_subset_separator(D / "simple.dot.fas") == "."
    assert PartitionHandler.Fasta.has_subsets(D / "simple.fas")
