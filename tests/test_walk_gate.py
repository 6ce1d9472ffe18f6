"""Host-side gate of the walk-strings aligned_pairs.txt path: the walkers copy sequence
bytes straight into the text, and the engine holds one latin-1 byte per character, while the
reference writes str to a UTF-8 text file (pairs.py SequencePairHandler.Formatted) -- so any
non-ASCII sequence, and every environment knob that makes the engine decline the packed aligner,
keeps the Python-formatted writer."""

from __future__ import annotations

import os

import pytest

from taxi2_amd.sequences import Sequence
from taxi2_amd.tasks.versus_all import walk_strings_ok

DEF = (1, -1, -8, -1, -1, -1)


def test_ascii_sequences_walk():
    assert walk_strings_ok(DEF, [Sequence("a", "ACGT"), Sequence("b", "ACGN")])


def test_latin1_sequence_keeps_python_writer():
    assert not walk_strings_ok(DEF, [Sequence("a", "ACGT"), Sequence("b", "ACGé")])


@pytest.mark.parametrize("knob", ["TAXI2_NO_ALIGNT", "TAXI2_NO_PACKED", "TAXI2_LONG", "TAXI2_NO_WALK_STRINGS"])
def test_engine_knobs_keep_python_writer(knob, monkeypatch):
    monkeypatch.setitem(os.environ, knob, "1")
    assert not walk_strings_ok(DEF, [Sequence("a", "ACGT")])


def test_linear_scores_and_long_sequences_do_not_walk():
    assert not walk_strings_ok((1, -1, -2, -2, -1, -1), [Sequence("a", "ACGT")])
    assert not walk_strings_ok(DEF, [Sequence("a", "A" * 2049)])
