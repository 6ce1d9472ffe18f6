"""Aligned strings from the packed aligner's walks (round 3, alignt2_kernel.hpp StrOut) against
the trace kernels (k_trace_fill + k_traceback, TAXI2_NO_WALK_STRINGS=1) and the oracle: the same
first Biopython alignment, byte for byte, in both orientations -- and VersusAll's
aligned_pairs.txt / metrics written from ONE walk per ordered pair identical to the round-2 path
(metrics from the triangle, strings re-aligned per pair).  Default and generic Gotoh scores,
tie-heavy two-letter families, N runs, empty and 1-base sequences, chains cut mid-row."""

from __future__ import annotations

import os

import numpy as np
import pytest

from tests.seqgen import family_sequences, mutate, random_sequences
from tests.test_gpu_parity import SCORE_SETS

pytestmark = pytest.mark.gpu


def _sets():
    return {
        "family": family_sequences(24, 700, 0x51, ancestors=3) + ["", "A", "NNNN"],
        "ties": random_sequences(40, 1, 90, 52, "AC") + mutate(random_sequences(10, 40, 300, 53, "ACGTN"), 54, 0.2),
    }


def _strings(engine, st, xs, ys, sc, both, walk: bool):
    if walk:
        os.environ.pop("TAXI2_NO_WALK_STRINGS", None)
    else:
        os.environ["TAXI2_NO_WALK_STRINGS"] = "1"
    try:
        return engine.align_strings(st, st, xs, ys, sc, both=both)
    finally:
        os.environ.pop("TAXI2_NO_WALK_STRINGS", None)


@pytest.mark.parametrize("name", ["family", "ties"])
@pytest.mark.parametrize("score", ["default", "generic"])
@pytest.mark.parametrize("both", [False, True])
def test_walk_strings_equal_trace_kernels(engine, name, score, both):
    seqs = _sets()[name]
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    rng = np.random.default_rng(7)
    xs = np.repeat(np.arange(n), n)  # x-major rows: chains of consecutive pairs sharing x
    ys = np.tile(np.arange(n), n)
    sel = np.sort(rng.choice(len(xs), min(len(xs), 1500), replace=False))
    xs, ys = xs[sel], ys[sel]
    sc = SCORE_SETS[score]
    got = _strings(engine, st, xs, ys, sc, both, True)
    exp = _strings(engine, st, xs, ys, sc, both, False)
    assert got == exp
    st.free()


def test_walk_strings_vs_oracle_restatement(engine):
    from oracle import restatement as R

    seqs = _sets()["ties"][:30]
    st = engine.upload(seqs, align=True)
    xs = np.repeat(np.arange(30), 30)
    ys = np.tile(np.arange(30), 30)
    got = engine.align_strings(st, st, xs, ys, SCORE_SETS["default"], both=True)
    for k, (x, y) in enumerate(zip(xs, ys)):
        if not seqs[x] or not seqs[y]:
            continue
        ax, ay, _ = R.align(seqs[x], seqs[y])
        bx, by, _ = R.align(seqs[x], seqs[y], swapped=True)
        assert got[k][0] == (ax, ay) and got[k][1] == (bx, by), (x, y)
    st.free()


TASK_VARIANTS = ["default", "generic", "percent"]


@pytest.mark.parametrize("variant", TASK_VARIANTS)
@pytest.mark.parametrize("stream", [False, True])
def test_task_pairs_from_walks_equal_round2_path(tmp_path, engine, variant, stream):
    from taxi2_amd.align import Scores
    from taxi2_amd.partitions import Partition
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    raw = family_sequences(20, 400, 0x61, ancestors=2) + random_sequences(8, 1, 60, 62, "ACGTN") + ["A"]
    seqs = [Sequence(f"s{k}", s, {"v": str(k % 3)}) for k, s in enumerate(raw)]
    if not stream:  # an identical full tuple (the diagonal rule); the streamed path needs unique ids
        seqs.append(Sequence("s3", raw[3], {"v": "0"}))

    def run(out, walk):
        if walk:
            os.environ.pop("TAXI2_NO_WALK_STRINGS", None)
        else:
            os.environ["TAXI2_NO_WALK_STRINGS"] = "1"
        try:
            t = VersusAll()
            t.engine, t.progress_handler, t.work_dir = engine, None, out
            t.input.sequences = Sequences(seqs)
            t.params.engine.stream = stream
            t.params.engine.block_bytes = 7 * len(seqs) * 1000  # a few rows per block
            t.params.engine.launch_pairs = 0
            if variant == "generic":
                t.params.pairs.scores = dict(Scores(match_score=2, mismatch_score=-3, internal_open_gap_score=-5,
                                                    internal_extend_gap_score=-2, end_open_gap_score=-1,
                                                    end_extend_gap_score=-1))
            if variant == "percent":
                t.params.format.percentage_multiply = True
                t.input.genera = Partition({s.id: "g%d" % (k % 2) for k, s in enumerate(seqs)})
            t.start()
            return t
        finally:
            os.environ.pop("TAXI2_NO_WALK_STRINGS", None)

    a = run(tmp_path / "walk", True)
    b = run(tmp_path / "r2", False)
    if not stream:
        assert a.pairs_walked and not b.pairs_walked
    files = sorted(p.relative_to(tmp_path / "r2") for p in (tmp_path / "r2").rglob("*") if p.is_file())
    assert files
    for f in files:
        assert (tmp_path / "walk" / f).read_bytes() == (tmp_path / "r2" / f).read_bytes(), f


@pytest.mark.parametrize("pipeline", ["fused_dma", "fused_kernel", "streams", "streams_mask"])
@pytest.mark.parametrize("mode", ["one_block", "small_blocks", "switch", "split_text", "tail_row"])
@pytest.mark.parametrize("variant", ["default", "generic"])
def test_task_pairs_one_fill_equals_rect_path(tmp_path, engine, mode, variant, pipeline, monkeypatch):
    """Dense aligned_pairs.txt from ONE fill per unordered pair (taxi2_tri_strings_dev: both
    orientations walked, the (b, a) strings kept in HBM until row b, text through per-pair pointers)
    == the rect path that aligns every ordered pair once (TAXI2_PAIRS_RECT=1), every output file
    byte for byte: one block, many small blocks (the pipeline two blocks deep, the writers formatting
    each block from HBM), a keep budget that runs out mid-way (the remaining rows switch to the rect
    path), and a block's text split over many formatter calls (a one-row bound per call).  Every
    text pipeline (params.engine.text_pipeline): the text queued on the fill stream and moved by the
    DMA engine or the copy kernel, and the second-stream text beside the fills (plain or CU-masked
    streams)."""
    from taxi2_amd.tasks import versus_all as VA

    env = {"fused_dma": {"TAXI2_TEXT_PIPELINE": "fused", "TAXI2_TEXT_COPY": "1"},
           "fused_kernel": {"TAXI2_TEXT_PIPELINE": "fused", "TAXI2_TEXT_COPY": "2"},
           "streams": {"TAXI2_TEXT_PIPELINE": "streams", "TAXI2_TEXT_COPY": "0"},
           "streams_mask": {"TAXI2_TEXT_PIPELINE": "streams", "TAXI2_TEXT_COPY": "2", "TAXI2_TEXT_MASK": "1"}}
    for k, v in env[pipeline].items():
        monkeypatch.setenv(k, v)

    if mode == "split_text":
        monkeypatch.setattr(VA, "TEXT_CALL_BYTES", 1)
    from taxi2_amd.align import Scores
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    raw = family_sequences(26, 500, 0x71, ancestors=3) + random_sequences(6, 1, 80, 72, "ACGTN") + ["A", ""]
    seqs = [Sequence(f"q{k}", s, {"v": str(k % 4)}) for k, s in enumerate(raw)]
    seqs.append(Sequence("q5", raw[5], {"v": "1"}))  # an identical full tuple (the diagonal rule)

    def run(out, rect):
        if rect:
            os.environ["TAXI2_PAIRS_RECT"] = "1"
        try:
            t = VersusAll()
            t.engine, t.progress_handler, t.work_dir = engine, None, out
            t.input.sequences = Sequences(seqs)
            t.params.engine.stream = False
            if variant == "generic":
                t.params.pairs.scores = dict(Scores(match_score=2, mismatch_score=-3, internal_open_gap_score=-5,
                                                    internal_extend_gap_score=-2, end_open_gap_score=-1,
                                                    end_extend_gap_score=-1))
            if mode == "tail_row":  # blocks ... (28, 34), (34, 35): the last row alone, no pairs of its own
                t.params.engine.launch_pairs = 60
            elif mode != "one_block":
                t.params.engine.launch_pairs = 97  # a few rows per block
            if mode == "switch":
                t.params.engine.keep_bytes = 40_000  # runs out after the first blocks
            t.start()
            return t
        finally:
            os.environ.pop("TAXI2_PAIRS_RECT", None)

    a = run(tmp_path / "tri", False)
    b = run(tmp_path / "rect", True)
    assert a.pairs_walked and b.pairs_walked
    files = sorted(p.relative_to(tmp_path / "rect") for p in (tmp_path / "rect").rglob("*") if p.is_file())
    assert files
    for f in files:
        assert (tmp_path / "tri" / f).read_bytes() == (tmp_path / "rect" / f).read_bytes(), f
