"""GPU parity of the column-tiled aligner (taxi2_amd/csrc/alignlong_kernel.hpp): sequences of any
length, as the reference's PairwiseAligner.Biopython.align (/root/reference/src/itaxotools/taxi2/
align.py:151-157) aligns them.

* TAXI2_LONG=1 forces it on short inputs and TAXI2_LONG_TILE=256 cuts them into many 256-column
  tiles, so tile hand-offs, the end-gap column inside a later tile and pairs narrower than one tile
  are all exercised cheaply: every result against the C oracle AND the register-resident kernels.
* 5 000 and 10 000 bp pairs (past every register-resident shape) against the oracle.
* Aligned strings (aligned_pairs.txt, NCD on aligned strings) from its walkers equal the trace
  kernel's (k_traceback) where both exist, and past 4 095 bp their columns reproduce the walk's
  own counters (pre-aligned metrics of the strings == the aligned metrics).
"""

from __future__ import annotations

import os

import numpy as np
import pytest

from tests.seqgen import family_sequences, mutate, random_sequences
from tests.test_gpu_parity import METRICS, SCORE_SETS, assert_metrics_equal

pytestmark = pytest.mark.gpu


def _env(env: dict, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


LONG256 = {"TAXI2_LONG": "1", "TAXI2_LONG_TILE": "256"}


@pytest.mark.parametrize("scores", ["default", "generic", "linear"])
@pytest.mark.parametrize("tile", ["256", "1024", "2048"])
def test_tiled_triangle_small(engine, oracle_c, scores, tile):
    from taxi2_amd._native import tri_pairs

    base = random_sequences(6, 150, 900, 0x4C + int(tile), "ACGT", n_rate=0.02)
    seqs = base + mutate(base, 0x4D, rate=0.15) + ["", "A", "NNNN", "acgtRYacgt" * 30]
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    sc = SCORE_SETS[scores]
    got, gsc = _env({"TAXI2_LONG": "1", "TAXI2_LONG_TILE": tile},
                    lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    ref, rsc = engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)  # empty sequences included: the end-gap score (restated)
    assert np.array_equal(gsc, rsc)
    assert_metrics_equal(got, exp)
    assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(ref, nan=9.0))
    st.free()


def test_tiled_rectangle_and_list(engine, oracle_c):
    q = random_sequences(5, 200, 700, 0x4E, "ACGT")
    r = mutate(q[:3], 0x4F, rate=0.2) + random_sequences(4, 100, 800, 0x50, "ACGTN")
    qs, rs = engine.upload(q, align=True), engine.upload(r, align=True)
    got = _env(LONG256, lambda: engine.rect_pairs(qs, rs, 0, len(q), METRICS, None))
    allseq = q + r
    pa = np.repeat(np.arange(len(q)), len(r))
    pb = np.tile(np.arange(len(r)), len(q)) + len(q)
    exp, _ = oracle_c.batch(allseq, pa, pb, align=True, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp[:, 0, :])
    xs = np.array([0, 4, 2, 2]), np.array([1, 0, 5, 2])
    got = _env(LONG256, lambda: engine.list_pairs(qs, rs, xs[0], xs[1], METRICS, None))
    exp, _ = oracle_c.batch(allseq, xs[0], xs[1] + len(q), align=True, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp)
    qs.free()
    rs.free()


@pytest.mark.parametrize("length,scores", [(5000, "default"), (10000, "default"), (5000, "linear")])
def test_long_sequences(engine, oracle_c, length, scores):
    from taxi2_amd._native import tri_pairs

    fam = family_sequences(4, length, 0x51 + length, ancestors=2, max_sub=0.1, indel_rate=0.01)
    seqs = [fam[0], fam[1][: length - 300], fam[2], fam[3][: length // 2]]
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    sc = SCORE_SETS[scores]
    got, gsc = engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    st.free()


def test_tiled_aligned_strings_equal_traceback(engine):
    base = random_sequences(5, 100, 600, 0x52, "ACGTN")
    seqs = base + mutate(base, 0x53, rate=0.2) + ["", "ACGT"]
    st = engine.upload(seqs, align=True)
    xs = np.array([0, 1, 2, 3, 4, 5, 10, 11, 0])
    ys = np.array([5, 6, 7, 8, 9, 0, 1, 10, 0])
    for sc in (SCORE_SETS["default"], SCORE_SETS["generic"], SCORE_SETS["linear"]):
        ref = engine.align_strings(st, st, xs, ys, sc, both=True)
        got = _env(LONG256, lambda: engine.align_strings(st, st, xs, ys, sc, both=True))
        assert got == ref
    st.free()


@pytest.mark.parametrize("scores", ["default", "linear"])
def test_long_aligned_strings_match_counters(engine, oracle_c, scores):
    """Past 4 095 bp: the strings the walkers write have the columns the walks counted."""
    fam = family_sequences(3, 6000, 0x54, ancestors=1, max_sub=0.08, indel_rate=0.01)
    seqs = [fam[0], fam[1][:5500], fam[2]]
    st = engine.upload(seqs, align=True)
    xs, ys = np.array([0, 1, 0]), np.array([1, 2, 2])
    sc = SCORE_SETS[scores]
    strings = engine.align_strings(st, st, xs, ys, sc, both=True)
    aligned = engine.list_pairs(st, st, xs, ys, METRICS, sc)
    for k, pair in enumerate(strings):
        for o, (ax, ay) in enumerate(pair):
            assert ax.replace("-", "") == seqs[xs[k]] and ay.replace("-", "") == seqs[ys[k]]
            assert len(ax) == len(ay)
            pre, _ = oracle_c.batch([ax, ay], [0], [1], align=False, scores=SCORE_SETS["default"])
            assert_metrics_equal(aligned[k, o][None, :], pre[0, 0][None, :])
    st.free()


def test_versus_all_long_sequences(tmp_path, engine, oracle_c):
    """The task end to end on 4 800-5 200 bp sequences (distances + aligned_pairs.txt)."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll
    from taxi2_amd._native import tri_pairs

    fam = family_sequences(4, 5200, 0x55, ancestors=2, max_sub=0.1, indel_rate=0.01)
    raw = [s[: 4800 + 100 * k] for k, s in enumerate(fam)]
    t = VersusAll()
    t.engine, t.progress_handler, t.work_dir = engine, None, tmp_path
    t.input.sequences = Sequences([Sequence(f"s{k}", s) for k, s in enumerate(raw)])
    t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.Kimura2P()]
    t.start()
    D = t.distances
    a, b = tri_pairs(len(raw))
    exp, _ = oracle_c.batch(raw, a, b, align=True, scores=SCORE_SETS["default"], metrics=("p", "k2p"))
    assert_metrics_equal(D[a, b][:, None, :], exp[:, 0][:, None, :], ("p", "k2p"))
    assert_metrics_equal(D[b, a][:, None, :], exp[:, 1][:, None, :], ("p", "k2p"))
    text = (tmp_path / "align" / "aligned_pairs.txt").read_text()
    assert text.count("\n") > 16 * 3
