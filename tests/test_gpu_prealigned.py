"""The tiled pre-aligned kernel (k_prealigned_tile, round 3) against the C restatement and the
one-thread-per-pair kernel (TAXI2_PRE_NOTILE=1), bit for bit: triangle blocks that start and end
inside a row, rectangles (host and device outputs), ragged lengths (plane words past a sequence's
end), leading / trailing gaps and N (the gap plane restricted to each sequence's own ACGT range),
the packed counter slots of the streamed path, and tiles narrower than 64 sequences."""

from __future__ import annotations

import os

import numpy as np
import pytest

from tests.seqgen import random_sequences
from tests.test_gpu_parity import SCORE_SETS, assert_metrics_equal

pytestmark = pytest.mark.gpu

METRICS = ("p", "p-gaps", "jc", "k2p")


def _sets():
    rng = np.random.default_rng(21)
    ragged = random_sequences(190, 0, 420, 22, "ACGTacgtN--?RY")
    edges = []
    for k in range(145):  # gaps / N at the ends, inside the range, whole-gap rows
        core = "".join(rng.choice(list("ACGT-"), size=int(rng.integers(1, 300))))
        edges.append("-" * int(rng.integers(0, 40)) + "N" * int(rng.integers(0, 3)) + core + "-" * int(rng.integers(0, 40)))
    edges += ["-" * 50, "", "A", "N" * 70, "ACGT" * 80]
    return {"ragged": ragged, "edges": edges}


def _notile(flag: bool):
    if flag:
        os.environ["TAXI2_PRE_NOTILE"] = "1"
    else:
        os.environ.pop("TAXI2_PRE_NOTILE", None)


@pytest.mark.parametrize("name", ["ragged", "edges"])
def test_tile_triangle_vs_oracle_and_notile(engine, oracle_c, name):
    from taxi2_amd._native import tri_pairs

    seqs = _sets()[name]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    total = n * (n - 1) // 2
    a, b = tri_pairs(n)
    exp, _ = oracle_c.batch(seqs, a, b, align=False, scores=SCORE_SETS["default"])
    got = engine.all_pairs(st, 0, total, METRICS)
    assert_metrics_equal(got, exp[:, 0, :])
    # blocks starting / ending inside rows, one tile row or many
    for k0, cnt in ((0, 4096), (777, 5000), (total // 3 + 13, 4200), (total - 4100, 4100)):
        cnt = min(cnt, total - k0)
        blk = engine.all_pairs(st, k0, cnt, METRICS)
        assert np.array_equal(blk.view(np.int64), got[k0 : k0 + cnt].view(np.int64))
    try:
        _notile(True)
        ref = engine.all_pairs(st, 0, total, METRICS)
    finally:
        _notile(False)
    assert np.array_equal(ref.view(np.int64), got.view(np.int64))
    st.free()


def test_tile_rect_host_and_device(engine, oracle_c):
    import torch

    seqs = _sets()["ragged"]
    q, r = seqs[:70], seqs[70:]
    sq = engine.upload(q, align=False)
    sr = engine.upload(r, align=False)
    R = len(r)
    qa = np.repeat(np.arange(len(q)), R)
    rb = np.tile(np.arange(R), len(q))
    exp, _ = oracle_c.batch(q + r, qa, rb + len(q), align=False, scores=SCORE_SETS["default"])
    got = engine.rect_pairs(sq, sr, 0, len(q), METRICS)
    assert_metrics_equal(got, exp[:, 0, :])
    for q0, q1 in ((0, len(q)), (5, 41), (69, 70)):
        out = torch.empty(((q1 - q0) * R, len(METRICS)), dtype=torch.float64, device="cuda")
        s = torch.cuda.Stream()
        engine.rect_pairs_dev(sq, sr, q0, q1, METRICS, out.data_ptr(), None, None, s.cuda_stream)
        s.synchronize()
        dev = out.cpu().numpy()
        assert np.array_equal(dev.view(np.int64), got[q0 * R : q1 * R].view(np.int64))
    sq.free()
    sr.free()


def test_tile_counts_slots(engine):
    """TAXI2_METRIC_COUNTS through the tile: the packed counters give the metrics bit for bit."""
    import torch

    seqs = _sets()["edges"]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    cnt = torch.empty((n * n,), dtype=torch.float64, device="cuda")
    met = torch.empty((n * n, len(METRICS)), dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    engine.rect_pairs_dev(st, st, 0, n, ("counts",), cnt.data_ptr(), None, None, s.cuda_stream)
    engine.rect_pairs_dev(st, st, 0, n, METRICS, met.data_ptr(), None, None, s.cuda_stream)
    out = torch.empty_like(met)
    engine.counts_metrics_dev(cnt.data_ptr(), n * n, METRICS, out.data_ptr(), 1.0, s.cuda_stream)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.int64), met.cpu().numpy().view(np.int64))
    st.free()
