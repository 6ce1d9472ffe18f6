"""The oracle pinned against the reference's own vectors (CPU only)."""

from __future__ import annotations

import json
import math
import random

import numpy as np
import pytest

from oracle import restatement as R
from tests.conftest import GOLDEN

ALIGN_ROWS = json.loads((GOLDEN / "align_tests.json").read_text())


@pytest.mark.parametrize("row", ALIGN_ROWS, ids=lambda r: f"{r['x']}-{r['y']}-{tuple(r['scores'].values())}")
def test_restatement_align_vectors(row):
    """tests/test_align.py:49-163: the first alignment is one of the accepted solutions."""
    sc = R.Scores(*row["scores"].values())
    ax, ay, score = R.align(row["x"], row["y"], sc)
    assert len(ax) == len(ay)
    assert [ax, ay] in row["solutions"]
    # every accepted solution has the optimal score under these scores
    assert ax.replace("-", "") == row["x"] and ay.replace("-", "") == row["y"]


def _metrics_rows():
    lines = (GOLDEN / "metrics.tsv").read_text().splitlines()
    hdr = lines[0].split("\t")
    for ln in lines[1:]:
        f = ln.split("\t")
        for lab, v in zip(hdr[2:], f[2:]):
            yield f[0], f[1], lab, (None if v == "NA" else float(v))


@pytest.mark.parametrize("x,y,label,expected", list(_metrics_rows()))
def test_restatement_metrics_fixture(x, y, label, expected):
    """tests/test_distances/metrics.tsv at the reference's tolerance 0.00051."""
    got = R.metric(label, x, y)
    if expected is None:
        assert got is None
    else:
        assert got is not None and abs(got - expected) <= 0.00051


def test_restatement_metric_tests_exact():
    """tests/test_distances.py:515-521 (precision 0)."""
    labels = {"Uncorrected": "p", "UncorrectedWithGaps": "p-gaps"}
    for r in json.loads((GOLDEN / "metric_tests.json").read_text()):
        assert R.metric(labels[r["metric"]], r["x"], r["y"]) == r["d"]


def test_normalize():
    assert R.normalize("ac-g?t--n") == "ACGNTN"
    assert R.normalize("") == ""


def test_jc_k2p_negative_zero():
    """p = 0 gives -0.0 for jc and k2p (printed '-0.0000' by '{:.4f}')."""
    c = R.counts("ACGT", "ACGT")
    assert math.copysign(1.0, R.metric_value("jc", c)) == -1.0
    assert math.copysign(1.0, R.metric_value("k2p", c)) == -1.0
    assert "{:.4f}".format(R.metric_value("jc", c)) == "-0.0000"


def test_c_oracle_matches_python_traceback(oracle_c):
    """The C restatement's forward-carried counters == explicit traceback + counting, both
    orientations, across score regimes (Gotoh, NW, generic)."""
    rng = random.Random(7)
    score_sets = [R.Scores(), R.Scores(1, 0, 0, 0, 0, 0), R.Scores(1, -1, -1, -1, -1, -1),
                  R.Scores(2, -3, -5, -2, -1, -1), R.Scores(10, 0, -10, -6, 0, 0), R.Scores(1, 0, -1, 0, 0, -1)]
    for _ in range(600):
        sc = rng.choice(score_sets)
        alpha = rng.choice(["ACGT", "AC", "ACGTN", "ACGTNRY"])
        x = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 25)))
        y = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 25)))
        if rng.random() < 0.5:
            y = "".join(c if rng.random() > 0.2 else rng.choice(alpha) for c in x)
        a, b, s = R.aligned_counts(x, y, sc)
        ca, cb, cs = oracle_c.align_counts(x, y, sc)
        assert (tuple(a), tuple(b), s) == (ca, cb, cs), (x, y, sc)


def test_c_oracle_prealigned_and_metrics(oracle_c):
    rng = random.Random(3)
    for _ in range(600):
        x = "".join(rng.choice("ACGTacgtN-?") for _ in range(rng.randint(0, 30)))
        y = "".join(rng.choice("ACGTacgtN-?") for _ in range(rng.randint(0, 30)))
        c = R.counts(x, y)
        assert tuple(c) == oracle_c.prealigned_counts(x, y)
        for lab in R.METRICS:
            pv = R.metric_value(lab, c)
            cv = oracle_c.metric(lab, tuple(c))
            assert (math.isnan(pv) and math.isnan(cv)) or pv == cv, (lab, x, y, pv, cv)


def test_c_oracle_batch_threads_agree(oracle_c):
    from taxi2_amd.synth import family_sequences

    seqs = family_sequences(12, 150, 11)
    a = np.repeat(np.arange(12), 12)
    b = np.tile(np.arange(12), 12)
    o1, s1 = oracle_c.batch(seqs, a, b, align=True, scores=(1, -1, -8, -1, -1, -1), threads=1)
    o4, s4 = oracle_c.batch(seqs, a, b, align=True, scores=(1, -1, -8, -1, -1, -1), threads=4)
    assert np.array_equal(np.nan_to_num(o1, nan=9.0), np.nan_to_num(o4, nan=9.0))
    assert np.array_equal(s1, s4)
