"""GPU parity of the packed aligners' trace band (the row-shared k_alignr, alignr_kernel.hpp, for the
default and one-extend scores up to 1 024 columns; k_alignt2, alignt2_kernel.hpp a2_band_blocks, for the other
score sets and shapes; both requeue escapes to k_alignt2_queued's full-trace pass):
the fill stores only the diagonal strip j - i in [min(0, nB - nA) - band, max(0, nB - nA) + band]
of each pair's trace, a walk that would leave it queues the pair, and a second launch redoes the
queued pairs with the full trace.  Results must not depend on the band: every case against the
C oracle and against band = 0 (full trace), bit for bit, including bands so narrow that most
pairs take the second launch, and pairs whose first path leaves any strip (long deletions).
Reference: /root/reference/src/itaxotools/taxi2/align.py:151-157 (one global alignment per pair).
"""

from __future__ import annotations

import re

import numpy as np
import pytest

from tests.seqgen import family_sequences, random_sequences
from tests.test_gpu_alignt import _tie_heavy, _with_env
from tests.test_gpu_parity import METRICS, SCORE_SETS, assert_metrics_equal

pytestmark = pytest.mark.gpu


def _indel_family(length: int, seed: int) -> list[str]:
    """A family plus copies whose first paths leave the diagonal: a long deletion with a
    compensating insertion further on (same length, so the strip's length-difference side does
    not cover the shift), a long insertion, and unrelated sequences of other lengths."""
    fam = family_sequences(6, length, seed, ancestors=2, max_sub=0.08, indel_rate=0.01)
    rng = np.random.default_rng(seed)
    out = list(fam)
    for k in range(4):
        s = fam[k]
        d = int(rng.integers(60, length // 4))
        at = int(rng.integers(10, length // 3))
        at2 = int(rng.integers(at + d + 10, length - 10))
        ins = "".join("ACGT"[int(c)] for c in rng.integers(0, 4, d))
        out.append(s[:at] + s[at + d:at2] + ins + s[at2:])  # shifted by d between at and at2
        out.append(s[:at] + ins + s[at:])                   # long insertion (longer than the family)
    out += random_sequences(3, length // 2, length, seed + 1, "ACGT")
    return out


def _queued(err: str) -> int:
    return sum(int(m) for m in re.findall(r"band \d+: (\d+) of \d+ pairs took the full-trace pass", err))


@pytest.mark.parametrize("band", ["8", "40", "default"])
@pytest.mark.parametrize("scores", ["default", "generic", "generic1"])
def test_band_triangle(engine, oracle_c, capfd, band, scores):
    from taxi2_amd._native import tri_pairs

    seqs = _indel_family(900, 0x71) + _tie_heavy(6, 900, 0x72) + ["", "A", "N" * 30]
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    sc = SCORE_SETS[scores]
    env = {"TAXI2_AT_BAND_STATS": "1"}
    if band != "default":
        env["TAXI2_AT_BAND"] = band
    capfd.readouterr()
    got, gsc = _with_env(env, lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    queued = _queued(capfd.readouterr().err)
    full, fsc = _with_env({"TAXI2_AT_BAND": "0"}, lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)  # empty sequences included: the end-gap score (restated)
    assert_metrics_equal(got, exp)
    assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(full, nan=9.0))
    assert np.array_equal(gsc, fsc)
    # the long deletions / insertions leave every strip tried here: the second launch really ran
    assert queued > 0
    if band == "8":
        assert queued >= 10


@pytest.mark.parametrize("band", ["8", "default"])
def test_band_rectangle_and_list(engine, oracle_c, band):
    q = _indel_family(800, 0x73)[:10]
    r = _indel_family(700, 0x74)
    qs, rs = engine.upload(q, align=True), engine.upload(r, align=True)
    env = {} if band == "default" else {"TAXI2_AT_BAND": band}
    allseq = q + r
    pa = np.repeat(np.arange(len(q)), len(r))
    pb = np.tile(np.arange(len(r)), len(q)) + len(q)
    for name in ("default", "generic", "generic1"):
        sc = SCORE_SETS[name]
        got = _with_env(env, lambda: engine.rect_pairs(qs, rs, 0, len(q), METRICS, sc))
        exp, _ = oracle_c.batch(allseq, pa, pb, align=True, scores=sc)
        assert_metrics_equal(got, exp[:, 0, :])
        xs = np.array([0, 9, 3, 3, 7]), np.array([1, 0, 12, 3, 5])
        got = _with_env(env, lambda: engine.list_pairs(qs, rs, xs[0], xs[1], METRICS, sc))
        exp, _ = oracle_c.batch(allseq, xs[0], xs[1] + len(q), align=True, scores=sc)
        assert_metrics_equal(got, exp)
    qs.free()
    rs.free()


def test_band_two_thousand_columns(engine, oracle_c):
    """The 1 025-2 048-column shape (four fill waves) with a narrow band and long indels."""
    from taxi2_amd._native import tri_pairs

    seqs = _indel_family(1600, 0x75)[:9]
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    got, gsc = _with_env({"TAXI2_AT_BAND": "24"}, lambda: engine.all_pairs(st, 0, len(a), METRICS, None, with_scores=True))
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=SCORE_SETS["default"])
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)


def test_band_device_buffers(engine, oracle_c):
    """The *_dev entry point (what bench.py times): queue and second launch on the caller's stream."""
    import torch

    from taxi2_amd._native import tri_pairs

    seqs = _indel_family(1000, 0x76)
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    k = len(a)
    out = torch.empty((k, 2, len(METRICS)), dtype=torch.float64, device="cuda")
    sco = torch.empty((k,), dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        _with_env({"TAXI2_AT_BAND": "16"}, lambda: engine.all_pairs_dev(st, 0, k, METRICS, out.data_ptr(), None,
                                                                        sco.data_ptr(), s.cuda_stream))
    s.synchronize()
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=SCORE_SETS["default"])
    assert np.array_equal(sco.cpu().numpy(), esc)
    assert_metrics_equal(out.cpu().numpy(), exp)
