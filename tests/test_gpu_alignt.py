"""GPU parity of the trace-and-walk aligners: the fill stores the tie information of every cell and
a walker wave traces both Biopython first paths (priority M>Ix>Iy for (a, b), M>Iy>Ix for (b, a)).
Which kernel runs a case: with the DEFAULT scores and every sequence <= 1 024 columns, the
row-shared packed aligner k_alignr (alignr_kernel.hpp, the headline kernel) for the triangle, the
rectangle and the string-emitting launches; other Gotoh score sets within int16, and 1 025 - 2 048
columns, the packed k_alignt2 (alignt2_kernel.hpp); TAXI2_NO_PACKED=1 the 32-bit k_alignt
(alignt_kernel.hpp); TAXI2_NO_ALIGNR=1 keeps default scores on k_alignt2
(test_alignr_off_matches_default pins that k_alignt2 default-score path bit for bit).

Every case is checked against the C restatement (oracle/taxi2_oracle.c, scores bit-exact,
p / p-gaps bit-exact, jc / k2p within 1e-12) AND against the forward-carry kernels
(TAXI2_NO_ALIGNT=1), bit for bit; the packed kernel also against the 32-bit one
(TAXI2_NO_PACKED=1).  TAXI2_AT_CHUNK forces long chains on small inputs and
TAXI2_AT_HOPS=1 starves the walker so that most walks finish in the post-chain drain.
"""

from __future__ import annotations

import os

import numpy as np
import pytest

from tests.seqgen import family_sequences
from tests.test_gpu_parity import METRICS, SCORE_SETS, assert_metrics_equal

pytestmark = pytest.mark.gpu


def _with_env(env: dict, fn):
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


def _tie_heavy(n: int, length: int, seed: int) -> list[str]:
    """Near-identical families with ragged ends, lowercase runs and IUPAC bytes: many Ix / Iy
    ties (the (a, b) and (b, a) alignments differ), and the byte-compare substitution path."""
    fam = family_sequences(n, length, seed, ancestors=3, max_sub=0.05, indel_rate=0.02)
    rng = np.random.default_rng(seed)
    out = []
    for k, s in enumerate(fam):
        s = s[: length - 200 + int(rng.integers(0, 200))]
        if k % 4 == 1:
            s = s[:100] + s[100:160].lower() + s[160:]
        if k % 5 == 2:
            b = bytearray(s.encode())
            for pos in rng.integers(0, len(b), 6):
                b[pos] = ord("NRYKM"[int(rng.integers(0, 5))])
            s = b.decode()
        out.append(s)
    return out


@pytest.mark.parametrize("env", [{}, {"TAXI2_AT_CHUNK": "8"}, {"TAXI2_AT_CHUNK": "3", "TAXI2_AT_HOPS": "1"}])
def test_alignt_triangle(engine, oracle_c, env):
    from taxi2_amd._native import tri_pairs

    seqs = _tie_heavy(18, 900, 0x61)
    seqs += ["ACGT" * 256, "A", "", "N" * 40, seqs[0]]  # 1024 (capacity), 1, empty, no ACGT, duplicate
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    for name in ("default", "generic", "generic1"):
        sc = SCORE_SETS[name]
        got, gsc = _with_env(env, lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
        old, osc = _with_env({"TAXI2_NO_ALIGNT": "1"},
                             lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
        t32, t32sc = _with_env(dict(env, TAXI2_NO_PACKED="1"),
                               lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
        exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
        assert np.array_equal(gsc, esc)  # empty sequences included: the end-gap score (restated)
        assert_metrics_equal(got, exp)
        assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(old, nan=9.0))
        assert np.array_equal(gsc, osc)
        assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(t32, nan=9.0))
        assert np.array_equal(gsc, t32sc)
        asym = ~np.all(np.isclose(np.nan_to_num(exp[:, 0]), np.nan_to_num(exp[:, 1])), axis=1)
        assert asym.sum() > 0  # the two orientations really differ somewhere
    # an offset block of the triangle (chunks start mid-row)
    k0, cnt = 57, 83
    got = _with_env(env, lambda: engine.all_pairs(st, k0, cnt, METRICS, None))
    exp, _ = oracle_c.batch(seqs, a[k0 : k0 + cnt], b[k0 : k0 + cnt], align=True, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp)
    st.free()


@pytest.mark.parametrize("scores", ["default", "generic"])
@pytest.mark.parametrize("env", [{}, {"TAXI2_AT_CHUNK": "5"}, {"TAXI2_NO_PACKED": "1"}])
def test_alignt_rectangle(engine, oracle_c, env, scores):
    """One ordered orientation per pair (versusReference): the walk of the (query, ref) slot,
    with queries longer and shorter than the references (rows / columns swapped; under generic
    scores the swapped walk reads the stored tagF)."""
    seqs = _tie_heavy(14, 700, 0x62)
    qseq = seqs[:6]
    rseq = [s[:350] if k % 2 else s for k, s in enumerate(seqs[6:])]
    qs = engine.upload(qseq, align=True)
    rs = engine.upload(rseq, align=True)
    sc = SCORE_SETS[scores]
    got = _with_env(env, lambda: engine.rect_pairs(qs, rs, 0, len(qseq), METRICS, sc))
    allseq = qseq + rseq
    pa = np.repeat(np.arange(len(qseq)), len(rseq))
    pb = np.tile(np.arange(len(rseq)), len(qseq)) + len(qseq)
    exp, _ = oracle_c.batch(allseq, pa, pb, align=True, scores=sc)
    assert_metrics_equal(got, exp[:, 0, :])
    qs.free()
    rs.free()


@pytest.mark.parametrize("packed", [True, False])
def test_alignt_bench_shape(engine, oracle_c, packed):
    """The bench generator (config 3, 1 000 bp, unrelated families) with chains of 8 pairs."""
    from taxi2_amd._native import tri_pairs

    seqs = family_sequences(30, 1000, 0x7A12, ancestors=6)
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    env = {"TAXI2_AT_CHUNK": "8"} if packed else {"TAXI2_AT_CHUNK": "8", "TAXI2_NO_PACKED": "1"}
    got, gsc = _with_env(env, lambda: engine.all_pairs(st, 0, len(a), METRICS, None, with_scores=True))
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=SCORE_SETS["default"])
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    st.free()


def test_alignt2_value_range_extremes(engine, oracle_c):
    """The default-score best-open fill stores its cells as f16 bit patterns (bias 20480, one
    v_pk_maximum3_f16 per cell pair, alignt2_kernel.hpp A2_MAX3): exact only while every value is a
    positive normal f16 pattern.  The extremes of that range at the packed shape's 1 024-column
    capacity: identical full-length sequences (the largest drifted values), full-length all-mismatch
    pairs, full-length against 1-base sequences (the longest end gaps), long internal runs, non-ACGT
    rows and empty sequences -- every pair in both orientations against the oracle."""
    from taxi2_amd._native import tri_pairs

    L = 1024
    seqs = ["A" * L, "A" * L, "C" * L, "T" * L, "A" * (L // 2) + "C" * (L // 2), "ACGT" * (L // 4),
            "A", "C", "AC" * 8, "A" * (L - 24) + "N" * 24, "G" * 3 + "A" * (L - 6) + "G" * 3, "", "N" * L]
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    sc = SCORE_SETS["default"]
    got, gsc = engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)  # empty sequences included: the end-gap score (restated)
    assert_metrics_equal(got, exp)
    # the identical full-length pair scores its length (the largest value the fill holds)
    k = int(np.flatnonzero((a == 0) & (b == 1))[0])
    assert int(gsc[k]) == L
    st.free()


def test_alignr_off_matches_default(engine, oracle_c):
    """TAXI2_NO_ALIGNR=1 runs the default scores on k_alignt2 instead of k_alignr: both must give the
    same scores and metrics bit for bit (triangle and rectangle, tie-heavy ragged sets up to the
    1 024-column capacity), and the oracle's."""
    from taxi2_amd._native import tri_pairs

    seqs = _tie_heavy(20, 1000, 0x6A) + ["ACGT" * 256, "A", "", "N" * 40]
    seqs.append(seqs[0])
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    sc = SCORE_SETS["default"]
    got, gsc = engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True)
    off, osc = _with_env({"TAXI2_NO_ALIGNR": "1"},
                         lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    assert np.array_equal(got.view(np.int64), off.view(np.int64)) and np.array_equal(gsc, osc)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    r_on = engine.rect_pairs(st, st, 3, 9, METRICS, sc)
    r_off = _with_env({"TAXI2_NO_ALIGNR": "1"}, lambda: engine.rect_pairs(st, st, 3, 9, METRICS, sc))
    assert np.array_equal(r_on.view(np.int64), r_off.view(np.int64))
    st.free()


def test_alignr_swapped_units_match_default(engine):
    """TAXI2_AR_SWAP=1 (k_alignr pairs a launch's unshared row with itself: units of two of its pairs
    on the row's sequence, walked in the other orientation) gives the default's scores, metrics and
    aligned strings bit for bit: whole triangles (every odd column count leaves a row alone), a
    mid-row launch, a rectangle (one orientation), and both orientations' strings."""
    from taxi2_amd._native import tri_pairs

    seqs = _tie_heavy(24, 1000, 0x6B) + ["ACGT" * 200, "A", "", "N" * 40]
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    sc = SCORE_SETS["default"]
    swap = {"TAXI2_AR_SWAP": "1"}
    for k0, cnt in ((0, len(a)), (7, len(a) - 19)):
        got, gsc = engine.all_pairs(st, k0, cnt, METRICS, sc, with_scores=True)
        sw, ssc = _with_env(swap, lambda: engine.all_pairs(st, k0, cnt, METRICS, sc, with_scores=True))
        assert np.array_equal(got.view(np.int64), sw.view(np.int64)) and np.array_equal(gsc, ssc)
    r_on = engine.rect_pairs(st, st, 3, 11, METRICS, sc)
    r_sw = _with_env(swap, lambda: engine.rect_pairs(st, st, 3, 11, METRICS, sc))
    assert np.array_equal(r_on.view(np.int64), r_sw.view(np.int64))
    import torch

    cnt = len(a)
    cap = 2 * max(len(s) for s in seqs) + 1

    def strings():
        d = torch.empty((cnt, 2, len(METRICS)), dtype=torch.float64, device="cuda")
        sx = torch.zeros((cnt, 2, cap), dtype=torch.uint8, device="cuda")
        sy = torch.zeros((cnt, 2, cap), dtype=torch.uint8, device="cuda")
        sl = torch.zeros((cnt, 2), dtype=torch.int32, device="cuda")
        engine.tri_strings_dev(st, 0, cnt, METRICS, d.data_ptr(), cap, sx.data_ptr(), sy.data_ptr(), sl.data_ptr(),
                               sc)
        torch.cuda.synchronize()
        return [t.cpu().numpy() for t in (d, sx, sy, sl)]

    s_def = strings()
    s_sw = _with_env(swap, strings)
    for u, v in zip(s_def, s_sw):
        assert np.array_equal(u.view(np.uint8), v.view(np.uint8))
    st.free()
