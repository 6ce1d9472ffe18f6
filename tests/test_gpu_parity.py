"""GPU parity: the HIP engine (through the C ABI) against the C restatement.

Bar (BASELINE.json north_star): alignment scores and p / p-gaps bit-exact; jc / k2p within
1e-12 absolute; undefined (NaN/inf -> None) in exactly the same places.
"""

from __future__ import annotations

import json

import numpy as np
import pytest

from tests.conftest import GOLDEN
from tests.seqgen import family_sequences, mutate, random_sequences

pytestmark = pytest.mark.gpu

METRICS = ("p", "p-gaps", "jc", "k2p")
TOL_LOG = 1e-12  # jc / k2p (f64 log on GPU vs glibc)

SCORE_SETS = {
    "default": (1, -1, -8, -1, -1, -1),
    "generic": (2, -3, -5, -2, -1, -1),
    # one extend for internal and end gaps: the packed aligner's best-open fill (capi.hip bopen_ok)
    "generic1": (2, -3, -5, -2, -3, -2),
    "linear": (1, -1, -2, -2, -1, -1),
}


def assert_metrics_equal(got: np.ndarray, exp: np.ndarray, metrics=METRICS):
    assert got.shape == exp.shape
    for mi, m in enumerate(metrics):
        g = got[..., mi].ravel()
        e = exp[..., mi].ravel()
        gu, eu = ~np.isfinite(g), ~np.isfinite(e)
        bad = np.nonzero(gu != eu)[0]
        assert bad.size == 0, f"{m}: undefined mismatch at {bad[:10]} got={g[bad[:5]]} exp={e[bad[:5]]}"
        gd, ed = g[~gu], e[~eu]
        if m in ("p", "p-gaps"):
            diff = np.nonzero(gd != ed)[0]
            assert diff.size == 0, f"{m}: {diff.size} values differ, e.g. {gd[diff[:5]]} vs {ed[diff[:5]]}"
        else:
            err = np.max(np.abs(gd - ed)) if gd.size else 0.0
            assert err <= TOL_LOG, f"{m}: max abs err {err}"
        # sign of zero (jc/k2p print -0.0000 for p = 0)
        assert np.array_equal(np.signbit(gd[gd == 0]), np.signbit(ed[ed == 0]))


# ----------------------------------------------------------------------------- golden vectors
def test_align_golden_vectors(engine, oracle_c):
    """tests/test_align.py:49-163 vectors: GPU counters == restatement (whose alignment is one
    of the accepted solutions for every vector)."""
    from oracle import restatement as R

    rows = json.loads((GOLDEN / "align_tests.json").read_text())
    for r in rows:
        sc = tuple(r["scores"].values())
        s = engine.upload([r["x"], r["y"]], align=True)
        got, score = engine.list_pairs(s, s, [0], [1], METRICS, sc, with_scores=True)
        exp, escore = oracle_c.batch([r["x"], r["y"]], [0], [1], align=True, scores=sc, threads=1)
        assert_metrics_equal(got, exp)
        ax, ay, bs = R.align(r["x"], r["y"], R.Scores(*sc))
        assert [ax, ay] in r["solutions"]
        assert int(score[0]) == int(escore[0]) == int(bs), r
        s.free()


def test_prealigned_metrics_fixture(engine):
    """tests/test_distances/metrics.tsv (26 rows x 4 metrics, tolerance 0.00051 as in
    tests/test_distances.py:524) and the exact metric_tests (test_distances.py:515-521)."""
    lines = (GOLDEN / "metrics.tsv").read_text().splitlines()
    hdr = lines[0].split("\t")
    xs, ys, exp = [], [], []
    for ln in lines[1:]:
        f = ln.split("\t")
        xs.append(f[0])
        ys.append(f[1])
        exp.append([np.nan if v == "NA" else float(v) for v in f[2:]])
    labels = tuple(hdr[2:])
    s = engine.upload(xs + ys, align=False)
    n = len(xs)
    got = engine.list_pairs(s, s, np.arange(n), np.arange(n) + n, labels)
    exp = np.asarray(exp)
    for k in range(n):
        for m in range(len(labels)):
            g, e = got[k, m], exp[k, m]
            if np.isnan(e):
                assert not np.isfinite(g), (xs[k], ys[k], labels[m], g)
            else:
                assert abs(g - e) <= 0.00051, (xs[k], ys[k], labels[m], g, e)
    s.free()
    for r in json.loads((GOLDEN / "metric_tests.json").read_text()):
        label = {"Uncorrected": "p", "UncorrectedWithGaps": "p-gaps"}[r["metric"]]
        s = engine.upload([r["x"], r["y"]], align=False)
        g = engine.list_pairs(s, s, [0], [1], [label])[0, 0]
        if r["d"] is None:
            assert not np.isfinite(g)
        else:
            assert g == r["d"]
        s.free()


# ----------------------------------------------------------------------------- aligned, random
BUCKETS = [  # (lo, hi) lengths chosen to exercise every (K, W) kernel variant
    (1, 40), (60, 250), (300, 380), (420, 512), (600, 760), (900, 1024), (1100, 1500), (1700, 2048),
    (2200, 2600),
]


@pytest.mark.parametrize("bucket", BUCKETS)
@pytest.mark.parametrize("scores", list(SCORE_SETS))
def test_align_all_pairs_random(engine, oracle_c, bucket, scores):
    lo, hi = bucket
    if lo >= 2200 and scores != "default":
        pytest.skip("long buckets: default scores only (oracle time)")
    n = 10 if hi > 1100 else 16
    seed = hash((lo, hi, scores)) & 0xFFFF
    base = random_sequences(n // 2, lo, hi, seed, "ACGT", n_rate=0.02)
    seqs = base + mutate(base, seed + 1, rate=0.15)
    seqs = [s if s else "A" for s in seqs]
    sc = SCORE_SETS[scores]
    st = engine.upload(seqs, align=True)
    total = n * (n - 1) // 2
    got, gsc = engine.all_pairs(st, 0, total, METRICS, sc, with_scores=True)
    from taxi2_amd._native import tri_pairs

    a, b = tri_pairs(n)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    st.free()


def test_align_family_1000bp(engine, oracle_c):
    """The bench workload shape (config 3 generator, 1 000 bp) on a small sample."""
    seqs = family_sequences(24, 1000, 0x7A12, ancestors=4)
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    got, gsc = engine.all_pairs(st, 0, n * (n - 1) // 2, METRICS, None, with_scores=True)
    from taxi2_amd._native import tri_pairs

    a, b = tri_pairs(n)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=SCORE_SETS["default"])
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    # the (x, y) / (y, x) asymmetry the survey found (~1 % of aligned pairs) must be reproduced
    st.free()


def test_align_edge_cases(engine, oracle_c):
    seqs = ["", "A", "N", "NNNN", "ACGT", "ACGT", "TTTT", "ACGTNNACGT", "GATTACA" * 3, "-" * 0, "C"]
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    from taxi2_amd._native import tri_pairs

    a, b = tri_pairs(n)
    for sc in SCORE_SETS.values():
        got, gsc = engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True)
        exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc, threads=1)
        assert_metrics_equal(got, exp)
        assert np.array_equal(gsc, esc)  # empty sequences included: the end-gap score (restated)
        # a pair with an empty side is the other sequence against one end gap: eo + ee (n - 1),
        # 0 for two empty sequences (the restated fill's row / column 0, oracle/restatement.py _gotoh)
        for k, (i, j) in enumerate(zip(a, b)):
            ne = len(seqs[i]) + len(seqs[j])
            if not seqs[i] or not seqs[j]:
                assert gsc[k] == (0 if ne == 0 else sc[4] + sc[5] * (ne - 1)), (seqs[i], seqs[j], gsc[k])
    st.free()


# ----------------------------------------------------------------------------- pre-aligned
def test_prealigned_all_pairs_random(engine, oracle_c):
    seqs = random_sequences(150, 0, 300, 5, "ACGTacgtN--?RY")
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    from taxi2_amd._native import tri_pairs

    a, b = tri_pairs(n)
    got = engine.all_pairs(st, 0, len(a), METRICS)
    exp, _ = oracle_c.batch(seqs, a, b, align=False, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp[:, 0, :])
    assert_metrics_equal(got, exp[:, 1, :])
    st.free()


def test_prealigned_samples_ca200(engine, oracle_c):
    """samples/Taxi2test1_ca200.tab (unaligned 416-618 bp, acgt + n) pre-aligned, config-2 shape."""
    from taxi2_amd.sequences import Sequences, SequenceHandler

    seqs = [s.seq for s in Sequences.fromPath(GOLDEN / "samples" / "Taxi2test1_ca200.tab",
                                              SequenceHandler.Tabfile, idHeader="seqid", seqHeader="sequence")]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    from taxi2_amd._native import tri_pairs

    a, b = tri_pairs(n)
    got = engine.all_pairs(st, 0, len(a), ("p", "jc", "k2p"))
    exp, _ = oracle_c.batch(seqs, a, b, align=False, scores=SCORE_SETS["default"], metrics=("p", "jc", "k2p"))
    assert_metrics_equal(got, exp[:, 0, :], ("p", "jc", "k2p"))
    st.free()


def test_prealigned_samples_ca2000(engine, oracle_c):
    """The full samples/Taxi2test1_ca2000.tab (BASELINE.md's stand-in for the missing ca9000 of
    config 2; 1 999 sequences) pre-aligned, p / jc / k2p over all 1 997 001 unordered pairs against
    the oracle."""
    from taxi2_amd.sequences import Sequences, SequenceHandler
    from taxi2_amd._native import tri_pairs

    seqs = [s.seq for s in Sequences.fromPath(GOLDEN / "samples" / "Taxi2test1_ca2000.tab",
                                              SequenceHandler.Tabfile, idHeader="seqid", seqHeader="sequence")]
    assert len(seqs) == 1999
    st = engine.upload(seqs, align=False)
    a, b = tri_pairs(len(seqs))
    got = engine.all_pairs(st, 0, len(a), ("p", "jc", "k2p"))
    exp, _ = oracle_c.batch(seqs, a, b, align=False, scores=SCORE_SETS["default"], metrics=("p", "jc", "k2p"),
                            threads=16)
    assert_metrics_equal(got, exp[:, 0, :], ("p", "jc", "k2p"))
    assert_metrics_equal(got, exp[:, 1, :], ("p", "jc", "k2p"))
    st.free()


def test_config4_generator_rect_closest(engine, oracle_c):
    """Config 4's generator (BASELINE.json configs[3]: 650 bp family sequences, references seed
    0x7A13, queries 0x7A14, as bench_secondary.leg_config4) on a slice: every (query, reference)
    pair's four metrics, and the closest reference + extras (versus_reference.py:119-129, 184-188)
    against the oracle."""
    from taxi2_amd.synth import family_sequences

    refs = family_sequences(400, 650, 0x7A13)
    qs_ = family_sequences(24, 650, 0x7A13 + 1)
    sq = engine.upload(qs_, align=True)
    sr = engine.upload(refs, align=True)
    sc = SCORE_SETS["default"]
    got = engine.rect_pairs(sq, sr, 0, len(qs_), METRICS, sc)
    pa = np.repeat(np.arange(len(qs_)), len(refs))
    pb = np.tile(np.arange(len(refs)), len(qs_)) + len(qs_)
    exp, _ = oracle_c.batch(qs_ + refs, pa, pb, align=True, scores=sc, threads=16)
    assert_metrics_equal(got, exp[:, 0, :])
    idx, d, ex, _ = engine.closest(sq, sr, 0, len(qs_), "p", ("p-gaps", "jc", "k2p"), sc)
    prim = exp[:, 0, 0].reshape(len(qs_), len(refs))
    for k in range(len(qs_)):
        row = prim[k]
        ok = np.isfinite(row)
        j = int(np.nonzero(ok & (row == row[ok].min()))[0][0])
        assert idx[k] == j and d[k] == row[j]
        assert_metrics_equal(ex[k][None, :], exp[k * len(refs) + j, 0, 1:][None, :], ("p-gaps", "jc", "k2p"))
    sq.free()
    sr.free()


# ----------------------------------------------------------------------------- rect / closest
@pytest.mark.parametrize("align", [True, False])
def test_rect_and_closest(engine, oracle_c, align):
    q = random_sequences(20, 50, 200, 11, "ACGTN")
    r = mutate(q[:7], 12, rate=0.2) + random_sequences(9, 50, 200, 13, "ACGT")
    if not align:
        q = [s.lower() for s in q]
    qs = engine.upload(q, align=align)
    rs = engine.upload(r, align=align)
    sc = SCORE_SETS["default"]
    got = engine.rect_pairs(qs, rs, 0, len(q), METRICS, sc)
    allseq = q + r
    pa = np.repeat(np.arange(len(q)), len(r))
    pb = np.tile(np.arange(len(r)), len(q)) + len(q)
    exp, _ = oracle_c.batch(allseq, pa, pb, align=align, scores=sc)
    assert_metrics_equal(got, exp[:, 0, :])
    # closest: first minimum of the primary metric over defined values (versus_reference.py:184-188)
    idx, d, ex, mat = engine.closest(qs, rs, 0, len(q), "p", ("p-gaps", "jc", "k2p"), sc, want_matrix=True)
    prim = exp[:, 0, 0].reshape(len(q), len(r))
    assert_metrics_equal(mat[..., None], prim[..., None], ("p",))
    for k in range(len(q)):
        row = prim[k]
        ok = np.isfinite(row)
        if not ok.any():
            assert idx[k] == -1
            continue
        j = int(np.nonzero(ok & (row == row[ok].min()))[0][0])
        assert idx[k] == j and d[k] == row[j]
        e = exp[k * len(r) + j, 0, 1:]
        assert_metrics_equal(ex[k][None, :], e[None, :], ("p-gaps", "jc", "k2p"))
    qs.free()
    rs.free()


# ----------------------------------------------------------------------------- single orientation
def _with_env(name, value, fn):
    import os

    old = os.environ.get(name)
    if value is None:
        os.environ.pop(name, None)
    else:
        os.environ[name] = value
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop(name, None)
        else:
            os.environ[name] = old


def test_single_orientation_divergent_pairs(engine, oracle_c):
    """Sequences <= 1023 run the single-orientation kernel (align1_kernel.hpp): orientation A for
    every pair, orientation B re-run only for pairs whose A path passes a divergent Ix/Iy tie.
    Tie-heavy families (identical ancestors, short indels), ragged lengths, lowercase and IUPAC
    bytes (the byte-compare path of the substitution score): counters must equal the oracle's
    AND the two-orientation kernel's, and the (a, b) / (b, a) results must actually differ for
    some pairs so pass 2 is exercised."""
    from taxi2_amd._native import tri_pairs

    fam = family_sequences(20, 700, 0x51, ancestors=3, max_sub=0.05, indel_rate=0.02)
    rng = np.random.default_rng(5)
    seqs = []
    for k, s in enumerate(fam):
        s = s[: 500 + int(rng.integers(0, 200))]
        if k % 4 == 1:
            s = s[:100] + s[100:160].lower() + s[160:]
        if k % 5 == 2:
            b = bytearray(s.encode())
            for pos in rng.integers(0, len(b), 6):
                b[pos] = ord("NRYKM"[int(rng.integers(0, 5))])
            s = b.decode()
        seqs.append(s)
    seqs += ["ACGT" * 255 + "ACG", "A"]  # 1023 (capacity limit) and 1
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    a, b = tri_pairs(n)
    for sc in (SCORE_SETS["default"], SCORE_SETS["generic"], SCORE_SETS["generic1"]):
        got, gsc = engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True)
        two, tsc = _with_env("TAXI2_NO_ALIGN1", "1",
                             lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
        exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
        assert np.array_equal(gsc, esc) and np.array_equal(tsc, esc)
        assert_metrics_equal(got, exp)
        assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(two, nan=9.0))
        asym = ~np.all(np.isclose(np.nan_to_num(exp[:, 0]), np.nan_to_num(exp[:, 1])), axis=1)
        assert asym.sum() > 0
    # rectangular (one ordered orientation only), longer query than reference: swapped rows
    qs = engine.upload(seqs[:6], align=True)
    rs = engine.upload([s[:300] for s in seqs[6:14]], align=True)
    got = engine.rect_pairs(qs, rs, 0, 6, METRICS, SCORE_SETS["default"])
    allseq = seqs[:6] + [s[:300] for s in seqs[6:14]]
    pa = np.repeat(np.arange(6), 8)
    pb = np.tile(np.arange(8), 6) + 6
    exp, _ = oracle_c.batch(allseq, pa, pb, align=True, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp[:, 0, :])
    for s in (st, qs, rs):
        s.free()


def test_single_orientation_long_counters(engine, oracle_c):
    """1 024-4 095 bp run the three-word-counter variant (NW = 3): a tie-heavy 1 500 bp family
    with ragged ends and IUPAC bytes against the oracle and the two-orientation kernel."""
    from taxi2_amd._native import tri_pairs

    fam = family_sequences(10, 1500, 0x52, ancestors=2, max_sub=0.05, indel_rate=0.02)
    rng = np.random.default_rng(6)
    seqs = []
    for k, s in enumerate(fam):
        s = s[: 1100 + int(rng.integers(0, 400))]
        if k % 3 == 1:
            b = bytearray(s.encode())
            for pos in rng.integers(0, len(b), 5):
                b[pos] = ord("NRY"[int(rng.integers(0, 3))])
            s = b.decode()
        seqs.append(s)
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    got, gsc = engine.all_pairs(st, 0, len(a), METRICS, None, with_scores=True)
    two = _with_env("TAXI2_NO_ALIGN1", "1", lambda: engine.all_pairs(st, 0, len(a), METRICS, None))
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=SCORE_SETS["default"])
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(two, nan=9.0))
    st.free()


@pytest.mark.parametrize("chunk", [16, 7])
def test_chained_pairs(engine, oracle_c, chunk):
    """k_align1c streams the rows of consecutive pairs that share their column sequence through
    the same lanes.  Small inputs get chunks of one pair automatically, so TAXI2_A1_CHUNK forces
    long chains here: ragged lengths (len(b) > len(a) breaks a chain), empty and 1-base sequences
    inside chunks, a triangle row boundary mid-chunk, both counter widths, both passes, and the
    rectangle (query-major) source; every result against the oracle and the unchained kernel."""
    from taxi2_amd._native import tri_pairs

    rng = np.random.default_rng(chunk)
    fam = family_sequences(18, 600, 0x53 + chunk, ancestors=3, max_sub=0.05, indel_rate=0.02)
    seqs = [s[: 300 + int(rng.integers(0, 300))] for s in fam]
    seqs[3] = ""
    seqs[7] = "A"
    seqs[11] = seqs[10]  # identical neighbours: a full-tie pair inside a chain
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    for sc in (SCORE_SETS["default"], SCORE_SETS["generic"], SCORE_SETS["generic1"]):
        got, gsc = _with_env("TAXI2_A1_CHUNK", str(chunk),
                             lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
        one = _with_env("TAXI2_A1_NOCHAIN", "1", lambda: engine.all_pairs(st, 0, len(a), METRICS, sc))
        exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
        assert_metrics_equal(got, exp)
        assert np.array_equal(gsc, esc)  # empty sequences included: the end-gap score (restated)
        assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(one, nan=9.0))
    # an offset block of the triangle (chunks start mid-row)
    k0, cnt = 40, 61
    got = _with_env("TAXI2_A1_CHUNK", str(chunk), lambda: engine.all_pairs(st, k0, cnt, METRICS, None))
    exp, _ = oracle_c.batch(seqs, a[k0 : k0 + cnt], b[k0 : k0 + cnt], align=True, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp)
    # rectangle: query-major pairs share the query as their column sequence
    qs = engine.upload(seqs[:5], align=True)
    rs = engine.upload(seqs[5:], align=True)
    got = _with_env("TAXI2_A1_CHUNK", str(chunk), lambda: engine.rect_pairs(qs, rs, 0, 5, METRICS, None))
    pa = np.repeat(np.arange(5), len(seqs) - 5)
    pb = np.tile(np.arange(5, len(seqs)), 5)
    exp, _ = oracle_c.batch(seqs, pa, pb, align=True, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp[:, 0, :])
    # three-word counters (lengths > 1023)
    long = [s * 3 for s in seqs[:8] if s]
    lt = engine.upload(long, align=True)
    la, lb = tri_pairs(len(long))
    got = _with_env("TAXI2_A1_CHUNK", str(chunk), lambda: engine.all_pairs(lt, 0, len(la), METRICS, None))
    exp, _ = oracle_c.batch(long, la, lb, align=True, scores=SCORE_SETS["default"])
    assert_metrics_equal(got, exp)
    for s in (st, qs, rs, lt):
        s.free()


@pytest.mark.parametrize("scores", ["default", "generic", "generic1"])
@pytest.mark.parametrize("chunk", [16, 5])
def test_chained_long_ragged_rect(engine, oracle_c, chunk, scores):
    """2 100-2 600 bp (past the packed kernel's 2 048 columns, so k_align1c with three-word
    counters) query x reference with forced chains: references both shorter and longer than each
    query, so chains start, break and restart in both orientations, and the chain rule (at_swap)
    puts rows up to 1/8 longer than columns.  Round 1's version of that rule faulted here: pass 2
    re-decided the orientation and wrote the other orientation's (null) slot; pass 2 now reuses
    pass 1's choice.  Every result against the oracle."""
    rng = np.random.default_rng(0x2100 + chunk)
    fam = family_sequences(12, 2600, 0x54 + chunk, ancestors=2, max_sub=0.05, indel_rate=0.02)
    seqs = [s[: 2100 + int(rng.integers(0, 500))] for s in fam]
    q, r = seqs[:4], seqs[4:]
    qs = engine.upload(q, align=True)
    rs = engine.upload(r, align=True)
    sc = SCORE_SETS[scores]
    got = _with_env("TAXI2_A1_CHUNK", str(chunk), lambda: engine.rect_pairs(qs, rs, 0, len(q), METRICS, sc))
    pa = np.repeat(np.arange(len(q)), len(r))
    pb = np.tile(np.arange(len(r)), len(q)) + len(q)
    exp, _ = oracle_c.batch(seqs, pa, pb, align=True, scores=sc)
    assert_metrics_equal(got, exp[:, 0, :])
    for s in (qs, rs):
        s.free()
