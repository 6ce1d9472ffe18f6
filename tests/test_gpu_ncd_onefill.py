"""GPU: NCD from the aligners' own string slots -- every metric of a pair from ONE fill, as
versus_all.py:546-552 feeds one alignment per ordered pair to p / p-gaps / jc / k2p AND ncd
(distances.py:351-358).

The oracle is the Python restatement (oracle/restatement.py: the first Biopython alignment of each
ordered pair + alfpy's NCD over Python's zlib 1.2.11).  The packed walkers' strings
(all_pairs / tri_strings_dev / rect_strings_dev with "ncd", taxi2_ncd_slots_dev) are also checked
against the round-1 trace kernels' strings (TAXI2_NO_WALK_STRINGS=1 forces them), bit for bit.
"""

from __future__ import annotations

import os
import random

import numpy as np
import pytest

from tests.seqgen import family_sequences, mutate, random_sequences

pytestmark = pytest.mark.gpu

DEFAULT = (1, -1, -8, -1, -1, -1)
GENERIC1 = (2, -3, -5, -2, -3, -2)  # best-open fill, one extend for internal and end gaps
GENERIC = (2, -3, -5, -2, -1, -1)   # tagged sign-digit fill
FOUR = ("p", "p-gaps", "jc", "k2p")


def tie_heavy(seed: int) -> list[str]:
    """Two-letter runs, families with indels, N runs, one short / one long sequence whose alignment
    is mostly end gaps (its concatenation exceeds the first zlen pass's likely length: the redo
    pass), and an empty sequence."""
    from oracle import restatement as R

    rng = random.Random(seed)
    fam = family_sequences(4, 300, seed, ancestors=2)
    two = ["".join(rng.choice("AC") for _ in range(rng.randrange(40, 160))) for _ in range(4)]
    base = random_sequences(3, 60, 260, seed + 1, "ACGTN", n_rate=0.05)
    seqs = fam + two + base + mutate(base[:2], seed + 2, rate=0.2)
    seqs += ["A" * 150 + "C" * 150, "C" * 150 + "G" * 150, ""]
    return [R.normalize(s) for s in seqs]


def oracle_ncd(seqs, a, b, scores):
    from oracle import restatement as R

    sc = R.Scores(*scores)
    out = np.empty((len(a), 2))
    for k, (i, j) in enumerate(zip(a, b)):
        ax, ay, _ = R.align(seqs[i], seqs[j], sc)
        by, bx, _ = R.align(seqs[j], seqs[i], sc)
        out[k, 0] = R.ncd(ax, ay)
        out[k, 1] = R.ncd(by, bx)
    return out


def same(x, y) -> bool:
    """Bit-identical, NaN positions included."""
    return np.array_equal(np.asarray(x).view(np.int64), np.asarray(y).view(np.int64))


@pytest.mark.parametrize("scores", [DEFAULT, GENERIC1, GENERIC])
def test_all_pairs_with_ncd_one_fill(engine, scores):
    from taxi2_amd._native import tri_pairs

    seqs = tie_heavy(3)
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    npairs = n * (n - 1) // 2
    five = engine.all_pairs(st, 0, npairs, FOUR + ("ncd",), scores)
    four = engine.all_pairs(st, 0, npairs, FOUR, scores)
    assert same(five[..., :4], four), "the counter metrics change when NCD rides the same fill"
    a, b = tri_pairs(n)
    exp = oracle_ncd(seqs, a, b, scores)
    assert np.array_equal(five[..., 4], exp), "NCD differs from the restatement"
    # NCD first in the list, twice: every NCD column is written, the others stay the counters
    mixed = engine.all_pairs(st, 0, npairs, ("ncd", "p", "ncd"), scores)
    assert np.array_equal(mixed[..., 0], exp) and np.array_equal(mixed[..., 2], exp)
    assert same(mixed[..., 1], four[..., 0])
    st.free()


def test_walker_ncd_equals_trace_kernel_ncd(engine):
    """ncd_pairs on the packed walkers' strings == on the trace kernels' strings (TAXI2_NO_WALK_STRINGS),
    both orientations, tie-heavy pairs; and the host all_pairs fallback (trace strings) agrees too."""
    seqs = tie_heavy(5)
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    rng = random.Random(7)
    xs = np.array([rng.randrange(n) for _ in range(300)])
    ys = np.array([rng.randrange(n) for _ in range(300)])
    npairs = n * (n - 1) // 2
    for scores in (DEFAULT, GENERIC1):
        walk = engine.ncd_pairs(st, st, xs, ys, scores, aligned=True, both=True)
        os.environ["TAXI2_NO_WALK_STRINGS"] = "1"
        try:
            trace = engine.ncd_pairs(st, st, xs, ys, scores, aligned=True, both=True)
            fb = engine.all_pairs(st, 0, npairs, FOUR + ("ncd",), scores)
        finally:
            del os.environ["TAXI2_NO_WALK_STRINGS"]
        assert np.array_equal(walk, trace)
        assert same(fb, engine.all_pairs(st, 0, npairs, FOUR + ("ncd",), scores))
    st.free()


def test_all_pairs_dev_with_ncd_and_slots_entry(engine):
    """The device form (caller's stream) and taxi2_ncd_slots_dev on tri_strings_dev slots give the
    host path's values; rect_strings_dev with "ncd" gives the (q, r) orientation."""
    import torch

    from taxi2_amd._native import tri_pairs

    seqs = family_sequences(12, 700, 9, ancestors=3) + tie_heavy(11)[:6]
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    npairs = n * (n - 1) // 2
    host = engine.all_pairs(st, 0, npairs, FOUR + ("ncd",), DEFAULT)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        out = torch.empty((npairs, 2, 5), dtype=torch.float64, device=dev)
        engine.all_pairs_dev(st, 0, npairs, FOUR + ("ncd",), out.data_ptr(), DEFAULT, None, s.cuda_stream)
        cap = 2 * max(len(x) for x in seqs) + 1
        d = torch.empty((npairs, 2, 2), dtype=torch.float64, device=dev)
        sx = torch.empty((npairs, 2, cap), dtype=torch.uint8, device=dev)
        sy = torch.empty((npairs, 2, cap), dtype=torch.uint8, device=dev)
        sl = torch.empty((npairs, 2), dtype=torch.int32, device=dev)
        engine.tri_strings_dev(st, 0, npairs, ("p", "ncd"), d.data_ptr(), cap, sx.data_ptr(), sy.data_ptr(),
                               sl.data_ptr(), DEFAULT, s.cuda_stream)
        a, b = tri_pairs(n)
        lens = np.array([len(x) for x in seqs])
        end = torch.as_tensor(lens[a] + lens[b], device=dev)
        v = torch.empty((npairs, 2), dtype=torch.float64, device=dev)
        engine.ncd_slots_dev(sx.data_ptr(), sy.data_ptr(), sl.data_ptr(), cap, 2, 2, end.data_ptr(), npairs,
                             int(lens.max()), v.data_ptr(), stream=s.cuda_stream)
        v1 = torch.empty((npairs,), dtype=torch.float64, device=dev)
        engine.ncd_slots_dev(sx.data_ptr(), sy.data_ptr(), sl.data_ptr(), cap, 2, 1, end.data_ptr(), npairs,
                             int(lens.max()), v1.data_ptr(), stream=s.cuda_stream)
        R_ = n
        rc = torch.empty((3 * R_, 2), dtype=torch.float64, device=dev)
        rsx = torch.empty((3 * R_, cap), dtype=torch.uint8, device=dev)
        rsy = torch.empty((3 * R_, cap), dtype=torch.uint8, device=dev)
        rsl = torch.empty((3 * R_,), dtype=torch.int32, device=dev)
        engine.rect_strings_dev(st, st, 2, 5, ("ncd", "k2p"), rc.data_ptr(), cap, rsx.data_ptr(), rsy.data_ptr(),
                                rsl.data_ptr(), DEFAULT, s.cuda_stream)
    s.synchronize()
    assert same(out.cpu().numpy(), host)
    assert same(d.cpu().numpy()[..., 1], host[..., 4]) and same(d.cpu().numpy()[..., 0], host[..., 0])
    assert same(v.cpu().numpy(), host[..., 4])
    assert same(v1.cpu().numpy(), host[:, 0, 4])
    exp = oracle_ncd(seqs, np.repeat(np.arange(2, 5), R_), np.tile(np.arange(R_), 3), DEFAULT)
    assert np.array_equal(rc.cpu().numpy()[:, 0], exp[:, 0])
    st.free()


@pytest.mark.parametrize("scores", [DEFAULT, GENERIC1])
def test_task_ncd_with_aligned_pairs_walked(tmp_path, engine, scores):
    """VersusAll with aligned_pairs.txt on (the walked one-fill path) and p + ncd: the NCD values come
    from the walks' own strings and equal the restatement; the files equal the non-walked path's."""
    from oracle import restatement as R
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    raw = tie_heavy(13)[:12]
    seqs = [Sequence(f"s{k}", s) for k, s in enumerate(raw)]

    def run(out, env):
        if env:
            os.environ["TAXI2_PAIRS_RECT"] = "1"
        try:
            t = VersusAll()
            t.engine, t.progress_handler, t.work_dir = engine, None, out
            t.input.sequences = Sequences(seqs)
            t.params.pairs.scores = dict(zip(("match_score", "mismatch_score", "internal_open_gap_score",
                                              "internal_extend_gap_score", "end_open_gap_score",
                                              "end_extend_gap_score"), scores))
            t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.NCD()]
            t.start()
            return t
        finally:
            os.environ.pop("TAXI2_PAIRS_RECT", None)

    t1 = run(tmp_path / "tri", False)
    t2 = run(tmp_path / "rect", True)
    assert t1.pairs_walked and t2.pairs_walked
    sc = R.Scores(*scores)
    n = len(raw)
    for i in range(n):
        for j in range(n):
            if i == j:
                continue
            ax, ay, _ = R.align(R.normalize(raw[i]), R.normalize(raw[j]), sc)
            assert t1.distances[i, j, 1] == R.ncd(ax, ay), (i, j)
    for f in ("distances/linear.tsv", "distances/matricial/ncd.tsv", "align/aligned_pairs.txt", "summary.tsv"):
        assert (tmp_path / "tri" / f).read_bytes() == (tmp_path / "rect" / f).read_bytes(), f


def test_self_strings_mismatch_above_match(engine):
    """with mismatch > match the self alignment need not be the identity (a one-column
    shift of a 10-base sequence scores 9 * 5 - 2 = 43 against 10): self_strings must align."""
    from oracle import restatement as R
    from taxi2_amd.tasks.versus_all import self_strings
    from taxi2_amd.sequences import Sequence

    scores = (1, 5, -1, -1, -1, -1)
    raw = ["ACGTACGTAC", "AAAACCCCGG", "ACGT" * 20, "A"]
    seqs = [Sequence(f"s{k}", s) for k, s in enumerate(raw)]
    st = engine.upload(raw, align=True)
    got = self_strings(engine, st, seqs, np.arange(len(raw)), scores)
    ref = engine.align_strings(st, st, np.arange(len(raw)), np.arange(len(raw)), scores)
    assert got == ref
    for k, s in enumerate(raw):
        ax, ay, _ = R.align(s, s, R.Scores(*scores))
        assert got[k] == (ax, ay)
    assert got[0] != (raw[0], raw[0])  # the shifted alignment, not the identity
    st.free()


def test_ncd_slots_fused_lengths_edges(engine):
    """taxi2_ncd_slots_dev on crafted slot strings: every orientation's NCD equals alfpy's formula over
    Python's zlib, where the fused deflate pass (C(x) from the parse of x + y, forked MIN_LOOKAHEAD
    before x's end) meets its edges -- x shorter than the fork margin (0, 1, 3, 200, 261, 262, 263
    bytes), matches running through the fork point and across x's end (periodic x, y = x, y a
    suffix of x), long literal runs, gaps, and orientation pairs that differ (the singles)."""
    import torch

    from oracle import restatement as R

    rng = random.Random(17)

    def dna(n, alpha="ACGT"):
        return "".join(rng.choice(alpha) for _ in range(n))

    xs, ys = [], []
    for L in (0, 1, 3, 200, 261, 262, 263, 264, 300, 520, 777, 1000):
        xs.append(dna(L))
        ys.append(dna(rng.randrange(0, 600)))
    per = "ACGTTGCA" * 120
    xs += [per[:500], per[:700], per[:1000], "A" * 900, dna(400, "AC-")]
    ys += [per[:500], per[200:900], per[:30], "A" * 5, dna(380, "AC-")]
    base = dna(800)
    xs += [base, base[:600] + dna(200)]
    ys += [base[300:], base[100:]]
    xs += ["", ""]  # both strings empty (an empty sequence against itself): C(x) = C(x + y)
    ys += ["", ""]
    n = len(xs)
    # two orientations per pair: the second one is (x, y) itself (same alignment) for even k, a
    # different pair of strings for odd k -- the skipped and the computed singles
    o1 = [(xs[k], ys[k]) if k % 2 == 0 else (dna(len(xs[k]) // 2 + 5), dna(len(ys[k]) // 2 + 3)) for k in range(n)]
    lens = [max(len(xs[k]), len(ys[k]), len(o1[k][0]), len(o1[k][1])) for k in range(n)]
    cap = 2 * max(lens) + 8
    end = np.array([cap - 4] * n, dtype=np.int64)
    sx = np.zeros((n, 2, cap), dtype=np.uint8)
    sy = np.zeros((n, 2, cap), dtype=np.uint8)
    sl = np.zeros((n, 2), dtype=np.int32)
    for k in range(n):
        # slot strings are the two aligned strings, equal length: pad the shorter with gaps
        for o, (a, b) in enumerate(((xs[k], ys[k]), o1[k])):
            m = max(len(a), len(b))
            a, b = a.ljust(m, "-"), b.ljust(m, "-")
            sx[k, o, end[k] - m:end[k]] = np.frombuffer(a.encode(), np.uint8)
            sy[k, o, end[k] - m:end[k]] = np.frombuffer(b.encode(), np.uint8)
            sl[k, o] = m
    dev = torch.device("cuda", 0)
    t = {k: torch.as_tensor(v, device=dev) for k, v in (("sx", sx), ("sy", sy), ("sl", sl), ("end", end))}
    out = torch.empty((n, 2), dtype=torch.float64, device=dev)
    engine.ncd_slots_dev(t["sx"].data_ptr(), t["sy"].data_ptr(), t["sl"].data_ptr(), cap, 2, 2, t["end"].data_ptr(), n,
                         cap // 2, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for k in range(n):
        m0 = int(sl[k, 0])
        a0 = bytes(sx[k, 0, end[k] - m0:end[k]]).decode()
        b0 = bytes(sy[k, 0, end[k] - m0:end[k]]).decode()
        m1 = int(sl[k, 1])
        a1 = bytes(sx[k, 1, end[k] - m1:end[k]]).decode()
        b1 = bytes(sy[k, 1, end[k] - m1:end[k]]).decode()
        e0, e1 = R.ncd(a0, b0), R.ncd(b1, a1)  # orientation 1 is the (b, a) metric
        assert (np.isnan(got[k, 0]) and e0 is None) or got[k, 0] == e0, (k, len(a0))
        assert (np.isnan(got[k, 1]) and e1 is None) or got[k, 1] == e1, (k, len(a1))
