"""GPU: NCD (distances.py:351-358) against the oracle (Python zlib 1.2.11 + the alignment
restatement), per pair, through both tasks."""

from __future__ import annotations

import random
import zlib

import numpy as np
import pytest

from tests.seqgen import family_sequences, mutate, random_sequences

pytestmark = pytest.mark.gpu

DEFAULT = (1, -1, -8, -1, -1, -1)


def test_zlib_lengths_exact(engine):
    rng = random.Random(21)
    seqs = []
    for L in (0, 1, 2, 3, 7, 64, 500, 1000, 3000, 8000):
        for alpha in ("ACGT", "ACGTN-", "acgtNRYKM", "AC"):
            seqs.append("".join(rng.choice(alpha) for _ in range(L)))
    seqs += family_sequences(6, 1000, 5, ancestors=2)
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    got1 = engine.zlib_lengths(st, np.arange(n))
    exp1 = [len(zlib.compress(s.upper().encode())) for s in seqs]
    assert got1.tolist() == exp1
    xs = np.array([rng.randrange(n) for _ in range(200)])
    ys = np.array([rng.randrange(n) for _ in range(200)])
    got2 = engine.zlib_lengths(st, xs, st, ys)
    exp2 = [len(zlib.compress((seqs[a] + seqs[b]).upper().encode())) for a, b in zip(xs, ys)]
    assert got2.tolist() == exp2
    st.free()


def test_ncd_pairs_raw_both_orders(engine):
    from oracle import restatement as R

    base = random_sequences(10, 50, 900, 4, "ACGTN", n_rate=0.03)
    seqs = base + [s.lower() for s in mutate(base, 5, rate=0.1)] + ["", "-A-C-"]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    rng = random.Random(2)
    xs = np.array([rng.randrange(n) for _ in range(120)])
    ys = np.array([rng.randrange(n) for _ in range(120)])
    got = engine.ncd_pairs(st, st, xs, ys, aligned=False, both=True)
    for k, (a, b) in enumerate(zip(xs, ys)):
        assert got[k, 0] == R.ncd(seqs[a], seqs[b])
        assert got[k, 1] == R.ncd(seqs[b], seqs[a])
    st.free()


@pytest.mark.parametrize("scores", [DEFAULT, (2, -3, -5, -2, -1, -1), (1, -1, -2, -2, -1, -1)])
def test_ncd_pairs_aligned_both_orders(engine, scores):
    """On the gapped strings of the first alignment of each ordered pair (the strings VersusAll
    hands the metric)."""
    from oracle import restatement as R

    base = random_sequences(6, 20, 140, 8, "ACGT", n_rate=0.02)
    seqs = [R.normalize(s) for s in base + mutate(base, 9, rate=0.15)]
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    xs = np.repeat(np.arange(n), n)
    ys = np.tile(np.arange(n), n)
    got = engine.ncd_pairs(st, st, xs, ys, scores, aligned=True, both=True)
    sc = R.Scores(*scores)
    for k, (a, b) in enumerate(zip(xs, ys)):
        ax, ay, _ = R.align(seqs[a], seqs[b], sc)
        by, bx, _ = R.align(seqs[b], seqs[a], sc)
        assert got[k, 0] == R.ncd(ax, ay), (a, b)
        assert got[k, 1] == R.ncd(by, bx), (a, b)
    st.free()


def test_ncd_metric_calculate(engine):
    from oracle import restatement as R
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence

    x, y = Sequence("a", "gg-ccnccta" * 7), Sequence("b", "GGACCACCAA" * 7)
    d = DistanceMetric.NCD().calculate(x, y)
    assert d.metric == DistanceMetric.NCD() and d.d == R.ncd(x.seq, y.seq)


@pytest.mark.parametrize("align", [True, False])
def test_versus_all_with_ncd(tmp_path, engine, oracle_c, align):
    from oracle import restatement as R
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    raw = random_sequences(5, 40, 120, 31, "ACGTN", n_rate=0.05)
    raw = raw + mutate(raw[:3], 32, rate=0.1)
    seqs = [Sequence(f"s{k}", s, {"voucher": str(k)}) for k, s in enumerate(raw)]
    seqs.append(Sequence("s0", raw[0], {"voucher": "0"}))  # duplicate tuple -> None row/col
    task = VersusAll()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input.sequences = Sequences(seqs)
    task.params.pairs.align = align
    task.params.pairs.write = False
    task.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.NCD()]
    work = [s.normalize() for s in seqs] if align else seqs
    D = task.compute_distances(work)
    n = len(work)
    for i in range(n):
        for j in range(n):
            same = (work[i].id, work[i].seq, work[i].extras) == (work[j].id, work[j].seq, work[j].extras)
            if same and (not align or R.align(work[i].seq, work[j].seq)[0] == R.align(work[i].seq, work[j].seq)[1]):
                assert np.isnan(D[i, j]).all()
                continue
            if align:
                ax, ay, _ = R.align(work[i].seq, work[j].seq)
            else:
                ax, ay = work[i].seq, work[j].seq
            assert D[i, j, 1] == R.ncd(ax, ay), (i, j)
            p = R.metric("p", ax, ay)
            assert (np.isnan(D[i, j, 0]) and p is None) or D[i, j, 0] == p
    task.start()
    assert (tmp_path / "out/distances/matricial/ncd.tsv").exists()


def test_versus_reference_ncd_primary_and_extra(tmp_path, engine):
    from oracle import restatement as R
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusReference

    q = random_sequences(6, 40, 110, 41, "ACGT")
    r = mutate(q[:4], 42, rate=0.2) + random_sequences(3, 40, 110, 43, "ACGT")
    for primary, extras in ((DistanceMetric.NCD(), [DistanceMetric.Uncorrected()]),
                            (DistanceMetric.Uncorrected(), [DistanceMetric.NCD(), DistanceMetric.JukesCantor()])):
        task = VersusReference()
        task.engine = engine
        task.progress_handler = None
        task.work_dir = tmp_path / f"out_{primary}"
        task.input.data = Sequences([Sequence(f"q{k}", s) for k, s in enumerate(q)])
        task.input.reference = Sequences([Sequence(f"r{k}", s) for k, s in enumerate(r)])
        task.params.pairs.write = False
        task.params.distances.metric = primary
        task.params.distances.extra_metrics = list(extras)
        task.start()
        for qi, ri, d, ext in task.closest:
            vals = []
            for rj in range(len(r)):
                ax, ay, _ = R.align(R.normalize(q[qi]), R.normalize(r[rj]))
                vals.append(R.ncd(ax, ay) if str(primary) == "ncd" else R.metric("p", ax, ay))
            ok = [v for v in vals if v is not None]
            assert ri == vals.index(min(ok)) and d == min(ok)
            ax, ay, _ = R.align(R.normalize(q[qi]), R.normalize(r[ri]))
            for k, m in enumerate(task.params.distances.extra_metrics):
                exp = R.ncd(ax, ay) if str(m) == "ncd" else R.metric(str(m), ax, ay)
                # ncd, p, p-gaps exact; jc / k2p within north_star's 1e-12 (the GPU's log)
                tol = 1e-12 if str(m) in ("jc", "k2p") else 0.0
                assert (exp is None and np.isnan(ext[k])) or abs(ext[k] - exp) <= tol


def test_scratch_regrowth_interleaved(engine):
    """Context scratch regrows across entry points (formatter buffers, NCD slabs): interleaved calls
    with growing sizes stay correct (regression: a regrowth once freed an unrelated buffer)."""
    seqs = ["ACGT" * 50, "ACGA" * 60, "TTGCA" * 30]
    st = engine.upload(seqs, align=False)
    vals = np.array([[0.5, np.nan], [1.25, -0.0]])
    for n in (1, 70, 300, 5000):
        idx = np.arange(n) % 3
        assert engine.zlib_lengths(st, idx).tolist() == [len(zlib.compress(seqs[i].encode())) for i in idx]
        assert engine.format_rows(vals, ["a", "b"], None, decimals=2).decode() == "a\t0.50\tNA\nb\t1.25\t-0.00\n"
    st.free()


def test_zlib_lengths_multi_block(engine):
    """Concatenations of 10-32 kB (several deflate blocks, one window) against Python's zlib."""
    rng = random.Random(23)
    seqs = ["".join(rng.choice("ACGT") for _ in range(L)) for L in (9000, 10000, 12000, 16383, 20000, 32000)]
    seqs += ["".join(rng.choice("ACGTN-") for _ in range(11000)), "ACGT" * 4000]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    got1 = engine.zlib_lengths(st, np.arange(n))
    assert got1.tolist() == [len(zlib.compress(s.upper().encode())) for s in seqs]
    xs = np.array([0, 1, 2, 3, 6, 7, 1, 4])
    ys = np.array([1, 0, 3, 2, 0, 6, 6, 5])
    got2 = engine.zlib_lengths(st, xs, st, ys)
    assert got2.tolist() == [len(zlib.compress((seqs[a] + seqs[b]).upper().encode())) for a, b in zip(xs, ys)]
    st.free()


def test_ncd_aligned_long_sequences(engine):
    """NCD on the aligned strings of 9 000-10 000 bp pairs: ~20 kB concatenations (multi-block), from
    the column-tiled aligner's strings, against Python's zlib on those same strings."""
    from oracle import restatement as R

    fam = family_sequences(3, 10000, 0x56, ancestors=1, max_sub=0.1, indel_rate=0.01)
    seqs = [fam[0], fam[1][:9000], fam[2]]
    st = engine.upload(seqs, align=True)
    xs, ys = np.array([0, 1, 2]), np.array([1, 2, 0])
    got = engine.ncd_pairs(st, st, xs, ys, DEFAULT, aligned=True, both=True)
    strings = engine.align_strings(st, st, xs, ys, DEFAULT, both=True)
    for k, pair in enumerate(strings):
        (ax, ay), (bx, by) = pair
        assert len(ax) + len(ay) > 16383
        assert got[k, 0] == R.ncd(ax, ay)
        assert got[k, 1] == R.ncd(by, bx)
    st.free()


def test_zlib_lengths_wave_path_edges(engine):
    """The one-wave-per-stream path (k_zlen_wave, streams <= 16 384 bytes): high-entropy inputs
    near its 16 384-byte limit (mostly literals: up to the 16 383-symbol block flush), DNA
    families with long repeats (matches reaching nice_match / MAX_MATCH, second candidate round),
    tiny inputs; against Python's zlib and against the one-thread-per-stream path."""
    import os

    rng = random.Random(29)
    wide = "".join(chr(c) for c in list(range(33, 97)) + list(range(123, 127)))

    def no_repeat(L: int) -> str:  # no 3-gram twice: every byte a literal, 16 383 of them flush a block
        out, seen = ["!", "#"], set()
        while len(out) < L:
            c = rng.choice(wide)
            g = out[-2] + out[-1] + c
            if g not in seen:
                seen.add(g)
                out.append(c)
        return "".join(out)

    seqs = [no_repeat(16384), no_repeat(16383), "".join(rng.choice(wide) for _ in range(16200))]
    fam = family_sequences(4, 2500, 0x29, ancestors=1, max_sub=0.01, indel_rate=0.002)
    seqs += fam + ["ACGT" * 600, "A" * 3000, "", "AC", "ACG", "ACGTACGT"]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    exp1 = [len(zlib.compress(s.upper().encode())) for s in seqs]
    assert engine.zlib_lengths(st, np.arange(n)).tolist() == exp1
    xs = np.array([3, 4, 5, 6, 7, 8, 9, 3, 10])
    ys = np.array([4, 3, 6, 5, 8, 7, 3, 9, 10])
    exp2 = [len(zlib.compress((seqs[a] + seqs[b]).upper().encode())) for a, b in zip(xs, ys)]
    assert engine.zlib_lengths(st, xs, st, ys).tolist() == exp2
    os.environ["TAXI2_ZLEN_SERIAL"] = "1"
    try:
        assert engine.zlib_lengths(st, xs, st, ys).tolist() == exp2
    finally:
        os.environ.pop("TAXI2_ZLEN_SERIAL")
    st.free()


def test_zlib_lengths_sliding_window(engine):
    """Streams past one 64 KiB window (65 273 bytes): the one-thread parse slides the window as
    zlib's fill_window does; single streams and concatenations up to 300 kB vs Python's zlib."""
    rng = random.Random(31)
    dna = "".join(rng.choice("ACGT") for _ in range(300000))
    rep = (dna[:173] * 1800)[:300000]
    seqs = [dna[:65274], dna[:65537], dna[:98305], dna[:131073], dna, rep[:200000], rep[:70001],
            mutate([rep[:150000]], 3, rate=0.02)[0], "ACGT" * 10]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    got1 = engine.zlib_lengths(st, np.arange(n))
    assert got1.tolist() == [len(zlib.compress(s.upper().encode())) for s in seqs]
    xs, ys = np.array([0, 1, 6, 8, 5]), np.array([6, 8, 2, 3, 7])
    got2 = engine.zlib_lengths(st, xs, st, ys)
    assert got2.tolist() == [len(zlib.compress((seqs[a] + seqs[b]).upper().encode())) for a, b in zip(xs, ys)]
    st.free()


def test_ncd_latin1_sequences(engine):
    """Non-ASCII (latin-1) sequences: alfpy compresses str.upper().encode() -- two UTF-8 bytes per
    accented letter, "ß" -> "SS" -- raw pairs (cached and per-pair paths) and aligned pairs."""
    from oracle import restatement as R

    rng = random.Random(37)
    alpha = "ACGTNacgtéÉßµÿñ-"
    seqs = ["".join(rng.choice(alpha) for _ in range(rng.randrange(0, 400))) for _ in range(14)] + ["ß", "ÿ" * 40]
    st = engine.upload(seqs, align=False)
    n = len(seqs)
    assert engine.zlib_lengths(st, np.arange(n)).tolist() == [len(zlib.compress(s.upper().encode())) for s in seqs]
    xs = np.repeat(np.arange(n), n)
    ys = np.tile(np.arange(n), n)
    got = engine.ncd_pairs(st, st, xs, ys, aligned=False, both=True)  # pairs >> sequences: cached C(x)
    few = engine.ncd_pairs(st, st, xs[:5], ys[:5], aligned=False, both=True)  # per-pair streams
    for k, (a, b) in enumerate(zip(xs, ys)):
        assert got[k, 0] == R.ncd(seqs[a], seqs[b]) and got[k, 1] == R.ncd(seqs[b], seqs[a]), (a, b)
    assert np.array_equal(few, got[:5])
    st.free()
    al = [s.replace("-", "") for s in seqs[:8]]
    st = engine.upload(al, align=True)
    xs = np.repeat(np.arange(8), 8)
    ys = np.tile(np.arange(8), 8)
    got = engine.ncd_pairs(st, st, xs, ys, DEFAULT, aligned=True, both=True)
    for k, (a, b) in enumerate(zip(xs, ys)):
        ax, ay, _ = R.align(al[a], al[b])
        by, bx, _ = R.align(al[b], al[a])
        assert got[k, 0] == R.ncd(ax, ay) and got[k, 1] == R.ncd(by, bx), (a, b)
    st.free()
