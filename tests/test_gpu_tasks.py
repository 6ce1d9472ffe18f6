"""GPU: aligned strings, per-pair API and the end-to-end tasks against the oracle."""

from __future__ import annotations

import json
import random

import numpy as np
import pytest

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

SAMPLES = GOLDEN / "samples"


def read_tab(name):
    from taxi2_amd.sequences import SequenceHandler, Sequences

    return list(Sequences.fromPath(SAMPLES / name, SequenceHandler.Tabfile, idHeader="seqid", seqHeader="sequence"))


# ----------------------------------------------------------------------------- aligned strings
def test_aligner_golden_vectors(engine):
    """PairwiseAligner.Biopython.align on tests/test_align.py:49-163 vectors."""
    from taxi2_amd.align import PairwiseAligner, Scores
    from taxi2_amd.pairs import SequencePair
    from taxi2_amd.sequences import Sequence

    for r in json.loads((GOLDEN / "align_tests.json").read_text()):
        al = PairwiseAligner.Biopython(Scores(**r["scores"]), engine=engine)
        ax, ay = al.align(SequencePair(Sequence("idx", r["x"]), Sequence("idy", r["y"])))
        assert ax.id == "idx" and ay.id == "idy"
        assert [ax.seq, ay.seq] in r["solutions"], (r, ax.seq, ay.seq)


@pytest.mark.parametrize("scores", [(1, -1, -8, -1, -1, -1), (2, -3, -5, -2, -1, -1), (1, -1, -2, -2, -1, -1),
                                    (1, 0, 0, 0, 0, 0)])
def test_align_strings_both_orientations(engine, scores):
    """GPU trace + walk == the restatement's traceback, for (x, y) and for (y, x)."""
    from oracle import restatement as R

    rng = random.Random(sum(scores) + 17)
    seqs = []
    for _ in range(24):
        x = "".join(rng.choice("ACGTN") for _ in range(rng.randint(1, 120)))
        seqs.append(x)
    for k in range(12):
        seqs.append("".join(c if rng.random() > 0.15 else rng.choice("ACGT") for c in seqs[k]))
    st = engine.upload(seqs, align=True)
    xs = np.array([rng.randrange(len(seqs)) for _ in range(60)])
    ys = np.array([rng.randrange(len(seqs)) for _ in range(60)])
    got = engine.align_strings(st, st, xs, ys, scores, both=True)
    sc = R.Scores(*scores)
    for (a, b), (ab, ba) in zip(zip(xs, ys), got):
        ax, ay, _ = R.align(seqs[a], seqs[b], sc)
        assert ab == (ax, ay)
        # the (y, x) alignment Biopython returns, in (x, y) column order
        by, bx, _ = R.align(seqs[b], seqs[a], sc)
        assert ba == (bx, by)
    st.free()


def test_distance_metric_calculate_per_pair(engine, oracle_c):
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence

    x, y = Sequence("idx", "gg-ccnccta"), Sequence("idy", "ggaccaccaa")
    assert DistanceMetric.Uncorrected().calculate(x, y).d == 1.0 / 8.0
    assert DistanceMetric.UncorrectedWithGaps().calculate(x, y).d == 2.0 / 9.0
    assert DistanceMetric.Uncorrected().calculate(Sequence("a", "---"), Sequence("b", "nnn")).d is None
    r = DistanceMetric.Kimura2P().calculate(x, y)
    assert r.metric == DistanceMetric.Kimura2P() and r.x.id == "idx" and r.y.id == "idy"


# ----------------------------------------------------------------------------- tasks
def expected_versus_all(seqs, labels, align, oracle_c):
    """(N, N, M) expected matrix from the C oracle + the diagonal rule."""
    from oracle import restatement as R

    work = [s.normalize() for s in seqs] if align else seqs
    n = len(work)
    a = np.repeat(np.arange(n), n)
    b = np.tile(np.arange(n), n)
    out, _ = oracle_c.batch([s.seq for s in work], a, b, align=align, scores=(1, -1, -8, -1, -1, -1),
                            metrics=labels)
    D = out[:, 0, :].reshape(n, n, len(labels))
    for i in range(n):
        for j in range(n):
            if (work[i].id, work[i].seq, work[i].extras) == (work[j].id, work[j].seq, work[j].extras):
                if not align or R.align(work[i].seq, work[j].seq)[0] == R.align(work[i].seq, work[j].seq)[1]:
                    D[i, j] = np.nan
    return work, D


def render_expected(tmp, work, D, metrics, fmt="{:.4f}", missing="NA"):
    from taxi2_amd.distances import Distance, DistanceHandler

    lin = tmp / "exp_linear.tsv"
    with DistanceHandler.Linear.WithExtras(lin, "w", missing=missing, formatter=fmt) as fh:
        for i, x in enumerate(work):
            for j, y in enumerate(work):
                for m, metric in enumerate(metrics):
                    v = D[i, j, m]
                    fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))
    mats = {}
    for m, metric in enumerate(metrics):
        p = tmp / f"exp_{metric}.tsv"
        with DistanceHandler.Matrix(p, "w", missing=missing, formatter=fmt) as fh:
            for i, x in enumerate(work):
                for j, y in enumerate(work):
                    v = D[i, j, m]
                    fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))
        mats[str(metric)] = p
    return lin, mats


def test_versus_all_config1(tmp_path, engine, oracle_c):
    """Config 1: samples/Taxi2test1_10.tab, versusAll, p only, align=True (reference default),
    100 ordered rows; plus aligned_pairs.txt on a truncated copy (pure-Python traceback oracle)."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequences
    from taxi2_amd.tasks import VersusAll

    seqs = read_tab("Taxi2test1_10.tab")
    task = VersusAll()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input.sequences = Sequences(seqs)
    task.params.distances.metrics = [DistanceMetric.Uncorrected()]
    task.params.pairs.write = False
    res = task.start()
    assert res.seconds_taken > 0
    work, D = expected_versus_all(seqs, ("p",), True, oracle_c)
    lin, mats = render_expected(tmp_path, work, D, task.params.distances.metrics)
    assert (tmp_path / "out/distances/linear.tsv").read_text() == lin.read_text()
    assert (tmp_path / "out/distances/matricial/p.tsv").read_text() == mats["p"].read_text()


@pytest.mark.parametrize("latin1", [False, True])
def test_versus_all_aligned_pairs_file(tmp_path, engine, latin1):
    """aligned_pairs.txt file-exact against the restatement; with a latin-1 character in a
    sequence the file must stay the reference's UTF-8 text (the walk-strings path,
    which copies single latin-1 bytes, is gated off for it: versus_all.walk_strings_ok)."""
    from oracle import restatement as R
    from taxi2_amd.pairs import SequencePair, SequencePairHandler
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    seqs = [Sequence(s.id, s.seq[:80], s.extras) for s in read_tab("Taxi2test1_10.tab")[:5]]
    if latin1:
        seqs[2] = Sequence(seqs[2].id, seqs[2].seq[:30] + "é" + seqs[2].seq[30:], seqs[2].extras)
    task = VersusAll()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input.sequences = Sequences(seqs)
    task.start()
    exp = tmp_path / "exp_pairs.txt"
    with SequencePairHandler.Formatted(exp, "w") as fh:
        for x in seqs:
            for y in seqs:
                xn, yn = x.normalize(), y.normalize()
                ax, ay, _ = R.align(xn.seq, yn.seq)
                fh.write(SequencePair(Sequence(x.id, ax), Sequence(y.id, ay)))
    got = (tmp_path / "out/align/aligned_pairs.txt").read_bytes()
    assert got == exp.read_bytes()
    got.decode("utf-8")  # valid UTF-8


def test_versus_all_prealigned_ca200(tmp_path, engine, oracle_c):
    """Config-2 shape (pre-aligned p / jc / k2p) on samples/Taxi2test1_ca200.tab."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequences
    from taxi2_amd.tasks import VersusAll

    seqs = read_tab("Taxi2test1_ca200.tab")
    metrics = [DistanceMetric.Uncorrected(), DistanceMetric.JukesCantor(), DistanceMetric.Kimura2P()]
    task = VersusAll()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input.sequences = Sequences(seqs)
    task.params.pairs.align = False
    task.params.distances.metrics = metrics
    task.params.format.percentage_multiply = True
    task.start()
    work, D = expected_versus_all(seqs, ("p", "jc", "k2p"), False, oracle_c)
    lin, mats = render_expected(tmp_path, work, D * 100.0, metrics)
    assert (tmp_path / "out/distances/linear.tsv").read_text() == lin.read_text()
    for m in ("p", "jc", "k2p"):
        assert (tmp_path / f"out/distances/matricial/{m}.tsv").read_text() == mats[m].read_text()


@pytest.mark.parametrize("align", [True, False])
def test_versus_reference(tmp_path, engine, oracle_c, align):
    from taxi2_amd.distances import Distance, DistanceHandler, DistanceMetric
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusReference

    allseqs = read_tab("Taxi2test1_120.tab")
    data = allseqs[:30]
    refs = allseqs[30:75]
    # duplicate consecutive query ids merge in groupby (versus_reference.py:185)
    data = data[:5] + [Sequence(data[4].id, data[10].seq, data[10].extras)] + data[5:]
    task = VersusReference()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input.data = Sequences(data)
    task.input.reference = Sequences(refs)
    task.params.pairs.align = align
    task.params.pairs.write = False
    task.start()
    wd = [s.normalize() for s in data] if align else data
    wr = [s.normalize() for s in refs] if align else refs
    seqs = [s.seq for s in wd] + [s.seq for s in wr]
    Q, R = len(wd), len(wr)
    pa = np.repeat(np.arange(Q), R)
    pb = np.tile(np.arange(R), Q) + Q
    out, _ = oracle_c.batch(seqs, pa, pb, align=align, scores=(1, -1, -8, -1, -1, -1))
    vals = out[:, 0, :].reshape(Q, R, 4)
    metrics = [DistanceMetric.Uncorrected(), DistanceMetric.UncorrectedWithGaps(), DistanceMetric.JukesCantor(),
               DistanceMetric.Kimura2P()]
    exp = tmp_path / "exp_closest.tsv"
    with DistanceHandler.Linear.WithExtras(exp, "w", missing="NA", formatter="{:.4f}") as fh:
        q = 0
        while q < Q:
            g = q
            while g + 1 < Q and wd[g + 1].id == wd[q].id:
                g += 1
            best = None
            for qq in range(q, g + 1):
                for r in range(R):
                    v = vals[qq, r, 0]
                    if np.isfinite(v) and (best is None or v < best[0]):
                        best = (v, qq, r)
            _, qq, r = best
            for m, metric in enumerate(metrics):
                v = vals[qq, r, m]
                fh.write(Distance(metric, wd[qq], wr[r], float(v) if np.isfinite(v) else None))
            q = g + 1
    assert (tmp_path / "out/closest.tsv").read_text() == exp.read_text()
    lin = tmp_path / "exp_lin.tsv"
    with DistanceHandler.Linear.WithExtras(lin, "w", missing="NA", formatter="{:.4f}") as fh:
        for qq in range(Q):
            for r in range(R):
                v = vals[qq, r, 0]
                fh.write(Distance(metrics[0], wd[qq], wr[r], float(v) if np.isfinite(v) else None))
    assert (tmp_path / "out/distances/p.linear.tsv").read_text() == lin.read_text()


@pytest.mark.parametrize("pct", [False, True])
def test_decontaminate(tmp_path, engine, oracle_c, pct):
    """decontaminate.py:336-371 on sample sequences: duplicate consecutive query ids (groupby +
    zip pairing), an all-N query (every distance None -> the group's first distance), x100 before
    the threshold; every output file against the oracle's distances."""
    from taxi2_amd.distances import Distance, DistanceHandler, DistanceMetric
    from taxi2_amd.handlers import FileHandler
    from taxi2_amd.sequences import Sequence, SequenceHandler, Sequences
    from taxi2_amd.tasks import Decontaminate

    allseqs = read_tab("Taxi2test1_120.tab")
    data = allseqs[:12]
    data = data[:4] + [Sequence(data[3].id, data[8].seq, data[8].extras)] + data[4:]
    data.append(Sequence("allN", "NNNNNNNNNN", dict(data[0].extras)))
    outgroup = allseqs[40:48] + [Sequence("twin", data[1].seq, dict(data[1].extras))]
    task = Decontaminate()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input = Sequences(data)
    task.outgroup = Sequences(outgroup)
    task.params.pairs.write = False
    task.params.thresholds.similarity = 8.0 if pct else 0.08
    task.params.format.percentage_multiply = pct
    task.start()

    dn = [s.normalize() for s in data]
    on = [s.normalize() for s in outgroup]
    Q, R = len(dn), len(on)
    seqs = [s.seq for s in dn] + [s.seq for s in on]
    pa = np.repeat(np.arange(Q), R)
    pb = np.tile(np.arange(R), Q) + Q
    out, _ = oracle_c.batch(seqs, pa, pb, align=True, scores=(1, -1, -8, -1, -1, -1), metrics=("p",))
    A = out[:, 0, 0].reshape(Q, R) * (100.0 if pct else 1.0)
    # groups of consecutive ids, min(key=d or inf)
    minima, g0 = [], 0
    for k in range(1, Q + 1):
        if k == Q or dn[k].id != dn[g0].id:
            best = None
            for q in range(g0, k):
                for r in range(R):
                    v = A[q, r] if np.isfinite(A[q, r]) else np.inf
                    if best is None or v < best[0]:
                        best = (v, q, r)
            v, q, r = best
            minima.append((on[r].id, None if v == np.inf else float(v)))
            g0 = k
    verdicts = [(s, d is not None and d <= task.params.thresholds.similarity) for s, (_, d) in zip(data, minima)]
    assert any(c for _, c in verdicts) and not all(c for _, c in verdicts)
    exp_sum = tmp_path / "exp_summary.tsv"
    with FileHandler.Tabfile(exp_sum, "w", columns=("query_id", "outgroup_id", "outgroup_distance", "contaminant")) as fh:
        for (s, c), (oid, d) in zip(verdicts, minima):
            fh.write((s.id, oid, "NA" if d is None else "{:.4f}".format(d), "Yes" if c else "No"))
    assert (tmp_path / "out/summary.tsv").read_text() == exp_sum.read_text()
    for name, want in (("decontaminated.tsv", False), ("contaminants.tsv", True)):
        exp = tmp_path / f"exp_{name}"
        with SequenceHandler.Tabfile(exp, "w", idHeader="seqid", seqHeader="sequence") as fh:
            for s, c in verdicts:
                if c == want:
                    fh.write(s)
        assert (tmp_path / "out" / name).read_text() == exp.read_text(), name
    lin = tmp_path / "exp_lin.tsv"
    with DistanceHandler.Linear.WithExtras(lin, "w", missing="NA", formatter="{:.4f}") as fh:
        for q in range(Q):
            for r in range(R):
                v = A[q, r]
                fh.write(Distance(DistanceMetric.Uncorrected(), dn[q], on[r], float(v) if np.isfinite(v) else None))
    assert (tmp_path / "out/distances/p.linear.tsv").read_text() == lin.read_text()


@pytest.mark.parametrize("pct", [False, True])
def test_decontaminate2(tmp_path, engine, oracle_c, pct):
    """decontaminate2.py:390-434: outgroup AND ingroup minima per group of consecutive query ids,
    x100 on the outgroup side only, side weights, contaminant = out defined and (in undefined or
    out < in); summary, sequence files and all four distance files against the oracle."""
    from taxi2_amd.distances import Distance, DistanceHandler, DistanceMetric
    from taxi2_amd.handlers import FileHandler
    from taxi2_amd.sequences import Sequence, SequenceHandler, Sequences
    from taxi2_amd.tasks import Decontaminate2

    allseqs = read_tab("Taxi2test1_120.tab")
    data = allseqs[:12]
    data = data[:4] + [Sequence(data[3].id, data[8].seq, data[8].extras)] + data[4:]
    data.append(Sequence("allN", "NNNNNNNNNN", dict(data[0].extras)))
    outgroup = allseqs[40:48] + [Sequence("twin", data[1].seq, dict(data[1].extras))]
    ingroup = allseqs[60:70] + [Sequence("inN", "NNNN", dict(data[0].extras))]
    task = Decontaminate2()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input = Sequences(data)
    task.outgroup = Sequences(outgroup)
    task.ingroup = Sequences(ingroup)
    task.params.pairs.write = False
    task.params.weights.outgroup = 1.0
    task.params.weights.ingroup = 100.0 if pct else 1.5
    task.params.format.percentage_multiply = pct
    task.start()

    dn = [s.normalize() for s in data]
    Q = len(dn)

    def side(refs, scale):
        rn = [s.normalize() for s in refs]
        R = len(rn)
        seqs = [s.seq for s in dn] + [s.seq for s in rn]
        pa = np.repeat(np.arange(Q), R)
        pb = np.tile(np.arange(R), Q) + Q
        out, _ = oracle_c.batch(seqs, pa, pb, align=True, scores=(1, -1, -8, -1, -1, -1), metrics=("p",))
        A = out[:, 0, 0].reshape(Q, R) * scale
        minima, g0 = [], 0
        for k in range(1, Q + 1):
            if k == Q or dn[k].id != dn[g0].id:
                best = None
                for q in range(g0, k):
                    for r in range(R):
                        v = A[q, r] if np.isfinite(A[q, r]) else np.inf
                        if best is None or v < best[0]:
                            best = (v, r)
                minima.append((rn[best[1]].id, None if best[0] == np.inf else float(best[0])))
                g0 = k
        return rn, A, minima

    on, AO, omin = side(outgroup, 100.0 if pct else 1.0)
    inn, AI, imin = side(ingroup, 1.0)
    rows = []
    for s, (oid, od), (iid, idd) in zip(data, omin, imin):
        od = None if od is None else od * task.params.weights.outgroup
        idd = None if idd is None else idd * task.params.weights.ingroup
        c = False if od is None else True if idd is None else od < idd
        rows.append((s, oid, od, iid, idd, c))
    assert any(r[5] for r in rows) and not all(r[5] for r in rows)
    exp_sum = tmp_path / "exp_summary.tsv"
    cols = ("query_id", "outgroup_id", "outgroup_distance", "ingroup_id", "ingroup_distance", "contaminant")
    with FileHandler.Tabfile(exp_sum, "w", columns=cols) as fh:
        for s, oid, od, iid, idd, c in rows:
            fh.write((s.id, oid, "NA" if od is None else "{:.4f}".format(od), iid,
                      "NA" if idd is None else "{:.4f}".format(idd), "Yes" if c else "No"))
    assert (tmp_path / "out/summary.tsv").read_text() == exp_sum.read_text()
    for name, want in (("decontaminated.tsv", False), ("contaminants.tsv", True)):
        exp = tmp_path / f"exp_{name}"
        with SequenceHandler.Tabfile(exp, "w", idHeader="seqid", seqHeader="sequence") as fh:
            for r in rows:
                if r[5] == want:
                    fh.write(r[0])
        assert (tmp_path / "out" / name).read_text() == exp.read_text(), name
    for label, refs, A in (("outgroup", on, AO), ("ingroup", inn, AI)):
        lin = tmp_path / f"exp_{label}_lin.tsv"
        with DistanceHandler.Linear.WithExtras(lin, "w", missing="NA", formatter="{:.4f}") as fh:
            for q in range(Q):
                for r in range(len(refs)):
                    v = A[q, r]
                    fh.write(Distance(DistanceMetric.Uncorrected(), dn[q], refs[r], float(v) if np.isfinite(v) else None))
        assert (tmp_path / f"out/distances/{label}.p.linear.tsv").read_text() == lin.read_text(), label
        mat = tmp_path / f"exp_{label}_mat.tsv"
        with DistanceHandler.Matrix(mat, "w", missing="NA", formatter="{:.4f}") as fh:
            for q in range(Q):
                for r in range(len(refs)):
                    v = A[q, r]
                    fh.write(Distance(DistanceMetric.Uncorrected(), dn[q], refs[r], float(v) if np.isfinite(v) else None))
        assert (tmp_path / f"out/distances/{label}.p.matricial.tsv").read_text() == mat.read_text(), label
