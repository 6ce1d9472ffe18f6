"""Dereplicate (tasks/dereplicate.py:393-440) against the restated greedy walk (oracle A10).

CPU: the task's replay and writers with the pair distances supplied by the C oracle (the GPU
distance pass is swapped out).  GPU: the whole task on the engine, every output file."""

from __future__ import annotations

import random

import numpy as np
import pytest

from oracle import restatement as R

DEFAULT = (1, -1, -8, -1, -1, -1)


def make_data(seed: int, dup_id: bool = True):
    """Clusters of near-identical short sequences (1-2 substitutions, trimmed ends -> ties and
    longer/shorter branches), unrelated singletons, a sequence under the length threshold, a
    duplicated consecutive id and an all-N sequence (every distance None)."""
    from taxi2_amd.sequences import Sequence

    rng = random.Random(seed)
    out = []
    for c in range(6):
        base = "".join(rng.choice("ACGT") for _ in range(rng.randint(34, 50)))
        for v in range(rng.randint(1, 4)):
            s = list(base)
            for _ in range(rng.randint(0, 2)):
                k = rng.randrange(len(s))
                s[k] = rng.choice("ACGT")
            a, b = rng.randint(0, 3), rng.randint(0, 3)
            out.append(Sequence(f"c{c}v{v}", "".join(s[a : len(s) - b]), {"organism": f"org{c}"}))
    rng.shuffle(out)
    out.insert(3, Sequence("short", "ACGTACG", {"organism": "x"}))
    if dup_id:  # the distance writers fall back to the handlers (line grouping by id)
        out.insert(5, Sequence(out[4].id, out[4].seq[:-1], {"organism": "dup"}))
    out.append(Sequence("allN", "N" * 20, {"organism": "n"}))
    return out


def expected(tmp, data, D, params, aligned_pairs=None):
    """Expected output texts from the oracle walk and the handler writers."""
    from taxi2_amd.distances import Distance, DistanceHandler, DistanceMetric
    from taxi2_amd.handlers import FileHandler
    from taxi2_amd.sequences import SequenceHandler

    keep = [s for s in data if len(s.seq) >= params["length"]]
    work = [s.normalize() for s in keep]

    def dist(i, j):
        v = D[i, j]
        return float(v) if np.isfinite(v) else None

    lines, kept, excluded = R.dereplicate([(s.id, len(s.seq)) for s in keep], dist, params["similarity"])
    fmt, missing = "{:.4f}", "NA"
    files = {}

    def txt(d):
        return missing if d is None else fmt.format(d)

    p = tmp / "exp_summary.tsv"
    cols = ("query_id", "query_length", "included_id", "included_length", "included_distance", "excluded_id",
            "excluded_length", "excluded_distance")
    with FileHandler.Tabfile(p, "w", columns=cols) as fh:
        for ln in lines:
            fh.write((ln.query_id, str(ln.query_length), ln.included[0], str(ln.included[1]), txt(ln.included[2]),
                      ln.excluded[0], str(ln.excluded[1]), txt(ln.excluded[2])))
    files["summary.tsv"] = p.read_text()
    for name, want in (("dereplicated.tsv", False), ("excluded.tsv", True)):
        p = tmp / f"exp_{name}"
        with SequenceHandler.Tabfile(p, "w", idHeader="seqid", seqHeader="sequence") as fh:
            for s in keep:
                if (s.id in excluded) == want:
                    fh.write(s)
        files[name] = p.read_text()
    if kept:
        m = DistanceMetric.Uncorrected()
        p = tmp / "exp_lin.tsv"
        with DistanceHandler.Linear.WithExtras(p, "w", missing=missing, formatter=fmt) as fh:
            for i, j in kept:
                fh.write(Distance(m, work[i], work[j], dist(i, j)))
        files["distances/p.linear.tsv"] = p.read_text()
        p = tmp / "exp_mat.tsv"
        with DistanceHandler.Matrix(p, "w", missing=missing, formatter=fmt) as fh:
            for i, j in kept:
                fh.write(Distance(m, work[i], work[j], dist(i, j)))
        files["distances/p.matricial.tsv"] = p.read_text()
        if aligned_pairs:
            from taxi2_amd.pairs import SequencePair, SequencePairHandler
            from taxi2_amd.sequences import Sequence

            p = tmp / "exp_pairs.txt"
            sc = R.Scores(*DEFAULT)
            with SequencePairHandler.Formatted(p, "w") as fh:
                for i, j in kept:
                    ax, ay, _ = R.align(work[i].seq, work[j].seq, sc)
                    fh.write(SequencePair(Sequence(work[i].id, ax, work[i].extras),
                                          Sequence(work[j].id, ay, work[j].extras)))
            files["aligned_pairs.txt"] = p.read_text()
    return files, lines, kept, excluded


def oracle_matrix(oracle_c, seqs, pct):
    n = len(seqs)
    pa, pb = np.nonzero(np.triu(np.ones((n, n), dtype=bool), 1))
    out, _ = oracle_c.batch(seqs, pa, pb, align=True, scores=DEFAULT, metrics=("p",))
    D = np.full((n, n), np.nan)
    D[pa, pb], D[pb, pa] = out[:, 0, 0], out[:, 1, 0]
    return D * (100.0 if pct else 1.0)


def run_task(tmp, data, engine, pct, write_pairs):
    from taxi2_amd.sequences import Sequences
    from taxi2_amd.tasks import Dereplicate

    task = Dereplicate()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp / "out"
    task.input = Sequences(data)
    task.params.pairs.write = write_pairs
    task.params.thresholds.similarity = 7.0 if pct else 0.07
    task.params.format.percentage_multiply = pct
    task.start()
    return task


def check(tmp, files):
    for name, text in files.items():
        assert (tmp / "out" / name).read_text() == text, name


class _HostOnly:
    """Stands in for the engine where the CPU test swaps out the GPU distance pass."""

    class _Set:
        def free(self):
            pass

    def upload(self, seqs, align):
        return self._Set()


@pytest.mark.parametrize("seed,pct", [(1, False), (2, True), (3, False)])
def test_dereplicate_replay_cpu(tmp_path, oracle_c, monkeypatch, seed, pct):
    """The task's native walk + summary / sequence files, with the oracle's distances."""
    import taxi2_amd.tasks.dereplicate as mod

    data = make_data(seed)
    keep = [s for s in data if len(s.seq) >= 10]
    D = oracle_matrix(oracle_c, [s.normalize().seq for s in keep], pct)
    monkeypatch.setattr(mod, "pair_matrix", lambda eng, st, metric, align, scores: D / (100.0 if pct else 1.0))
    from taxi2_amd.sequences import Sequences
    from taxi2_amd.tasks import Dereplicate

    task = Dereplicate()
    task.engine = _HostOnly()
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input = Sequences(data)
    task.params.pairs.write = False
    task.params.distances.write_linear = task.params.distances.write_matricial = False
    task.params.thresholds.similarity = 7.0 if pct else 0.07
    task.params.format.percentage_multiply = pct
    task.start()
    files, lines, kept, excluded = expected(tmp_path, data, D, {"length": 10, "similarity": task.params.thresholds.similarity})
    assert lines and excluded and len(kept) < len(keep) * (len(keep) - 1)  # exclusions pruned later pairs
    check(tmp_path, {k: v for k, v in files.items() if not k.startswith("distances")})
    assert not (tmp_path / "out/distances").exists()
    assert task.excluded == excluded


def test_walk_native_vs_oracle():
    """taxi2_dereplicate_walk (host code in the engine library) == the restated walk on random
    matrices: None values, length ties, repeated ids (adjacent and apart), dense similarity."""
    from taxi2_amd._native import dereplicate_walk

    rng = np.random.default_rng(5)
    for case in range(300):
        n = int(rng.integers(0, 40))
        D = rng.random((n, n)) * 0.2
        D[rng.random((n, n)) < 0.1] = np.nan
        D[rng.random((n, n)) < 0.02] = np.inf
        names = [f"s{k}" for k in range(max(1, n))]
        ids = [names[int(rng.integers(0, max(1, n - n // 4)))] for _ in range(n)]
        lens = rng.integers(10, 14, n)
        sim = float(rng.choice([0.0, 0.02, 0.07, 0.2]))

        def dist(i, j):
            return float(D[i, j]) if np.isfinite(D[i, j]) else None

        lines, kept, excluded = R.dereplicate(list(zip(ids, lens.tolist())), dist, sim)
        codes = {}
        w = dereplicate_walk(D, [codes.setdefault(i, len(codes)) for i in ids], lens, sim)
        got_kept = list(zip(np.repeat(np.arange(n), w.row_kept).tolist(), w.kept_cols.tolist()))
        assert got_kept == kept, case
        got = [(q, a, b, None if np.isnan(da) else da, None if np.isnan(db) else db)
               for (q, a, b), (da, db) in zip(w.line_idx.tolist(), w.line_d.tolist())]
        want = [(q, a, b, da, db) for q, a, b, da, db in _line_rows(lines, ids, lens)]
        assert [(ids[q], ids[a], ids[b], da, db) for q, a, b, da, db in got] == \
            [(q, a, b, da, db) for q, a, b, da, db in want], case
        assert {i for i, e in zip(ids, w.excluded) if e} == excluded, case


def _line_rows(lines, ids, lens):
    for ln in lines:
        yield ln.query_id, ln.included[0], ln.excluded[0], ln.included[2], ln.excluded[2]


def test_dereplicate_oracle_walk():
    """Hand-checked walk: a (len 5) ~ b (len 6) ~ c (len 6); d unrelated."""
    items = [("a", 5), ("b", 6), ("c", 6), ("d", 4)]
    near = {frozenset("ab"), frozenset("bc"), frozenset("ac")}

    def dist(i, j):
        return 0.01 if frozenset((items[i][0], items[j][0])) in near else 0.5

    lines, kept, excluded = R.dereplicate(items, dist, 0.07)
    # query a: (a,b) -> b longer: include b, exclude a; a is excluded -> its other pairs vanish
    # query b: (b,c) -> same length: include b, exclude c; (b,d) unrelated
    assert [(ln.query_id, ln.included[0], ln.excluded[0]) for ln in lines] == [("a", "b", "a"), ("b", "b", "c")]
    assert excluded == {"a", "c"}
    assert kept == [(0, 1), (1, 2), (1, 3), (3, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,pct,dup", [(1, False, True), (2, True, True), (4, False, False), (5, True, False)])
def test_dereplicate_gpu(tmp_path, engine, oracle_c, seed, pct, dup):
    """Whole task on the GPU; unique ids take the GPU text formatter (ragged rows) for the distance
    files, a repeated id the handler writers."""
    data = make_data(seed, dup)
    keep = [s for s in data if len(s.seq) >= 10]
    D = oracle_matrix(oracle_c, [s.normalize().seq for s in keep], pct)
    task = run_task(tmp_path, data, engine, pct, write_pairs=True)
    files, lines, kept, excluded = expected(tmp_path, data, D, {"length": 10, "similarity": task.params.thresholds.similarity},
                                            aligned_pairs=True)
    assert lines and excluded
    check(tmp_path, files)


@pytest.mark.gpu
def test_format_ragged(engine):
    """taxi2_format_ragged == Python formatting: empty rows, chunk offsets, NaN / inf / -0.0."""
    rng = np.random.default_rng(3)
    n = 17
    row_kept = rng.integers(0, 6, n)
    row_kept[[0, 5]] = 0
    starts = np.concatenate([[0], np.cumsum(row_kept)])
    cols = rng.integers(0, n, int(starts[-1])).astype(np.int32)
    vals = rng.normal(size=(int(starts[-1]), 2)) * 10
    vals[::7, 0] = np.nan
    vals[3, 1] = -0.0
    vals[4, 0] = np.inf
    rp = [f"r{k}\tx" for k in range(n)]
    cp = [f"c{k}" for k in range(n)]

    def t(v):
        return "NA" if not np.isfinite(v) else "{:.4f}".format(v)

    for r0, r1 in ((0, n), (3, 11)):
        lin = engine.format_ragged(vals, starts[r0 : r1 + 1], cols, rp[r0:r1], cp, decimals=4, missing="NA")
        want = "".join(f"{rp[r]}\t{cp[cols[g]]}\t{t(vals[g, 0])}\t{t(vals[g, 1])}\n"
                       for r in range(r0, r1) for g in range(starts[r], starts[r + 1]))
        assert lin.decode() == want
        mat = engine.format_ragged(vals[:, 0], starts[r0 : r1 + 1], cols, rp[r0:r1], None, ncols=n, decimals=4,
                                   missing="NA")
        want = "".join(rp[r] + "".join("\t" + t(vals[g, 0]) for g in range(starts[r], starts[r + 1])) + "\n"
                       for r in range(r0, r1) if starts[r + 1] > starts[r])
        assert mat.decode() == want
