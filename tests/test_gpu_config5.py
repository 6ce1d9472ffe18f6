"""Config 5 (BASELINE.json configs[4]: versusAll 200 000 x 1 000 bp) through VersusAll.start(),
pre-aligned p / jc / k2p, reductions only ("gather only reductions" at that size).

* Full size, one GPU: every ordered pair evaluated on the streamed pre-aligned path; the row
  minima of 64 sampled rows equal the C restatement's first minimum over the whole row (x100 and
  None rules applied), the genus and species statistics cover the same number of values, and the
  per-phase times are reported (tools/bench_config5_task.py writes the same as JSON).
* Mid size (N = 4 000): the streamed subset statistics (exact parallel sums, subset_kernels.hpp)
  equal the dense path's sequential host aggregation bit for bit (means, minima, maxima, counts).
Reference: /root/reference/src/itaxotools/taxi2/tasks/versus_all.py:57-96, 617-640, 732-773."""

from __future__ import annotations

import json
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def _bits(a):
    return np.ascontiguousarray(a).view(np.int64)


@pytest.mark.timeout(900)
def test_config5_task_full_size(tmp_path, engine, oracle_c):
    from bench_secondary import build_config5_task as build_task

    n, L = 200_000, 1000
    task, buf, offs = build_task(n, L, engine, tmp_path, 2.0)
    res = task.start()
    t = task.timings
    print(json.dumps({"n": n, "seconds": res.seconds_taken, "phases_s": t}))
    idx, d = task.row_minima
    rng = np.random.default_rng(5)
    rows = np.sort(rng.choice(n, 64, replace=False))
    for x in rows:
        pa = np.full(n, x, dtype=np.int64)
        pb = np.arange(n, dtype=np.int64)
        exp, _ = oracle_c.batch((buf, offs), pa, pb, align=False, scores=(1, -1, -8, -1, -1, -1), metrics=("p",),
                                threads=16)
        v = exp[:, 0, 0] * 100.0
        v[x] = np.nan  # diagonal rule (unique full tuples)
        v = np.where(np.isfinite(v), v, np.inf)
        j = int(np.argmin(v))
        if np.isfinite(v[j]):
            assert idx[x] == j and _bits(d[x]) == _bits(v[j]), (x, idx[x], j, d[x], v[j])
        else:
            assert idx[x] == -1
    g, s = task.subset_stats["genera"], task.subset_stats["species"]
    assert len(g.subsets) == 2 and len(s.subsets) > 900
    assert np.array_equal(g.count.sum(axis=(0, 1)), s.count.sum(axis=(0, 1)))
    assert (g.count.sum(axis=(0, 1)) <= n * (n - 1)).all()
    assert {"compute_s", "reduce_s", "text_s", "comm_s", "upload_s", "prepare_s", "finish_s"} <= set(t)


def test_streamed_subsets_exact_vs_dense(tmp_path, engine):
    from bench_secondary import build_config5_task as build_task

    n, L = 4000, 600
    dense, _, _ = build_task(n, L, engine, tmp_path / "dense", 0.05)
    dense.params.engine.stream = False
    dense.params.engine.row_minima = None
    dense.start()
    streamed, _, _ = build_task(n, L, engine, tmp_path / "stream", 0.05)  # ~1 MB blocks: many blocks
    streamed.start()
    for name in ("genera", "species"):
        a, b = dense.subset_stats[name], streamed.subset_stats[name]
        assert a.subsets == b.subsets
        assert np.array_equal(a.count, b.count)
        for x, y in ((a.mean, b.mean), (a.min, b.min), (a.max, b.max)):
            assert np.array_equal(_bits(np.nan_to_num(x, nan=-7.0)), _bits(np.nan_to_num(y, nan=-7.0))), name
    for f in sorted((tmp_path / "dense" / "subsets").rglob("*.tsv")):
        rel = f.relative_to(tmp_path / "dense")
        assert (tmp_path / "stream" / rel).read_bytes() == f.read_bytes(), rel


def test_column_view_matches_task_order(tmp_path, engine, monkeypatch):
    """The reductions-only stream stores its blocks' columns in species order (taxi2_set_permuted);
    with duplicated rows (the diagonal rule's NaN groups), row minima and every subset statistic
    equal the run that keeps the task's column order (TAXI2_NO_COLPERM), bit for bit."""
    from bench_secondary import build_config5_task as build_task
    from taxi2_amd.sequences import Sequences

    n, L = 3000, 400

    def run(sub, perm):
        if perm:
            monkeypatch.delenv("TAXI2_NO_COLPERM", raising=False)
        else:
            monkeypatch.setenv("TAXI2_NO_COLPERM", "1")
        task, _, _ = build_task(n, L, engine, tmp_path / sub, 0.02)
        seqs = list(task.input.sequences)
        for k in range(0, 60, 3):  # 20 duplicated full tuples (id, sequence, extras)
            seqs[k + 1] = seqs[k]
        task.input.sequences = Sequences(seqs)
        task.start()
        return task

    a, b = run("perm", True), run("plain", False)
    ia, da = a.row_minima
    ib, db = b.row_minima
    assert np.array_equal(ia, ib)
    assert np.array_equal(_bits(np.nan_to_num(da, nan=-7.0)), _bits(np.nan_to_num(db, nan=-7.0)))
    for name in ("genera", "species"):
        x, y = a.subset_stats[name], b.subset_stats[name]
        assert np.array_equal(x.count, y.count)
        for u, v in ((x.mean, y.mean), (x.min, y.min), (x.max, y.max)):
            assert np.array_equal(_bits(np.nan_to_num(u, nan=-7.0)), _bits(np.nan_to_num(v, nan=-7.0))), name


@pytest.mark.timeout(600)
def test_aligned_streamed_reductions_vs_dense_and_oracle(tmp_path, engine, oracle_c):
    """Config 5's aligned form (NW / Gotoh on a stated subset) through the streamed
    reductions path at N = 2 000 x 600 bp of its generator: every subset statistic equals the dense
    path's sequential host aggregation bit for bit, the row minima equal the dense matrix's first
    minima (x100, diagonal None), and sampled rows equal the C restatement's alignments."""
    from bench_secondary import build_config5_task as build_task

    n, L = 2000, 600
    streamed, _, _ = build_task(n, L, engine, tmp_path / "stream", 0.05, aligned=True)  # many blocks
    streamed.start()
    dense, _, _ = build_task(n, L, engine, tmp_path / "dense", 0.05, aligned=True)
    dense.params.engine.stream = False
    dense.params.engine.row_minima = None
    dense.start()
    for name in ("genera", "species"):
        a, b = dense.subset_stats[name], streamed.subset_stats[name]
        assert a.subsets == b.subsets
        assert np.array_equal(a.count, b.count)
        for x, y in ((a.mean, b.mean), (a.min, b.min), (a.max, b.max)):
            assert np.array_equal(_bits(np.nan_to_num(x, nan=-7.0)), _bits(np.nan_to_num(y, nan=-7.0))), name
    D = dense.distances
    v = D[:, :, 0] * 100.0
    v[np.arange(n), np.arange(n)] = np.nan
    v = np.where(np.isfinite(v), v, np.inf)
    j = np.argmin(v, axis=1)
    idx, d = streamed.row_minima
    fin = np.isfinite(v[np.arange(n), j])
    assert np.array_equal(idx[fin], j[fin]) and (idx[~fin] == -1).all()
    assert np.array_equal(_bits(d[fin]), _bits(v[np.arange(n), j][fin]))
    seqs = [s.normalize().seq for s in streamed.input.sequences]
    for x in (0, 777, n - 1):
        pa = np.full(n, x, dtype=np.int64)
        pb = np.arange(n, dtype=np.int64)
        exp, _ = oracle_c.batch(seqs, pa, pb, align=True, scores=(1, -1, -8, -1, -1, -1), metrics=("p",),
                                threads=16)
        e = exp[:, 0, 0]
        got = D[x, :, 0]
        m = np.arange(n) != x
        assert np.array_equal(np.isfinite(e[m]), np.isfinite(got[m]))
        assert np.array_equal(_bits(e[m][np.isfinite(e[m])]), _bits(got[m][np.isfinite(got[m])]))


@pytest.mark.timeout(900)
def test_streamed_subsets_exact_vs_dense_16000(tmp_path, engine):
    """the streamed subset statistics (exact parallel sums) against the dense
    path's sequential host aggregation at N = 16 000 (2.56e8 ordered pairs, 6 GB dense), bit for bit
    -- 16x the pairs of the N = 4 000 check, every block boundary and binade change of a long run."""
    from bench_secondary import build_config5_task as build_task

    n, L = 16_000, 300
    dense, _, _ = build_task(n, L, engine, tmp_path / "dense", 0.5)
    dense.params.engine.stream = False
    dense.params.engine.row_minima = None
    dense.start()
    streamed, _, _ = build_task(n, L, engine, tmp_path / "stream", 0.5)
    streamed.start()
    for name in ("genera", "species"):
        a, b = dense.subset_stats[name], streamed.subset_stats[name]
        assert a.subsets == b.subsets
        assert np.array_equal(a.count, b.count)
        for x, y in ((a.mean, b.mean), (a.min, b.min), (a.max, b.max)):
            assert np.array_equal(_bits(np.nan_to_num(x, nan=-7.0)), _bits(np.nan_to_num(y, nan=-7.0))), name
