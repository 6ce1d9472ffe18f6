"""Exact parallel subset aggregation on the GPU (taxi2_subset_aggregate_dev, subset_kernels.hpp)
against the reference's sequential SimpleAggregator (versus_all.py:57-96, fed x-major by
_aggregate_distances :617-640), restated below as a plain Python loop: every key's running
``sum += v`` in x-major order, min from +inf (first of equal values kept, so the sign of a zero
minimum is the first zero's), max from 0.0, count; None (non-finite) skipped.

Bit-level comparisons (sums and minima compared as int64 patterns), on inputs built to defeat
the integer fast path: dyadic values whose grid quotient is exactly halfway (ties), negative
values, tiny and huge magnitudes (binade changes at every step), -0.0 minima, few and many
subsets, row blocks of 1 .. n rows."""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def seq_aggregate(A: np.ndarray, code: np.ndarray, ns: int):
    n, _, m = A.shape
    s = np.zeros((ns, ns, m))
    lo = np.full((ns, ns, m), np.inf)
    hi = np.zeros((ns, ns, m))
    c = np.zeros((ns, ns, m), dtype=np.int64)
    for x in range(n):
        a = code[x]
        for y in range(n):
            b = code[y]
            for k in range(m):
                v = float(A[x, y, k])
                if not np.isfinite(v):
                    continue
                s[a, b, k] = float(s[a, b, k]) + v
                if v < lo[a, b, k]:
                    lo[a, b, k] = v
                if v > hi[a, b, k]:
                    hi[a, b, k] = v
                c[a, b, k] += 1
    return s, lo, hi, c


def run_dev(engine, A, code, ns, block):
    import torch

    n, _, m = A.shape
    dev = torch.device("cuda", engine.device)
    order = np.argsort(code, kind="stable")
    start = np.zeros(ns + 1, dtype=np.int64)
    start[1:] = np.cumsum(np.bincount(code, minlength=ns))
    rc = torch.as_tensor(code.astype(np.int32), device=dev)
    cs = torch.as_tensor(start, device=dev)
    ci = torch.as_tensor(order.astype(np.int32), device=dev)
    shape = (ns, ns, m)
    s = torch.empty(shape, dtype=torch.float64, device=dev)
    lo = torch.empty(shape, dtype=torch.float64, device=dev)
    hi = torch.empty(shape, dtype=torch.float64, device=dev)
    c = torch.empty(shape, dtype=torch.int64, device=dev)
    D = torch.as_tensor(A, device=dev)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        for x0 in range(0, n, block):
            x1 = min(n, x0 + block)
            Db = D[x0:x1].contiguous()
            engine.subset_aggregate_dev(Db.data_ptr(), x1 - x0, n, m, rc[x0:x1].data_ptr(), cs.data_ptr(),
                                        ci.data_ptr(), ns, x0 == 0, s.data_ptr(), lo.data_ptr(), hi.data_ptr(),
                                        c.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    return tuple(t.cpu().numpy() for t in (s, lo, hi, c))


def assert_bits(got, exp):
    g, e = np.ascontiguousarray(got), np.ascontiguousarray(exp)
    if g.dtype == np.float64:
        g, e = g.view(np.int64), e.view(np.int64)
    bad = np.argwhere(g != e)
    assert bad.size == 0, f"{len(bad)} keys differ, first {bad[:3].tolist()}: {got[tuple(bad[0])]!r} vs {exp[tuple(bad[0])]!r}"


def values(rng, n, m, kind):
    if kind == "uniform":
        A = rng.random((n, n, m)) * 30
    elif kind == "dyadic":  # k / 2^j: grid quotients land exactly halfway whenever the sum is large enough
        A = rng.integers(0, 64, (n, n, m)) / (2.0 ** rng.integers(0, 12, (n, n, m)))
    elif kind == "magnitudes":  # binade changes at every step
        A = rng.random((n, n, m)) * 10.0 ** rng.integers(-300, 300, (n, n, m)).astype(float)
    elif kind == "negative":
        A = rng.normal(0, 5, (n, n, m))
    else:  # "percent": p-distance-like quotients x 100
        A = rng.integers(0, 120, (n, n, m)) / rng.integers(80, 121, (n, n, m)) * 100.0
    A[rng.random((n, n, m)) < 0.08] = np.nan
    A[rng.random((n, n, m)) < 0.02] = np.inf
    A[rng.random((n, n, m)) < 0.05] = -0.0
    A[rng.random((n, n, m)) < 0.03] = 0.0
    return A


@pytest.mark.parametrize("kind", ["uniform", "dyadic", "magnitudes", "negative", "percent"])
@pytest.mark.parametrize("ns,block", [(1, 7), (2, 1), (3, 16), (17, 64), (40, 200)])
def test_subset_aggregate_exact(engine, kind, ns, block):
    rng = np.random.default_rng(hash((kind, ns, block)) % 2**32)
    n, m = 90, 3
    A = values(rng, n, m, kind)
    code = rng.integers(0, ns, n).astype(np.int32)
    code[:ns] = np.arange(ns)  # every subset present, first appearance order = code order
    exp = seq_aggregate(A, code, ns)
    got = run_dev(engine, A, code, ns, block)
    for g, e in zip(got, exp):
        assert_bits(g, e)


def test_subset_aggregate_long_chain(engine):
    """One subset, many rows: long sums that cross many binades inside one block and across
    blocks (the integer step, the combine's fallback row and the fixup all run)."""
    rng = np.random.default_rng(11)
    n, m = 400, 2
    A = rng.integers(1, 1000, (n, n, m)) / 7.0
    A[:, :, 1] = rng.random((n, n)) * 1e-3
    A[rng.random((n, n, m)) < 0.01] = 0.5  # exact halves
    code = np.zeros(n, np.int32)
    exp = seq_aggregate(A, code, 1)
    for block in (1, 33, 400):
        got = run_dev(engine, A, code, 1, block)
        for g, e in zip(got, exp):
            assert_bits(g, e)


def seq_aggregate_np(A: np.ndarray, code: np.ndarray, ns: int):
    """seq_aggregate for large n: per key the x-major value sequence, summed by np.add.accumulate
    (strictly left to right, as the reference's loop; None -> +0.0, an exact no-op on a sum that
    starts at +0.0), the first minimum (sign of a zero minimum from the first zero), max from 0.0."""
    n, _, m = A.shape
    s = np.zeros((ns, ns, m))
    lo = np.full((ns, ns, m), np.inf)
    hi = np.zeros((ns, ns, m))
    c = np.zeros((ns, ns, m), dtype=np.int64)
    for a in range(ns):
        xs = np.flatnonzero(code == a)
        for b in range(ns):
            ys = np.flatnonzero(code == b)
            for k in range(m):
                v = A[np.ix_(xs, ys)][:, :, k].ravel()  # x-major
                fin = np.isfinite(v)
                c[a, b, k] = int(fin.sum())
                if not c[a, b, k]:
                    continue
                s[a, b, k] = np.add.accumulate(np.where(fin, v, 0.0))[-1]
                d = v[fin]
                mn = d.min()
                if mn == 0.0:
                    mn = d[np.flatnonzero(d == 0.0)[0]]
                lo[a, b, k] = mn
                pos = d[d > 0.0]
                hi[a, b, k] = pos.max() if pos.size else 0.0
    return s, lo, hi, c


@pytest.mark.parametrize("path", ["natural", "gather"])
@pytest.mark.parametrize("kind", ["percent", "dyadic"])
@pytest.mark.parametrize("ns,block", [(1, 700), (2, 1999), (3, 5000)])
def test_subset_aggregate_wide_subsets(engine, monkeypatch, path, kind, ns, block):
    """Subsets wider than one chunk (2 048 columns): chunk partials merged per row in column order,
    multi-grid row partials across binade changes -- through the natural-order rows kernel that
    few subsets take (k_subset_rows_nat) and through the sorted-gather one (TAXI2_SUB_GATHER=1)."""
    if path == "gather":
        monkeypatch.setenv("TAXI2_SUB_GATHER", "1")
    rng = np.random.default_rng(hash(("wide", kind, ns, block)) % 2**32)
    n, m = 5000, 2
    A = values(rng, n, m, kind)
    code = rng.integers(0, ns, n).astype(np.int32)
    code[:ns] = np.arange(ns)
    exp = seq_aggregate_np(A, code, ns)
    got = run_dev(engine, A, code, ns, block)
    for g, e in zip(got, exp):
        assert_bits(g, e)
