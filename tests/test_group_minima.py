"""Host logic of Decontaminate / Decontaminate2 (taxi2_amd/tasks/decontaminate.py group_minima):
the reference's groupby(distance.x.id) + min(key=d or inf) over closest-reference rows
(/root/reference/src/itaxotools/taxi2/tasks/decontaminate2.py:294-306), CPU only."""

from __future__ import annotations

import numpy as np

from taxi2_amd.tasks.decontaminate import group_minima


def _ref(qids, M, scale):
    """Reference order over the full query-major product: first minimum of d (None -> inf) per group."""
    out, g0 = [], 0
    for k in range(1, len(qids) + 1):
        if k == len(qids) or qids[k] != qids[g0]:
            best = None
            for q in range(g0, k):
                for r in range(M.shape[1]):
                    v = M[q, r] * scale if np.isfinite(M[q, r]) else np.inf
                    if best is None or v < best[0]:
                        best = (v, q, r)
            v, q, r = best
            out.append((q, r, float(v)) if v != np.inf else (g0, 0, None))
            g0 = k
    return out


def test_group_minima_matches_reference_order():
    rng = np.random.default_rng(5)
    for trial in range(40):
        Q, R = int(rng.integers(1, 9)), int(rng.integers(1, 6))
        M = np.round(rng.random((Q, R)), 1)  # coarse values: many ties
        M[rng.random((Q, R)) < 0.3] = np.nan
        qids = [f"q{int(v)}" for v in np.sort(rng.integers(0, 4, Q))]
        # closest_rows contract: first minimum per row, -1 / NaN when the row has none
        ok = np.isfinite(M)
        idx = np.where(ok.any(1), np.argmin(np.where(ok, M, np.inf), 1), -1)
        d = np.where(idx >= 0, M[np.arange(Q), np.maximum(idx, 0)], np.nan)
        res = np.stack([idx.astype(float), d], 1)
        for scale in (1.0, 100.0):
            got = group_minima(qids, res, scale, R)
            exp = _ref(qids, M, scale)
            assert [(g[1], g[2]) for g in got] == [(e[1], e[2]) for e in exp], (trial, scale)


def test_group_minima_no_references():
    res = np.zeros((3, 2))
    assert group_minima(["a", "a", "b"], res, 1.0, 0) == []
