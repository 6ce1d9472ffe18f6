"""Rectangular (query x reference) building blocks shared by VersusReference and Decontaminate
(``versus_reference.py:119-188, 131-178``; ``decontaminate.py:170-294``): the closest-reference
search on the GPU and the three rectangular writers.
"""

from __future__ import annotations

from pathlib import Path
from typing import Callable

import numpy as np

from ..align import PairwiseAligner
from ..distances import Distance, DistanceHandler, DistanceMetric
from ..pairs import SequencePair, SequencePairHandler
from .common import create_parents, fixed_decimals, format_values, gpu_text_ok, write_rows_gpu


def first_minimum(block: np.ndarray, scale: float) -> tuple[np.ndarray, np.ndarray]:
    """Per row: index of the first minimum of ``scale * v`` over finite values (the reference's
    ``min`` over Distances after the x100 adjustment, versus_reference.py:184-188, 232) and the
    unscaled value; -1 / NaN for rows without a defined value (same contract as taxi2_closest)."""
    v = block * scale
    ok = np.isfinite(v)
    w = np.where(ok, v, np.inf)
    i = np.argmin(w, axis=1) if block.shape[1] else np.zeros(block.shape[0], dtype=np.int64)
    has = ok.any(axis=1)
    idx = np.where(has, i, -1).astype(np.int64)
    d = np.where(has, block[np.arange(block.shape[0]), np.maximum(idx, 0)], np.nan)
    return idx, d


def closest_rows(eng, qs, rs, qa: int, qb: int, primary: DistanceMetric, extras: list, scores, align: bool,
                 scale: float, want_matrix: bool, progress: Callable[[int], None] | None = None) -> np.ndarray:
    """Queries [qa, qb) of ``qs`` against every reference of ``rs``:
    rows [closest index (-1: none defined), its unscaled primary value, extras (E), primary row (R,
    only with ``want_matrix``)].  Counter metrics use taxi2_closest (argmin on the GPU); NCD as the
    primary metric takes the Q x R block from taxi2_ncd_pairs and the same first-minimum rule."""
    R, E = rs.n, len(extras)
    ncd_primary = str(primary) == "ncd"
    ncd_extra = [k for k, m in enumerate(extras) if str(m) == "ncd"]
    cextra = [k for k, m in enumerate(extras) if str(m) != "ncd"]
    width = 2 + E + (R if want_matrix else 0)
    res = np.full((qb - qa, width), np.nan)
    step = max(1, (1 << 16 if ncd_primary else 1 << 22) // max(R, 1))
    for q0 in range(qa, qb, step):
        q1 = min(qb, q0 + step)
        rows = res[q0 - qa : q1 - qa]
        rows[:, 0] = -1
        if R and not ncd_primary:
            cx = [str(extras[k]) for k in cextra]
            i, d, e, m = eng.closest(qs, rs, q0, q1, str(primary), cx, scores, scale=scale, want_matrix=want_matrix)
            rows[:, 0], rows[:, 1] = i, d
            if e is not None:
                rows[:, [2 + k for k in cextra]] = e
            if m is not None:
                rows[:, 2 + E :] = m
        elif R:
            nq = q1 - q0
            qv = np.repeat(np.arange(q0, q1, dtype=np.int64), R)
            rv = np.tile(np.arange(R, dtype=np.int64), nq)
            mat = eng.ncd_pairs(qs, rs, qv, rv, scores, aligned=align, both=False).reshape(nq, R)
            i, d = first_minimum(mat, scale)
            rows[:, 0], rows[:, 1] = i, d
            if want_matrix:
                rows[:, 2 + E :] = mat
            if cextra:
                ok = np.nonzero(i >= 0)[0]
                if len(ok):
                    e = eng.list_pairs(qs, rs, ok + q0, i[ok], [str(extras[k]) for k in cextra], scores)
                    rows[ok[:, None], np.array([2 + k for k in cextra])[None, :]] = e[:, 0, :] if align else e
        if ncd_extra and R:
            idxb = rows[:, 0].astype(np.int64)
            ok = np.nonzero(idxb >= 0)[0]
            if len(ok):
                v = eng.ncd_pairs(qs, rs, ok + q0, idxb[ok], scores, aligned=align, both=False)
                for k in ncd_extra:
                    rows[ok, 2 + k] = v
        if progress is not None:
            progress(q1)
    return res


def write_rect_pairs(path: Path, data: list, refs: list, align: bool, scores, eng) -> None:
    """aligned_pairs.txt (pairs.py:51-97 Formatted) for the query-major product."""
    create_parents(path)
    with SequencePairHandler.Formatted(path, "w") as fh:
        if not align:
            for x in data:
                for y in refs:
                    fh.write(SequencePair(x, y))
            return
        aligner = PairwiseAligner.Biopython(scores, engine=eng)
        for row in aligner.align_product_rows(data, refs):
            for pair in row:
                fh.write(pair)


def _pre(s, missing: str) -> str:
    return "\t".join([s.id, *[v if v is not None else missing for v in s.extras.values()]])


def write_rect_linear(path: Path, data: list, refs: list, A: np.ndarray, metric, fmt: str, missing: str, eng) -> None:
    """``DistanceHandler.Linear.WithExtras`` of one metric over the query-major product."""
    create_parents(path)
    dec = fixed_decimals(fmt)
    qids, rids = [s.id for s in data], [s.id for s in refs]
    if (data and refs and gpu_text_ok(A, dec) and len(set(qids)) == len(qids) and len(set(rids)) == len(rids)
            and all(list(s.extras) == list(data[0].extras) for s in data)
            and all(list(s.extras) == list(refs[0].extras) for s in refs)):
        # same text as the handler (one metric, no line merging), formatted on the GPU
        head = ["seqid (query)", *[k + " (query)" for k in data[0].extras], "seqid (reference)",
                *[k + " (reference)" for k in refs[0].extras], str(metric)]
        with open(path, "wb") as fh:
            fh.write(("\t".join(head) + "\n").encode("utf-8"))
            write_rows_gpu(fh, eng, np.ascontiguousarray(A)[:, :, None], [_pre(s, missing) for s in data],
                           [_pre(s, missing) for s in refs], dec, missing)
        return
    with DistanceHandler.Linear.WithExtras(path, "w", missing=missing, formatter=fmt) as fh:
        for i, x in enumerate(data):
            for j, y in enumerate(refs):
                v = A[i, j]
                fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))


def write_rect_matrix(path: Path, data: list, refs: list, A: np.ndarray, metric, fmt: str, missing: str, eng) -> None:
    """``DistanceHandler.Matrix`` of one metric over the query-major product."""
    create_parents(path)
    ids = [s.id for s in data]
    if len(set(ids)) != len(ids):
        with DistanceHandler.Matrix(path, "w", missing=missing, formatter=fmt) as fh:
            for i, x in enumerate(data):
                for j, y in enumerate(refs):
                    v = A[i, j]
                    fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))
        return
    dec = fixed_decimals(fmt)
    if data and refs and gpu_text_ok(A, dec):
        with open(path, "wb") as fh:
            fh.write(("\t".join(["", *[s.id for s in refs]]) + "\n").encode("utf-8"))
            write_rows_gpu(fh, eng, np.ascontiguousarray(A), ids, None, dec, missing)
        return
    text = format_values(A, fmt, missing)
    with open(path, "w") as fh:
        if data and refs:
            fh.write("\t".join(["", *[s.id for s in refs]]) + "\n")
        for i, x in enumerate(data):
            if refs:
                fh.write("\t".join((x.id, *text[i])) + "\n")
