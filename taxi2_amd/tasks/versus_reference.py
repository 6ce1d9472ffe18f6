"""VersusReference task (``src/itaxotools/taxi2/tasks/versus_reference.py:33-247``), GPU-backed.

``start`` computes, for the Q x R product (query outer, reference inner):
  * the primary metric for every pair (default p, :83-86), x100 when percentage_multiply;
  * per group of consecutive queries with equal id (``groupby(x.id)``, :184-188) the first
    minimum over defined values (``min`` raises ValueError when a group has none);
  * the extra metrics (default p-gaps / jc / k2p minus the primary, :87-93) for that closest
    pair only, on the same alignment (:124-129);
and writes ``distances/<metric>.linear.tsv``, ``distances/<metric>.matricial.tsv``,
``closest.tsv`` and (``params.pairs.write``) ``aligned_pairs.txt``.
Argmin runs on the GPU (``taxi2_closest``), so the Q x R block never round-trips through
Python unless a writer needs it.  With NCD as the primary metric the Q x R NCD block comes from
``taxi2_ncd_pairs`` and the same first-minimum rule runs on the host; NCD as an extra metric is
computed for the closest pairs only.
"""

from __future__ import annotations

from pathlib import Path
from time import perf_counter
from typing import Callable

import numpy as np

from ..align import PairwiseAligner, Scores
from ..distances import ENGINE_LABELS, Distance, DistanceHandler, DistanceMetric, check_ncd_strings
from ..pairs import SequencePair, SequencePairHandler
from ..types import AttrDict
from ..sharding import distributed_rows, world_info
from .common import (Results, console_report, create_parents, fixed_decimals, format_values, gpu_text_ok,
                     report, write_rows_gpu)


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


class VersusReference:
    def __init__(self):
        self.work_dir: Path = None
        self.paths = AttrDict()
        self.progress_handler: Callable = console_report
        self.progress_interval: float = 0.015
        self.engine = None

        self.input = AttrDict()
        self.input.data = None
        self.input.reference = None

        self.params = AttrDict()
        self.params.pairs = AttrDict()
        self.params.pairs.align = True
        self.params.pairs.write = True
        self.params.pairs.scores = None

        self.params.distances = AttrDict()
        self.params.distances.metric = None
        self.params.distances.extra_metrics = None
        self.params.distances.write_linear = True
        self.params.distances.write_matricial = True

        self.params.format = AttrDict()
        self.params.format.float = "{:.4f}"
        self.params.format.percentage = "{:.2f}"
        self.params.format.missing = "NA"
        self.params.format.percentage_multiply = False

        self.closest: list | None = None  # [(query index range, ref index, d, extras)] after start()

    def generate_paths(self):
        assert self.work_dir
        w = Path(self.work_dir)
        create_parents(w)
        metric = str(self.params.distances.metric)
        self.paths.closest = w / "closest.tsv"
        self.paths.aligned_pairs = w / "aligned_pairs.txt"
        self.paths.distances_linear = w / "distances" / f"{metric}.linear.tsv"
        self.paths.distances_matricial = w / "distances" / f"{metric}.matricial.tsv"

    def check_metrics(self):
        self.params.distances.metric = self.params.distances.metric or DistanceMetric.Uncorrected()
        self.params.distances.extra_metrics = self.params.distances.extra_metrics or [
            DistanceMetric.UncorrectedWithGaps(),
            DistanceMetric.JukesCantor(),
            DistanceMetric.Kimura2P(),
        ]
        if self.params.distances.metric in self.params.distances.extra_metrics:
            self.params.distances.extra_metrics.remove(self.params.distances.metric)
        for m in [self.params.distances.metric, *self.params.distances.extra_metrics]:
            if str(m) not in ENGINE_LABELS:
                raise NotImplementedError(f"metric {m} is not computed by the MI355X engine (DESIGN.md)")

    def _engine(self):
        if self.engine is None:
            from .._native import Engine

            self.engine = Engine.default()
        return self.engine

    def start(self) -> Results:
        ts = perf_counter()
        self.check_metrics()
        self.generate_paths()
        align = bool(self.params.pairs.align)
        data = list(self.input.data)
        refs = list(self.input.reference)
        if align:
            data = [s.normalize() for s in data]
            refs = [s.normalize() for s in refs]
        Q, R = len(data), len(refs)
        primary = self.params.distances.metric
        extras = list(self.params.distances.extra_metrics)
        scores = Scores(**(self.params.pairs.scores or {})).as_tuple()
        pct = bool(self.params.format.percentage_multiply)
        want_matrix = bool(self.params.distances.write_linear or self.params.distances.write_matricial)
        total = Q * R
        eng = self._engine()
        ncd_primary = str(primary) == "ncd"
        ncd_extra = [k for k, m in enumerate(extras) if str(m) == "ncd"]
        cextra = [k for k, m in enumerate(extras) if str(m) != "ncd"]
        if ncd_primary or ncd_extra:
            check_ncd_strings(s.seq for s in data)
            check_ncd_strings(s.seq for s in refs)
        qs = eng.upload([s.seq for s in data], align=align)
        rs = eng.upload([s.seq for s in refs], align=align)
        E = len(extras)
        scale = 100.0 if pct else 1.0

        def block(qa: int, qb: int) -> np.ndarray:
            """Queries [qa, qb) -> rows [idx, dmin, extras (E), primary row (R if want_matrix)]."""
            width = 2 + E + (R if want_matrix else 0)
            res = np.full((qb - qa, width), np.nan)
            step = max(1, (1 << 22) // max(R, 1))
            if ncd_primary:
                step = max(1, (1 << 16) // max(R, 1))
            for q0 in range(qa, qb, step):
                q1 = min(qb, q0 + step)
                rows = res[q0 - qa : q1 - qa]
                rows[:, 0] = -1
                if R and not ncd_primary:
                    cx = [str(extras[k]) for k in cextra]
                    i, d, e, m = eng.closest(qs, rs, q0, q1, str(primary), cx, scores, scale=scale,
                                             want_matrix=want_matrix)
                    rows[:, 0], rows[:, 1] = i, d
                    if e is not None:
                        rows[:, [2 + k for k in cextra]] = e
                    if m is not None:
                        rows[:, 2 + E :] = m
                elif R:
                    nq = q1 - q0
                    qv = np.repeat(np.arange(q0, q1, dtype=np.int64), R)
                    rv = np.tile(np.arange(R, dtype=np.int64), nq)
                    mat_b = eng.ncd_pairs(qs, rs, qv, rv, scores, aligned=align, both=False).reshape(nq, R)
                    i, d = first_minimum(mat_b, scale)
                    rows[:, 0], rows[:, 1] = i, d
                    if want_matrix:
                        rows[:, 2 + E :] = mat_b
                    if cextra:
                        ok = np.nonzero(i >= 0)[0]
                        if len(ok):
                            e = eng.list_pairs(qs, rs, ok + q0, i[ok], [str(extras[k]) for k in cextra], scores)
                            rows[ok[:, None], np.array([2 + k for k in cextra])[None, :]] = e[:, 0, :] if align else e
                if ncd_extra:
                    idxb = rows[:, 0].astype(np.int64)
                    ok = np.nonzero(idxb >= 0)[0]
                    if len(ok):
                        v = eng.ncd_pairs(qs, rs, ok + q0, idxb[ok], scores, aligned=align, both=False)
                        for k in ncd_extra:
                            rows[ok, 2 + k] = v
                report(self.progress_handler, "distance.x.id", q1 * R, total)
            return res

        try:
            distributed, rank = world_info()
            if distributed:  # queries sharded across ranks, references replicated
                import torch
                import torch.distributed as dist

                device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
                res = distributed_rows(Q, block, device=device)
            else:
                res = block(0, Q)
        finally:
            qs.free()
            rs.free()
        idx = res[:, 0].astype(np.int64)
        dmin = res[:, 1]
        ext = res[:, 2 : 2 + E]
        mat = res[:, 2 + E :] if want_matrix else None

        # groupby(x.id) over consecutive queries, first minimum wins (versus_reference.py:184-188)
        groups = []
        g0 = 0
        for k in range(1, Q + 1):
            if k == Q or data[k].id != data[g0].id:
                groups.append((g0, k))
                g0 = k
        closest = []
        for a, b in groups:
            best = None
            for q in range(a, b):
                if idx[q] < 0:
                    continue
                v = dmin[q] * (100.0 if pct else 1.0)
                if best is None or v < best[0]:
                    best = (v, q)
            if best is None:
                raise ValueError("min() arg is an empty sequence")  # the reference's min() on all-None
            q = best[1]
            closest.append((q, int(idx[q]), float(dmin[q]), ext[q].copy()))
        self.closest = closest

        if world_info()[1] == 0:  # rank 0 writes (every rank holds the gathered results)
            if self.params.pairs.write:
                self.write_pairs(data, refs)
            if mat is not None:
                A = mat * 100.0 if pct else mat
                self.write_distances_linear(data, refs, A)
                self.write_distances_matrix(data, refs, A)
            self.write_closest(data, refs, closest)
        report(self.progress_handler, "Finalizing...", total, total)
        return Results(self.work_dir, perf_counter() - ts)

    # ------------------------------------------------------------------ writers
    def write_pairs(self, data, refs):
        create_parents(self.paths.aligned_pairs)
        with SequencePairHandler.Formatted(self.paths.aligned_pairs, "w") as fh:
            if not self.params.pairs.align:
                for x in data:
                    for y in refs:
                        fh.write(SequencePair(x, y))
                return
            aligner = PairwiseAligner.Biopython(self.params.pairs.scores, engine=self._engine())
            for x in data:
                for pair in aligner.align_many([SequencePair(x, y) for y in refs]):
                    fh.write(pair)

    def write_distances_linear(self, data, refs, A):
        if not self.params.distances.write_linear:
            return
        create_parents(self.paths.distances_linear)
        fmt, missing = self.params.format.float, self.params.format.missing
        metric = self.params.distances.metric
        dec = fixed_decimals(fmt)
        qids, rids = [s.id for s in data], [s.id for s in refs]
        if (data and refs and gpu_text_ok(A, dec) and len(set(qids)) == len(qids) and len(set(rids)) == len(rids)
                and all(list(s.extras) == list(data[0].extras) for s in data)
                and all(list(s.extras) == list(refs[0].extras) for s in refs)):
            # same text as DistanceHandler.Linear.WithExtras (one metric, no line merging), GPU-formatted
            exq, exr = list(data[0].extras), list(refs[0].extras)
            head = ["seqid (query)", *[k + " (query)" for k in exq], "seqid (reference)",
                    *[k + " (reference)" for k in exr], str(metric)]

            def pre(s):
                return "\t".join([s.id, *[v if v is not None else missing for v in s.extras.values()]])

            with open(self.paths.distances_linear, "wb") as fh:
                fh.write(("\t".join(head) + "\n").encode("utf-8"))
                write_rows_gpu(fh, self._engine(), np.ascontiguousarray(A)[:, :, None], [pre(s) for s in data],
                               [pre(s) for s in refs], dec, missing)
            return
        with DistanceHandler.Linear.WithExtras(self.paths.distances_linear, "w", missing=missing,
                                               formatter=fmt) as fh:
            for i, x in enumerate(data):
                for j, y in enumerate(refs):
                    v = A[i, j]
                    fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))

    def write_distances_matrix(self, data, refs, A):
        if not self.params.distances.write_matricial:
            return
        create_parents(self.paths.distances_matricial)
        fmt, missing = self.params.format.float, self.params.format.missing
        ids = [s.id for s in data]
        if len(set(ids)) != len(ids):
            metric = self.params.distances.metric
            with DistanceHandler.Matrix(self.paths.distances_matricial, "w", missing=missing, formatter=fmt) as fh:
                for i, x in enumerate(data):
                    for j, y in enumerate(refs):
                        v = A[i, j]
                        fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))
            return
        dec = fixed_decimals(fmt)
        if data and refs and gpu_text_ok(A, dec):
            with open(self.paths.distances_matricial, "wb") as fh:
                fh.write(("\t".join(["", *[s.id for s in refs]]) + "\n").encode("utf-8"))
                write_rows_gpu(fh, self._engine(), np.ascontiguousarray(A), ids, None, dec, missing)
            return
        text = format_values(A, fmt, missing)
        with open(self.paths.distances_matricial, "w") as fh:
            if data and refs:
                fh.write("\t".join(["", *[s.id for s in refs]]) + "\n")
            for i, x in enumerate(data):
                if refs:
                    fh.write("\t".join((x.id, *text[i])) + "\n")

    def write_closest(self, data, refs, closest):
        create_parents(self.paths.closest)
        fmt, missing = self.params.format.float, self.params.format.missing
        pct = bool(self.params.format.percentage_multiply)
        primary = self.params.distances.metric
        extras = list(self.params.distances.extra_metrics)
        with DistanceHandler.Linear.WithExtras(self.paths.closest, "w", missing=missing, formatter=fmt) as fh:
            for q, r, d, ex in closest:
                x, y = data[q], refs[r]
                fh.write(Distance(primary, x, y, d * 100.0 if pct else d))
                for metric, v in zip(extras, ex):
                    fv = float(v) if np.isfinite(v) else None
                    if fv is not None and pct:
                        fv *= 100.0
                    fh.write(Distance(metric, x, y, fv))
