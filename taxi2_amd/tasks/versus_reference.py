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

from ..align import Scores
from ..distances import ENGINE_LABELS, Distance, DistanceHandler, DistanceMetric, check_ncd_strings
from ..types import AttrDict
from ..sharding import distributed_rows, world_info
from .common import Results, console_report, create_parents, report
from .rect import closest_rows, first_minimum, write_rect_linear, write_rect_matrix, write_rect_pairs  # noqa: F401


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
        if str(primary) == "ncd" or any(str(m) == "ncd" for m in extras):
            check_ncd_strings(s.seq for s in data)
            check_ncd_strings(s.seq for s in refs)
        qs = eng.upload([s.seq for s in data], align=align)
        rs = eng.upload([s.seq for s in refs], align=align)
        E = len(extras)
        scale = 100.0 if pct else 1.0

        def block(qa: int, qb: int) -> np.ndarray:
            return closest_rows(eng, qs, rs, qa, qb, primary, extras, scores, align, scale, want_matrix,
                                lambda q1: report(self.progress_handler, "distance.x.id", q1 * R, total))

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
        write_rect_pairs(self.paths.aligned_pairs, data, refs, self.params.pairs.align, self.params.pairs.scores,
                         self._engine())

    def write_distances_linear(self, data, refs, A):
        if self.params.distances.write_linear:
            write_rect_linear(self.paths.distances_linear, data, refs, A, self.params.distances.metric,
                              self.params.format.float, self.params.format.missing, self._engine())

    def write_distances_matrix(self, data, refs, A):
        if self.params.distances.write_matricial:
            write_rect_matrix(self.paths.distances_matricial, data, refs, A, self.params.distances.metric,
                              self.params.format.float, self.params.format.missing, self._engine())

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
