"""Dereplicate task (``src/itaxotools/taxi2/tasks/dereplicate.py:108-440``), GPU-backed.

The reference is a lazily pulled generator chain in which ``find_replicates`` (:289-337) adds ids
to ``self.excluded`` while ``drop_excluded_pairs`` (:188-196) -- upstream in the same chain --
filters every later pair of ``fromProduct(data, data)`` (x outer) against that set.  Following the
pulls through ``multiply`` / ``zip`` / ``groupby`` (:393-425): pair k is filtered after every
pair before it has been processed, and consecutive queries with equal ids share one group.

Here every ordered pair's distance (one metric, x100 when ``percentage_multiply``) is computed up
front on the GPU (the versusAll triangle, both orientations in one pass); the sequential walk over
those values runs natively (``taxi2_dereplicate_walk``, about a nanosecond per pair), and the
pairs it keeps -- the only ones the reference aligns and writes -- go to ``aligned_pairs.txt``
(GPU traceback) and the distance files (GPU text formatter, ragged rows).
"""

from __future__ import annotations

from pathlib import Path
from time import perf_counter
from typing import Callable, NamedTuple

import numpy as np

from ..align import Scores
from ..distances import ENGINE_LABELS, Distance, DistanceHandler, DistanceMetric, check_ncd_strings
from ..handlers import FileHandler
from ..pairs import SequencePair, SequencePairHandler
from ..sequences import Sequence
from ..types import AttrDict
from .common import Results, console_report, create_parents, fixed_decimals, gpu_text_ok, report
from .decontaminate import FileFormat, _OrganismFasta, format_from_path


class SummaryLine(NamedTuple):
    query_id: str
    query_length: str
    included_id: str
    included_length: int
    included_distance: float | None
    excluded_id: str
    excluded_length: int
    excluded_distance: float | None


def pair_matrix(eng, st, metric: DistanceMetric, align: bool, scores) -> np.ndarray:
    """(n, n) values of ``metric`` for every ordered pair (i, j) of the uploaded set ``st``,
    i != j (NaN = None): one pass of the versusAll triangle (both orientations)."""
    from .._native import tri_pairs

    n = st.n
    D = np.full((n, n), np.nan)
    if n < 2:
        return D
    npairs = n * (n - 1) // 2
    step = 1 << 16 if str(metric) == "ncd" else 1 << 20
    for k0 in range(0, npairs, step):
        c = min(step, npairs - k0)
        a, b = tri_pairs(n, k0, c)
        if str(metric) == "ncd":
            v = eng.ncd_pairs(st, st, a, b, scores, aligned=align, both=True)
            D[a, b], D[b, a] = v[:, 0], v[:, 1]
        else:
            v = eng.all_pairs(st, k0, c, [str(metric)], scores)
            if align:
                D[a, b], D[b, a] = v[:, 0, 0], v[:, 1, 0]
            else:
                D[a, b] = D[b, a] = v[:, 0]
    return D


class Dereplicate:
    def __init__(self):
        self.work_dir: Path = None
        self.paths = AttrDict()
        self.progress_handler: Callable = console_report
        self.progress_interval: float = 0.015
        self.engine = None

        self.input = None
        self.output_format = None
        self.excluded: set[str] = set()

        self.params = AttrDict()
        self.params.thresholds = AttrDict()
        self.params.thresholds.similarity = 0.07
        self.params.thresholds.length = 10
        self.params.pairs = AttrDict()
        self.params.pairs.align = True
        self.params.pairs.write = True
        self.params.pairs.scores = None
        self.params.distances = AttrDict()
        self.params.distances.metric = None
        self.params.distances.write_linear = True
        self.params.distances.write_matricial = True
        self.params.format = AttrDict()
        self.params.format.float = "{:.4f}"
        self.params.format.missing = "NA"
        self.params.format.percentage_multiply = False

    def set_output_format_from_path(self, path: Path):
        self.output_format = format_from_path(path)

    def get_output_handler(self, path: Path):
        if self.output_format == FileFormat.Fasta:
            return _OrganismFasta(path)
        from ..sequences import SequenceHandler

        return SequenceHandler.Tabfile(path, "w", idHeader="seqid", seqHeader="sequence")

    def check_params(self):
        self.output_format = self.output_format or FileFormat.Tabfile
        self.params.distances.metric = self.params.distances.metric or DistanceMetric.Uncorrected()
        if str(self.params.distances.metric) not in ENGINE_LABELS:
            raise NotImplementedError(f"metric {self.params.distances.metric} is not computed by the MI355X engine")

    def generate_paths(self):
        assert self.work_dir
        create_parents(self.work_dir)
        metric = str(self.params.distances.metric)
        ext = self.output_format[1]
        w = Path(self.work_dir)
        self.paths.summary = w / "summary.tsv"
        self.paths.dereplicated = w / f"dereplicated{ext}"
        self.paths.excluded = w / f"excluded{ext}"
        self.paths.aligned_pairs = w / "aligned_pairs.txt"
        self.paths.distances_linear = w / "distances" / f"{metric}.linear.tsv"
        self.paths.distances_matricial = w / "distances" / f"{metric}.matricial.tsv"

    def _engine(self):
        if self.engine is None:
            from .._native import Engine

            self.engine = Engine.default()
        return self.engine

    def start(self) -> Results:
        from .._native import dereplicate_walk

        ts = perf_counter()
        self.excluded = set()
        self.check_params()
        self.generate_paths()
        align = bool(self.params.pairs.align)
        metric = self.params.distances.metric
        scores = Scores(**(self.params.pairs.scores or {})).as_tuple()
        pct = bool(self.params.format.percentage_multiply)
        fmt, missing = self.params.format.float, self.params.format.missing

        data = [s for s in self.input if len(s.seq) >= self.params.thresholds.length]  # :180-183
        work = [s.normalize() for s in data] if align else data
        n = len(data)
        if str(metric) == "ncd":
            check_ncd_strings(s.seq for s in work)
        eng = self._engine()
        st = eng.upload([s.seq for s in work], align=align)
        try:
            D = pair_matrix(eng, st, metric, align, scores)
            if pct:
                D *= 100.0
            report(self.progress_handler, "distance.x.id", n * n, n * n)
            codes: dict[str, int] = {}
            idc = np.array([codes.setdefault(s.id, len(codes)) for s in data], dtype=np.int64)
            walk = dereplicate_walk(D, idc, [len(s.seq) for s in data], self.params.thresholds.similarity)
            rows = np.repeat(np.arange(n, dtype=np.int64), walk.row_kept)
            cols = walk.kept_cols.astype(np.int64)
            if len(rows):
                if self.params.pairs.write:
                    self._write_pairs(work, rows, cols, align, scores, eng, st)
                vals = D[rows, cols]
                if self.params.distances.write_linear:
                    self._write_linear(work, walk.row_kept, rows, cols, vals, metric, fmt, missing, eng)
                if self.params.distances.write_matricial:
                    self._write_matrix(work, walk.row_kept, rows, cols, vals, metric, fmt, missing, eng)
        finally:
            st.free()

        def dist(v):
            return float(v) if np.isfinite(v) else None

        lines = [SummaryLine(data[q].id, len(data[q].seq), data[a].id, len(data[a].seq), dist(da), data[b].id,
                             len(data[b].seq), dist(db))
                 for (q, a, b), (da, db) in zip(walk.line_idx.tolist(), walk.line_d.tolist())]
        self.excluded = {s.id for s, e in zip(data, walk.excluded) if e}

        def text(d):
            return missing if d is None else fmt.format(d)

        with FileHandler.Tabfile(self.paths.summary, "w", columns=SummaryLine._fields) as fh:
            for ln in lines:
                fh.write((ln.query_id, str(ln.query_length), ln.included_id, str(ln.included_length),
                          text(ln.included_distance), ln.excluded_id, str(ln.excluded_length),
                          text(ln.excluded_distance)))
        self.summary = lines
        with self.get_output_handler(self.paths.dereplicated) as fh:
            for s, e in zip(data, walk.excluded):
                if not e:
                    fh.write(s)
        with self.get_output_handler(self.paths.excluded) as fh:
            for s, e in zip(data, walk.excluded):
                if e:
                    fh.write(s)
        report(self.progress_handler, "Finalizing...", n * n, n * n)
        return Results(self.work_dir, perf_counter() - ts)

    # ------------------------------------------------------------------ writers (:226-287)
    def _write_pairs(self, work, rows, cols, align, scores, eng, st, chunk: int = 1 << 16) -> None:
        create_parents(self.paths.aligned_pairs)
        with SequencePairHandler.Formatted(self.paths.aligned_pairs, "w") as fh:
            for k0 in range(0, len(rows), chunk):
                r, c = rows[k0 : k0 + chunk], cols[k0 : k0 + chunk]
                if not align:
                    for i, j in zip(r.tolist(), c.tolist()):
                        fh.write(SequencePair(work[i], work[j]))
                    continue
                for i, j, (ax, ay) in zip(r.tolist(), c.tolist(), eng.align_strings(st, st, r, c, scores)):
                    fh.write(SequencePair(Sequence(work[i].id, ax, work[i].extras),
                                          Sequence(work[j].id, ay, work[j].extras)))

    @staticmethod
    def _gpu_ok(work, vals, fmt) -> bool:
        dec = fixed_decimals(fmt)
        ids = [s.id for s in work]
        keys = list(work[0].extras) if work else []
        return (gpu_text_ok(vals, dec) and len(set(ids)) == len(ids)
                and all(list(s.extras) == keys for s in work))

    def _write_linear(self, work, row_kept, rows, cols, vals, metric, fmt, missing, eng) -> None:
        path = self.paths.distances_linear
        create_parents(path)
        if self._gpu_ok(work, vals, fmt):
            keys = list(work[0].extras)
            head = ["seqid (query)", *[k + " (query)" for k in keys], "seqid (reference)",
                    *[k + " (reference)" for k in keys], str(metric)]
            pre = [_pre(s, missing) for s in work]
            with open(path, "wb") as fh:
                fh.write(("\t".join(head) + "\n").encode("utf-8"))
                _ragged_chunks(fh, eng, vals, row_kept, cols, pre, pre, fixed_decimals(fmt), missing)
            return
        with DistanceHandler.Linear.WithExtras(path, "w", missing=missing, formatter=fmt) as fh:
            for i, j, v in zip(rows.tolist(), cols.tolist(), vals.tolist()):
                fh.write(Distance(metric, work[i], work[j], v if np.isfinite(v) else None))

    def _write_matrix(self, work, row_kept, rows, cols, vals, metric, fmt, missing, eng) -> None:
        path = self.paths.distances_matricial
        create_parents(path)
        if self._gpu_ok(work, vals, fmt):
            first = int(rows[0])
            with open(path, "wb") as fh:
                fh.write(("\t".join(["", *[work[j].id for j in cols[: row_kept[first]].tolist()]]) + "\n")
                         .encode("utf-8"))
                _ragged_chunks(fh, eng, vals, row_kept, cols, [s.id for s in work], None, fixed_decimals(fmt),
                               missing)
            return
        with DistanceHandler.Matrix(path, "w", missing=missing, formatter=fmt) as fh:
            for i, j, v in zip(rows.tolist(), cols.tolist(), vals.tolist()):
                fh.write(Distance(metric, work[i], work[j], v if np.isfinite(v) else None))


def _pre(s, missing: str) -> str:
    return "\t".join([s.id, *[v if v is not None else missing for v in s.extras.values()]])


def _ragged_chunks(fh, eng, vals, row_kept, cols, row_pre, col_pre, decimals, missing,
                   max_values: int = 1 << 23) -> None:
    """Formatter text of the kept pairs (row r: its row_kept[r] tokens), in row chunks of about
    ``max_values`` tokens."""
    starts = np.concatenate([[0], np.cumsum(row_kept)]).astype(np.int64)
    n = len(row_kept)
    r0 = 0
    while r0 < n:
        r1 = int(np.searchsorted(starts, starts[r0] + max_values, side="right")) - 1
        r1 = min(n, max(r1, r0 + 1))
        fh.write(eng.format_ragged(vals, starts[r0 : r1 + 1], cols, row_pre[r0:r1], col_pre, ncols=len(row_pre),
                                   decimals=decimals, missing=missing, view=True))
        r0 = r1
