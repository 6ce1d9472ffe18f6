"""Decontaminate task (``src/itaxotools/taxi2/tasks/decontaminate.py:93-371``), GPU-backed.

For every query: the closest outgroup sequence under one metric (default p) over the query-major
product (``fromProduct(data, outgroup)``, aligned when ``params.pairs.align``), x100 when
``percentage_multiply``; consecutive queries with equal ids form one group
(``groupby(distance.x.id)``, :255-259) whose minimum is the reference's ``min(.., key=d or inf)``
(:261-268: first minimum, and the group's first distance when none is defined).  The k-th input
sequence is paired with the k-th group minimum (``zip(sequences, minimums)``, :279) and is a
contaminant when that distance is <= ``params.thresholds.similarity`` (:275-277).  Writes
``summary.tsv``, ``decontaminated.<ext>``, ``contaminants.<ext>``, and (params) ``aligned_pairs.txt``
and ``distances/<metric>.{linear,matricial}.tsv``.  The distance search is the versusReference
closest kernel (``taxi2_closest``), query-sharded across ranks under torch.distributed.
"""

from __future__ import annotations

from math import inf
from pathlib import Path
from time import perf_counter
from typing import Callable, NamedTuple

import numpy as np

from ..align import Scores
from ..distances import ENGINE_LABELS, DistanceMetric, check_ncd_strings
from ..handlers import FileHandler
from ..sequences import Sequence, SequenceHandler
from ..sharding import distributed_rows, world_info
from ..types import AttrDict
from .common import Results, console_report, create_parents, report
from .rect import closest_rows, write_rect_linear, write_rect_matrix, write_rect_pairs


class Verdict(NamedTuple):
    sequence: Sequence
    contaminant: bool


class SummaryLine(NamedTuple):
    query_id: str
    outgroup_id: str
    outgroup_distance: float | None
    contaminant: bool


class FileFormat:
    """``file_types.py:12-14`` output formats (label, extension)."""

    Fasta = ("Fasta", ".fas")
    Tabfile = ("Tabfile", ".tsv")


def format_from_path(path: Path) -> tuple[str, str]:
    return FileFormat.Fasta if Path(path).suffix.lower() in (".fas", ".fasta", ".fa") else FileFormat.Tabfile


class _OrganismFasta:
    """``SequenceHandler.Fasta(path, "w", write_organism=True)`` (sequences.py:104-134):
    '>' id ['|' organism] then the sequence in 60-column lines and a blank line."""

    def __init__(self, path: Path, line_width: int = 60):
        self.fh = open(path, "w")
        self.w = line_width

    def write(self, s: Sequence) -> None:
        ident = s.id
        org = s.extras.get("organism", None)
        if org:
            ident += "|" + org
        self.fh.write(">" + ident + "\n")
        for k in range(0, len(s.seq), self.w):
            self.fh.write(s.seq[k : k + self.w] + "\n")
        self.fh.write("\n")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.fh.close()


def group_minima(qids: list[str], res: np.ndarray, scale: float, R: int) -> list[tuple[int, int, float | None]]:
    """Per group of consecutive equal query ids (``groupby(distance.x.id)``, decontaminate.py:255-259):
    ``min(distances, key=d or inf)`` (:261-268) -- the first minimum as (query, reference, scaled
    value), or (the group's first query, reference 0, None) when no distance is defined.  ``res`` rows
    are closest_rows output (closest index, unscaled value); nothing when there are no references
    (the reference's groupby then yields no group and zip stops)."""
    idx = res[:, 0].astype(np.int64)
    dmin = res[:, 1]
    minima: list[tuple[int, int, float | None]] = []
    Q = len(qids)
    if R:
        g0 = 0
        for k in range(1, Q + 1):
            if k == Q or qids[k] != qids[g0]:
                best = None
                for q in range(g0, k):
                    v = dmin[q] * scale if idx[q] >= 0 else inf
                    if best is None or v < best[0]:
                        best = (v, q)
                v, q = best
                minima.append((q, int(idx[q]), v) if v != inf else (g0, 0, None))
                g0 = k
    return minima


class Decontaminate:
    def __init__(self):
        self.work_dir: Path = None
        self.paths = AttrDict()
        self.progress_handler: Callable = console_report
        self.progress_interval: float = 0.015
        self.engine = None

        self.input = None
        self.outgroup = None
        self.output_format = None

        self.params = AttrDict()
        self.params.thresholds = AttrDict()
        self.params.thresholds.similarity = 0.07
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
        self.paths.decontaminated = w / f"decontaminated{ext}"
        self.paths.contaminants = w / f"contaminants{ext}"
        self.paths.aligned_pairs = w / "aligned_pairs.txt"
        self.paths.distances_linear = w / "distances" / f"{metric}.linear.tsv"
        self.paths.distances_matrix = w / "distances" / f"{metric}.matricial.tsv"

    def _engine(self):
        if self.engine is None:
            from .._native import Engine

            self.engine = Engine.default()
        return self.engine

    def start(self) -> Results:
        ts = perf_counter()
        self.check_params()
        self.generate_paths()
        align = bool(self.params.pairs.align)
        data = list(self.input)
        outgroup = list(self.outgroup)
        dn = [s.normalize() for s in data] if align else data
        on = [s.normalize() for s in outgroup] if align else outgroup
        metric = self.params.distances.metric
        scores = Scores(**(self.params.pairs.scores or {})).as_tuple()
        pct = bool(self.params.format.percentage_multiply)
        scale = 100.0 if pct else 1.0
        want_matrix = bool(self.params.distances.write_linear or self.params.distances.write_matricial)
        Q, R = len(dn), len(on)
        if str(metric) == "ncd":
            check_ncd_strings(s.seq for s in dn)
            check_ncd_strings(s.seq for s in on)
        eng = self._engine()
        qs = eng.upload([s.seq for s in dn], align=align)
        rs = eng.upload([s.seq for s in on], align=align)

        def block(qa: int, qb: int) -> np.ndarray:
            return closest_rows(eng, qs, rs, qa, qb, metric, [], scores, align, scale, want_matrix,
                                lambda q1: report(self.progress_handler, "distance.x.id", q1 * R, Q * R))

        try:
            distributed, rank = world_info()
            if distributed:
                import torch
                import torch.distributed as dist

                device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
                res = distributed_rows(Q, block, device=device)
            else:
                res = block(0, Q)
        finally:
            qs.free()
            rs.free()
        minima = group_minima([s.id for s in dn], res, scale, R)
        threshold = self.params.thresholds.similarity
        verdicts, lines = [], []
        for sequence, (q, r, d) in zip(data, minima):
            is_contaminant = d is not None and bool(d <= threshold)
            verdicts.append(Verdict(sequence, is_contaminant))
            lines.append(SummaryLine(sequence.id, on[r].id, d, is_contaminant))
        self.verdicts, self.summary = verdicts, lines

        if rank == 0:
            fmt, missing = self.params.format.float, self.params.format.missing
            if self.params.pairs.write:
                write_rect_pairs(self.paths.aligned_pairs, dn, on, align, self.params.pairs.scores, eng)
            if want_matrix:
                A = res[:, 2:] * scale if pct else res[:, 2:]
                if self.params.distances.write_linear:
                    write_rect_linear(self.paths.distances_linear, dn, on, A, metric, fmt, missing, eng)
                if self.params.distances.write_matricial:
                    write_rect_matrix(self.paths.distances_matrix, dn, on, A, metric, fmt, missing, eng)
            with self.get_output_handler(self.paths.decontaminated) as fh:
                for v in verdicts:
                    if not v.contaminant:
                        fh.write(v.sequence)
            with self.get_output_handler(self.paths.contaminants) as fh:
                for v in verdicts:
                    if v.contaminant:
                        fh.write(v.sequence)
            with FileHandler.Tabfile(self.paths.summary, "w", columns=SummaryLine._fields) as fh:
                for ln in lines:
                    d = missing if ln.outgroup_distance is None else fmt.format(ln.outgroup_distance)
                    fh.write((ln.query_id, ln.outgroup_id, d, "Yes" if ln.contaminant else "No"))
        report(self.progress_handler, "Finalizing...", len(data), len(data))
        return Results(self.work_dir, perf_counter() - ts)
