"""Decontaminate2 task (``src/itaxotools/taxi2/tasks/decontaminate2.py:99-434``), GPU-backed.

Every query is compared with an outgroup AND an ingroup (two query-major products,
``fromProduct(data, outgroup)`` / ``fromProduct(data, ingroup)``, aligned when
``params.pairs.align``).  Per group of consecutive equal query ids each side's minimum is the
reference's ``min(.., key=d or inf)`` (``group_minima``); only the outgroup distances are x100 with
``percentage_multiply`` (``adjust_distances`` sits on the outgroup chain alone, :404-412); each minimum
is then multiplied by its side's weight (:321-330).  A query is a contaminant when its outgroup
distance is defined and either the ingroup distance is undefined or outgroup < ingroup (:314-319).
Writes ``summary.tsv`` (query, outgroup id / distance, ingroup id / distance, Yes / No),
``decontaminated.<ext>``, ``contaminants.<ext>`` and, per params, ``aligned_pairs/{outgroup,ingroup}.txt``
and ``distances/{outgroup,ingroup}.<metric>.{linear,matricial}.tsv``.  Both searches are the
versusReference closest kernel (``taxi2_closest``), query-sharded across ranks under torch.distributed.
"""

from __future__ import annotations

from pathlib import Path
from time import perf_counter
from typing import Callable, NamedTuple

import numpy as np

from ..align import Scores
from ..distances import ENGINE_LABELS, DistanceMetric, check_ncd_strings
from ..handlers import FileHandler
from ..sharding import distributed_rows, world_info
from ..types import AttrDict
from .common import Results, console_report, create_parents, report
from .decontaminate import Decontaminate, FileFormat, Verdict, group_minima
from .rect import closest_rows, write_rect_linear, write_rect_matrix, write_rect_pairs


class SummaryLine(NamedTuple):
    query_id: str
    outgroup_id: str
    outgroup_distance: float | None
    ingroup_id: str
    ingroup_distance: float | None
    contaminant: bool


class Decontaminate2:
    def __init__(self):
        self.work_dir: Path = None
        self.paths = AttrDict()
        self.progress_handler: Callable = console_report
        self.progress_interval: float = 0.015
        self.engine = None

        self.input = None
        self.outgroup = None
        self.ingroup = None
        self.output_format = None

        self.params = AttrDict()
        self.params.weights = AttrDict()
        self.params.weights.outgroup = 1.0
        self.params.weights.ingroup = 1.0
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

    # same output formats and handlers as Decontaminate (decontaminate2.py:133-143)
    set_output_format_from_path = Decontaminate.set_output_format_from_path
    get_output_handler = Decontaminate.get_output_handler
    _engine = Decontaminate._engine

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
        self.paths.outgroup_aligned_pairs = w / "aligned_pairs" / "outgroup.txt"
        self.paths.ingroup_aligned_pairs = w / "aligned_pairs" / "ingroup.txt"
        self.paths.outgroup_linear = w / "distances" / f"outgroup.{metric}.linear.tsv"
        self.paths.outgroup_matrix = w / "distances" / f"outgroup.{metric}.matricial.tsv"
        self.paths.ingroup_linear = w / "distances" / f"ingroup.{metric}.linear.tsv"
        self.paths.ingroup_matrix = w / "distances" / f"ingroup.{metric}.matricial.tsv"

    def _search(self, eng, qs, refs: list, align: bool, scores, scale: float, want_matrix: bool,
                done: int, total: int) -> np.ndarray:
        """closest_rows of every query against one side (query-sharded under torch.distributed)."""
        metric = self.params.distances.metric
        Q, R = qs.n, len(refs)
        rs = eng.upload([s.seq for s in refs], align=align)

        def block(qa: int, qb: int) -> np.ndarray:
            return closest_rows(eng, qs, rs, qa, qb, metric, [], scores, align, scale, want_matrix,
                                lambda q1: report(self.progress_handler, "distance.x.id", done + q1 * R, total))

        try:
            distributed, _ = world_info()
            if distributed:
                import torch
                import torch.distributed as dist

                device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
                return distributed_rows(Q, block, device=device)
            return block(0, Q)
        finally:
            rs.free()

    def start(self) -> Results:
        ts = perf_counter()
        self.check_params()
        self.generate_paths()
        align = bool(self.params.pairs.align)
        data, outgroup, ingroup = list(self.input), list(self.outgroup), list(self.ingroup)
        dn = [s.normalize() for s in data] if align else data
        on = [s.normalize() for s in outgroup] if align else outgroup
        inn = [s.normalize() for s in ingroup] if align else ingroup
        metric = self.params.distances.metric
        scores = Scores(**(self.params.pairs.scores or {})).as_tuple()
        pct = bool(self.params.format.percentage_multiply)
        oscale = 100.0 if pct else 1.0  # the ingroup chain has no adjust_distances (:414-421)
        want_matrix = bool(self.params.distances.write_linear or self.params.distances.write_matricial)
        Q, RO, RI = len(dn), len(on), len(inn)
        if str(metric) == "ncd":
            for side in (dn, on, inn):
                check_ncd_strings(s.seq for s in side)
        eng = self._engine()
        qs = eng.upload([s.seq for s in dn], align=align)
        total = Q * (RO + RI)
        try:
            res_o = self._search(eng, qs, on, align, scores, oscale, want_matrix, 0, total)
            res_i = self._search(eng, qs, inn, align, scores, 1.0, want_matrix, Q * RO, total)
        finally:
            qs.free()
        qids = [s.id for s in dn]
        out_min = group_minima(qids, res_o, oscale, RO)
        in_min = group_minima(qids, res_i, 1.0, RI)

        w_out, w_in = self.params.weights.outgroup, self.params.weights.ingroup
        verdicts, lines = [], []
        for sequence, (_, ro, od), (_, ri, idd) in zip(data, out_min, in_min):
            if od is not None:
                od *= w_out
            if idd is not None:
                idd *= w_in
            is_contaminant = False if od is None else True if idd is None else bool(od < idd)
            verdicts.append(Verdict(sequence, is_contaminant))
            lines.append(SummaryLine(sequence.id, on[ro].id, od, inn[ri].id, idd, is_contaminant))
        self.verdicts, self.summary = verdicts, lines

        _, rank = world_info()
        if rank == 0:
            fmt, missing = self.params.format.float, self.params.format.missing
            if self.params.pairs.write:
                write_rect_pairs(self.paths.outgroup_aligned_pairs, dn, on, align, self.params.pairs.scores, eng)
                write_rect_pairs(self.paths.ingroup_aligned_pairs, dn, inn, align, self.params.pairs.scores, eng)
            if want_matrix:
                for res, refs, scale, lin, mat in ((res_o, on, oscale, self.paths.outgroup_linear, self.paths.outgroup_matrix),
                                                   (res_i, inn, 1.0, self.paths.ingroup_linear, self.paths.ingroup_matrix)):
                    A = res[:, 2:] * scale if scale != 1.0 else res[:, 2:]
                    if self.params.distances.write_linear:
                        write_rect_linear(lin, dn, refs, A, metric, fmt, missing, eng)
                    if self.params.distances.write_matricial:
                        write_rect_matrix(mat, dn, refs, A, metric, fmt, missing, eng)
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
                    fh.write((ln.query_id, ln.outgroup_id,
                              missing if ln.outgroup_distance is None else fmt.format(ln.outgroup_distance),
                              ln.ingroup_id,
                              missing if ln.ingroup_distance is None else fmt.format(ln.ingroup_distance),
                              "Yes" if ln.contaminant else "No"))
        report(self.progress_handler, "Finalizing...", len(data), len(data))
        return Results(self.work_dir, perf_counter() - ts)

