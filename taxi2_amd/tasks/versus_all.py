"""VersusAll task (``src/itaxotools/taxi2/tasks/versus_all.py:374-773``), GPU-backed.

Same public surface: ``task.work_dir``, ``task.input.sequences``, ``task.params`` (same names),
``task.progress_handler``, ``task.start() -> Results(output_directory, seconds_taken)``.

What ``start`` computes is the reference's hot path (``versus_all.py:732-753``):
normalize (when aligning) -> ordered product x-major -> Biopython global alignment ->
p / p-gaps / jc / k2p for every ordered pair, ``None`` where the aligned pair is identical
(``x != y`` on full tuples, :549-552), x100 when ``percentage_multiply`` (:554-562) ->
``distances/linear.tsv`` (Linear.WithExtras) and ``distances/matricial/<metric>.tsv``, plus
``align/aligned_pairs.txt`` (Formatted) when ``params.pairs.write``, ``summary.tsv`` (always, with
genus / species / comparison type from ``input.genera`` / ``input.species``) and, per given
partition, the subset statistics under ``subsets/{genera,species}`` (``tasks/subsets.py``).

The N(N-1)/2 unordered pairs run on the MI355X engine in blocks; one DP fill gives both ordered
pairs.  With torch.distributed initialised (one process per GPU) the pair space is sharded by
row blocks and gathered over RCCL (``taxi2_amd/sharding.py``).

Out of scope: per-sequence statistics (``stats/*.tsv``) and histograms.
Their params exist with the reference's names but default to False here; setting one raises
NotImplementedError.
"""

from __future__ import annotations

from pathlib import Path
from time import perf_counter
from typing import Callable

import numpy as np

from ..align import PairwiseAligner, Scores
from ..distances import ENGINE_LABELS, Distance, DistanceHandler, DistanceMetric, check_ncd_strings
from ..pairs import SequencePair, SequencePairHandler
from ..sequences import Sequences
from ..types import AttrDict
from .common import (Results, console_report, create_parents, fixed_decimals, format_values, gpu_text_ok,
                     report, seq_key, write_rows_gpu)


class VersusAll:
    def __init__(self):
        self.work_dir: Path = None
        self.paths = AttrDict()
        self.progress_handler: Callable = console_report
        self.progress_interval: float = 0.015
        self.engine = None  # taxi2_amd._native.Engine (default: one per local GPU)

        self.input = AttrDict()
        self.input.sequences: Sequences = None
        self.input.species = None
        self.input.genera = None

        self.params = AttrDict()
        self.params.pairs = AttrDict()
        self.params.pairs.align = True
        self.params.pairs.write = True
        self.params.pairs.scores = None

        self.params.distances = AttrDict()
        self.params.distances.metrics = None
        self.params.distances.write_linear = True
        self.params.distances.write_matricial = True

        self.params.plot = AttrDict()
        self.params.plot.histograms = False  # reference default True: out of scope
        self.params.plot.binwidth = 0.05
        self.params.plot.formats = None
        self.params.plot.palette = None

        self.params.format = AttrDict()
        self.params.format.float = "{:.4f}"
        self.params.format.percentage = "{:.2f}"
        self.params.format.missing = "NA"
        self.params.format.stats_template = "{mean} ({min}-{max})"
        self.params.format.percentage_multiply = False

        self.params.stats = AttrDict()
        self.params.stats.all = False  # reference default True: out of scope
        self.params.stats.species = False
        self.params.stats.genera = False

        self.distances: np.ndarray | None = None  # (N, N, M) after start(), NaN = None

    # ------------------------------------------------------------------ reference steps
    def generate_paths(self):
        assert self.work_dir
        w = Path(self.work_dir)
        self.paths.summary = w / "summary.tsv"
        self.paths.stats_all = w / "stats" / "all.tsv"
        self.paths.stats_species = w / "stats" / "species.tsv"
        self.paths.stats_genera = w / "stats" / "genera.tsv"
        self.paths.aligned_pairs = w / "align" / "aligned_pairs.txt"
        self.paths.distances_linear = w / "distances" / "linear.tsv"
        self.paths.distances_matricial = w / "distances" / "matricial"
        self.paths.subsets = w / "subsets"
        self.paths.plots = w / "plots"
        create_parents(self.paths.summary)

    def check_metrics(self):
        self.params.distances.metrics = self.params.distances.metrics or [
            DistanceMetric.Uncorrected(),
            DistanceMetric.UncorrectedWithGaps(),
            DistanceMetric.JukesCantor(),
            DistanceMetric.Kimura2P(),
        ]
        for m in self.params.distances.metrics:
            if str(m) not in ENGINE_LABELS:
                raise NotImplementedError(f"metric {m} is not computed by the MI355X engine (DESIGN.md)")

    def _check_scope(self):
        for flag, name in ((self.params.stats.all, "stats.all"), (self.params.stats.species, "stats.species"),
                           (self.params.stats.genera, "stats.genera"), (self.params.plot.histograms, "plot.histograms")):
            if flag:
                raise NotImplementedError(f"params.{name} is outside the MI355X hot path (SURVEY.md §2)")

    def _engine(self):
        if self.engine is None:
            from .._native import Engine

            self.engine = Engine.default()
        return self.engine

    # ------------------------------------------------------------------ compute
    def compute_distances(self, seqs: list) -> np.ndarray:
        """(N, N, M) float64 matrix, NaN where the reference yields None (before x100)."""
        from .._native import tri_pairs

        labels = [str(m) for m in self.params.distances.metrics]
        M = len(labels)
        cidx = [k for k, lab in enumerate(labels) if lab != "ncd"]  # counter metrics
        nidx = [k for k, lab in enumerate(labels) if lab == "ncd"]
        clabels = [labels[k] for k in cidx]
        align = bool(self.params.pairs.align)
        scores = Scores(**(self.params.pairs.scores or {})).as_tuple()
        n = len(seqs)
        D = np.full((n, n, M), np.nan)
        total = M * n * n
        if n == 0:
            return D
        if nidx:
            check_ncd_strings(s.seq for s in seqs)
        eng = self._engine()
        st = eng.upload([s.seq for s in seqs], align=align)
        try:
            npairs = n * (n - 1) // 2

            def compute(k0: int, count: int) -> np.ndarray:
                """Unordered pairs [k0, k0 + count) -> (count, 2 * M): (a, b) row then (b, a) row."""
                out = np.empty((count, 2, M))
                step = (1 << 20) if align else (1 << 24)
                if nidx:
                    step = min(step, 1 << 16)
                for c0 in range(0, count, step):
                    c = min(step, count - c0)
                    if cidx:
                        blk = eng.all_pairs(st, k0 + c0, c, clabels, scores)
                        if align:
                            out[c0 : c0 + c][:, :, cidx] = blk
                        else:  # counters are symmetric: one value serves both ordered rows
                            out[c0 : c0 + c][:, 0, cidx] = blk
                            out[c0 : c0 + c][:, 1, cidx] = blk
                    if nidx:
                        a, b = tri_pairs(n, k0 + c0, c)
                        v = eng.ncd_pairs(st, st, a, b, scores, aligned=align, both=True)
                        for k in nidx:
                            out[c0 : c0 + c][:, :, k] = v
                    report(self.progress_handler, "distance.x.id", min(total, 2 * M * (k0 + c0 + c)), total)
                return out.reshape(count, 2 * M)

            res = self._run_pairs(n, npairs, compute)
            a, b = tri_pairs(n)
            D[a, b] = res[:, :M]
            D[b, a] = res[:, M:]
            # diagonal rule on full tuples: identical (id, seq, extras) -> None unless the
            # alignment of the sequence with itself is not the identity (non-default scores)
            groups: dict = {}
            for i, s in enumerate(seqs):
                groups.setdefault(seq_key(s), []).append(i)
            dup = [g for g in groups.values()]
            if align:
                reps = np.array([g[0] for g in dup], dtype=np.int64)
                strings = eng.align_strings(st, st, reps, reps, scores)
                self_vals = np.empty((len(reps), M))
                if cidx:
                    self_vals[:, cidx] = eng.list_pairs(st, st, reps, reps, clabels, scores)[:, 0, :]
                if nidx:
                    v = eng.ncd_pairs(st, st, reps, reps, scores, aligned=True, both=False)
                    for k in nidx:
                        self_vals[:, k] = v
            for gi, g in enumerate(dup):
                if align and strings[gi][0] != strings[gi][1]:
                    for i in g:
                        D[i, i] = self_vals[gi]
                    continue
                for i in g:
                    D[i, g] = np.nan
        finally:
            st.free()
        return D

    def _run_pairs(self, n: int, npairs: int, compute) -> np.ndarray:
        try:
            import torch.distributed as dist

            dist_on = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        except Exception:
            dist_on = False
        if not dist_on:
            return compute(0, npairs)
        import torch
        import torch.distributed as dist

        from ..sharding import distributed_all_pairs

        device = None
        if dist.get_backend() == "nccl":
            device = torch.device("cuda", torch.cuda.current_device())
        return distributed_all_pairs(n, compute, device=device)

    # ------------------------------------------------------------------ outputs
    def _adjusted(self, D: np.ndarray) -> np.ndarray:
        return D * 100.0 if self.params.format.percentage_multiply else D

    def write_distances_linear(self, seqs: list, D: np.ndarray):
        if not self.params.distances.write_linear:
            return
        create_parents(self.paths.distances_linear)
        fmt, missing = self.params.format.float, self.params.format.missing
        metrics = self.params.distances.metrics
        ids = [s.id for s in seqs]
        if len(set(ids)) != len(ids):  # duplicate ids: exact reference line grouping
            with DistanceHandler.Linear.WithExtras(self.paths.distances_linear, "w", missing=missing,
                                                   formatter=fmt) as fh:
                for i, x in enumerate(seqs):
                    for j, y in enumerate(seqs):
                        for m, metric in enumerate(metrics):
                            v = D[i, j, m]
                            fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))
            return
        n = len(seqs)
        if n == 0:
            open(self.paths.distances_linear, "w").close()
            return
        ex0 = list(seqs[0].extras.keys())
        head = ["seqid (query)", *[k + " (query)" for k in ex0], "seqid (reference)",
                *[k + " (reference)" for k in ex0], *[str(m) for m in metrics]]
        pre = ["\t".join([s.id, *[v if v is not None else missing for v in s.extras.values()]]) for s in seqs]
        dec = fixed_decimals(fmt)
        if gpu_text_ok(D, dec):  # text formatted on the GPU (taxi2_format_rows)
            with open(self.paths.distances_linear, "wb") as fh:
                fh.write(("\t".join(head) + "\n").encode("utf-8"))
                write_rows_gpu(fh, self._engine(), D, pre, pre, dec, missing)
            return
        text = format_values(D, fmt, missing)
        with open(self.paths.distances_linear, "w") as fh:
            fh.write("\t".join(head) + "\n")
            for i in range(n):
                rows = ["\t".join((pre[i], pre[j], *text[i, j])) for j in range(n)]
                fh.write("\n".join(rows) + "\n")

    def write_distances_multimatrix(self, seqs: list, D: np.ndarray):
        if not self.params.distances.write_matricial:
            return
        create_parents(self.paths.distances_matricial)
        fmt, missing = self.params.format.float, self.params.format.missing
        ids = [s.id for s in seqs]
        for m, metric in enumerate(self.params.distances.metrics):
            path = self.paths.distances_matricial / f"{metric}.tsv"
            if len(set(ids)) != len(ids):
                with DistanceHandler.Matrix(path, "w", missing=missing, formatter=fmt) as fh:
                    for i, x in enumerate(seqs):
                        for j, y in enumerate(seqs):
                            v = D[i, j, m]
                            fh.write(Distance(metric, x, y, float(v) if np.isfinite(v) else None))
                continue
            dec = fixed_decimals(fmt)
            if gpu_text_ok(D[:, :, m], dec):
                with open(path, "wb") as fh:
                    if seqs:
                        fh.write(("\t".join(["", *ids]) + "\n").encode("utf-8"))
                        write_rows_gpu(fh, self._engine(), np.ascontiguousarray(D[:, :, m]), ids, None, dec,
                                       missing)
                continue
            text = format_values(D[:, :, m], fmt, missing)
            with open(path, "w") as fh:
                if seqs:
                    fh.write("\t".join(["", *ids]) + "\n")
                for i in range(len(seqs)):
                    fh.write("\t".join((ids[i], *text[i])) + "\n")

    def write_pairs(self, seqs: list):
        if not self.params.pairs.write:
            return
        create_parents(self.paths.aligned_pairs)
        n = len(seqs)
        with SequencePairHandler.Formatted(self.paths.aligned_pairs, "w") as fh:
            if not self.params.pairs.align:
                for x in seqs:
                    for y in seqs:
                        fh.write(SequencePair(x, y))
                return
            aligner = PairwiseAligner.Biopython(self.params.pairs.scores, engine=self._engine())
            for x in seqs:  # row x: (x, y) for every y, x-major like fromProduct
                for pair in aligner.align_many([SequencePair(x, y) for y in seqs]):
                    fh.write(pair)

    def write_summary(self, seqs: list, A: np.ndarray):
        from .subsets import write_summary

        write_summary(self.paths.summary, seqs, A, self.params.distances.metrics, self.input.genera,
                      self.input.species, self.params.format.float, self.params.format.missing,
                      self._engine() if seqs else None)

    def write_subsets(self, seqs: list, A: np.ndarray):
        from .subsets import aggregate, write_subset_statistics

        ids = [s.id for s in seqs]
        for partition, name in ((self.input.genera, "genera"), (self.input.species, "species")):
            if partition:
                write_subset_statistics(self.paths.subsets / name, aggregate(A, ids, partition),
                                        self.params.distances.metrics, self.params.format.float,
                                        self.params.format.stats_template)

    # ------------------------------------------------------------------ driver
    def start(self) -> Results:
        ts = perf_counter()
        self.generate_paths()
        self.check_metrics()
        self._check_scope()
        seqs = list(self.input.sequences)
        if self.params.pairs.align:
            seqs = [s.normalize() for s in seqs]
        D = self.compute_distances(seqs)
        self.distances = D
        rank0 = True
        try:
            import torch.distributed as dist

            rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
        except Exception:
            pass
        if rank0:
            A = self._adjusted(D)
            self.write_pairs(seqs)
            self.write_distances_linear(seqs, A)
            self.write_distances_multimatrix(seqs, A)
            self.write_summary(seqs, A)
            self.write_subsets(seqs, A)
        n = len(seqs)
        total = len(self.params.distances.metrics) * n * n
        report(self.progress_handler, "Finalizing...", total, total)
        return Results(self.work_dir, perf_counter() - ts)
