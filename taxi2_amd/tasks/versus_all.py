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

import os
import sys
from pathlib import Path
from time import perf_counter
from typing import Callable

import numpy as np

from ..align import PairwiseAligner, Scores
from ..distances import ENGINE_LABELS, Distance, DistanceHandler, DistanceMetric, check_ncd_strings
from ..pairs import SequencePair, SequencePairHandler
from ..sequences import Sequences
from ..types import AttrDict
from .common import (Results, console_report, create_parents, fixed_decimals, format_values, full_tuple_groups,
                     gpu_text_ok, report, write_rows_gpu)


def self_strings(eng, st, seqs: list, idx, scores: tuple) -> list:
    """Each sequence idx[k] aligned with itself (versus_all.py:549's diagonal rule, the diagonal pairs
    of aligned_pairs.txt).  When a match scores > 0, no mismatch scores more than a match and no gap
    score is positive, the first alignment is the identity -- the diagonal scores len * match, a
    path with gaps trades at least one match for gaps and a shifted diagonal pairs mismatching bytes
    at most -- so no alignment is run; otherwise the aligner's own strings (e.g. mismatch > match:
    a one-column shift of a 10-base sequence can outscore the identity)."""
    m, mi, io, ie, eo, ee = scores
    if m > 0 and mi <= m and max(io, ie, eo, ee) <= 0:
        return [(seqs[i].seq, seqs[i].seq) for i in np.asarray(idx).tolist()]
    return eng.align_strings(st, st, idx, idx, scores)


def walk_strings_ok(scores: tuple, seqs: list) -> bool:
    """Does the packed trace-and-walk aligner (which can write the aligned strings while its walks
    give the metrics) cover this run?  Gotoh scores (not every open == extend), pairs up to 2 048
    columns, every DP difference within int16 (alignt2_kernel.hpp at_fits16, restated), and the
    same environment knobs that make the engine decline the shape (capi.hip launch_packed_strings).

    Only all-ASCII sequences: the walkers copy sequence bytes straight into the aligned_pairs.txt
    text, and the engine stores one latin-1 byte per character, while the reference writes str to a
    UTF-8 text file (SequencePairHandler.Formatted) -- a character in U+0080..U+00FF must become two
    bytes there, which the Python-formatted writer does."""
    ma, mi, io, ie, eo, ee = scores
    if io == ie and eo == ee:
        return False
    if any(os.environ.get(k) for k in ("TAXI2_NO_ALIGNT", "TAXI2_NO_PACKED", "TAXI2_LONG", "TAXI2_NO_WALK_STRINGS")):
        return False
    if not all(s.seq.isascii() for s in seqs):
        return False
    L = max((len(s.seq) for s in seqs), default=0)
    if L > 2048:
        return False
    P = max(abs(ma), abs(mi), abs(ie), abs(ee))
    O = max(abs(io), abs(eo))
    lo = 2 * (P * 2 * L + 2 * O + 2)
    hi = 2 * abs(ma) * L + 2 + 2 * abs(ie) * 2 * L
    return lo + 2 * O + 2 * P + 16384 + 8 < 32767 and hi + 2 * O + 2 * P + 16384 + 8 < 32767



WALK_LAUNCH_PAIRS = 1 << 19  # ordered pairs per string-emitting aligner launch (the bench's batch)
WALK_BLOCK_BYTES = 8 << 30   # HBM for one block's string slots + metrics
DEVICE_D_BYTES = 16 << 30    # the walked path's device copy of the counter metrics, at most
TEXT_CALL_BYTES = 1 << 30    # aligned_pairs.txt text per formatter call (bound), i.e. its pinned buffer
PIPE_DEPTH = 2               # one-fill aligned_pairs path: blocks aligned ahead of the block being written


def walk_block_rows(n: int, per_pair: int, block_bytes: int, launch_pairs: int = WALK_LAUNCH_PAIRS) -> int:
    """Rows per block of the string-emitting row-block path: at least what ``block_bytes`` allows,
    and enough rows for ~``launch_pairs`` pairs per launch (a 12-row block of N = 5 000 left the
    GPU mostly idle between syncs) as long as the block's slots fit WALK_BLOCK_BYTES."""
    per_row = max(1, n * per_pair)
    b_bytes = block_bytes // per_row
    b_fill = min(-(-int(launch_pairs) // max(1, n)), WALK_BLOCK_BYTES // per_row)
    return max(1, min(n, max(b_bytes, b_fill)))

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

        # MI355X engine options (no reference counterpart).  stream: None = automatic (row-block
        # streaming when the dense N x N x M host matrix would exceed dense_limit bytes, or with
        # more than one rank), True / False force it; block_bytes sizes the streamed row blocks;
        # launch_pairs: the string-emitting row blocks grow to about this many pairs per launch
        # (0: block_bytes alone).
        self.params.engine = AttrDict()
        self.params.engine.launch_pairs = WALK_LAUNCH_PAIRS
        # HBM for the (b, a) aligned strings the one-fill aligned_pairs path keeps until row b
        self.params.engine.keep_bytes = 160 << 30
        # CUs' worth of workgroup slots the one-fill aligned_pairs path leaves free beside each
        # block's fill, for the previous block's text kernel (host-link bound: it needs few CUs)
        self.params.engine.text_reserve_cus = 32
        # text_cu_mask: the fill and the text on disjoint CU ranges (CU-masked streams);
        # text_copy: how the pair text reaches pinned host memory (0 kernel stores, 1 device buffer +
        # DMA, 2 device buffer + 16-byte copy kernel; taxi2_set_text_copy)
        self.params.engine.text_cu_mask = False
        self.params.engine.text_copy = 0
        # text_pipeline "fused": each block's compaction and text queued on the fill stream behind
        # its fill (whole chip, ~1 ms per GB), the text moved to the host beside the next fills by
        # a copy kernel (text_copy 2, the default there: no LDS, so it co-runs with a persistent
        # fill) or the DMA engine (1), no CUs reserved; "streams": the text
        # kernels on a second stream beside the fills, in text_reserve_cus CUs (round 5)
        self.params.engine.text_pipeline = "fused"
        self.params.engine.stream = None
        self.params.engine.dense_limit = 4 << 30
        self.params.engine.block_bytes = 256 << 20
        # reductions instead of (or beside) the N x N text: write_summary False skips summary.tsv
        # (the reference always writes it); row_minima = a metric label gathers, per sequence, the
        # closest other sequence by that metric (first minimum, None skipped) into
        # task.row_minima = (index, value) and distances/row_minima.tsv (streamed path)
        self.params.engine.write_summary = True
        self.params.engine.row_minima = None
        self.row_minima = None
        # streamed pre-aligned path: a sharded rank keeps its computed row blocks in HBM for the
        # rank-ordered subset chain when they fit this many bytes (else recomputes them);
        # timings = True synchronises after each phase and fills task.timings (seconds)
        self.params.engine.hold_bytes = 160 << 30
        self.params.engine.timings = False
        self.timings = None
        self.subset_stats = None  # {"genera" / "species": SubsetStats} after start() (engine extra)
        self.pairs_walked = False  # aligned_pairs.txt came from the metric walks (dense path)

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
    def compute_distances(self, seqs: list, pairs_fh=None) -> np.ndarray:
        """(N, N, M) float64 matrix, NaN where the reference yields None (before x100).  With
        ``pairs_fh`` (a binary file, aligning, one rank) the metrics and aligned_pairs.txt come from
        the same walks when the packed aligner covers the shape (``self.pairs_walked``)."""
        from .._native import tri_pairs

        labels = [str(m) for m in self.params.distances.metrics]
        M = len(labels)
        cidx = [k for k, lab in enumerate(labels) if lab != "ncd"]  # counter metrics
        nidx = [k for k, lab in enumerate(labels) if lab == "ncd"]
        clabels = [labels[k] for k in cidx]
        align = bool(self.params.pairs.align)
        scores = Scores(**(self.params.pairs.scores or {})).as_tuple()
        n = len(seqs)
        # every entry is written below (each path fills every ordered pair's row, the diagonal rule
        # every (x, x)): no N^2 NaN fill up front -- the pages are touched as the rows arrive
        D = np.empty((n, n, M))
        total = M * n * n
        if n == 0:
            return D
        if nidx:
            check_ncd_strings(s.seq for s in seqs)
        eng = self._engine()
        st = eng.upload([s.seq for s in seqs], align=align)
        t_up = perf_counter()
        try:
            npairs = n * (n - 1) // 2

            def compute(k0: int, count: int) -> np.ndarray:
                """Unordered pairs [k0, k0 + count) -> (count, 2 * M): (a, b) row then (b, a) row."""
                out = np.empty((count, 2, M))
                step = (1 << 20) if align else (1 << 24)
                if nidx:
                    step = min(step, 1 << 18 if align else 1 << 16)
                for c0 in range(0, count, step):
                    c = min(step, count - c0)
                    if align:  # every metric, NCD included, from the one alignment of each ordered pair
                        out[c0 : c0 + c] = eng.all_pairs(st, k0 + c0, c, labels, scores)
                    else:
                        if cidx:  # counters are symmetric: one value serves both ordered rows
                            blk = eng.all_pairs(st, k0 + c0, c, clabels, scores)
                            out[c0 : c0 + c][:, 0, cidx] = blk
                            out[c0 : c0 + c][:, 1, cidx] = blk
                        if nidx:
                            a, b = tri_pairs(n, k0 + c0, c)
                            v = eng.ncd_pairs(st, st, a, b, scores, aligned=False, both=True)
                            for k in nidx:
                                out[c0 : c0 + c][:, :, k] = v
                    report(self.progress_handler, "distance.x.id", min(total, 2 * M * (k0 + c0 + c)), total)
                return out.reshape(count, 2 * M)

            walked = False
            if pairs_fh is not None and walk_strings_ok(scores, seqs):
                # every metric (NCD from the same walks' strings) and aligned_pairs.txt from one fill
                every = list(range(M))
                walked = (self._tri_with_pairs(seqs, eng, st, D, every, labels, scores, pairs_fh)
                          or self._rows_with_pairs(seqs, eng, st, D, every, labels, scores, pairs_fh))
            if not walked:
                res = self._run_pairs(n, npairs, compute)
                a, b = tri_pairs(n)
                D[a, b] = res[:, :M]
                D[b, a] = res[:, M:]
            self.pairs_walked = walked
            t_walk = perf_counter()
            # diagonal rule on full tuples: identical (id, seq, extras) -> None unless the
            # alignment of the sequence with itself is not the identity (non-default scores)
            dup = full_tuple_groups(seqs)
            if align:
                reps = np.array([g[0] for g in dup], dtype=np.int64)
                strings = self_strings(eng, st, seqs, reps, scores)
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
        if isinstance(self.timings, dict):  # sub-phases of compute_s (walk includes the pairs text)
            self.timings["walk_s"] = t_walk - t_up
            self.timings["diag_s"] = perf_counter() - t_walk
        return D

    def _tri_with_pairs(self, seqs, eng, st, D, cidx, clabels, scores, fh) -> bool:
        """_tri_with_pairs_on with its two streams.  With text_reserve_cus = R > 0 the fill stream
        runs on CUs [R, num_cus) and the text stream on CUs [0, R) (taxi2_stream_create_cus): the
        fill's persistent launch leaves R CUs' worth of workgroup slots free, and without a CU mask
        the dispatcher spreads both kernels' workgroups over every CU, so the text kernel's VALU
        work can take issue slots from the fill waves on all of them (params.engine.text_cu_mask,
        TAXI2_TEXT_MASK=1; profiles/r6/task/)."""
        import torch

        dev = torch.device("cuda", eng.device)
        # CUs' worth of workgroup slots the fill leaves free for the previous block's text kernel
        pipeline = os.environ.get("TAXI2_TEXT_PIPELINE", self.params.engine.text_pipeline)
        if pipeline not in ("fused", "streams"):
            raise ValueError(f"params.engine.text_pipeline: 'fused' or 'streams', not {pipeline!r}")
        reserve = int(os.environ.get("TAXI2_TEXT_RESERVE_CUS", self.params.engine.text_reserve_cus))
        copy_mode = int(os.environ.get("TAXI2_TEXT_COPY", self.params.engine.text_copy))
        if pipeline == "fused":  # the fill takes every CU; nothing runs beside it but the host copies
            reserve = 0
            copy_mode = copy_mode or 2
        ncu = eng.num_cus()
        raw = []
        mask = os.environ.get("TAXI2_TEXT_MASK", "1" if self.params.engine.text_cu_mask else "") not in ("", "0")
        eng.set_text_copy(copy_mode if pipeline == "streams" else 0)
        if 0 < reserve < ncu and mask:
            # fill, text, and the block writers' formatters (on the text CUs, their own queue)
            raw = [eng.cu_stream(reserve, ncu - reserve), eng.cu_stream(0, reserve), eng.cu_stream(0, reserve)]
            stream, tstream, wstream = (torch.cuda.ExternalStream(h, device=dev) for h in raw)
        else:
            wstream = None
            stream = torch.cuda.Stream(dev)
            # high priority: a queue of its own beside the fill's (HIP multiplexes streams onto
            # GPU_MAX_HW_QUEUES hardware queues, and two streams sharing one run their kernels in
            # order), and the dispatcher hands freed slots to the text first
            tstream = torch.cuda.Stream(dev, priority=0 if os.environ.get("TAXI2_TEXT_PRIO") == "0" else -1)
        try:
            # the fused pipeline's host copies: a stream of their own (the DMA engine, or the copy
            # kernel, beside the queued fills)
            cstream = torch.cuda.Stream(dev)
            return self._tri_with_pairs_on(seqs, eng, st, D, cidx, clabels, scores, fh, stream, tstream, wstream,
                                           cstream, reserve, pipeline, copy_mode)
        finally:
            eng.set_text_copy(0)
            if raw:
                for s_ in (stream, tstream, wstream):
                    s_.synchronize()
                for h in raw:
                    eng.destroy_stream(h)

    def _tri_with_pairs_on(self, seqs, eng, st, D, cidx, clabels, scores, fh, stream, tstream, wstream, cstream,
                           reserve, pipeline, copy_mode) -> bool:
        """aligned_pairs.txt and the counter metrics from ONE fill per unordered pair: the triangle
        in row blocks (taxi2_tri_strings_dev: the walkers walk both orientations, as the metric
        kernel does), the (a, b) strings formatted with row a's block, the (b, a) strings compacted
        and kept in HBM until row b's block is written (the text kernel reads each pair's strings
        through a pointer).  Two streams: block b aligns while block b - 1's compaction, text (the
        kernel writes it straight into pinned host memory) and complete rows run on the other; the
        linear / matricial / summary writers take each block's rows in a worker thread.  False
        (nothing written) when TAXI2_PAIRS_RECT is set or the packed aligner does not cover the
        shape -- then _rows_with_pairs aligns every ordered pair once instead; when the kept strings
        outgrow params.engine.keep_bytes, the remaining rows switch to it."""
        import torch

        from .._native import NativeError, pack_strings

        n = len(seqs)
        lens_h = np.array([len(s.seq) for s in seqs], dtype=np.int64)
        if os.environ.get("TAXI2_PAIRS_RECT") or n < 2:
            return False
        keep_limit = int(self.params.engine.keep_bytes)
        kept_bytes = 0
        dev = torch.device("cuda", eng.device)
        cap = 2 * int(lens_h.max()) + 1
        Mc = len(cidx)
        npairs = n * (n - 1) // 2
        ids = pack_strings([s.id for s in seqs])
        # text bytes of row x, bounded above: per pair "idx / idy" + 4 LF + 3 lines of at most
        # len(x) + len(y) columns
        idl = np.diff(ids[1]).astype(np.int64)
        row_text_bound = n * (idl + 8 + 3 * lens_h + 3) + int(idl.sum()) + 3 * int(lens_h.sum())
        total = len(self.params.distances.metrics) * n * n
        launch = int(self.params.engine.launch_pairs or 0)
        slot_budget = max(int(self.params.engine.block_bytes), WALK_BLOCK_BYTES if launch else 0)
        per_pair = 4 * cap + 16 * Mc + 8
        # a triangle block fills each pair once for both orientations: twice launch_pairs of them
        # per launch (fewer launch tails and per-block host steps; the slots still fit slot_budget)
        target = max(1, min(2 * launch, slot_budget // per_pair) if launch else slot_budget // per_pair)
        # the counter metrics land in a device copy of D (scattered on the GPU) unless that copy
        # would be large.  Rows [x0, x1) are complete once their block is scattered (the (r, c < r)
        # values come from earlier blocks): they go to a pinned staging buffer behind the block's
        # text, and into D while the GPU aligns the next block
        Dd = None
        if n * n * Mc * 8 <= DEVICE_D_BYTES:
            with torch.cuda.stream(stream):  # filled on `stream`, ahead of the scatters queued there
                Dd = torch.full((n, n, Mc), float("nan"), dtype=torch.float64, device=dev)
        # the row blocks: rows [x0, x1) hold about `target` triangle pairs, at most 2 * target ordered
        # pairs of text.  Known up front, so that every per-block buffer is allocated once at its
        # largest size: an allocation inside the loop (a pinned buffer, a device segment of the
        # caching allocator) can synchronise the device and serialise the two streams
        blocks = []
        x0 = 0
        while x0 < n:
            x1, cnt = x0, 0
            while x1 < n and (x1 == x0 or (cnt + (n - 1 - x1) <= target and (x1 + 1 - x0) * n <= 2 * target)):
                cnt += n - 1 - x1
                x1 += 1
            blocks.append((x0, x1, cnt))
            x0 = x1
        rows_max = max(b[1] - b[0] for b in blocks)
        fused = pipeline == "fused"
        if fused:
            # kept (b, a) storage bound per row a: sum over b > a of la + lb columns
            suf = np.concatenate([np.cumsum(lens_h[::-1])[::-1], [0]])
            keep_bound = (n - 1 - np.arange(n)) * lens_h + suf[1:]
            ids_d = torch.as_tensor(ids[0].copy(), device=dev)
            ioffs_d = torch.as_tensor(ids[1], device=dev)
            nch = -(-n // 256)
            tb_max = max(int(row_text_bound[b[0]:b[1]].sum()) for b in blocks) + 16
            # PIPE_DEPTH + 1 text buffers: block k + PIPE_DEPTH + 1 is launched after post(k) has
            # moved block k's text out
            tslots = [dict(text=torch.empty(tb_max, dtype=torch.uint8, device=dev),
                           total=torch.zeros(2, dtype=torch.int64, device=dev),
                           scratch=torch.empty(2 * rows_max * nch, dtype=torch.int64, device=dev))
                      for _ in range(PIPE_DEPTH + 1)]
            b_index = [0]
            htot = torch.zeros(2, dtype=torch.int64, pin_memory=True)
            pins = []
        stage = [None, None, None]  # pinned buffer, its event, the rows (x0, x1) it holds
        if Dd is not None:
            stage[0] = torch.empty((rows_max, n, Mc), dtype=torch.float64, pin_memory=True)

        def rows_out(x0: int, x1: int) -> None:  # queue rows [x0, x1) of Dd to the staging buffer
            if Dd is None or x1 <= x0:
                return
            with torch.cuda.stream(tstream):  # after the block's event (post() waits on it)
                stage[0][: x1 - x0].copy_(Dd[x0:x1], non_blocking=True)
                stage[1] = torch.cuda.Event()
                stage[1].record(tstream)
            stage[2] = (x0, x1)

        def rows_in() -> None:  # the staged rows into D (waits for their copy only)
            if stage[2] is None:
                return
            x0, x1 = stage[2]
            stage[1].synchronize()
            D[x0:x1, :, cidx] = stage[0][: x1 - x0].numpy()
            stage[2] = None

        # Two streams: blocks k + 1 .. k + PIPE_DEPTH align on `stream` while block k's post-processing
        # -- compaction of its kept (b, a) strings, the text kernel (straight into pinned host
        # memory) and the file write, the staging of its complete rows -- runs on `tstream` after
        # block k's event.  Tensors of a block are
        # record_stream()'d on tstream before they are dropped, so the caching allocator never hands
        # their memory to the next block while the text still reads it.
        with torch.cuda.stream(stream):
            lens = torch.as_tensor(lens_h, device=dev)
            # self alignments (x, x) for the diagonal pairs' text
            t_self = perf_counter()
            strings = self_strings(eng, st, seqs, np.arange(n), scores)
            sa = [a.encode("latin-1") for a, _ in strings]
            sb = [b.encode("latin-1") for _, b in strings]
            slen_self = torch.as_tensor(np.array([len(a) for a in sa], dtype=np.int32), device=dev)
            soff = np.zeros(n, dtype=np.int64)
            soff[1:] = np.cumsum([len(a) for a in sa])[:-1]
            self_x = torch.as_tensor(np.frombuffer(b"".join(sa) + b"\0", dtype=np.uint8).copy(), device=dev)
            self_y = torch.as_tensor(np.frombuffer(b"".join(sb) + b"\0", dtype=np.uint8).copy(), device=dev)
            soff_d = torch.as_tensor(soff, device=dev)
            px_self = self_x.data_ptr() + soff_d
            py_self = self_y.data_ptr() + soff_d
            if isinstance(self.timings, dict):
                self.timings["walk_self_s"] = perf_counter() - t_self
            # (b, a) strings of every pair, kept until row b: pointers per triangle pair
            kpx = torch.zeros(npairs, dtype=torch.int64, device=dev)
            kpy = torch.zeros(npairs, dtype=torch.int64, device=dev)
            klen = torch.zeros(npairs, dtype=torch.int32, device=dev)
        tstream.wait_stream(stream)  # the tables above
        kept = []  # the arena's chunks: every block's kept strings are carved from the newest one
        kept_b = [0]
        arena = [None, 0]  # current chunk, its next free byte

        def carve(nbytes: int, cnt: int, k_end: int):
            """nbytes of kept-string storage (stream-ordered on tstream).  A new chunk holds what the
            rest of the triangle will keep at this block's bytes per pair (one or two allocations per
            task instead of one per block), bounded by the keep budget."""
            if arena[0] is None or arena[1] + nbytes > arena[0].numel():
                left = npairs - k_end
                est = int(1.05 * nbytes / max(1, cnt) * left) + nbytes
                size = max(nbytes, min(est, max(nbytes, keep_limit - kept_b[0])), 1)
                arena[0] = torch.empty(size, dtype=torch.uint8, device=dev)
                arena[1] = 0
                kept.append(arena[0])
            t = arena[0][arena[1]:arena[1] + nbytes]
            arena[1] += (nbytes + 255) // 256 * 256
            return t
        # linear.tsv, the matricial files, summary.tsv and the subset statistics per row block, while
        # the next blocks align and their aligned_pairs.txt text is written: the writers' own engine
        # context (formatting on its own stream, its own lock) in a worker thread, fed each block's
        # adjusted rows (x100, diagonal rule) once they are complete
        sink = writers = None
        futs = []
        if Dd is not None and not os.environ.get("TAXI2_NO_BLOCK_WRITERS") and n > 1:
            from concurrent.futures import ThreadPoolExecutor

            from .._native import Engine

            sink = _BlockWriters(self, seqs, Engine(eng.device), files=True, walk=False, pairs=False)
            sink.rmin_k = None  # (row minima: the streamed path's extra, not the dense path's)
            sink._wstream = wstream  # None: the writers make their own
            sink.diag = self._diag_info(seqs, eng, st, True, scores, [str(m) for m in self.params.distances.metrics])
            writers = ThreadPoolExecutor(1, thread_name_prefix="taxi2-writers")
            scale = 100.0 if self.params.format.percentage_multiply else 1.0
            # three block buffers: a writer reads block k's while block k + 1 is being written and
            # block k + 2's is filled (at most two blocks queued for the thread)
            with torch.cuda.stream(tstream):
                Abuf = [torch.empty((rows_max, n, Mc), dtype=torch.float64, device=dev) for _ in range(3)]
            nblk = [0]

        # `reserve`: CUs' worth of workgroup slots the fill leaves free, so that the previous block's
        # text kernel runs beside it instead of after it (round 5, unmasked streams, N = 5 000:
        # 0 -> 4.9 s, 16 -> 4.2 s, 32 -> 3.6 s, 48 -> 3.6 s, profiles/r5/task_reserve/)
        fill_ev = []  # (start, end) events of every block's fill: the fills' GPU time for task.timings

        def launch(x0: int, x1: int, cnt: int):
            """Block rows [x0, x1) (cnt triangle pairs) on `stream`: the fill (metrics + both
            orientations' strings) and the metrics' scatter into Dd; returns the block record."""
            k0 = x0 * (2 * n - x0 - 1) // 2
            with torch.cuda.stream(stream):
                d = torch.empty((cnt, 2, Mc), dtype=torch.float64, device=dev)
                sx = torch.empty((cnt, 2, cap), dtype=torch.uint8, device=dev)
                sy = torch.empty((cnt, 2, cap), dtype=torch.uint8, device=dev)
                sl = torch.empty((cnt, 2), dtype=torch.int32, device=dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                eng.tri_strings_dev(st, k0, cnt, clabels, d.data_ptr(), cap, sx.data_ptr(), sy.data_ptr(),
                                    sl.data_ptr(), scores, stream.cuda_stream, reserve_cus=reserve)
                e1.record(stream)
                fill_ev.append((e0, e1))
                # pair (a, b) of the block: a in [x0, x1), b > a
                rows = torch.arange(x0, x1, device=dev)
                per = n - 1 - rows
                # (output_size: repeat_interleave would otherwise read the total back -- a host sync
                # behind this block's fill, which kept block k's text from running beside it)
                ra = torch.repeat_interleave(rows, per, output_size=cnt)
                first = torch.cumsum(per, 0) - per
                rb = ra + 1 + torch.arange(cnt, device=dev) - torch.repeat_interleave(first, per, output_size=cnt)
                if Dd is not None:
                    Dd[ra, rb] = d[:, 0, :]
                    Dd[rb, ra] = d[:, 1, :]
                ev = torch.cuda.Event()
                ev.record(stream)
                blk = dict(x0=x0, x1=x1, k0=k0, cnt=cnt, d=d, sx=sx, sy=sy, sl=sl, ra=ra, rb=rb, ev=ev)
                if fused:
                    text_on_fill_stream(blk)
            return blk

        def text_on_fill_stream(b) -> None:
            """Fused pipeline: block b's compaction of its kept (b, a) strings and its whole
            aligned_pairs.txt text (taxi2_format_pairs_ptr_async: lengths, offsets and text on the
            device, no host synchronisation) queued on the fill stream right behind its fill, so they
            run on the whole chip between two fills (~1 ms of text kernel per GB) instead of waiting
            for CU slots beside a persistent fill; the text lands in one of NT device buffers and
            post() moves it to the host beside the next fills (DMA engine or copy kernel)."""
            x0, x1, k0, cnt = b["x0"], b["x1"], b["k0"], b["cnt"]
            end = L1 = off = None
            if cnt:
                sx, sy, sl, ra, rb = b["sx"], b["sy"], b["sl"], b["ra"], b["rb"]
                end = (lens[ra] + lens[rb]).to(torch.int64)
                L1 = sl[:, 1].to(torch.int64)
                off = torch.cumsum(L1, 0) - L1
                # kept storage by the host bound (an alignment has at most la + lb columns): no
                # read-back of the exact total behind the fill
                nb = int(keep_bound[x0:x1].sum())
                kxy = carve(2 * max(1, nb), cnt, k0 + cnt)
                kx, ky = kxy[:max(1, nb)], kxy[max(1, nb):]
                eng.pack_slots_dev(sx.data_ptr(), sy.data_ptr(), sl.data_ptr(), cap, 2, 1, end.data_ptr(),
                                   off.data_ptr(), cnt, kx.data_ptr(), ky.data_ptr(), stream.cuda_stream)
                kpx[k0:k0 + cnt] = kx.data_ptr() + off
                kpy[k0:k0 + cnt] = ky.data_ptr() + off
                klen[k0:k0 + cnt] = sl[:, 1]
                kept_b[0] += 2 * nb
                px, py, ln = pointers(x0, x1, k0, cnt, sx, sy, sl, end)
            else:
                px, py, ln = pointers(x0, x1, k0, 0)
            slot = tslots[b_index[0] % len(tslots)]
            b_index[0] += 1
            eng.format_pairs_ptr_async(x1 - x0, n, px.data_ptr(), py.data_ptr(), ln.data_ptr(), ids_d.data_ptr(),
                                       ioffs_d.data_ptr() + 8 * x0, ids_d.data_ptr(), ioffs_d.data_ptr(),
                                       first=x0 == 0, text_ptr=slot["text"].data_ptr(), cap=slot["text"].numel(),
                                       total_ptr=slot["total"].data_ptr(), scratch_ptr=slot["scratch"].data_ptr(),
                                       stream=stream.cuda_stream)
            tev = torch.cuda.Event()
            tev.record(stream)
            b.update(tslot=slot, tev=tev, keep=(end, L1, off, px, py, ln))

        def ensure_pins() -> None:
            if not pins:
                # (a multiple of 16: every piece's source stays 16-aligned for the copy kernel)
                psz = (min(max(TEXT_CALL_BYTES, 1 << 20), int(row_text_bound.sum()) + 16) + 15) // 16 * 16
                pins.extend(torch.empty(psz, dtype=torch.uint8, pin_memory=True) for _ in range(2))

        def text_to_host(b) -> None:
            """Block b's text from its device buffer to the file: its length read back on the copy
            stream once the text kernel is done, then <= TEXT_CALL_BYTES pieces through two pinned
            buffers (piece j's transfer runs while piece j - 1 is written)."""
            slot = b["tslot"]
            with torch.cuda.stream(cstream):
                cstream.wait_event(b["tev"])
                htot.copy_(slot["total"], non_blocking=True)
                cstream.synchronize()
                total_b, fit = int(htot[0]), int(htot[1])
                if not fit:
                    raise NativeError(f"aligned_pairs text of rows {b['x0']}-{b['x1']} outgrew its bound")
                if not pins:  # (a keep-budget switch before the pipeline's setup)
                    ensure_pins()
                prev = None
                piece = pins[0].numel()
                for j, o in enumerate(range(0, total_b, piece)):
                    nbj = min(piece, total_b - o)
                    buf = pins[j % 2]
                    if copy_mode == 2:
                        eng.copy_text_dev(slot["text"].data_ptr() + o, buf.data_ptr(), nbj, cstream.cuda_stream)
                    else:
                        buf[:nbj].copy_(slot["text"][o:o + nbj], non_blocking=True)
                    evj = torch.cuda.Event()
                    evj.record(cstream)
                    if prev is not None:
                        prev[0].synchronize()
                        fh.write(memoryview(prev[1].numpy()[:prev[2]]))
                    prev = (evj, buf, nbj)
                if prev is not None:
                    prev[0].synchronize()
                    fh.write(memoryview(prev[1].numpy()[:prev[2]]))

        prof = {} if os.environ.get("TAXI2_TASK_PROFILE") else None

        def pointers(x0, x1, k0, cnt, sx=None, sy=None, sl=None, end=None):
            """Per-pair string pointers and lengths of the text of rows [x0, x1) x every y: (x, y > x)
            from this block's slot 0, (x, y < x) from the kept (y, x) strings -- x's aligned string
            is the pair's b side (sy) -- and (x, x) from the self alignments (on tstream)."""
            xs_ = torch.arange(x0, x1, device=dev)[:, None]
            ys_ = torch.arange(n, device=dev)[None, :]
            up = ys_ > xs_
            lo = ys_ < xs_
            pu = xs_ * (2 * n - xs_ - 1) // 2 + (ys_ - xs_ - 1)   # pair (x, y) for y > x
            pl = ys_ * (2 * n - ys_ - 1) // 2 + (xs_ - ys_ - 1)   # pair (y, x) for y < x
            px = torch.where(lo, kpy[pl.clamp(0, npairs - 1)], px_self[xs_.expand(-1, n)])
            py = torch.where(lo, kpx[pl.clamp(0, npairs - 1)], py_self[xs_.expand(-1, n)])
            ln = torch.where(lo, klen[pl.clamp(0, npairs - 1)], slen_self[xs_.expand(-1, n)])
            if cnt:
                q = (pu - k0).clamp(0, max(0, cnt - 1))
                L0 = sl[:, 0].to(torch.int64)
                start0 = q * 2 * cap + end[q] - L0[q]
                px = torch.where(up, sx.data_ptr() + start0, px)
                py = torch.where(up, sy.data_ptr() + start0, py)
                ln = torch.where(up, sl[:, 0][q], ln)
            return px.contiguous(), py.contiguous(), ln.to(torch.int32).contiguous()

        def post(b) -> None:
            """Block b's compaction, text and rows on tstream (after its fill)."""
            x0, x1, k0, cnt = b["x0"], b["x1"], b["k0"], b["cnt"]
            t0 = perf_counter()
            pt = {}  # TAXI2_TASK_PROFILE: host time per step of post()
            tl = [t0]

            def mark(name):
                if prof is not None:
                    t = perf_counter()
                    pt[name] = t - tl[0]
                    tl[0] = t

            with torch.cuda.stream(tstream):
                if fused:
                    if cnt:
                        tstream.wait_event(b["ev"])
                        if Dd is None:
                            b["d"].record_stream(tstream)
                            dd = b["d"].cpu().numpy()
                            a_h, b_h = b["ra"].cpu().numpy(), b["rb"].cpu().numpy()
                            for q, kk in enumerate(cidx):
                                D[a_h, b_h, kk] = dd[:, 0, q]
                                D[b_h, a_h, kk] = dd[:, 1, q]
                    mark("wait")
                    text_to_host(b)
                    mark("text")
                elif cnt:
                    tstream.wait_event(b["ev"])
                    for key in ("d", "sx", "sy", "sl", "ra", "rb"):
                        b[key].record_stream(tstream)
                    sx, sy, sl, ra, rb = b["sx"], b["sy"], b["sl"], b["ra"], b["rb"]
                    if Dd is None:
                        dd = b["d"].cpu().numpy()
                        a_h, b_h = ra.cpu().numpy(), rb.cpu().numpy()
                        for q, kk in enumerate(cidx):
                            D[a_h, b_h, kk] = dd[:, 0, q]
                            D[b_h, a_h, kk] = dd[:, 1, q]
                    end = (lens[ra] + lens[rb]).to(torch.int64)
                    # keep the (b, a) orientation compacted (taxi2_pack_slots_dev: each slot's
                    # right-aligned bytes to a running offset)
                    L1 = sl[:, 1].to(torch.int64)
                    off = torch.cumsum(L1, 0) - L1
                    tot = int(L1.sum().item())  # waits for tstream only (this block's fill is done)
                    mark("wait")
                    kxy = carve(2 * max(1, tot), cnt, k0 + cnt)
                    kx, ky = kxy[:max(1, tot)], kxy[max(1, tot):]
                    eng.pack_slots_dev(sx.data_ptr(), sy.data_ptr(), sl.data_ptr(), cap, 2, 1, end.data_ptr(),
                                       off.data_ptr(), cnt, kx.data_ptr(), ky.data_ptr(), tstream.cuda_stream)
                    kpx[k0:k0 + cnt] = kx.data_ptr() + off
                    kpy[k0:k0 + cnt] = ky.data_ptr() + off
                    klen[k0:k0 + cnt] = sl[:, 1]
                    kept_b[0] += 2 * tot
                if not fused:
                    mark("pack")
                    px, py, ln = pointers(x0, x1, k0, cnt, sx, sy, sl, end) if cnt else pointers(x0, x1, k0, 0)
                    mark("pointers")
                # the text in row runs of at most TEXT_CALL_BYTES (an upper bound from the lengths):
                # the pinned buffer the kernel writes into stays ~1 GB, allocated once -- a block's
                # whole text (~4 GB at N = 5 000) took ~1 s to pin, twice as the buffer grew
                r0 = x0
                while r0 < x1 and not fused:
                    r1 = r0 + 1
                    tot_b = row_text_bound[r0]
                    while r1 < x1 and tot_b + row_text_bound[r1] <= TEXT_CALL_BYTES:
                        tot_b += row_text_bound[r1]
                        r1 += 1
                    o = (r0 - x0) * n
                    fh.write(eng.format_pairs_ptr_dev(r1 - r0, n, px.data_ptr() + 8 * o, py.data_ptr() + 8 * o,
                                                      ln.data_ptr() + 4 * o, (ids[0], ids[1][r0:r1 + 1]), ids,
                                                      first=r0 == 0, stream=tstream.cuda_stream))
                    r0 = r1
                if not fused:
                    mark("text")
                rows_in()  # the previous block's staged rows into D
                rows_out(x0, x1)
                mark("rows")
                if sink is not None:  # rows [x0, x1) are complete: adjusted on the GPU, text in the thread
                    while len(futs) >= 2:  # at most two blocks queued for the thread
                        futs.pop(0).result()
                    A = Abuf[nblk[0] % 3][: x1 - x0]
                    nblk[0] += 1
                    if scale != 1.0:
                        torch.mul(Dd[x0:x1], scale, out=A)
                    else:
                        A.copy_(Dd[x0:x1])
                    sink.diagonal(x0, x1, A, scale)
                    sink.aggregate(x0, x1, A)
                    ready = torch.cuda.Event()
                    ready.record(tstream)
                    # the writers format the block where it is (taxi2_format_rows_dev): no D2H of the
                    # values and no H2D of them again per file
                    futs.append(writers.submit(sink.write_text_dev, x0, x1, A, ready))
                    mark("writers")
            if prof is not None:
                print(f"taxi2 task block {x0}-{x1}: " + " ".join(f"{k} {v * 1e3:.1f}" for k, v in pt.items()),
                      file=sys.stderr)
            if isinstance(self.timings, dict):
                self.timings["pairs_text_s"] = self.timings.get("pairs_text_s", 0.0) + perf_counter() - t0
            report(self.progress_handler, "distance.x.id", min(total, len(self.params.distances.metrics) * n * x1),
                   total)

        # blocks launched and not yet posted: the fills run PIPE_DEPTH blocks ahead of the text, so
        # the fill stream never waits for the host to finish a block's text before its next launch
        from collections import deque

        pending = deque()
        first = True
        for x0, x1, cnt in blocks:
            try:
                blk = launch(x0, x1, cnt) if cnt else dict(x0=x0, x1=x1, k0=0, cnt=0)
                if fused and not cnt:  # a block of the last row alone: its text still needs queueing
                    with torch.cuda.stream(stream):
                        text_on_fill_stream(blk)
            except NativeError as e:
                if x0 == 0 and "walker strings need" in str(e):
                    return False
                raise
            pending.append(blk)
            if first and (len(pending) == 2 or x1 >= n):
                # while the first two blocks align: the text calls' pinned buffer, and the kept-string
                # arena at its estimated size (both orientations' strings of every pair below the
                # diagonal: 2 x 1.04 x the longer sequence of each pair; a short estimate only means
                # a second chunk later)
                first = False
                tp = [perf_counter()]
                if fused:  # two pinned pieces for text_to_host (the arena: carve() on block 0)
                    ensure_pins()
                else:
                    eng._pinned_view(min(TEXT_CALL_BYTES, int(row_text_bound.sum())))
                tp.append(perf_counter())
                ls = np.sort(lens_h)
                est = int(2.08 * float(np.dot(ls, np.arange(n, dtype=np.float64)))) + (1 << 20)
                with torch.cuda.stream(tstream):
                    if not fused:
                        arena[0] = torch.empty(max(1, min(est, keep_limit)), dtype=torch.uint8, device=dev)
                    tp.append(perf_counter())
                    # the first use of each torch kernel of post() loads its code object (~0.2 s in
                    # all): a one-row dummy block here, while the GPU aligns
                    z8, z32 = torch.zeros((1, 2, cap), dtype=torch.uint8, device=dev), torch.zeros(
                        (1, 2), dtype=torch.int32, device=dev)
                    pointers(0, 1, 0, 1, z8, z8, z32, torch.zeros(1, dtype=torch.int64, device=dev))
                tp.append(perf_counter())
                if not fused:
                    arena[1] = 0
                    kept.append(arena[0])
                if prof is not None:
                    print("taxi2 task setup: pinned %.1f arena %.1f warm %.1f ms" % tuple(
                        1e3 * (tp[i + 1] - tp[i]) for i in range(3)), file=sys.stderr)
            if len(pending) > PIPE_DEPTH:
                post(pending.popleft())  # block k's text while blocks k + 1 .. k + PIPE_DEPTH align
            if x1 < n and kept_b[0] > keep_limit:
                # the kept strings outgrew their budget: the remaining rows align every ordered pair
                # once (row blocks of the rect path), nothing kept
                while pending:
                    post(pending.popleft())
                rows_in()
                tstream.synchronize()
                stream.synchronize()
                del kept, kpx, kpy, klen, Dd
                if sink is not None:  # the end-of-task writers redo every file from the full matrix
                    for f in futs:
                        f.result()
                    writers.shutdown()
                    sink.abandon()
                return self._rows_with_pairs(seqs, eng, st, D, cidx, clabels, scores, fh, x_start=x1)
        while pending:
            post(pending.popleft())
        rows_in()
        tstream.synchronize()
        stream.synchronize()
        del kept
        if isinstance(self.timings, dict):  # the fills' own GPU time (they overlap the text)
            self.timings["fill_gpu_s"] = sum(a.elapsed_time(b) for a, b in fill_ev) / 1e3
        if sink is not None:
            t0 = perf_counter()
            for f in futs:
                f.result()
            writers.shutdown()
            sink.close()
            self._written_by_blocks = True
            if isinstance(self.timings, dict):
                self.timings["writers_drain_s"] = perf_counter() - t0
        return True

    def _rows_with_pairs(self, seqs, eng, st, D, cidx, clabels, scores, fh, x_start: int = 0) -> bool:
        """versus_all.py:746-750 as the reference runs it: each ORDERED pair aligned once, its aligned
        strings fed to both the metrics and aligned_pairs.txt.  Row blocks [x0, x1) x [0, N) on the
        packed aligner with string output (taxi2_rect_strings_dev), the text formatted on the GPU
        (taxi2_format_pairs_dev) and written in x-major order.  False (nothing written) when that
        kernel does not cover the shape (linear scores, past 2 048 bp, scores outside int16)."""
        import torch

        from .._native import NativeError, pack_strings

        n = len(seqs)
        cap = 2 * max(len(s.seq) for s in seqs) + 1
        B = walk_block_rows(n, 2 * cap + 8 * len(cidx) + 4, int(self.params.engine.block_bytes),
                            int(self.params.engine.launch_pairs or 0))
        ids = pack_strings([s.id for s in seqs])
        dev = torch.device("cuda", eng.device)
        stream = torch.cuda.Stream(dev)
        total = len(self.params.distances.metrics) * n * n
        with torch.cuda.stream(stream):
            for x0 in range(x_start, n, B):
                x1 = min(n, x0 + B)
                c = (x1 - x0) * n
                d = torch.empty((c, len(cidx)), dtype=torch.float64, device=dev)
                sx = torch.empty(c * cap, dtype=torch.uint8, device=dev)
                sy = torch.empty(c * cap, dtype=torch.uint8, device=dev)
                sl = torch.empty(c, dtype=torch.int32, device=dev)
                try:
                    eng.rect_strings_dev(st, st, x0, x1, clabels, d.data_ptr(), cap, sx.data_ptr(), sy.data_ptr(),
                                         sl.data_ptr(), scores, stream.cuda_stream)
                except NativeError as e:
                    if x0 == 0 and "walker strings need" in str(e):
                        return False
                    raise
                stream.synchronize()  # the alignment kernel counts as compute, not text
                t0 = perf_counter()
                fh.write(eng.format_pairs_dev(st, st, x0, x1, cap, sx.data_ptr(), sy.data_ptr(), sl.data_ptr(),
                                              (ids[0], ids[1][x0 : x1 + 1]), ids, first=x0 == 0,
                                              stream=stream.cuda_stream))
                if isinstance(self.timings, dict):  # format + D2H + file write (the kernel was waited for)
                    self.timings["pairs_text_s"] = self.timings.get("pairs_text_s", 0.0) + perf_counter() - t0
                D[x0:x1, :, cidx] = d.cpu().numpy().reshape(x1 - x0, n, len(cidx))
                report(self.progress_handler, "distance.x.id", min(total, len(self.params.distances.metrics) * n * x1),
                       total)
        return True

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
            for row in aligner.align_product_rows(seqs, seqs):  # x-major like fromProduct
                for pair in row:
                    fh.write(pair)

    def write_summary(self, seqs: list, A: np.ndarray):
        from .subsets import write_summary

        if not self.params.engine.write_summary:
            return

        write_summary(self.paths.summary, seqs, A, self.params.distances.metrics, self.input.genera,
                      self.input.species, self.params.format.float, self.params.format.missing,
                      self._engine() if seqs else None)

    def write_subsets(self, seqs: list, A: np.ndarray):
        from .subsets import aggregate, write_subset_statistics

        ids = [s.id for s in seqs]
        self.subset_stats = {}
        for partition, name in ((self.input.genera, "genera"), (self.input.species, "species")):
            if partition:
                st = self.subset_stats[name] = aggregate(A, ids, partition)
                write_subset_statistics(self.paths.subsets / name, st, self.params.distances.metrics,
                                        self.params.format.float, self.params.format.stats_template,
                                        eng=self._engine())

    # ------------------------------------------------------------------ streamed driver
    def _streaming(self, seqs: list) -> bool:
        """Row-block streaming (taxi2_amd/streaming.py) instead of the dense (N, N, M) matrix."""
        n, M = len(seqs), len(self.params.distances.metrics)
        want = self.params.engine.stream
        if want is None:  # multi-rank runs too: small ones gather the dense matrix (sharding.py)
            want = n * n * M * 8 > self.params.engine.dense_limit
        return bool(want) and n > 0

    def _start_streaming(self, seqs: list) -> None:
        """versus_all.py:732-773 with bounded memory: every rank computes its triangle rows into a
        TriangleStore (packed counters, + NCD), then the ordered product is assembled on rank 0 one
        row block at a time (x-major) and every writer / aggregator consumes the block."""
        import torch

        from ..sharding import world_info
        from ..streaming import TriangleStore

        dist_on, rank = world_info()
        world = 1
        group_backend = None
        if dist_on:
            import torch.distributed as dist

            world = dist.get_world_size()
            group_backend = dist.get_backend()
        labels = [str(m) for m in self.params.distances.metrics]
        M = len(labels)
        cidx = [k for k, lab in enumerate(labels) if lab != "ncd"]
        nidx = [k for k, lab in enumerate(labels) if lab == "ncd"]
        clabels = [labels[k] for k in cidx]
        align = bool(self.params.pairs.align)
        scores = Scores(**(self.params.pairs.scores or {})).as_tuple()
        n = len(seqs)
        total = M * n * n
        if nidx:
            check_ncd_strings(s.seq for s in seqs)
        eng = self._engine()
        cuda = torch.device("cuda", eng.device)
        store_dev = cuda if group_backend in (None, "nccl") else torch.device("cpu")
        t_up = perf_counter()
        st = eng.upload([s.seq for s in seqs], align=align)
        self._upload_s = perf_counter() - t_up
        # one real stream for the torch ops and the engine's *_dev calls of this path (the legacy
        # default stream has handle 0, which the engine would read as "its own stream")
        stream = torch.cuda.Stream(cuda)
        with torch.cuda.stream(stream):
            walk = (align and self.params.pairs.write and not nidx and walk_strings_ok(scores, seqs)
                    and not os.environ.get("TAXI2_NO_WALK_STRINGS"))
            if (not align and not nidx) or walk:
                self._stream_rows(seqs, eng, st, stream, scores, labels, world, rank, group_backend, walk)
                return
            store = TriangleStore(n, world, rank, device=store_dev)
            self._stream_blocks(seqs, eng, st, store, stream, align, scores, labels, cidx, nidx, clabels,
                                world, rank, total)

    def _diag_info(self, seqs, eng, st, align, scores, labels):
        """Inputs of the diagonal rule (versus_all.py:549): groups of identical full tuples, and when
        aligning each group's first alignment with itself (strings) and its values -- a sequence
        whose self-alignment is not the identity (non-default scores) keeps its own values."""
        dup = full_tuple_groups(seqs)
        if not align:
            return dup, None, None
        cidx = [k for k, lab in enumerate(labels) if lab != "ncd"]
        nidx = [k for k, lab in enumerate(labels) if lab == "ncd"]
        reps = np.array([g[0] for g in dup], dtype=np.int64)
        strings = self_strings(eng, st, seqs, reps, scores)
        self_vals = np.empty((len(reps), len(labels)))
        if cidx:
            self_vals[:, cidx] = eng.list_pairs(st, st, reps, reps, [labels[k] for k in cidx], scores)[:, 0, :]
        if nidx:
            sv = eng.ncd_pairs(st, st, reps, reps, scores, aligned=True, both=False)
            for kk in nidx:
                self_vals[:, kk] = sv
        return dup, self_vals, strings

    def _stream_rows(self, seqs, eng, st, stream, scores, labels, world, rank, backend, walk) -> None:
        """Row-block streamed versusAll.  Pre-aligned (config 5: 200 000 x 1 000 bp, p / jc / k2p):
        every x-major row block [x0, x1) x [0, N) is computed directly by the tiled pre-aligned
        kernel (taxi2_rect_pairs_dev).  That evaluates each unordered pair once per orientation
        instead of once, but a pre-aligned pair costs a few hundred VALU ops: recomputing is far
        cheaper than storing the triangle (16 B per pair, 320 GB at N = 200 000) and gathering it.
        Aligned with aligned_pairs.txt (``walk``): every ordered pair aligned once by the packed
        aligner, whose walkers write the strings the block's text is formatted from
        (taxi2_rect_strings_dev + taxi2_format_pairs_dev) while the same walks give the metrics --
        the reference's own one alignment per ordered pair (versus_all.py:746-750).

        One rank: the blocks in order, each fed to the diagonal rule, the writers and the
        reductions.  Several ranks, reductions only: each rank takes a contiguous row range; the
        row minima are per row (gathered at the end), and the subset statistics -- whose sums must
        follow the reference's x-major order -- are passed rank to rank: rank r accumulates its rows
        into the state it receives from rank r - 1 (the blocks it computed are kept in HBM when they
        fit params.engine.hold_bytes, else recomputed).  With N x N text to write the funnel is the
        host's file stream anyway, and rank 0 computes every block itself."""
        import torch

        from ..sharding import gather_blocks, shard_range
        from ..streaming import block_rows

        p = self.params
        n, M = len(seqs), len(labels)
        text = bool(p.distances.write_linear or p.distances.write_matricial or p.pairs.write or p.engine.write_summary)
        sharded = world > 1 and not text
        if not sharded and rank != 0:
            return
        rows = shard_range(n, world) if sharded else [(0, n)]
        r0, r1 = rows[rank if sharded else 0]
        times = dict(compute_s=0.0, reduce_s=0.0, text_s=0.0, comm_s=0.0)
        timed = bool(p.engine.timings)
        cuda = stream.device

        def tick(key, t0):
            if timed:
                stream.synchronize()
                times[key] += perf_counter() - t0
            return perf_counter()

        t_prep = perf_counter()
        sink = _BlockWriters(self, seqs, eng, files=(rank == 0), walk=walk)
        times["prepare_sink_s"] = perf_counter() - t_prep
        t_d = perf_counter()
        sink.diag = self._diag_info(seqs, eng, st, bool(p.pairs.align), scores, labels)
        times["prepare_diag_s"] = perf_counter() - t_d
        # host-side phases outside the block loop: the set upload, the writers' and aggregators' set-up
        # with the diagonal rule's groups, and the close (subset statistics files, row_minima.tsv)
        times["upload_s"] = getattr(self, "_upload_s", 0.0)
        times["prepare_s"] = perf_counter() - t_prep
        scale = 100.0 if p.format.percentage_multiply else 1.0
        cap = 2 * max((len(s.seq) for s in seqs), default=0) + 1
        B = (walk_block_rows(n, 8 * M + 2 * cap + 4, int(p.engine.block_bytes), int(p.engine.launch_pairs or 0)) if walk
             else block_rows(n, 8 * M, int(p.engine.block_bytes)))
        hold = sharded and (r1 - r0) * n * M * 8 <= int(p.engine.hold_bytes)
        held = []
        total = M * n * n
        if walk:
            from .._native import pack_strings

            ids = pack_strings(sink.ids)
        pairs_text = None

        fused = [None]  # the block's fused row minima (pre-aligned, taxi2_rect_block_dev)
        # Pre-aligned reductions without text: the blocks' columns are stored in the order of the
        # partition with the most subsets (a column view of the set, taxi2_set_permuted), so its
        # aggregation reads each subset as one contiguous run instead of gathering it column by
        # column; the diagonal rule, the row minima and the other partition follow the task's columns
        cols_view = col_nat = None
        big = [agg for _, agg in sink.aggs if agg.ns > 4]
        if not walk and not p.pairs.align and not text and big and not os.environ.get("TAXI2_NO_COLPERM"):
            order = max(big, key=lambda a: a.ns).order.astype(np.int64)
            col_nat = torch.as_tensor(order, device=cuda)
            cols_view = eng.permuted_view(st, col_nat.data_ptr())
            inv = np.empty(n, dtype=np.int64)
            inv[order] = np.arange(n, dtype=np.int64)
            for _, agg in sink.aggs:
                agg.set_storage(inv, col_nat)
            sink.col_map = (order, inv, col_nat)
        times["prepare_s"] = perf_counter() - t_prep  # + the column view

        def block(x0, x1):
            nonlocal pairs_text
            t = perf_counter()
            D = torch.empty((x1 - x0, n, M), dtype=torch.float64, device=cuda)
            if walk:
                c = (x1 - x0) * n
                sx = torch.empty(c * cap, dtype=torch.uint8, device=cuda)
                sy = torch.empty(c * cap, dtype=torch.uint8, device=cuda)
                sl = torch.empty(c, dtype=torch.int32, device=cuda)
                eng.rect_strings_dev(st, st, x0, x1, labels, D.data_ptr(), cap, sx.data_ptr(), sy.data_ptr(),
                                     sl.data_ptr(), scores, stream.cuda_stream)
                t = tick("compute_s", t)
                pairs_text = eng.format_pairs_dev(st, st, x0, x1, cap, sx.data_ptr(), sy.data_ptr(), sl.data_ptr(),
                                                  (ids[0], ids[1][x0 : x1 + 1]), ids, first=x0 == 0,
                                                  stream=stream.cuda_stream)
                del sx, sy, sl
                t = tick("text_s", t)
            elif not p.pairs.align:
                # pre-aligned: x100, the diagonal's NaN and the row minima fused into the tile kernel
                k = sink.rmin_k if sink.rmin_k is not None else -1
                if k >= 0:
                    fused[0] = (torch.empty(x1 - x0, dtype=torch.int64, device=cuda),
                                torch.empty(x1 - x0, dtype=torch.float64, device=cuda))
                eng.rect_block_dev(st, x0, x1, labels, D.data_ptr(), scale, True, k,
                                   fused[0][0].data_ptr() if k >= 0 else None,
                                   fused[0][1].data_ptr() if k >= 0 else None, stream.cuda_stream, cols=cols_view,
                                   col_nat_ptr=col_nat.data_ptr() if col_nat is not None else None)
                sink.diagonal(x0, x1, D, scale, main=False)
                tick("compute_s", t)
                return D
            else:
                eng.rect_pairs_dev(st, st, x0, x1, labels, D.data_ptr(), scores, None, stream.cuda_stream)
            if scale != 1.0:
                D.mul_(scale)
            sink.diagonal(x0, x1, D, scale)
            tick("compute_s", t)
            return D

        # Reductions only on one rank (config 5): block b's reductions (row minima, subset partials --
        # short latency-bound waves) run on a second stream while block b + 1's tile kernel runs;
        # at most two blocks in flight.  The row minima stay on the device until the end.
        overlap = (not walk and not p.pairs.align and not text and not sharded and rank == 0
                   and not os.environ.get("TAXI2_NO_OVERLAP"))
        # one reduction stream per partition (each aggregator with its own scratch): genus and
        # species partials of a block run side by side
        reds = [torch.cuda.Stream(cuda) for _ in range(max(1, len(sink.aggs)))] if overlap else []
        red = reds[0] if overlap else None
        if overlap and len(sink.aggs) > 1:
            for _, agg in sink.aggs:
                agg.use_own_scratch()
        red_done = []  # per block: events of its reductions (one per stream)
        if overlap and sink.rmin_k is not None:
            sink.rmin_dev = (torch.full((n,), -1, dtype=torch.int64, device=cuda),
                             torch.full((n,), float("nan"), dtype=torch.float64, device=cuda))
        t_loop = perf_counter()
        try:
            for x0 in range(r0, r1, B):
                x1 = min(r1, x0 + B)
                fused[0] = None
                if overlap and len(red_done) >= 2:
                    for e in red_done.pop(0):  # block b - 2's D can be reused
                        e.synchronize()
                D = block(x0, x1)
                t = perf_counter()
                if overlap:
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    dones = []
                    for k, rs in enumerate(reds):
                        rs.wait_event(ev)
                        with torch.cuda.stream(rs):
                            D.record_stream(rs)
                            if k == 0:
                                for tt in fused[0] or ():
                                    tt.record_stream(rs)
                                sink.row_minima(x0, x1, D, fused[0])
                            if k < len(sink.aggs):
                                sink.aggs[k][1].add(D, x0, x1)
                            done = torch.cuda.Event()
                            done.record(rs)
                            dones.append(done)
                    red_done.append(dones)
                    del D
                    report(self.progress_handler, "distance.x.id", min(total, M * n * x1), total)
                    continue
                sink.row_minima(x0, x1, D, fused[0])
                if not sharded:
                    sink.aggregate(x0, x1, D)
                t = tick("reduce_s", t)
                if not sharded:
                    sink.write_text(x0, x1, D, pairs_text)
                    tick("text_s", t)
                elif hold:
                    held.append((x0, x1, D))
                del D
                report(self.progress_handler, "distance.x.id", min(total, M * n * x1 * (world if sharded else 1)),
                       total)
            if sharded:
                comm = torch.device("cuda", eng.device) if backend == "nccl" else torch.device("cpu")
                t = perf_counter()
                if sink.aggs:
                    if rank > 0:
                        sink.recv_state(rank - 1, comm)
                    t = tick("comm_s", t)
                    for x0 in range(r0, r1, B):
                        x1 = min(r1, x0 + B)
                        D = held.pop(0)[2] if hold else block(x0, x1)
                        t = perf_counter()
                        sink.aggregate(x0, x1, D)
                        t = tick("reduce_s", t)
                        del D
                    sink.send_state((rank + 1) % world, comm)
                    if rank == 0:
                        sink.recv_state(world - 1, comm)
                    t = tick("comm_s", t)
                if sink.rmin_k is not None:  # the row minima to rank 0, which writes them (a gather)
                    lo, hi = r0, r1
                    loc = np.stack([sink.rmin_idx[lo:hi].astype(np.float64), sink.rmin_d[lo:hi]], axis=1)
                    allr = gather_blocks(loc, [b - a for a, b in rows],
                                         device=comm if backend == "nccl" else None, dst=0)
                    if rank == 0:
                        sink.rmin_idx[:] = allr[:, 0].astype(np.int64)
                        sink.rmin_d[:] = allr[:, 1]
                    tick("comm_s", t)
            if overlap:
                for rs in reds:
                    rs.synchronize()
                stream.synchronize()
                # the loop's time not spent waiting for the tile kernels: reductions not hidden
                times["reduce_s"] = max(0.0, perf_counter() - t_loop - times["compute_s"])
                if sink.rmin_dev is not None:
                    sink.rmin_idx[:] = sink.rmin_dev[0].cpu().numpy()
                    sink.rmin_d[:] = sink.rmin_dev[1].cpu().numpy()
            if rank == 0:
                t_cl = perf_counter()
                sink.close()
                times["finish_s"] = perf_counter() - t_cl
                times["finish_subsets_s"] = sink.subsets_s
        finally:
            if cols_view is not None:
                cols_view.free()  # before its parent set
            st.free()
        self.timings = times

    def _stream_blocks(self, seqs, eng, st, store, stream, align, scores, labels, cidx, nidx, clabels, world,
                       rank, total) -> None:
        import torch

        from .._native import tri_pairs
        from ..streaming import block_rows

        n, M = len(seqs), len(labels)
        cuda = stream.device
        store_dev = store.device
        times = dict(compute_s=0.0, assemble_s=0.0, reduce_text_s=0.0)
        t_c = perf_counter()
        try:
            # ---- 1. this rank's triangle rows
            # packed 16-bit counters (TAXI2_METRIC_COUNTS) up to 32 767 bp; past that, one f64 plane
            # per counter metric (the metrics themselves)
            wide = max((len(s.seq) for s in seqs), default=0) > 32767
            cpl = store.add_plane("counts", torch.int64) if cidx and not wide else None
            mpl = [store.add_plane(f"m{k}", torch.float64) for k in cidx] if cidx and wide else None
            npl = store.add_plane("ncd", torch.float64) if nidx else None
            step = 1 << 22
            for c0 in range(0, store.count, step):
                c = min(step, store.count - c0)
                k = store.k0 + c0
                if cpl is not None:
                    out = torch.empty((c, 2 if align else 1), dtype=torch.float64, device=cuda)
                    eng.all_pairs_dev(st, k, c, ("counts",), out.data_ptr(), scores, None, stream.cuda_stream)
                    v = out.view(torch.int64)
                    cpl[c0 : c0 + c] = (v if align else v.expand(c, 2)).to(store_dev)
                if mpl is not None:
                    out = torch.empty((c, 2 if align else 1, len(cidx)), dtype=torch.float64, device=cuda)
                    eng.all_pairs_dev(st, k, c, clabels, out.data_ptr(), scores, None, stream.cuda_stream)
                    for q, pl in enumerate(mpl):
                        pl[c0 : c0 + c] = out[:, :, q].expand(c, 2).to(store_dev)
                if npl is not None:
                    a, b = tri_pairs(n, k, c)
                    npl[c0 : c0 + c] = torch.from_numpy(eng.ncd_pairs(st, st, a, b, scores, aligned=align, both=True))
                report(self.progress_handler, "distance.x.id", min(total, 2 * M * (k + c) * world), total)
            torch.cuda.synchronize(cuda)
            times["compute_s"] = perf_counter() - t_c
            # ---- 2. diagonal rule inputs (rank 0): identical full tuples -> None, unless the
            # alignment of the sequence with itself is not the identity (non-default scores)
            sink = _BlockWriters(self, seqs, eng) if rank == 0 else None
            if sink is not None:
                sink.diag = self._diag_info(seqs, eng, st, align, scores, labels)
            # ---- 3. row blocks, x-major
            per_entry = 8 * (len(store.planes) + M)
            B = block_rows(n, per_entry, int(self.params.engine.block_bytes))
            timed = bool(self.params.engine.timings)
            for x0 in range(0, n, B):
                x1 = min(n, x0 + B)
                t_a = perf_counter()
                blk = store.assemble(x0, x1)
                if timed:
                    torch.cuda.synchronize(cuda)
                    times["assemble_s"] += perf_counter() - t_a
                if sink is None:
                    continue
                t_r = perf_counter()
                D = torch.empty((x1 - x0, n, M), dtype=torch.float64, device=cuda)
                scale = 100.0 if self.params.format.percentage_multiply else 1.0
                if cidx and "counts" not in blk:  # wide: the metric planes themselves
                    for q, kk in enumerate(cidx):
                        mv = blk[f"m{kk}"].to(cuda)
                        D[:, :, kk] = mv * scale if scale != 1.0 else mv
                elif cidx:
                    cnt = blk["counts"].to(cuda).contiguous()
                    tmp = torch.empty((cnt.numel(), len(cidx)), dtype=torch.float64, device=cuda)
                    eng.counts_metrics_dev(cnt.data_ptr(), cnt.numel(), clabels, tmp.data_ptr(), scale,
                                           stream.cuda_stream)
                    D[:, :, cidx] = tmp.view(x1 - x0, n, len(cidx))
                if nidx:
                    nv = blk["ncd"].to(cuda)
                    for kk in nidx:
                        D[:, :, kk] = nv * scale if scale != 1.0 else nv
                sink.consume(x0, x1, D, scale)
                del D
                if timed:
                    torch.cuda.synchronize(cuda)
                    times["reduce_text_s"] += perf_counter() - t_r
                report(self.progress_handler, "distance.x.id", min(total, M * n * x1), total)
            if sink is not None:
                sink.close()
            self.timings = times
        finally:
            st.free()

    # ------------------------------------------------------------------ driver
    def start(self) -> Results:
        ts = perf_counter()
        self.generate_paths()
        self.check_metrics()
        self._check_scope()
        seqs = list(self.input.sequences)
        if self.params.pairs.align:
            seqs = [s.normalize() for s in seqs]
        if self._streaming(seqs):
            self.distances = None
            self._start_streaming(seqs)
            n = len(seqs)
            total = len(self.params.distances.metrics) * n * n
            report(self.progress_handler, "Finalizing...", total, total)
            return Results(self.work_dir, perf_counter() - ts)
        from ..sharding import world_info

        pairs_fh = None
        if self.params.pairs.write and self.params.pairs.align and seqs and not world_info()[0]:
            create_parents(self.paths.aligned_pairs)
            pairs_fh = open(self.paths.aligned_pairs, "wb")
        self.pairs_walked = False
        self._written_by_blocks = False
        self.timings = times = {"compute_s": 0.0, "pairs_text_s": 0.0}
        t0 = perf_counter()
        try:
            D = self.compute_distances(seqs, pairs_fh)
        finally:
            if pairs_fh is not None:
                pairs_fh.close()
        times["compute_s"] = perf_counter() - t0 - times["pairs_text_s"]
        self.distances = D
        rank0 = True
        try:
            import torch.distributed as dist

            rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
        except Exception:
            pass
        if rank0 and self._written_by_blocks:  # linear / matricial / summary / subsets per row block
            pass
        elif rank0:
            A = self._adjusted(D)
            for name, fn in (("pairs_s", None if self.pairs_walked else self.write_pairs),
                             ("linear_s", lambda s_: self.write_distances_linear(s_, A)),
                             ("matricial_s", lambda s_: self.write_distances_multimatrix(s_, A)),
                             ("summary_s", lambda s_: self.write_summary(s_, A)),
                             ("subsets_s", lambda s_: self.write_subsets(s_, A))):
                t0 = perf_counter()
                if fn is not None:
                    fn(seqs)
                times[name] = perf_counter() - t0
        n = len(seqs)
        total = len(self.params.distances.metrics) * n * n
        report(self.progress_handler, "Finalizing...", total, total)
        return Results(self.work_dir, perf_counter() - ts)


class _BlockWriters:
    """Rank 0's consumers of the streamed row blocks: aligned_pairs.txt, linear.tsv, matricial
    files, summary.tsv (GPU text formatter, unique ids) and the subset aggregators (on the GPU,
    taxi2_subset_aggregate_dev), each fed the rows [x0, x1) in x-major order -- the file contents
    are those of the dense path (tests/test_gpu_streaming.py)."""

    def __init__(self, task: VersusAll, seqs: list, eng, files: bool = True, walk: bool = False,
                 pairs: bool = True):
        import torch

        from .subsets import SubsetAggregatorDev, subset_codes

        self.task, self.seqs, self.eng = task, seqs, eng
        self.files = files  # False: a sharded rank's reductions only (rank 0 writes every file)
        p = task.params
        self.metrics = p.distances.metrics
        self.fmt, self.missing = p.format.float, p.format.missing
        self.dec = fixed_decimals(self.fmt)
        self.ids = [s.id for s in seqs]
        n = len(seqs)
        self.diag = None
        ex0 = list(seqs[0].extras.keys())
        # per-sequence text pieces only when a text writer needs them (N = 200 000: ~0.3 s of Python)
        want_rows = files and bool(p.distances.write_linear or p.distances.write_matricial)
        want_summary = files and bool(p.engine.write_summary)
        self.pre = (["\t".join([s.id, *[v if v is not None else self.missing for v in s.extras.values()]])
                     for s in seqs] if want_rows else None)
        self.lin = self.mats = None
        # duplicate ids: the reference's handlers merge consecutive lines of equal ids, and such a
        # run can span two row blocks -- the handler-shaped writers (kept open across blocks) and
        # the summary's run grouper carry it over
        self.dupids = len(set(self.ids)) != n
        if p.distances.write_linear and files:
            create_parents(task.paths.distances_linear)
            if self.dupids:
                self.lin = DistanceHandler.Linear.WithExtras(task.paths.distances_linear, "w", missing=self.missing,
                                                             formatter=self.fmt)
            else:
                self.lin = open(task.paths.distances_linear, "wb")
                head = ["seqid (query)", *[k + " (query)" for k in ex0], "seqid (reference)",
                        *[k + " (reference)" for k in ex0], *[str(m) for m in self.metrics]]
                self.lin.write(("\t".join(head) + "\n").encode("utf-8"))
        if p.distances.write_matricial and files:
            create_parents(task.paths.distances_matricial)
            self.mats = []
            for metric in self.metrics:
                path = task.paths.distances_matricial / f"{metric}.tsv"
                if self.dupids:
                    self.mats.append(DistanceHandler.Matrix(path, "w", missing=self.missing, formatter=self.fmt))
                    continue
                fh = open(path, "wb")
                fh.write(("\t".join(["", *self.ids]) + "\n").encode("utf-8"))
                self.mats.append(fh)
        # summary.tsv (always)
        genera, species = task.input.genera, task.input.species
        self.genera, self.species = genera, species
        self.suf = None
        if want_summary:
            gx = [genera.get(i, None) for i in self.ids] if genera else None
            sx = [species.get(i, None) for i in self.ids] if species else None
            ext = ["".join("\t" + (v if v is not None else self.missing) for v in s.extras.values()) for s in seqs]
            gs = ["\t" + ((gx[k] if gx else None) or "-") + "\t" + ((sx[k] if sx else None) or "-") for k in range(n)]
            self.suf = [t for pair in zip(ext, gs) for t in pair]
        # subset codes once per partition (summary.tsv and the aggregators)
        pcodes = {name: subset_codes(self.ids, part) for part, name in ((genera, "genera"), (species, "species")) if part}
        gcode = pcodes["genera"][0] if genera else np.zeros(n, np.int32)
        scode = pcodes["species"][0] if species else np.zeros(n, np.int32)
        self.codes = np.stack([gcode, scode], axis=1)
        self.summ = self.summ_runs = None
        if p.engine.write_summary and files:
            from .subsets import SummaryRuns

            create_parents(task.paths.summary)
            if self.dupids:
                self.summ = open(task.paths.summary, "w")
                self.summ_runs = SummaryRuns(self.summ, seqs, self.metrics, genera, species, self.fmt, self.missing)
            else:
                self.summ = open(task.paths.summary, "wb")
                head = ["seqid (query 1)", "seqid (query 2)", *[str(m) for m in self.metrics],
                        *[k + " (query 1)" for k in ex0], *[k + " (query 2)" for k in ex0],
                        "genus (query 1)", "species (query 1)", "genus (query 2)", "species (query 2)",
                        "comparison_type"]
                self.summ.write(("\t".join(head) + "\n").encode("utf-8"))
        self.rmin_k = None
        if p.engine.row_minima is not None:
            labels = [str(m) for m in self.metrics]
            if str(p.engine.row_minima) not in labels:
                raise ValueError(f"row_minima metric {p.engine.row_minima} is not one of {labels}")
            self.rmin_k = labels.index(str(p.engine.row_minima))
            self.rmin_idx = np.full(n, -1, dtype=np.int64)
            self.rmin_d = np.full(n, np.nan)
        self.aggs = [(name, SubsetAggregatorDev(eng, self.ids, part, len(self.metrics), codes=pcodes[name]))
                     for part, name in ((genera, "genera"), (species, "species")) if part]
        self.pairs_fh = None
        self._pair_sets = None
        if p.pairs.write and files and pairs:  # (pairs False: the caller writes aligned_pairs.txt)
            create_parents(task.paths.aligned_pairs)
            if walk:  # text from the metric kernel's walks, handed over per block (write_text)
                self.pairs_fh = open(task.paths.aligned_pairs, "wb")
            else:
                self.pairs_fh = SequencePairHandler.Formatted(task.paths.aligned_pairs, "w")
            self.aligner = (PairwiseAligner.Biopython(p.pairs.scores, engine=eng) if p.pairs.align else None)
        self.walk = walk
        self.torch = torch
        self.col_map = None  # (order, inverse, device order) when the blocks' columns are stored permuted
        self.rmin_dev = None  # (index, value) device arrays of the row minima (overlapped reductions)
        self.subsets_s = 0.0

    def consume(self, x0: int, x1: int, D, scale: float) -> None:
        """D: (x1 - x0, n, M) device tensor of the rows' values, x100 applied, diagonal not yet."""
        self.diagonal(x0, x1, D, scale)
        self.aggregate(x0, x1, D)
        self.row_minima(x0, x1, D)
        self.write_text(x0, x1, D)

    @property
    def has_text(self) -> bool:
        return any(f is not None for f in (self.lin, self.summ, self.pairs_fh)) or bool(self.mats)

    def diagonal(self, x0: int, x1: int, D, scale: float, main: bool = True) -> None:
        """Diagonal rule (versus_all.py:549) on rows [x0, x1): every (x, x) is None (one indexed
        store for the block), then the groups of identical full tuples with more than one member
        (every pair inside is None) and the sequences whose alignment with themselves is not the
        identity (their own values), from an index built once (N = 200 000: no per-row Python)."""
        torch = self.torch
        dup, self_vals, strings = self.diag
        if getattr(self, "_special", None) is None:
            special = []  # (row, group index) of rows whose group needs more than the NaN diagonal
            for gi, g in enumerate(dup):
                if len(g) > 1 or (strings is not None and strings[gi][0] != strings[gi][1]):
                    special.extend((i, gi) for i in g)
            special.sort()
            self._special = special
            self._special_rows = np.array([i for i, _ in special], dtype=np.int64)
        if main:  # (taxi2_rect_block_dev sets the diagonal's NaN itself)
            r = torch.arange(x1 - x0, device=D.device)
            D[r, r + x0] = float("nan")
        lo, hi = np.searchsorted(self._special_rows, [x0, x1])
        inv = self.col_map[1] if self.col_map is not None else None  # task column -> stored column
        for i, gi in self._special[lo:hi]:
            g = dup[gi]
            if strings is not None and strings[gi][0] != strings[gi][1]:
                D[i - x0, i if inv is None else int(inv[i])] = torch.as_tensor(
                    self_vals[gi] * scale if scale != 1.0 else self_vals[gi], device=D.device)
            else:
                cols = np.asarray(g) if inv is None else inv[np.asarray(g)]
                D[i - x0, torch.as_tensor(cols, device=D.device)] = float("nan")

    def aggregate(self, x0: int, x1: int, D) -> None:
        for _, agg in self.aggs:
            agg.add(D, x0, x1)

    def row_minima(self, x0: int, x1: int, D, fused=None) -> None:
        """Each row's first minimum over defined values (-0.0 == 0.0), None skipped.  `fused`: the
        (index, value) device tensors taxi2_rect_block_dev computed with the diagonal's NaN; rows of
        groups the diagonal rule changed afterwards (duplicate full tuples) are redone from D."""
        torch = self.torch
        if self.rmin_k is not None and fused is not None:
            idx, val = fused
            dev = self.rmin_dev is not None  # kept on the device (no host synchronisation per block)
            if dev:
                self.rmin_dev[0][x0:x1].copy_(idx)
                self.rmin_dev[1][x0:x1].copy_(val)
            else:
                self.rmin_idx[x0:x1] = idx.cpu().numpy()
                self.rmin_d[x0:x1] = val.cpu().numpy()
            lo, hi = np.searchsorted(self._special_rows, [x0, x1])
            rows = np.unique(self._special_rows[lo:hi])
            if rows.size:
                rr = torch.as_tensor(rows - x0, device=D.device)
                v = D[rr][:, :, self.rmin_k]
                v = torch.where(torch.isfinite(v), v, torch.full_like(v, float("inf")))
                if self.col_map is not None:  # stored columns permuted: back to the task's order
                    v = v[:, torch.as_tensor(self.col_map[1], device=D.device)]
                d, ix = torch.min(v, dim=1)
                ok = torch.isfinite(d)
                d = torch.gather(v, 1, ix[:, None])[:, 0]  # the first minimum's own value (-0.0 / 0.0)
                ri = torch.where(ok, ix, torch.full_like(ix, -1))
                rv = torch.where(ok, d, torch.full_like(d, float("nan")))
                if dev:
                    rr_abs = torch.as_tensor(rows, device=D.device)
                    self.rmin_dev[0][rr_abs] = ri
                    self.rmin_dev[1][rr_abs] = rv
                else:
                    self.rmin_idx[rows] = ri.cpu().numpy()
                    self.rmin_d[rows] = rv.cpu().numpy()
            return
        if self.rmin_k is not None:  # first minimum over defined values (-0.0 == 0.0), None skipped
            v = D[:, :, self.rmin_k]
            v = torch.where(torch.isfinite(v), v, torch.full_like(v, float("inf")))
            d, idx = torch.min(v, dim=1)
            ok = torch.isfinite(d)
            self.rmin_idx[x0:x1] = torch.where(ok, idx, torch.full_like(idx, -1)).cpu().numpy()
            self.rmin_d[x0:x1] = torch.where(ok, d, torch.full_like(d, float("nan"))).cpu().numpy()

    def send_state(self, dst: int, comm) -> None:
        """The subset aggregators' running state to rank `dst` (the sharded x-major chain)."""
        import torch.distributed as dist

        for _, agg in self.aggs:
            for t in agg.state():
                dist.send(t.to(comm), dst=dst)

    def recv_state(self, src: int, comm) -> None:
        import torch.distributed as dist

        for _, agg in self.aggs:
            for t in agg.state():
                buf = self.torch.empty_like(t, device=comm)
                dist.recv(buf, src=src)
                t.copy_(buf)

    def write_text(self, x0: int, x1: int, D, pairs_text: bytes | None = None) -> None:
        if not self.has_text:  # reductions only: the block never leaves HBM
            return
        self.write_text_host(x0, x1, D.cpu().numpy(), pairs_text)

    def write_text_dev(self, x0: int, x1: int, A, ready) -> None:
        """write_text from the block's adjusted values in HBM (a writer thread's entry): once `ready`
        (an event after their producer) has fired, the device formatters read them in place --
        linear rows, one matricial file per metric (a strided column of the block), summary lines.
        Blocks the formatters cannot take (duplicate ids, aligned pairs here, values too large for
        exact fixed-point text) go through write_text_host."""
        torch = self.torch
        ready.synchronize()
        dec = self.dec
        ok = dec is not None and not self.dupids and self.pairs_fh is None
        if getattr(self, "_wstream", None) is None:
            # the writers' own high-priority stream for the check and the formatters (not the
            # legacy default stream; not a hardware queue shared with the persistent fill, whose
            # kernels would otherwise hold the writers' behind it)
            self._wstream = torch.cuda.Stream(A.device, priority=-1)
        ws = self._wstream.cuda_stream
        if ok and A.numel():
            with torch.cuda.stream(self._wstream):
                big = float(torch.where(torch.isfinite(A), A.abs(), torch.zeros_like(A)).max())
            ok = big * 10.0 ** dec < 2.0 ** 62
        if not ok:
            self.write_text_host(x0, x1, A.cpu().numpy())
            return
        ids = self.ids
        if self.lin is not None:
            write_rows_gpu(self.lin, self.eng, A, self.pre[x0:x1], self.pre, dec, self.missing, stream=ws)
        if self.mats is not None:
            for m, fh in enumerate(self.mats):
                write_rows_gpu(fh, self.eng, A[:, :, m], ids[x0:x1], None, dec, self.missing, stream=ws)
        if self.summ is None:
            return
        from .subsets import SUMMARY_CHUNK_VALUES

        step = max(1, SUMMARY_CHUNK_VALUES // max(1, A.shape[1] * A.shape[2]))
        for r0 in range(0, x1 - x0, step):
            r1 = min(x1 - x0, r0 + step)
            self.summ.write(self.eng.format_summary(
                A[r0:r1], ids[x0 + r0 : x0 + r1], ids, self.suf[2 * (x0 + r0) : 2 * (x0 + r1)], self.suf,
                self.codes[x0 + r0 : x0 + r1], self.codes, has_genera=bool(self.genera),
                has_species=bool(self.species), decimals=dec, missing=self.missing, view=True, stream=ws))

    def write_text_host(self, x0: int, x1: int, A: np.ndarray, pairs_text: bytes | None = None) -> None:
        """write_text on the block's values already on the host (a writer thread's entry)."""
        seqs, ids = self.seqs, self.ids
        if self.walk and self.pairs_fh is not None:
            self.pairs_fh.write(pairs_text)
        elif self.pairs_fh is not None:
            if self.aligner is None:
                for x in seqs[x0:x1]:
                    for y in seqs:
                        self.pairs_fh.write(SequencePair(x, y))
            else:
                if self._pair_sets is None:  # uploaded once for every block
                    self._pair_sets = self.aligner.upload_sets(seqs, seqs)
                for row in self.aligner.align_product_rows(seqs, seqs, range(x0, x1), sets=self._pair_sets):
                    for pair in row:
                        self.pairs_fh.write(pair)
        if self.dupids:
            self._write_text_handlers(x0, x1, A)
            return
        ok = gpu_text_ok(A, self.dec)
        if self.lin is not None:
            if ok:
                write_rows_gpu(self.lin, self.eng, A, self.pre[x0:x1], self.pre, self.dec, self.missing)
            else:
                text = format_values(A, self.fmt, self.missing)
                for i in range(x1 - x0):
                    rows = ["\t".join((self.pre[x0 + i], self.pre[j], *text[i, j])) for j in range(len(seqs))]
                    self.lin.write(("\n".join(rows) + "\n").encode("utf-8"))
        if self.mats is not None:
            for m, fh in enumerate(self.mats):
                Am = np.ascontiguousarray(A[:, :, m])
                if ok:
                    write_rows_gpu(fh, self.eng, Am, ids[x0:x1], None, self.dec, self.missing)
                else:
                    text = format_values(Am, self.fmt, self.missing)
                    for i in range(x1 - x0):
                        fh.write(("\t".join((ids[x0 + i], *text[i])) + "\n").encode("utf-8"))
        if self.summ is None:
            return
        if ok:
            from .subsets import SUMMARY_CHUNK_VALUES

            step = max(1, SUMMARY_CHUNK_VALUES // max(1, A.shape[1] * A.shape[2]))
            for r0 in range(0, x1 - x0, step):
                r1 = min(x1 - x0, r0 + step)
                self.summ.write(self.eng.format_summary(
                    A[r0:r1], ids[x0 + r0 : x0 + r1], ids, self.suf[2 * (x0 + r0) : 2 * (x0 + r1)], self.suf,
                    self.codes[x0 + r0 : x0 + r1], self.codes, has_genera=bool(self.genera),
                    has_species=bool(self.species), decimals=self.dec, missing=self.missing, view=True))
        else:
            from .subsets import summary_lines

            self.summ.write(summary_lines(A, x0, seqs, self.metrics, self.genera, self.species, self.fmt,
                                          self.missing).encode("utf-8"))

    def _write_text_handlers(self, x0: int, x1: int, A) -> None:
        """Duplicate ids: every ordered pair through the reference-shaped handlers (distances.py
        Linear.WithExtras / Matrix: their open line carries over to the next block) and the
        summary's run grouper -- the dense path's writers, fed one block at a time."""
        seqs = self.seqs
        if self.lin is not None or self.mats:
            for r in range(x1 - x0):
                x = seqs[x0 + r]
                for j, y in enumerate(seqs):
                    for m, metric in enumerate(self.metrics):
                        v = A[r, j, m]
                        d = Distance(metric, x, y, float(v) if np.isfinite(v) else None)
                        if self.lin is not None:
                            self.lin.write(d)
                        if self.mats:
                            self.mats[m].write(d)
        if self.summ_runs is not None:
            self.summ_runs.feed(A, x0)

    def abandon(self) -> None:
        """Close the files without finishing them (the caller rewrites every one of them)."""
        for fh in [self.lin, self.summ, *(self.mats or [])]:
            if fh is not None:
                fh.close()
        self.lin = self.summ = self.mats = self.summ_runs = None

    def close(self) -> None:
        from .subsets import write_subset_statistics

        if not self.files:
            return
        if self.summ_runs is not None:
            self.summ_runs.close()

        for fh in [self.lin, self.summ, *(self.mats or [])]:
            if fh is not None:
                fh.close()
        if self.rmin_k is not None:
            self.task.row_minima = (self.rmin_idx, self.rmin_d)
            path = self.task.paths.distances_linear.parent / "row_minima.tsv"
            create_parents(path)
            fmt, missing = self.fmt, self.missing
            from .subsets import _tokens

            # values through the bulk formatter (Python-exact "{:.Nf}"), one join for the file
            fin = np.isfinite(self.rmin_d)
            vals = np.full(len(self.ids), missing, dtype=object)
            if fin.any():
                vals[fin] = _tokens(self.rmin_d[fin], fmt, self.eng)
            ids = self.ids
            close = [ids[j] if j >= 0 else missing for j in self.rmin_idx.tolist()]
            with open(path, "w") as fh:
                fh.write(f"seqid\tclosest\t{self.metrics[self.rmin_k]}\n")
                fh.write("".join(f"{a}\t{b}\t{c}\n" for a, b, c in zip(ids, close, vals.tolist())))
        if self.pairs_fh is not None:
            self.pairs_fh.close()
        if self._pair_sets is not None:
            self._pair_sets[0].free()
            self._pair_sets = None
        p = self.task.params
        self.task.subset_stats = {}
        t_sub = perf_counter()
        for name, agg in self.aggs:
            st = self.task.subset_stats[name] = agg.result()
            write_subset_statistics(self.task.paths.subsets / name, st, self.metrics, p.format.float,
                                    p.format.stats_template, eng=self.eng)
        self.subsets_s = perf_counter() - t_sub
