"""VersusAll's partition-aware outputs (``src/itaxotools/taxi2/tasks/versus_all.py``):

* ``summary.tsv`` -- ``SummaryHandler`` (:278-350) over every ordered pair: ids, the metrics,
  both sides' extras, genus / species of both (``partition.get(id) or "-"``) and the comparison
  type (``SubsetDistance.get_comparison_type``, :255-271).  Written unconditionally by the
  reference (:754-768).  Text on the GPU (``taxi2_format_summary``) when ids are unique (no line
  merging) and the formatter is ``{:.Nf}``; the handler's line grouping in Python otherwise.
* ``subsets/{species,genera}/linear/{pairs,identity}.tsv`` and ``.../matricial/<metric>.tsv`` --
  ``DistanceAggregator`` min / max / mean / count per (subset x, subset y) (:57-96, 605-684):
  accumulated natively in the reference's x-major order (``taxi2_subset_aggregate``), written by
  the Subset*StatisticsHandler rules (:98-236).
"""

from __future__ import annotations

from itertools import groupby
from pathlib import Path
from typing import NamedTuple

import math

import numpy as np

from .common import create_parents, fixed_decimals, gpu_text_ok


class ComparisonType:
    """``plot.py:15-27`` labels, in index order."""

    Unknown = "no info"
    IntraSpecies = "intra-species"
    InterSpecies = "inter-species"
    IntraGenus = "intra-genus"
    InterGenus = "inter-genus"


class SubsetPair(NamedTuple):
    x: str | None
    y: str | None


def comparison_type(genera: SubsetPair | None, species: SubsetPair | None) -> str:
    """``SubsetDistance.get_comparison_type`` (versus_all.py:255-271)."""
    same_g = bool(genera.x == genera.y) if genera else None
    same_s = bool(species.x == species.y) if species else None
    if same_g is False:
        return ComparisonType.InterGenus
    if same_s is True:
        return ComparisonType.IntraSpecies
    if same_s is False:
        return ComparisonType.InterSpecies
    return ComparisonType.IntraGenus if same_g else ComparisonType.Unknown


def subset_codes(ids: list[str], partition) -> tuple[np.ndarray, list]:
    """Per sequence: the code of ``partition.get(id, None)``, codes numbered in first-appearance
    order (= DistanceAggregator's dict order over the x-major product); and the subsets by code."""
    subsets: dict = {}
    code = np.array([subsets.setdefault(partition.get(i, None), len(subsets)) for i in ids], dtype=np.int32)
    return code, list(subsets)


# ----------------------------------------------------------------------------- summary.tsv
SUMMARY_CHUNK_VALUES = 1 << 22  # values per taxi2_format_summary call (rows of N * M values)


def write_summary(path: Path, seqs: list, A: np.ndarray, metrics: list, genera, species, fmt: str, missing: str,
                  eng=None) -> None:
    """``summary.tsv`` for the (N, N, M) adjusted values ``A`` (NaN = None)."""
    create_parents(path)
    n = len(seqs)
    if n == 0:  # no distances: the handler writes nothing (versus_all.py via distances.py:84-88)
        open(path, "w").close()
        return
    ids = [s.id for s in seqs]
    gx = [genera.get(i, None) for i in ids] if genera else None
    sx = [species.get(i, None) for i in ids] if species else None
    head = ["seqid (query 1)", "seqid (query 2)", *[str(m) for m in metrics],
            *[k + " (query 1)" for k in seqs[0].extras], *[k + " (query 2)" for k in seqs[0].extras],
            "genus (query 1)", "species (query 1)", "genus (query 2)", "species (query 2)", "comparison_type"]
    dec = fixed_decimals(fmt)
    if eng is not None and len(set(ids)) == n and gpu_text_ok(A, dec):
        ext = ["".join("\t" + (v if v is not None else missing) for v in s.extras.values()) for s in seqs]
        gs = ["\t" + ((gx[k] if gx else None) or "-") + "\t" + ((sx[k] if sx else None) or "-") for k in range(n)]
        suf = [t for pair in zip(ext, gs) for t in pair]
        gcode = subset_codes(ids, genera)[0] if genera else np.zeros(n, np.int32)
        scode = subset_codes(ids, species)[0] if species else np.zeros(n, np.int32)
        codes = np.stack([gcode, scode], axis=1)
        step = max(1, SUMMARY_CHUNK_VALUES // max(1, n * A.shape[2]))
        with open(path, "wb") as fh:
            fh.write(("\t".join(head) + "\n").encode("utf-8"))
            for r0 in range(0, n, step):
                r1 = min(n, r0 + step)
                fh.write(eng.format_summary(A[r0:r1], ids[r0:r1], ids, suf[2 * r0 : 2 * r1], suf, codes[r0:r1], codes,
                                            has_genera=bool(genera), has_species=bool(species), decimals=dec,
                                            missing=missing, view=True))
        return
    # line grouping of DistanceHandler.Linear (distances.py:96-111): runs of equal (x.id, y.id)
    text = _values_text(A, fmt, missing)

    def lines():
        pairs = ((i, j) for i in range(n) for j in range(n))
        for _, run in groupby(pairs, key=lambda ij: (ids[ij[0]], ids[ij[1]])):
            yield list(run)

    with open(path, "w") as fh:
        first = True
        for run in lines():
            i0, j0 = run[0]
            if first:
                labels = [str(m) for _ in run for m in metrics]
                head[2 : 2 + len(metrics)] = labels
                fh.write("\t".join(head) + "\n")
                first = False
            x, y = seqs[i0], seqs[j0]
            g = SubsetPair(gx[i0], gx[j0]) if gx is not None else None
            s = SubsetPair(sx[i0], sx[j0]) if sx is not None else None
            fh.write("\t".join((
                x.id, y.id, *[t for i, j in run for t in text[i, j]],
                *[v if v is not None else missing for v in x.extras.values()],
                *[v if v is not None else missing for v in y.extras.values()],
                (g.x if g else None) or "-", (s.x if s else None) or "-",
                (g.y if g else None) or "-", (s.y if s else None) or "-",
                comparison_type(g, s),
            )) + "\n")


class SummaryRuns:
    """summary.tsv with the handler's line grouping (runs of consecutive pairs with equal
    (x.id, y.id) share one line; the header repeats the metric labels for the FIRST run's length,
    as write_summary's grouped path) fed x-major row blocks: a run may span two blocks (the last
    pair of a block's last row and the first of the next block's first row), so the open run is
    carried over.  For duplicate ids on the streamed path."""

    def __init__(self, fh, seqs: list, metrics: list, genera, species, fmt: str, missing: str):
        self.fh, self.seqs, self.metrics = fh, seqs, metrics
        self.fmt, self.missing = fmt, missing
        self.ids = [s.id for s in seqs]
        self.gx = [genera.get(i, None) for i in self.ids] if genera else None
        self.sx = [species.get(i, None) for i in self.ids] if species else None
        self.head = ["seqid (query 1)", "seqid (query 2)", *[str(m) for m in metrics],
                     *[k + " (query 1)" for k in seqs[0].extras], *[k + " (query 2)" for k in seqs[0].extras],
                     "genus (query 1)", "species (query 1)", "genus (query 2)", "species (query 2)",
                     "comparison_type"]
        self.first = True
        self.run: list = []
        self.key = None

    def feed(self, A: np.ndarray, x0: int) -> None:
        text = _values_text(A, self.fmt, self.missing)
        ids = self.ids
        for r in range(A.shape[0]):
            i = x0 + r
            for j in range(len(ids)):
                k = (ids[i], ids[j])
                if self.run and k != self.key:
                    self._emit()
                self.key = k
                self.run.append((i, j, text[r, j]))

    def _emit(self) -> None:
        run, self.run = self.run, []
        i0, j0, _ = run[0]
        if self.first:
            self.head[2 : 2 + len(self.metrics)] = [str(m) for _ in run for m in self.metrics]
            self.fh.write("\t".join(self.head) + "\n")
            self.first = False
        x, y = self.seqs[i0], self.seqs[j0]
        gx, sx, missing = self.gx, self.sx, self.missing
        g = SubsetPair(gx[i0], gx[j0]) if gx is not None else None
        s = SubsetPair(sx[i0], sx[j0]) if sx is not None else None
        self.fh.write("\t".join((
            x.id, y.id, *[t for _, _, tt in run for t in tt],
            *[v if v is not None else missing for v in x.extras.values()],
            *[v if v is not None else missing for v in y.extras.values()],
            (g.x if g else None) or "-", (s.x if s else None) or "-",
            (g.y if g else None) or "-", (s.y if s else None) or "-",
            comparison_type(g, s),
        )) + "\n")

    def close(self) -> None:
        if self.run:
            self._emit()


def summary_lines(A: np.ndarray, x0: int, seqs: list, metrics: list, genera, species, fmt: str,
                  missing: str) -> str:
    """summary.tsv lines of the rows [x0, x0 + len(A)) x all columns, unique ids (one line per
    ordered pair: no (x.id, y.id) run spans two pairs), for the streamed writer."""
    ids = [s.id for s in seqs]
    gx = [genera.get(i, None) for i in ids] if genera else None
    sx = [species.get(i, None) for i in ids] if species else None
    text = _values_text(A, fmt, missing)
    out = []
    for r in range(A.shape[0]):
        i = x0 + r
        x = seqs[i]
        for j, y in enumerate(seqs):
            g = SubsetPair(gx[i], gx[j]) if gx is not None else None
            s = SubsetPair(sx[i], sx[j]) if sx is not None else None
            out.append("\t".join((
                x.id, y.id, *text[r, j],
                *[v if v is not None else missing for v in x.extras.values()],
                *[v if v is not None else missing for v in y.extras.values()],
                (g.x if g else None) or "-", (s.x if s else None) or "-",
                (g.y if g else None) or "-", (s.y if s else None) or "-",
                comparison_type(g, s),
            )) + "\n")
    return "".join(out)


def _values_text(A: np.ndarray, fmt: str, missing: str) -> np.ndarray:
    from .common import format_values

    return format_values(A, fmt, missing)


# ----------------------------------------------------------------------------- subset statistics
class SubsetStats(NamedTuple):
    subsets: list  # subset labels by code (None included)
    mean: np.ndarray  # [ns][ns][m], NaN where count == 0
    min: np.ndarray
    max: np.ndarray
    count: np.ndarray


def aggregate(A: np.ndarray, ids: list[str], partition) -> SubsetStats:
    """DistanceAggregator per metric over the (N, N, M) adjusted values (None skipped)."""
    from .._native import subset_aggregate

    code, subsets = subset_codes(ids, partition)
    agg = subset_aggregate(A, code, len(subsets))
    with np.errstate(invalid="ignore", divide="ignore"):
        mean = np.where(agg.count > 0, agg.sum / np.maximum(agg.count, 1), np.nan)
    mn = np.where(agg.count > 0, agg.min, np.nan)
    mx = np.where(agg.count > 0, agg.max, np.nan)
    return SubsetStats(subsets, mean, mn, mx, agg.count)


class SubsetAggregatorDev:
    """DistanceAggregator state of one partition on the GPU (versus_all.py:57-96, 617-640), fed the
    streamed row blocks in ascending order (taxi2_subset_aggregate_dev): the N x N values never
    exist on the host.  Same result as :func:`aggregate` over the full matrix, bit for bit."""

    def __init__(self, eng, ids: list[str], partition, m: int, codes: tuple | None = None):
        import torch

        code, self.subsets = codes if codes is not None else subset_codes(ids, partition)
        ns = len(self.subsets)
        dev = torch.device("cuda", eng.device)
        order = np.argsort(code, kind="stable")  # columns grouped by subset, ascending within one
        start = np.zeros(ns + 1, dtype=np.int64)
        start[1:] = np.cumsum(np.bincount(code, minlength=ns))
        self.eng, self.m, self.ns, self.n = eng, m, ns, len(ids)
        self.row_code = torch.as_tensor(code, dtype=torch.int32, device=dev)
        self.col_start = torch.as_tensor(start, dtype=torch.int64, device=dev)
        self.order = order  # the task's columns in subset order (ascending within a subset)
        self.col_idx = torch.as_tensor(order.astype(np.int32), dtype=torch.int32, device=dev)
        self.col_nat = None
        self.scratch = None  # own working memory (use_own_scratch): concurrent aggregators
        shape = (ns, ns, m)
        self.sum = torch.zeros(shape, dtype=torch.float64, device=dev)
        self.min = torch.full(shape, float("inf"), dtype=torch.float64, device=dev)
        self.max = torch.zeros(shape, dtype=torch.float64, device=dev)
        self.count = torch.zeros(shape, dtype=torch.int64, device=dev)
        self.torch = torch

    def set_storage(self, inv: np.ndarray, nat) -> None:
        """The blocks arrive with their columns stored permuted: stored column c is task column nat[c]
        (device int64), inv its inverse (host).  The subsets' columns are indexed by stored position
        from then on; sums are exact in any order and nat orders the minimum's ties."""
        self.col_idx = self.torch.as_tensor(inv[self.order].astype(np.int32), dtype=self.torch.int32,
                                            device=self.col_idx.device)
        self.col_nat = nat

    def use_own_scratch(self, nbytes: int = 384 << 20) -> None:
        """Give this aggregator its own working memory, so that several can run on separate
        streams at once (the library's default scratch is one per context)."""
        self.scratch = self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.col_idx.device)

    def add(self, D, x0: int, x1: int) -> None:
        """D: (x1 - x0, n, m) float64 device tensor of the rows' adjusted values (NaN = None),
        ordered after the work already queued on torch's current stream."""
        torch = self.torch
        D = D.contiguous()
        cur = torch.cuda.current_stream(D.device)
        side = None
        if cur.cuda_stream == 0:
            # the legacy default stream's handle is 0, which the engine reads as "its own stream":
            # run on a side stream ordered after `cur`, and order `cur` after it
            side = torch.cuda.Stream(D.device)
            side.wait_stream(cur)
        st = (side or cur).cuda_stream
        self.eng.subset_aggregate_dev(D.data_ptr(), x1 - x0, self.n, self.m, self.row_code[x0:x1].data_ptr(),
                                      self.col_start.data_ptr(), self.col_idx.data_ptr(), self.ns, False,
                                      self.sum.data_ptr(), self.min.data_ptr(), self.max.data_ptr(),
                                      self.count.data_ptr(), st,
                                      col_nat_ptr=self.col_nat.data_ptr() if self.col_nat is not None else None,
                                      scratch_ptr=self.scratch.data_ptr() if self.scratch is not None else None,
                                      scratch_bytes=self.scratch.numel() if self.scratch is not None else 0)
        if side is not None:
            cur.wait_stream(side)

    def state(self) -> tuple:
        """The running state tensors (sum, min, max, count), passed rank to rank by the sharded
        pre-aligned chain (VersusAll._stream_prealigned)."""
        return (self.sum, self.min, self.max, self.count)

    def result(self) -> SubsetStats:
        s, lo, hi, c = (t.cpu().numpy() for t in (self.sum, self.min, self.max, self.count))
        with np.errstate(invalid="ignore", divide="ignore"):
            mean = np.where(c > 0, s / np.maximum(c, 1), np.nan)
        return SubsetStats(self.subsets, mean, np.where(c > 0, lo, np.nan), np.where(c > 0, hi, np.nan), c)


def _text(v: float, fmt: str) -> str:
    return "NA" if not np.isfinite(v) else fmt.format(float(v))


def _tokens(arr: np.ndarray, fmt: str, eng=None) -> list:
    """``_text`` of every value of ``arr`` (flattened, C order) as a list of str.  A "{:.Nf}"
    formatter with an engine goes through taxi2_format_rows (Python-exact "%.Nf", one call);
    anything else through ``fmt.format`` on a Python list (no per-element numpy indexing)."""
    flat = np.ascontiguousarray(arr, dtype=np.float64).ravel()
    if not flat.size:
        return []
    dec = fixed_decimals(fmt)
    if eng is not None and gpu_text_ok(flat, dec):
        text = eng.format_rows(flat[None, :], [""], None, decimals=dec, missing="NA")
        return text.decode("utf-8")[1:-1].split("\t")
    return ["NA" if not math.isfinite(v) else fmt.format(v) for v in flat.tolist()]


def write_subset_statistics(path: Path, st: SubsetStats, metrics: list, fmt: str, template: str,
                            eng=None) -> None:
    """``linear/{pairs,identity}.tsv`` (versus_all.py:642-667) and ``matricial/<metric>.tsv``
    (:669-684) under ``path``; the handlers' missing text is always "NA".  Numbers are formatted
    in bulk (``_tokens``) and lines joined per row: the bytes of the handlers' per-value path,
    which took ~30 us per matrix cell (a 1 000-species partition has 3 M cells)."""
    lin = Path(path) / "linear"
    create_parents(lin)
    labels = [f"{m} {s}" for m in metrics for s in ("mean", "min", "max")]
    ns, m = len(st.subsets), len(metrics)
    names = ["?" if v is None else v for v in st.subsets]
    dec = fixed_decimals(fmt)
    if ns and dec is not None and all(gpu_text_ok(a, dec) for a in (st.mean, st.min, st.max)):
        _write_subset_statistics_native(path, st, metrics, names, labels, dec, template)
        return
    per = 3 * m
    # tok[(a * ns + b) * per + 3 k + s]: stat s (mean / min / max) of metric k for key (a, b)
    tok = _tokens(np.stack([st.mean, st.min, st.max], axis=-1), fmt, eng) if ns else []
    with open(lin / "pairs.tsv", "w") as fp, open(lin / "identity.tsv", "w") as fi:
        plines, ilines, head = [], [], False
        for a in range(ns):
            base, na = a * ns * per, names[a]
            for b in range(ns):
                cells = tok[base + b * per: base + (b + 1) * per]
                if a == b:  # bunch[0].idx == bunch[0].idy (one code per distinct subset)
                    ilines.append("\t".join((na, *cells)))
                else:
                    plines.append("\t".join((na, names[b], *cells)))
            if len(plines) >= 65536 or (a == ns - 1 and plines):
                if not head:
                    fp.write("\t".join(("target", "query", *labels)) + "\n")
                    head = True
                fp.write("\n".join(plines) + "\n")
                plines = []
        if ilines:
            fi.write("\t".join(("target", *labels)) + "\n")
            fi.write("\n".join(ilines) + "\n")
    mat = Path(path) / "matricial"
    create_parents(mat)
    simple = template == "{mean} ({min}-{max})"
    cnt = st.count.reshape(ns * ns, m).tolist() if ns else []
    for k, metric in enumerate(metrics):
        with open(mat / f"{metric}.tsv", "w") as fh:
            if ns:
                fh.write("\t".join(("", *names)) + "\n")
            rows = []
            for a in range(ns):
                cells = []
                for b in range(ns):
                    i = a * ns + b
                    if not cnt[i][k]:
                        cells.append("NA")
                        continue
                    q = i * per + 3 * k
                    if simple:
                        cells.append(f"{tok[q]} ({tok[q + 1]}-{tok[q + 2]})")
                    else:
                        cells.append(template.format(mean=tok[q], min=tok[q + 1], max=tok[q + 2]))
                rows.append("\t".join((names[a], *cells)))
                if len(rows) >= 256 or a == ns - 1:
                    fh.write("\n".join(rows) + "\n")
                    rows = []


def _write_subset_statistics_native(path: Path, st: SubsetStats, metrics: list, names: list, labels: list, dec: int,
                                    template: str) -> None:
    """write_subset_statistics through the engine library's host formatter (taxi2_format_subset_stats:
    the same bytes, "{:.Nf}" exact, threaded): a 1 000-species partition is 3 M formatted cells, ~2 s
    of Python string joins per partition otherwise."""
    from .._native import format_subset_stats

    from concurrent.futures import ThreadPoolExecutor

    lin = Path(path) / "linear"
    mean, mn, mx, cnt = st.mean, st.min, st.max, st.count
    simple = template == "{mean} ({min}-{max})"
    # every file's body at once (the library call releases the GIL), then the writes in order
    parts = [0, 1] + ([2 + k for k in range(len(metrics))] if simple else [])
    with ThreadPoolExecutor(max_workers=len(parts)) as ex:
        bodies = dict(zip(parts, ex.map(lambda q: format_subset_stats(mean, mn, mx, cnt, names, dec, q,
                                                                      threads=12 if q == 0 else 4), parts)))
    with open(lin / "pairs.tsv", "wb") as fp:
        body = bodies[0]
        if body:
            fp.write(("\t".join(("target", "query", *labels)) + "\n").encode())
            fp.write(body)
    with open(lin / "identity.tsv", "wb") as fi:
        fi.write(("\t".join(("target", *labels)) + "\n").encode())
        fi.write(bodies[1])
    mat = Path(path) / "matricial"
    create_parents(mat)
    for k, metric in enumerate(metrics):
        with open(mat / f"{metric}.tsv", "wb") as fh:
            fh.write(("\t".join(("", *names)) + "\n").encode())
            if simple:
                fh.write(bodies[2 + k])
                continue
            fmt = "{:.%df}" % dec
            for a in range(len(names)):
                cells = [template.format(mean=_text(mean[a, b, k], fmt), min=_text(mn[a, b, k], fmt),
                                         max=_text(mx[a, b, k], fmt)) if cnt[a, b, k] else "NA"
                         for b in range(len(names))]
                fh.write(("\t".join((names[a], *cells)) + "\n").encode())
