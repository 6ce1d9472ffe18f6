"""ctypes binding to ``libtaxi2_mi355x.so`` (the C ABI declared in ``include/taxi2_mi355x.h``).

This is the only way the product reaches the GPU.  There is no CPU fallback: if the library
is missing or no GPU is visible, constructing an :class:`Engine` raises
:class:`NativeError`.  ctypes releases the GIL for every call.

Replaces the reference's per-pair native crossings (``align.py:75,152`` Biopython C,
``distances.py:323-347`` Rust ``calc.seq_distances_*``) with batched calls.
"""

from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Iterable, NamedTuple, Sequence as Seq

import numpy as np

LIB_DIR = Path(__file__).resolve().parent / "_lib"
# TAXI2_LIB selects another in-tree build of the same ABI (the debug builds of
# taxi2_amd/csrc/Makefile: `make guard`, `make chunk16`), by file name inside _lib/.
LIB_PATH = LIB_DIR / os.path.basename(os.environ.get("TAXI2_LIB", "libtaxi2_mi355x.so"))
HEADER_PATH = Path(__file__).resolve().parent.parent / "include" / "taxi2_mi355x.h"

# Every symbol include/taxi2_mi355x.h declares.
EXPORTS = (
    "taxi2_device_count",
    "taxi2_ctx_create",
    "taxi2_ctx_destroy",
    "taxi2_last_error",
    "taxi2_version",
    "taxi2_set_create",
    "taxi2_set_destroy",
    "taxi2_set_info",
    "taxi2_all_pairs",
    "taxi2_all_pairs_dev",
    "taxi2_counts_metrics_dev",
    "taxi2_rect_pairs",
    "taxi2_rect_pairs_dev",
    "taxi2_rect_block_dev",
    "taxi2_set_permuted",
    "taxi2_rect_strings_dev",
    "taxi2_tri_strings_dev",
    "taxi2_format_pairs_ptr_dev",
    "taxi2_format_pairs_ptr_async",
    "taxi2_pack_slots_dev",
    "taxi2_stream_create_cus",
    "taxi2_stream_destroy",
    "taxi2_num_cus",
    "taxi2_set_text_copy",
    "taxi2_copy_text_dev",
    "taxi2_list_pairs",
    "taxi2_closest",
    "taxi2_align_strings",
    "taxi2_ncd_pairs",
    "taxi2_ncd_slots_dev",
    "taxi2_zlib_lengths",
    "taxi2_format_pairs_dev",
    "taxi2_format_rows",
    "taxi2_format_ragged",
    "taxi2_format_summary",
    "taxi2_format_rows_dev",
    "taxi2_format_summary_dev",
    "taxi2_subset_aggregate",
    "taxi2_format_subset_stats",
    "taxi2_subset_aggregate_dev",
    "taxi2_dereplicate_walk",
)

MODE_PREALIGNED = 0
MODE_ALIGN = 1

METRIC_CODES = {"p": 0, "p-gaps": 1, "jc": 2, "k2p": 3}
# Pseudo-metric: the packed column counters of each ordered pair (uint64 in the f64 slot:
# valid | ts << 16 | tv << 32 | gap << 48); must be the only metric of a call (taxi2_mi355x.h).
COUNTS = "counts"
COUNTS_CODE = 16
# NCD (distances.py:351-358) inside taxi2_all_pairs[_dev] on ALIGN sets: from the same fill's aligned
# strings (one fill per pair for every metric); other entry points take it through taxi2_ncd_pairs
NCD_CODE = 4
MAX_METRICS = 8


def _dev_vals(vals, stream):
    """(data pointer, (nrows, ncols, nm), value stride, stream) of a float64 CUDA tensor whose value
    slots (r, c) lie at a fixed stride -- (nrows, ncols, nm) with unit metric stride, or (nrows, ncols)
    -- else None (host values)."""
    if not (hasattr(vals, "is_cuda") and vals.is_cuda):
        return None
    import torch

    if vals.dtype != torch.float64:
        raise ValueError("device values must be float64")
    if vals.dim() == 2:
        nrows, ncols, nm = vals.shape[0], vals.shape[1], 1
    elif vals.dim() == 3 and (vals.shape[2] == 1 or vals.stride(2) == 1):
        nrows, ncols, nm = vals.shape
    else:
        raise ValueError("device values must be (nrows, ncols) or (nrows, ncols, nm) with unit metric stride")
    # slot g = r * ncols + c lies at g * vs: with one column the slots are the rows (stride(0)), else
    # the rows must be contiguous runs of slots
    vs = vals.stride(0) if ncols == 1 else vals.stride(1)
    if ncols > 1 and nrows > 1 and vals.stride(0) != ncols * vs:
        raise ValueError("device value rows must be contiguous slot runs")
    if nrows * ncols > 1 and vs < nm:
        raise ValueError("device value slots overlap")
    return vals.data_ptr(), (nrows, ncols, nm), int(max(vs, nm)), stream


class NativeError(RuntimeError):
    """The MI355X engine is unavailable or reported an error."""


class CScores(ctypes.Structure):
    _fields_ = [
        ("match_score", ctypes.c_int32),
        ("mismatch_score", ctypes.c_int32),
        ("internal_open_gap_score", ctypes.c_int32),
        ("internal_extend_gap_score", ctypes.c_int32),
        ("end_open_gap_score", ctypes.c_int32),
        ("end_extend_gap_score", ctypes.c_int32),
    ]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_INT = ctypes.c_int

_SIGNATURES = {
    "taxi2_device_count": (_INT, []),
    "taxi2_ctx_create": (_INT, [_INT, ctypes.POINTER(_P)]),
    "taxi2_ctx_destroy": (None, [_P]),
    "taxi2_last_error": (ctypes.c_char_p, [_P]),
    "taxi2_version": (ctypes.c_char_p, []),
    "taxi2_set_create": (_INT, [_P, _P, _P, _I64, _INT, ctypes.POINTER(_INT)]),
    "taxi2_set_destroy": (_INT, [_P, _INT]),
    "taxi2_set_info": (_INT, [_P, _INT, ctypes.POINTER(_I64), ctypes.POINTER(_I32), ctypes.POINTER(_INT)]),
    "taxi2_all_pairs": (_INT, [_P, _INT, _I64, _I64, ctypes.POINTER(CScores), _P, _INT, _P, _P]),
    "taxi2_all_pairs_dev": (_INT, [_P, _INT, _I64, _I64, ctypes.POINTER(CScores), _P, _INT, _P, _P, _P]),
    "taxi2_counts_metrics_dev": (_INT, [_P, _P, _I64, _P, _INT, ctypes.c_double, _P, _P]),
    "taxi2_rect_pairs": (_INT, [_P, _INT, _INT, _I64, _I64, ctypes.POINTER(CScores), _P, _INT, _P, _P]),
    "taxi2_rect_pairs_dev": (_INT, [_P, _INT, _INT, _I64, _I64, ctypes.POINTER(CScores), _P, _INT, _P, _P, _P]),
    "taxi2_set_permuted": (_INT, [_P, _INT, _P, _I64, ctypes.POINTER(_INT)]),
    "taxi2_rect_block_dev": (_INT, [_P, _INT, _INT, _I64, _I64, _P, _INT, ctypes.c_double, _INT, _INT, _P, _P, _P,
                                    _P, _P]),
    "taxi2_rect_strings_dev": (_INT, [_P, _INT, _INT, _I64, _I64, ctypes.POINTER(CScores), _P, _INT, _P, _I32, _P, _P,
                                      _P, _P]),
    "taxi2_format_pairs_dev": (_INT, [_P, _INT, _INT, _I64, _I64, _I32, _P, _P, _P, _P, _P, _P, _P, _INT, _P, _I64,
                                      ctypes.POINTER(_I64), _P]),
    "taxi2_tri_strings_dev": (_INT, [_P, _INT, _I64, _I64, ctypes.POINTER(CScores), _P, _INT, _P, _I32, _P, _P, _P,
                                     _INT, _P]),
    "taxi2_format_pairs_ptr_async": (_INT, [_P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _INT, _P, _I64, _P, _P,
                                            _P]),
    "taxi2_format_pairs_ptr_dev": (_INT, [_P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _INT, _P, _I64,
                                          ctypes.POINTER(_I64), _P]),
    "taxi2_pack_slots_dev": (_INT, [_P, _P, _P, _P, _I64, _INT, _INT, _P, _P, _I64, _P, _P, _P]),
    "taxi2_stream_create_cus": (_INT, [_P, _INT, _INT, ctypes.POINTER(_P)]),
    "taxi2_stream_destroy": (_INT, [_P, _P]),
    "taxi2_num_cus": (_INT, [_P]),
    "taxi2_set_text_copy": (_INT, [_P, _INT]),
    "taxi2_copy_text_dev": (_INT, [_P, _P, _P, _I64, _P]),
    "taxi2_list_pairs": (_INT, [_P, _INT, _INT, _P, _P, _I64, ctypes.POINTER(CScores), _P, _INT, _P, _P]),
    "taxi2_closest": (_INT, [_P, _INT, _INT, _I64, _I64, ctypes.POINTER(CScores), _I32, ctypes.c_double,
                             _P, _INT, _P, _P, _P, _P]),
    "taxi2_align_strings": (_INT, [_P, _INT, _INT, _P, _P, _I64, ctypes.POINTER(CScores), _INT, _I32, _P, _P, _P]),
    "taxi2_ncd_pairs": (_INT, [_P, _INT, _INT, _P, _P, _I64, _P, _INT, _P]),
    "taxi2_ncd_slots_dev": (_INT, [_P, _P, _P, _P, _I64, _INT, _INT, _P, _I64, _I32, _INT, _P, _P]),
    "taxi2_zlib_lengths": (_INT, [_P, _INT, _INT, _P, _P, _I64, _P]),
    "taxi2_format_rows": (_INT, [_P, _INT, _P, _I64, _I64, _INT, _P, _P, _P, _P, _INT, _P, _I32, _P, _I64,
                                 ctypes.POINTER(_I64)]),
    "taxi2_format_ragged": (_INT, [_P, _INT, _P, _I64, _P, _P, _I64, _INT, _P, _P, _P, _P, _INT, _P, _I32, _P,
                                   _I64, ctypes.POINTER(_I64)]),
    "taxi2_format_summary": (_INT, [_P, _P, _I64, _I64, _INT, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _INT, _INT,
                                    _P, _P, _INT, _P, _I32, _P, _I64, ctypes.POINTER(_I64)]),
    "taxi2_format_rows_dev": (_INT, [_P, _INT, _P, _I64, _I64, _I64, _INT, _P, _P, _P, _P, _INT, _P, _I32, _P, _I64,
                                     ctypes.POINTER(_I64), _P]),
    "taxi2_format_summary_dev": (_INT, [_P, _P, _I64, _I64, _I64, _INT, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                        _INT, _INT, _P, _P, _INT, _P, _I32, _P, _I64, ctypes.POINTER(_I64), _P]),
    "taxi2_subset_aggregate": (_INT, [_P, _I64, _INT, _P, _I32, _P, _P, _P, _P, _INT]),
    "taxi2_format_subset_stats": (_INT, [_I64, _INT, _P, _P, _P, _P, _P, _P, _INT, _INT, _P, _I64,
                                         ctypes.POINTER(_I64), _INT]),
    "taxi2_subset_aggregate_dev": (_INT, [_P, _P, _I64, _I64, _INT, _P, _P, _P, _I32, _INT, _P, _P, _P, _P, _P,
                                          _P, _I64, _P]),
    "taxi2_dereplicate_walk": (_INT, [_P, _I64, _P, _P, ctypes.c_double, _P, _P, _I64, ctypes.POINTER(_I64), _P,
                                      _P, _I64, ctypes.POINTER(_I64), _P]),
}

_lib = None
_lib_lock = threading.Lock()


def load_library() -> ctypes.CDLL:
    """Load the in-tree engine library (raises NativeError when it is absent)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise NativeError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or `make -C taxi2_amd/csrc`).  There is no CPU fallback."
            )
        lib = ctypes.CDLL(str(LIB_PATH))
        for name in EXPORTS:
            if "TAXI2_LIB" in os.environ and not hasattr(lib, name):
                continue  # a debug build of an older tree (tools/fault_*.sh): its own ABI subset
            fn = getattr(lib, name)  # AttributeError = missing export
            res, args = _SIGNATURES[name]
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def device_count() -> int:
    return int(load_library().taxi2_device_count())


def version() -> str:
    return load_library().taxi2_version().decode()


def build_info() -> dict:
    """The loaded library's source hash (baked in at build time) beside the hash of the sources in
    this tree (taxi2_amd/srchash.py): equal when the binary was built from these sources."""
    from .srchash import src_hash

    v = version()
    lib_hash = v.rsplit("src:", 1)[1] if "src:" in v else None
    tree = src_hash()
    return {"lib_src_hash": lib_hash, "tree_src_hash": tree, "lib_matches_tree": lib_hash == tree,
            "lib": str(LIB_PATH.relative_to(LIB_PATH.parent.parent.parent))}


def to_cscores(scores) -> CScores:
    """``align.Scores`` / mapping / 6-tuple -> C struct (field order = Scores.defaults)."""
    if scores is None:
        vals = (1, -1, -8, -1, -1, -1)
    elif isinstance(scores, dict):
        vals = tuple(
            scores[k]
            for k in (
                "match_score",
                "mismatch_score",
                "internal_open_gap_score",
                "internal_extend_gap_score",
                "end_open_gap_score",
                "end_extend_gap_score",
            )
        )
    else:
        vals = tuple(scores)
    ints = []
    for v in vals:
        if int(v) != v:
            raise ValueError(f"alignment scores must be integers (got {v!r})")
        ints.append(int(v))
    return CScores(*ints)


def metric_codes(metrics: Iterable, *, allow_ncd: bool = False) -> np.ndarray:
    codes = []
    for m in metrics:
        label = m if isinstance(m, str) else str(m)
        if label == COUNTS:
            codes.append(COUNTS_CODE)
            continue
        if label == "ncd" and allow_ncd:
            codes.append(NCD_CODE)
            continue
        if label not in METRIC_CODES:
            raise NativeError(f"metric {label!r} is not computed by the MI355X engine")
        codes.append(METRIC_CODES[label])
    if not 1 <= len(codes) <= MAX_METRICS:
        raise NativeError(f"between 1 and {MAX_METRICS} metrics per call")
    return np.asarray(codes, dtype=np.int32)


def encode_sequences(seqs: Seq[str], *, strict: bool) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate sequences as bytes + int64 offsets.

    Characters are handled as latin-1 bytes.  In align mode (``strict``) a character outside
    latin-1 raises ValueError instead of silently changing which letters compare equal.
    """
    errors = "strict" if strict else "replace"
    enc = [s.encode("latin-1", errors=errors) for s in seqs]
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        offs[1:] = np.cumsum(np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc)))
    buf = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8)
    return buf, offs


class SeqSet:
    """A sequence set resident in HBM (freed with the engine or by ``free``)."""

    def __init__(self, engine: "Engine", set_id: int, n: int, max_len: int, mode: int,
                 lengths: np.ndarray | None = None):
        self.engine = engine
        self.id = set_id
        self.n = n
        self.max_len = max_len
        self.mode = mode
        self._lengths = lengths

    def has_lengths(self) -> bool:
        return self._lengths is not None

    def lengths(self) -> np.ndarray:
        return self._lengths

    @property
    def aligned(self) -> bool:
        return self.mode == MODE_ALIGN

    def free(self) -> None:
        if self.id >= 0:
            self.engine._lib.taxi2_set_destroy(self.engine._ctx, self.id)
            self.id = -1


class Engine:
    """One engine context per GPU (one process per GPU for multi-GPU runs).

    Mixing with PyTorch in one process: import torch BEFORE the first Engine.  torch ships its own
    libamdhip64.so.7 (same soname as /opt/rocm's); whichever loads first serves the whole process,
    and torch only initialises its devices on the runtime it was built with.  Loaded that way the
    engine and torch share one runtime, so torch stream handles can be passed to the *_dev calls."""

    _default: dict[int, "Engine"] = {}

    def __init__(self, device: int | None = None):
        lib = load_library()
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        n = lib.taxi2_device_count()
        if n <= 0:
            raise NativeError("no HIP device visible; the MI355X engine has no CPU fallback")
        ctx = _P()
        rc = lib.taxi2_ctx_create(int(device), ctypes.byref(ctx))
        if rc != 0:
            raise NativeError(f"taxi2_ctx_create(device={device}) failed with {rc}")
        self._lib = lib
        self._ctx = ctx
        self.device = int(device)
        self._lock = threading.Lock()

    @classmethod
    def default(cls, device: int | None = None) -> "Engine":
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        eng = cls._default.get(device)
        if eng is None:
            eng = cls._default[device] = cls(device)
        return eng

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.taxi2_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = self._lib.taxi2_last_error(self._ctx)
            raise NativeError(f"{what}: {msg.decode() if msg else rc}")

    # ------------------------------------------------------------------ sets
    def upload(self, seqs: Seq[str], *, align: bool) -> SeqSet:
        buf, offs = encode_sequences(seqs, strict=align)
        return self.upload_packed(buf, offs, align=align)

    def upload_packed(self, buf: np.ndarray, offs: np.ndarray, *, align: bool) -> SeqSet:
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        n = len(offs) - 1
        sid = _INT()
        mode = MODE_ALIGN if align else MODE_PREALIGNED
        with self._lock:
            self._check(
                self._lib.taxi2_set_create(self._ctx, buf.ctypes.data, offs.ctypes.data, n, mode, ctypes.byref(sid)),
                "taxi2_set_create",
            )
            nn, ml, md = _I64(), _I32(), _INT()
            self._check(
                self._lib.taxi2_set_info(self._ctx, sid.value, ctypes.byref(nn), ctypes.byref(ml), ctypes.byref(md)),
                "taxi2_set_info",
            )
        return SeqSet(self, sid.value, nn.value, ml.value, md.value, np.diff(offs))

    def permuted_view(self, s: SeqSet, perm_ptr: int) -> SeqSet:
        """A column view of pre-aligned set ``s`` whose column c is s's sequence perm[c] (device int64
        array of s.n entries; taxi2_set_permuted).  Free it before ``s``."""
        vid = _INT()
        with self._lock:
            self._check(self._lib.taxi2_set_permuted(self._ctx, s.id, ctypes.c_void_p(perm_ptr), int(s.n),
                                                     ctypes.byref(vid)), "taxi2_set_permuted")
        return SeqSet(self, vid.value, s.n, s.max_len, s.mode, None)

    # ------------------------------------------------------------------ pair blocks
    def all_pairs(self, s: SeqSet, k0: int, count: int, metrics, scores=None, *, with_scores=False):
        """Upper-triangle block of ``s``.  ALIGN: (count, 2, M) [(a,b), (b,a)]; else (count, M).
        ALIGN sets also take "ncd": every metric of a pair from its one alignment (all_pairs_ncd)."""
        codes = metric_codes(metrics, allow_ncd=s.aligned)
        shape = (count, 2, len(codes)) if s.aligned else (count, len(codes))
        out = np.empty(shape, dtype=np.float64)
        sc_out = np.empty(count, dtype=np.int32) if (with_scores and s.aligned) else None
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_all_pairs(
                    self._ctx, s.id, int(k0), int(count), ctypes.byref(cs), codes.ctypes.data, len(codes),
                    out.ctypes.data, sc_out.ctypes.data if sc_out is not None else None,
                ),
                "taxi2_all_pairs",
            )
        return (out, sc_out) if with_scores else out

    def all_pairs_dev(self, s: SeqSet, k0: int, count: int, metrics, out_ptr: int, scores=None,
                      scores_ptr: int | None = None, stream: int | None = None) -> None:
        """Asynchronous device-output variant (pointers from e.g. torch tensors on this GPU)."""
        codes = metric_codes(metrics, allow_ncd=s.aligned)
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_all_pairs_dev(
                    self._ctx, s.id, int(k0), int(count), ctypes.byref(cs), codes.ctypes.data, len(codes),
                    ctypes.c_void_p(out_ptr), ctypes.c_void_p(scores_ptr) if scores_ptr else None,
                    ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_all_pairs_dev",
            )

    def counts_metrics_dev(self, counts_ptr: int, n: int, metrics, out_ptr: int, scale: float = 1.0,
                           stream: int | None = None) -> None:
        """out[k][m] = scale * metric m of the packed counters counts[k] (device pointers;
        asynchronous on ``stream``): the metrics of a TAXI2_METRIC_COUNTS launch."""
        codes = metric_codes(metrics)
        if COUNTS_CODE in codes:
            raise NativeError("counts_metrics_dev evaluates real metrics only")
        with self._lock:
            self._check(
                self._lib.taxi2_counts_metrics_dev(
                    self._ctx, ctypes.c_void_p(counts_ptr), int(n), codes.ctypes.data, len(codes), float(scale),
                    ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_counts_metrics_dev",
            )

    def subset_aggregate_dev(self, vals_ptr: int, nrows: int, ncols: int, m: int, row_code_ptr: int,
                             col_start_ptr: int, col_idx_ptr: int, ns: int, init: bool, sum_ptr: int, min_ptr: int,
                             max_ptr: int, count_ptr: int, stream: int | None = None, col_nat_ptr: int | None = None,
                             scratch_ptr: int | None = None, scratch_bytes: int = 0) -> None:
        """taxi2_subset_aggregate_dev on device buffers (see taxi2_amd/streaming.py); ``col_nat_ptr``:
        the task column of each stored column when the block is stored permuted."""
        with self._lock:
            self._check(
                self._lib.taxi2_subset_aggregate_dev(
                    self._ctx, ctypes.c_void_p(vals_ptr), int(nrows), int(ncols), int(m), ctypes.c_void_p(row_code_ptr),
                    ctypes.c_void_p(col_start_ptr), ctypes.c_void_p(col_idx_ptr), int(ns), 1 if init else 0,
                    ctypes.c_void_p(sum_ptr), ctypes.c_void_p(min_ptr), ctypes.c_void_p(max_ptr),
                    ctypes.c_void_p(count_ptr), ctypes.c_void_p(col_nat_ptr) if col_nat_ptr else None,
                    ctypes.c_void_p(scratch_ptr) if scratch_ptr else None, int(scratch_bytes),
                    ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_subset_aggregate_dev",
            )

    def rect_pairs(self, q: SeqSet, r: SeqSet, q0: int, q1: int, metrics, scores=None, *, with_scores=False):
        """(q1-q0)*R pairs (query, reference), row-major: (nq*R, M)."""
        codes = metric_codes(metrics)
        count = (q1 - q0) * r.n
        out = np.empty((count, len(codes)), dtype=np.float64)
        sc_out = np.empty(count, dtype=np.int32) if (with_scores and q.aligned) else None
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_rect_pairs(
                    self._ctx, q.id, r.id, int(q0), int(q1), ctypes.byref(cs), codes.ctypes.data, len(codes),
                    out.ctypes.data, sc_out.ctypes.data if sc_out is not None else None,
                ),
                "taxi2_rect_pairs",
            )
        return (out, sc_out) if with_scores else out

    def rect_pairs_dev(self, q: SeqSet, r: SeqSet, q0: int, q1: int, metrics, out_ptr: int, scores=None,
                       scores_ptr: int | None = None, stream: int | None = None) -> None:
        """Asynchronous device-output rectangle: out[(q - q0) * R + r][M] (orientation (q, r))."""
        codes = metric_codes(metrics)
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_rect_pairs_dev(
                    self._ctx, q.id, r.id, int(q0), int(q1), ctypes.byref(cs), codes.ctypes.data, len(codes),
                    ctypes.c_void_p(out_ptr), ctypes.c_void_p(scores_ptr) if scores_ptr else None,
                    ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_rect_pairs_dev",
            )

    def rect_block_dev(self, s: SeqSet, q0: int, q1: int, metrics, out_ptr: int, scale: float = 1.0,
                       diag: bool = True, rmin_metric: int = -1, rmin_idx_ptr: int | None = None,
                       rmin_val_ptr: int | None = None, stream: int | None = None, cols: SeqSet | None = None,
                       col_nat_ptr: int | None = None) -> None:
        """Row block [q0, q1) x set of the streamed pre-aligned versusAll with the task's epilogue on the
        GPU (taxi2_rect_block_dev): values x scale, NaN on the diagonal, each row's first minimum of
        metric index rmin_metric (idx -1 / NaN: none).  ``cols`` / ``col_nat_ptr``: the columns come
        from a permuted copy of ``s`` (stored in its order), column c being task column col_nat[c]."""
        codes = metric_codes(metrics)
        with self._lock:
            self._check(
                self._lib.taxi2_rect_block_dev(
                    self._ctx, s.id, (cols or s).id, int(q0), int(q1), codes.ctypes.data, len(codes), float(scale),
                    1 if diag else 0, int(rmin_metric), ctypes.c_void_p(rmin_idx_ptr) if rmin_idx_ptr else None,
                    ctypes.c_void_p(rmin_val_ptr) if rmin_val_ptr else None,
                    ctypes.c_void_p(col_nat_ptr) if col_nat_ptr else None, ctypes.c_void_p(out_ptr),
                    ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_rect_block_dev",
            )

    def rect_strings_dev(self, q: SeqSet, r: SeqSet, q0: int, q1: int, metrics, out_ptr: int | None, cap: int,
                         sx_ptr: int, sy_ptr: int, slen_ptr: int, scores=None, stream: int | None = None) -> None:
        """Metrics (may be empty) and aligned strings of rows [q0, q1) x every r, one fill per pair
        (device slots [(q - q0) * R + r][cap], right-aligned; see taxi2_rect_strings_dev)."""
        codes = metric_codes(metrics, allow_ncd=True) if metrics else np.zeros(0, dtype=np.int32)
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_rect_strings_dev(
                    self._ctx, q.id, r.id, int(q0), int(q1), ctypes.byref(cs), codes.ctypes.data if len(codes) else None,
                    len(codes), ctypes.c_void_p(out_ptr) if out_ptr else None, int(cap), ctypes.c_void_p(sx_ptr),
                    ctypes.c_void_p(sy_ptr), ctypes.c_void_p(slen_ptr), ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_rect_strings_dev",
            )

    def tri_strings_dev(self, s: SeqSet, k0: int, count: int, metrics, out_ptr: int | None, cap: int, sx_ptr: int,
                        sy_ptr: int, slen_ptr: int, scores=None, stream: int | None = None, reserve_cus: int = 0) -> None:
        """Metrics ([count][2][M], may be empty) and BOTH orientations' aligned strings of the
        triangle pairs [k0, k0 + count), one fill per pair (device slots [k][2][cap]; see
        taxi2_tri_strings_dev)."""
        codes = metric_codes(metrics, allow_ncd=True) if metrics else np.zeros(0, dtype=np.int32)
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_tri_strings_dev(
                    self._ctx, s.id, int(k0), int(count), ctypes.byref(cs), codes.ctypes.data if len(codes) else None,
                    len(codes), ctypes.c_void_p(out_ptr) if out_ptr else None, int(cap), ctypes.c_void_p(sx_ptr),
                    ctypes.c_void_p(sy_ptr), ctypes.c_void_p(slen_ptr), int(reserve_cus),
                    ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_tri_strings_dev",
            )

    def format_pairs_ptr_async(self, nrows: int, ncols: int, px_ptr: int, py_ptr: int, slen_ptr: int, rid_ptr: int,
                               roffs_ptr: int, cid_ptr: int, coffs_ptr: int, *, first: bool, text_ptr: int, cap: int,
                               total_ptr: int, scratch_ptr: int, stream: int) -> None:
        """Queue the aligned_pairs.txt text of an nrows x ncols block on ``stream``, every argument
        a device pointer (taxi2_format_pairs_ptr_async): text into ``text_ptr`` (``cap`` bytes),
        total_ptr[0] = its length, total_ptr[1] = 1 if it fit.  No host synchronisation."""
        with self._lock:
            self._check(
                self._lib.taxi2_format_pairs_ptr_async(
                    self._ctx, int(nrows), int(ncols), ctypes.c_void_p(px_ptr), ctypes.c_void_p(py_ptr),
                    ctypes.c_void_p(slen_ptr), ctypes.c_void_p(rid_ptr), ctypes.c_void_p(roffs_ptr),
                    ctypes.c_void_p(cid_ptr), ctypes.c_void_p(coffs_ptr), 1 if first else 0,
                    ctypes.c_void_p(text_ptr), int(cap), ctypes.c_void_p(total_ptr), ctypes.c_void_p(scratch_ptr),
                    ctypes.c_void_p(stream)),
                "taxi2_format_pairs_ptr_async",
            )

    def pack_slots_dev(self, sx_ptr: int, sy_ptr: int, slen_ptr: int, cap: int, nslot: int, slot: int, end_ptr: int,
                       off_ptr: int, count: int, dx_ptr: int, dy_ptr: int, stream: int) -> None:
        """Copy orientation ``slot`` of each pair's walker strings (the last slen bytes before end[k]
        of its slot) to dx / dy + off[k], on ``stream`` (taxi2_pack_slots_dev)."""
        with self._lock:
            self._check(
                self._lib.taxi2_pack_slots_dev(
                    self._ctx, ctypes.c_void_p(sx_ptr), ctypes.c_void_p(sy_ptr), ctypes.c_void_p(slen_ptr), int(cap),
                    int(nslot), int(slot), ctypes.c_void_p(end_ptr), ctypes.c_void_p(off_ptr), int(count),
                    ctypes.c_void_p(dx_ptr), ctypes.c_void_p(dy_ptr), ctypes.c_void_p(stream)),
                "taxi2_pack_slots_dev",
            )

    def num_cus(self) -> int:
        """Compute units of the engine's device (taxi2_num_cus)."""
        return int(self._lib.taxi2_num_cus(self._ctx))

    def cu_stream(self, cu_first: int, cu_count: int) -> int:
        """A raw hipStream_t whose kernels run only on CUs [cu_first, cu_first + cu_count)
        (taxi2_stream_create_cus); wrap it with torch.cuda.ExternalStream, release it with
        destroy_stream once its work is done."""
        out = _P()
        with self._lock:
            self._check(self._lib.taxi2_stream_create_cus(self._ctx, int(cu_first), int(cu_count), ctypes.byref(out)),
                        "taxi2_stream_create_cus")
        return int(out.value)

    def set_text_copy(self, mode: int) -> None:
        """Pair-text transfer into pinned memory (taxi2_set_text_copy): 0 kernel stores, 1 device
        buffer + DMA, 2 device buffer + 16-byte copy kernel; the bytes are the same."""
        with self._lock:
            self._check(self._lib.taxi2_set_text_copy(self._ctx, int(mode)), "taxi2_set_text_copy")

    def copy_text_dev(self, src_ptr: int, dst_ptr: int, nbytes: int, stream: int) -> None:
        """Device bytes -> pinned host bytes on ``stream`` (taxi2_copy_text_dev, asynchronous)."""
        with self._lock:
            self._check(self._lib.taxi2_copy_text_dev(self._ctx, ctypes.c_void_p(src_ptr), ctypes.c_void_p(dst_ptr),
                                                      int(nbytes), ctypes.c_void_p(stream)), "taxi2_copy_text_dev")

    def destroy_stream(self, stream: int) -> None:
        """Synchronise and destroy a stream from cu_stream (taxi2_stream_destroy)."""
        with self._lock:
            self._check(self._lib.taxi2_stream_destroy(self._ctx, ctypes.c_void_p(stream)), "taxi2_stream_destroy")

    def format_pairs_ptr_dev(self, nrows: int, ncols: int, px_ptr: int, py_ptr: int, slen_ptr: int, row_ids, col_ids,
                             *, first: bool, stream: int | None = None) -> memoryview:
        """aligned_pairs.txt text of an nrows x ncols block from per-pair string pointers
        (taxi2_format_pairs_ptr_dev); a memoryview of the pinned text buffer, valid until the next
        text call."""
        rb, ro = row_ids
        cb, co = col_ids
        need = _I64()
        buf = getattr(self, "_pairs_buf", None)
        if buf is None:
            buf = self._pinned(1 << 20)
        for _ in range(2):
            with self._lock:
                rc = self._lib.taxi2_format_pairs_ptr_dev(
                    self._ctx, int(nrows), int(ncols), ctypes.c_void_p(px_ptr), ctypes.c_void_p(py_ptr),
                    ctypes.c_void_p(slen_ptr), rb.ctypes.data, ro.ctypes.data, cb.ctypes.data, co.ctypes.data,
                    1 if first else 0, buf.ctypes.data, buf.size, ctypes.byref(need),
                    ctypes.c_void_p(stream) if stream else None)
            if rc == 1:
                self._pairs_buf = None
                buf = self._pinned(max(int(need.value), 2 * buf.size))
                continue
            self._check(rc, "taxi2_format_pairs_ptr_dev")
            self._pairs_buf = buf
            return memoryview(buf[: need.value])
        raise NativeError("taxi2_format_pairs_ptr_dev: output buffer sizing failed")

    def format_pairs_dev(self, q: SeqSet, r: SeqSet, q0: int, q1: int, cap: int, sx_ptr: int, sy_ptr: int,
                         slen_ptr: int, row_ids, col_ids, *, first: bool, stream: int | None = None) -> bytes:
        """aligned_pairs.txt text of the slots of rows [q0, q1) (taxi2_format_pairs_dev).  row_ids /
        col_ids: (bytes, offsets) from pack_strings.  Returns a memoryview of the engine's pinned
        text buffer, valid until the next call (write it out or copy it before then)."""
        rb, ro = row_ids
        cb, co = col_ids
        need = _I64()
        buf = getattr(self, "_pairs_buf", None)
        if buf is None:
            buf = self._pinned(1 << 20)
        for _ in range(2):
            with self._lock:
                rc = self._lib.taxi2_format_pairs_dev(
                    self._ctx, q.id, r.id, int(q0), int(q1), int(cap), ctypes.c_void_p(sx_ptr), ctypes.c_void_p(sy_ptr),
                    ctypes.c_void_p(slen_ptr), rb.ctypes.data, ro.ctypes.data, cb.ctypes.data, co.ctypes.data,
                    1 if first else 0, buf.ctypes.data, buf.size, ctypes.byref(need),
                    ctypes.c_void_p(stream) if stream else None)
            if rc == 1:
                self._pairs_buf = None
                buf = self._pinned(max(int(need.value), 2 * buf.size))
                continue
            self._check(rc, "taxi2_format_pairs_dev")
            self._pairs_buf = buf
            return memoryview(buf[: need.value])
        raise NativeError("taxi2_format_pairs_dev: output buffer sizing failed")

    def _pinned_view(self, nbytes: int) -> np.ndarray:
        """The first ``nbytes`` of the engine's pinned text buffer (grown as needed; valid until the
        next text call)."""
        buf = getattr(self, "_pairs_buf", None)
        if buf is None or buf.size < nbytes:
            self._pairs_buf = None
            buf = self._pairs_buf = self._pinned(max(int(nbytes), 1 << 20))
        return buf[: int(nbytes)]

    def _pinned(self, nbytes: int) -> np.ndarray:
        """A page-locked host buffer (the D2H of a block's text runs at full PCIe rate into it, no
        staging copy), kept alive by the engine; plain memory when torch cannot pin."""
        try:
            import torch

            t = torch.empty(int(nbytes), dtype=torch.uint8, pin_memory=True)
            self._pinned_keep = t
            return t.numpy()
        except Exception:
            return np.empty(int(nbytes), dtype=np.uint8)

    def list_pairs(self, x: SeqSet, y: SeqSet, xs, ys, metrics, scores=None, *, with_scores=False):
        """Explicit pairs.  ALIGN: (count, 2, M) [(x,y), (y,x)]; else (count, M)."""
        codes = metric_codes(metrics)
        xs = np.ascontiguousarray(xs, dtype=np.int64)
        ys = np.ascontiguousarray(ys, dtype=np.int64)
        if xs.shape != ys.shape:
            raise ValueError("xs and ys must have the same length")
        count = len(xs)
        shape = (count, 2, len(codes)) if x.aligned else (count, len(codes))
        out = np.empty(shape, dtype=np.float64)
        sc_out = np.empty(count, dtype=np.int32) if (with_scores and x.aligned) else None
        cs = to_cscores(scores)
        if count:
            with self._lock:
                self._check(
                    self._lib.taxi2_list_pairs(
                        self._ctx, x.id, y.id, xs.ctypes.data, ys.ctypes.data, count, ctypes.byref(cs),
                        codes.ctypes.data, len(codes), out.ctypes.data,
                        sc_out.ctypes.data if sc_out is not None else None,
                    ),
                    "taxi2_list_pairs",
                )
        return (out, sc_out) if with_scores else out

    def closest(self, q: SeqSet, r: SeqSet, q0: int, q1: int, primary, extras=(), scores=None, *,
                scale: float = 1.0, want_matrix: bool = False):
        """Per query: (idx[nq], d[nq], extras[nq, E] or None, matrix[nq, R] or None)."""
        pcode = int(metric_codes([primary])[0])
        nq = q1 - q0
        idx = np.empty(nq, dtype=np.int64)
        d = np.empty(nq, dtype=np.float64)
        ecodes = metric_codes(extras) if len(extras) else None
        ex = np.empty((nq, len(ecodes)), dtype=np.float64) if ecodes is not None else None
        mat = np.empty((nq, r.n), dtype=np.float64) if want_matrix else None
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_closest(
                    self._ctx, q.id, r.id, int(q0), int(q1), ctypes.byref(cs), pcode, float(scale),
                    ecodes.ctypes.data if ecodes is not None else None, len(ecodes) if ecodes is not None else 0,
                    idx.ctypes.data, d.ctypes.data, ex.ctypes.data if ex is not None else None,
                    mat.ctypes.data if mat is not None else None,
                ),
                "taxi2_closest",
            )
        return idx, d, ex, mat


    def ncd_pairs(self, x: SeqSet, y: SeqSet, xs, ys, scores=None, *, aligned: bool = True, both: bool = True):
        """NCD (distances.py:351-358) per pair: (count, 2) [(x, y), (y, x)] when ``both``, else (count,).
        ALIGN sets with ``aligned``: on the first alignment's gapped strings of each ordered pair
        (the strings VersusAll hands the metric); otherwise on the stored sequences."""
        xs = np.ascontiguousarray(xs, dtype=np.int64)
        ys = np.ascontiguousarray(ys, dtype=np.int64)
        if xs.shape != ys.shape:
            raise ValueError("xs and ys must have the same length")
        count = len(xs)
        out = np.empty((count, 2) if both else (count,), dtype=np.float64)
        use_aln = aligned and x.aligned
        cs = to_cscores(scores)
        if count:
            with self._lock:
                self._check(
                    self._lib.taxi2_ncd_pairs(
                        self._ctx, x.id, y.id, xs.ctypes.data, ys.ctypes.data, count,
                        ctypes.byref(cs) if use_aln else None, 1 if both else 0, out.ctypes.data,
                    ),
                    "taxi2_ncd_pairs",
                )
        return out

    def ncd_slots_dev(self, sx_ptr: int, sy_ptr: int, slen_ptr: int, cap: int, nslot: int, no: int, end_ptr: int,
                      count: int, max_len: int, out_ptr: int, *, latin1: bool = False,
                      stream: int | None = None) -> None:
        """NCD of walker string slots on the device (taxi2_ncd_slots_dev): out[k * no + o] for pair k's
        orientation o, from tri_strings_dev (nslot 2) / rect_strings_dev (nslot 1) slots whose strings
        end at end[k].  Asynchronous on ``stream``."""
        with self._lock:
            self._check(
                self._lib.taxi2_ncd_slots_dev(
                    self._ctx, ctypes.c_void_p(sx_ptr), ctypes.c_void_p(sy_ptr), ctypes.c_void_p(slen_ptr), int(cap),
                    int(nslot), int(no), ctypes.c_void_p(end_ptr), int(count), int(max_len), 1 if latin1 else 0,
                    ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream) if stream else None,
                ),
                "taxi2_ncd_slots_dev",
            )

    def zlib_lengths(self, x: SeqSet, xs, y: SeqSet | None = None, ys=None) -> np.ndarray:
        """len(zlib.compress(upper(x[xs[k]]) (+ upper(y[ys[k]])))) per k (zlib 1.2.11, level 6)."""
        xs = np.ascontiguousarray(xs, dtype=np.int64)
        yarr = None if ys is None else np.ascontiguousarray(ys, dtype=np.int64)
        out = np.empty(len(xs), dtype=np.int32)
        if len(xs):
            with self._lock:
                self._check(
                    self._lib.taxi2_zlib_lengths(
                        self._ctx, x.id, (y or x).id, xs.ctypes.data,
                        yarr.ctypes.data if yarr is not None else None, len(xs), out.ctypes.data,
                    ),
                    "taxi2_zlib_lengths",
                )
        return out

    def _check_dev_tensor(self, vals, dev) -> None:
        if dev is not None and vals.device.index is not None and vals.device.index != self.device:
            raise ValueError(f"device values live on cuda:{vals.device.index}, the engine on device {self.device}")

    def format_rows(self, vals, row_pre, col_pre=None, *, decimals: int = 4,
                    missing: str = "NA", view: bool = False, stream: int | None = None):
        """Writer text (taxi2_format_rows): ``vals`` (nrows, ncols, nm) -> linear rows
        ``row_pre TAB col_pre (TAB value){nm} LF`` per cell; (nrows, ncols) with ``col_pre=None``
        -> matrix rows ``row_pre (TAB value){ncols} LF``.  Values as Python "%.{decimals}f".
        ``vals`` may be a float64 CUDA tensor (slots at a fixed stride, e.g. one metric of a
        (rows, n, M) block): taxi2_format_rows_dev, ordered on ``stream``."""
        mode = 0 if col_pre is not None else 1
        dev = _dev_vals(vals, stream)
        self._check_dev_tensor(vals, dev)
        if dev is not None:  # a float64 CUDA tensor: taxi2_format_rows_dev reads it where it is
            v, nrows, ncols, nm = dev[0], *dev[1]
            if mode == 1 and nm != 1:
                raise ValueError("matrix text takes (nrows, ncols) values")
            return self._format(mode, v, nrows, None, None, ncols, nm, row_pre, col_pre, decimals, missing, view=view,
                                dev=dev)
        v = np.ascontiguousarray(vals, dtype=np.float64)
        if mode == 1 and v.ndim == 2:
            v = v[:, :, None]
        if v.ndim != 3:
            raise ValueError("vals must be (nrows, ncols, nm) (linear) or (nrows, ncols) (matrix)")
        nrows, ncols, nm = v.shape
        return self._format(mode, v, nrows, None, None, ncols, nm, row_pre, col_pre, decimals, missing, view=view)

    def format_ragged(self, vals: np.ndarray, row_start, cols, row_pre, col_pre=None, *, ncols: int | None = None,
                      decimals: int = 4, missing: str = "NA", view: bool = False):
        """Writer text for ragged rows (taxi2_format_ragged): row r formats tokens
        [row_start[r], row_start[r+1]) of ``vals`` (ntok, nm) / (ntok,), token g at column cols[g];
        linear with ``col_pre``, matrix rows otherwise (``ncols`` bounds cols then)."""
        v = np.ascontiguousarray(vals, dtype=np.float64)
        if v.ndim == 1:
            v = v[:, None]
        rs = np.ascontiguousarray(row_start, dtype=np.int64)
        cs = np.ascontiguousarray(cols, dtype=np.int32)
        nrows = len(rs) - 1
        if nrows < 0 or len(cs) < rs[-1] or len(v) < rs[-1]:
            raise ValueError("row_start must have nrows + 1 entries covering cols and vals")
        mode = 0 if col_pre is not None else 1
        if ncols is None:
            ncols = len(col_pre) if col_pre is not None else (int(cs.max()) + 1 if len(cs) else 0)
        return self._format(mode, v, nrows, rs, cs, ncols, v.shape[1], row_pre, col_pre, decimals, missing, view=view)

    def format_summary(self, vals: np.ndarray, row_pre, col_pre, row_suf, col_suf, row_codes, col_codes, *,
                       has_genera: bool, has_species: bool, decimals: int = 4, missing: str = "NA",
                       view: bool = False, stream: int | None = None):
        """summary.tsv lines (taxi2_format_summary) for ``vals`` (nrows, ncols, nm): row_suf / col_suf
        = 2 strings per row / column (extras with leading TABs; TAB genus TAB species),
        row_codes / col_codes (n, 2) = (genus, species) subset codes."""
        dev = _dev_vals(vals, stream)
        self._check_dev_tensor(vals, dev)
        if dev is not None:
            v, (nrows, ncols, nm) = dev[0], dev[1]
        else:
            v = np.ascontiguousarray(vals, dtype=np.float64)
            nrows, ncols, nm = v.shape
        rsb, rso = pack_strings(row_suf)
        csb, cso = pack_strings(col_suf)
        if len(rso) != 2 * nrows + 1 or len(cso) != 2 * ncols + 1:
            raise ValueError("two suffix strings per row and per column")
        rc_ = np.ascontiguousarray(row_codes, dtype=np.int32).reshape(nrows, 2)
        cc_ = np.ascontiguousarray(col_codes, dtype=np.int32).reshape(ncols, 2)
        lb, lo = pack_strings(COMPARISON_LABELS)
        extra = (rsb, rso, csb, cso, rc_, cc_, int(bool(has_genera)), int(bool(has_species)), lb, lo)
        sfx = int(rso[-1]) * ncols + int(cso[-1]) * nrows + nrows * ncols * 16
        return self._format(2, v, nrows, None, None, ncols, nm, row_pre, col_pre, decimals, missing, extra, sfx,
                            view=view, dev=dev)

    def _format(self, mode, v, nrows, rs, cs, ncols, nm, row_pre, col_pre, decimals, missing, summary=None,
                extra_cap: int = 0, view: bool = False, dev=None):
        """The formatter call; the text as bytes, or with ``view`` as a memoryview of the engine's
        pinned formatter buffer (valid until the next ``view`` call: write it out at once) -- the
        D2H then runs at full link rate into page-locked memory and no bytes copy is made."""
        pack = pack_strings
        rb, ro = pack(row_pre)
        if len(ro) != nrows + 1:
            raise ValueError("one row prefix per row")
        cb, co = pack(col_pre) if mode != 1 else (None, None)
        if mode != 1 and len(co) != ncols + 1:
            raise ValueError("one column prefix per column")
        miss = missing.encode("utf-8")
        need = _I64(0)
        ntok = nrows * ncols if rs is None else int(rs[-1] - rs[0])
        cap = max(1, ntok * (nm * (decimals + 8) + 4) + int(ro[-1]) * (ncols if rs is None else max(1, ntok))
                  + (int(co[-1]) * nrows if mode != 1 and rs is None else 0)
                  + (int(np.diff(co).max(initial=0)) * ntok if mode == 0 and rs is not None else 0) + extra_cap)
        name = "taxi2_format_summary" if summary else "taxi2_format_rows" if rs is None else "taxi2_format_ragged"
        if dev is not None:
            name += "_dev"
        for _ in range(2):
            if view:
                buf = getattr(self, "_fmt_buf", None)
                if buf is None or buf.size < cap:
                    self._fmt_buf = None
                    buf = self._fmt_buf = self._pinned(max(cap, 1 << 24))
                out = buf[:cap]
            else:
                out = np.empty(cap, dtype=np.uint8)
            cpre = (cb.ctypes.data if cb is not None else None, co.ctypes.data if co is not None else None)
            with self._lock:
                if dev is not None:
                    _, _, vstride, dst = dev
                    vp = ctypes.c_void_p(v)
                    if summary is not None:
                        rsb, rso, csb, cso, rc_, cc_, hg, hs, lb, lo = summary
                        rc = self._lib.taxi2_format_summary_dev(
                            self._ctx, vp, vstride, nrows, ncols, nm, rb.ctypes.data, ro.ctypes.data, *cpre,
                            rsb.ctypes.data, rso.ctypes.data, csb.ctypes.data, cso.ctypes.data, rc_.ctypes.data,
                            cc_.ctypes.data, hg, hs, lb.ctypes.data, lo.ctypes.data, int(decimals), miss, len(miss),
                            out.ctypes.data, cap, ctypes.byref(need), ctypes.c_void_p(dst) if dst else None,
                        )
                    else:
                        rc = self._lib.taxi2_format_rows_dev(
                            self._ctx, mode, vp, vstride, nrows, ncols, nm, rb.ctypes.data, ro.ctypes.data, *cpre,
                            int(decimals), miss, len(miss), out.ctypes.data, cap, ctypes.byref(need),
                            ctypes.c_void_p(dst) if dst else None,
                        )
                elif summary is not None:
                    rsb, rso, csb, cso, rc_, cc_, hg, hs, lb, lo = summary
                    rc = self._lib.taxi2_format_summary(
                        self._ctx, v.ctypes.data, nrows, ncols, nm, rb.ctypes.data, ro.ctypes.data, *cpre,
                        rsb.ctypes.data, rso.ctypes.data, csb.ctypes.data, cso.ctypes.data, rc_.ctypes.data,
                        cc_.ctypes.data, hg, hs, lb.ctypes.data, lo.ctypes.data, int(decimals), miss, len(miss),
                        out.ctypes.data, cap, ctypes.byref(need),
                    )
                elif rs is None:
                    rc = self._lib.taxi2_format_rows(
                        self._ctx, mode, v.ctypes.data, nrows, ncols, nm, rb.ctypes.data, ro.ctypes.data, *cpre,
                        int(decimals), miss, len(miss), out.ctypes.data, cap, ctypes.byref(need),
                    )
                else:
                    rc = self._lib.taxi2_format_ragged(
                        self._ctx, mode, v.ctypes.data, nrows, rs.ctypes.data, cs.ctypes.data, ncols, nm,
                        rb.ctypes.data, ro.ctypes.data, *cpre, int(decimals), miss, len(miss), out.ctypes.data,
                        cap, ctypes.byref(need),
                    )
            if rc == 1:
                cap = int(need.value)
                continue
            self._check(rc, name)
            return memoryview(out[: need.value]) if view else out[: need.value].tobytes()
        raise NativeError(f"{name}: output size changed between calls")

    def align_strings(self, x: SeqSet, y: SeqSet, xs, ys, scores=None, *, both: bool = False):
        """Gapped alignment strings: list of (ax, ay) per pair, plus the (y, x) alignment written
        in (x, y) column order when ``both`` (list of pairs of tuples)."""
        xs = np.ascontiguousarray(xs, dtype=np.int64)
        ys = np.ascontiguousarray(ys, dtype=np.int64)
        count = len(xs)
        if count == 0:
            return []
        cap = int(x.max_len + y.max_len) or 1
        ox = np.zeros((count, 2, cap), dtype=np.uint8)
        oy = np.zeros((count, 2, cap), dtype=np.uint8)
        ln = np.zeros((count, 2), dtype=np.int32)
        cs = to_cscores(scores)
        with self._lock:
            self._check(
                self._lib.taxi2_align_strings(
                    self._ctx, x.id, y.id, xs.ctypes.data, ys.ctypes.data, count, ctypes.byref(cs),
                    1 if both else 0, cap, ox.ctypes.data, oy.ctypes.data, ln.ctypes.data,
                ),
                "taxi2_align_strings",
            )
        lens_x = x.lengths()[xs] if x.has_lengths() else None
        lens_y = y.lengths()[ys] if y.has_lengths() else None
        out = []
        for k in range(count):
            end = int(lens_x[k] + lens_y[k])
            res = []
            for o in range(2 if both else 1):
                L = int(ln[k, o])
                res.append((ox[k, o, end - L:end].tobytes().decode("latin-1"),
                            oy[k, o, end - L:end].tobytes().decode("latin-1")))
            out.append(tuple(res) if both else res[0])
        return out


def unpack_counts(c: np.ndarray) -> np.ndarray:
    """TAXI2_METRIC_COUNTS slots (f64 or uint64 array) -> (..., 4) int64 (valid, ts, tv, gap)."""
    u = np.ascontiguousarray(c).view(np.uint64)
    return np.stack([(u >> np.uint64(s)) & np.uint64(0xFFFF) for s in (0, 16, 32, 48)], axis=-1).astype(np.int64)


def tri_index(a: np.ndarray, b: np.ndarray, n: int) -> np.ndarray:
    """Linear upper-triangle index of pairs a < b (row-major), as the C ABI numbers them."""
    a = np.asarray(a, dtype=np.int64)
    b = np.asarray(b, dtype=np.int64)
    return a * (2 * n - a - 1) // 2 + (b - a - 1)


def pack_strings(strings) -> tuple[np.ndarray, np.ndarray]:
    """UTF-8 bytes (NUL-terminated buffer) + int64 offsets [n + 1] of a list of str."""
    enc = [s.encode("utf-8") for s in strings]
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        offs[1:] = np.cumsum([len(e) for e in enc])
    return np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8), offs


COMPARISON_LABELS = ("no info", "intra-species", "inter-species", "intra-genus", "inter-genus")


class Aggregates(NamedTuple):
    """taxi2_subset_aggregate result, each [ns][ns][m]."""

    sum: np.ndarray
    min: np.ndarray
    max: np.ndarray
    count: np.ndarray


def subset_aggregate(d: np.ndarray, code, ns: int, threads: int = 0) -> Aggregates:
    """SimpleAggregator state per (subset x, subset y, metric) over the (n, n, m) adjusted values
    (taxi2_subset_aggregate: x-major summation order, host code in the engine library)."""
    lib = load_library()
    d = np.ascontiguousarray(d, dtype=np.float64)
    if d.ndim != 3 or d.shape[0] != d.shape[1]:
        raise ValueError("d must be (n, n, m)")
    n, _, m = d.shape
    code = np.ascontiguousarray(code, dtype=np.int32)
    if len(code) != n:
        raise ValueError("one subset code per sequence")
    out = [np.empty((ns, ns, m)) for _ in range(3)] + [np.empty((ns, ns, m), dtype=np.int64)]
    rc = lib.taxi2_subset_aggregate(d.ctypes.data, n, m, code.ctypes.data, ns, *[o.ctypes.data for o in out],
                                    int(threads))
    if rc != 0:
        raise NativeError(f"taxi2_subset_aggregate: bad arguments ({rc})")
    return Aggregates(*out)


def format_subset_stats(mean: np.ndarray, mn: np.ndarray, mx: np.ndarray, count: np.ndarray, names,
                        decimals: int, part: int, threads: int = 0) -> bytes:
    """Text of one subset statistics file (taxi2_format_subset_stats, host code: part 0 pairs.tsv
    lines, 1 identity.tsv lines, 2 + k matricial rows of metric k; no headers)."""
    lib = load_library()
    ns, _, m = mean.shape
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (mean, mn, mx)]
    cnt = np.ascontiguousarray(count, dtype=np.int64)
    nb, no = pack_strings(names)
    cap = ctypes.c_int64(0)
    est = int(ns * ns * (9 * m * 8 + 64) + 1024)
    for _ in range(2):
        buf = np.empty(max(1, est), dtype=np.uint8)
        rc = lib.taxi2_format_subset_stats(ns, m, *[a.ctypes.data for a in arrs], cnt.ctypes.data, nb.ctypes.data,
                                           no.ctypes.data, int(decimals), int(part), buf.ctypes.data, buf.size,
                                           ctypes.byref(cap), int(threads))
        if rc < 0:
            raise NativeError(f"taxi2_format_subset_stats: bad arguments ({rc})")
        if rc == 0:
            return buf[: cap.value].tobytes()
        est = cap.value
    raise NativeError("taxi2_format_subset_stats: output size changed")


class Walk(NamedTuple):
    """taxi2_dereplicate_walk result: kept pairs (row_kept per row, kept_cols row-major), summary
    lines (query, included, excluded rows; their distances, NaN = None) and the excluded flags."""

    row_kept: np.ndarray
    kept_cols: np.ndarray
    line_idx: np.ndarray
    line_d: np.ndarray
    excluded: np.ndarray


def dereplicate_walk(d: np.ndarray, ids, lens, similarity: float) -> Walk:
    """Dereplicate's greedy walk (taxi2_dereplicate_walk, host code in the engine library) over the
    (n, n) adjusted distance matrix; ``ids`` = id codes (equal <=> equal id), ``lens`` = unaligned
    lengths."""
    lib = load_library()
    d = np.ascontiguousarray(d, dtype=np.float64)
    n = len(d)
    if d.shape != (n, n):
        raise ValueError("d must be square")
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    if len(ids) != n or len(lens) != n:
        raise ValueError("one id code and one length per sequence")
    row_kept = np.zeros(n, dtype=np.int64)
    excluded = np.zeros(n, dtype=np.uint8)
    kcap, lcap = max(1, min(n * max(n - 1, 0), 1 << 24)), max(1, n)
    nk, nl = _I64(0), _I64(0)
    for _ in range(2):
        cols = np.empty(kcap, dtype=np.int32)
        li = np.empty((lcap, 3), dtype=np.int64)
        ld = np.empty((lcap, 2), dtype=np.float64)
        rc = lib.taxi2_dereplicate_walk(d.ctypes.data, n, ids.ctypes.data, lens.ctypes.data, float(similarity),
                                        row_kept.ctypes.data, cols.ctypes.data, kcap, ctypes.byref(nk),
                                        li.ctypes.data, ld.ctypes.data, lcap, ctypes.byref(nl), excluded.ctypes.data)
        if rc == 1:
            kcap, lcap = max(kcap, int(nk.value)), max(lcap, int(nl.value))
            continue
        if rc != 0:
            raise NativeError(f"taxi2_dereplicate_walk: bad arguments ({rc})")
        k, m = int(nk.value), int(nl.value)
        return Walk(row_kept, cols[:k], li[:m], ld[:m], excluded.astype(bool))
    raise NativeError("taxi2_dereplicate_walk: result size changed between calls")


def tri_pairs(n: int, k0: int = 0, count: int | None = None) -> tuple[np.ndarray, np.ndarray]:
    """Inverse of :func:`tri_index` for k in [k0, k0+count)."""
    total = n * (n - 1) // 2
    if count is None:
        count = total - k0
    k = np.arange(k0, k0 + count, dtype=np.int64)
    n2 = 2.0 * n - 1.0
    a = np.floor((n2 - np.sqrt(np.maximum(n2 * n2 - 8.0 * k, 0.0))) / 2).astype(np.int64)
    a = np.clip(a, 0, max(n - 2, 0))
    start = a * (2 * n - a - 1) // 2
    over = start > k
    while np.any(over):
        a[over] -= 1
        start = a * (2 * n - a - 1) // 2
        over = start > k
    nxt = (a + 1) * (2 * n - a - 2) // 2
    under = (nxt <= k) & (a + 1 <= n - 2)
    while np.any(under):
        a[under] += 1
        start = a * (2 * n - a - 1) // 2
        nxt = (a + 1) * (2 * n - a - 2) // 2
        under = (nxt <= k) & (a + 1 <= n - 2)
    b = a + 1 + (k - start)
    return a, b
