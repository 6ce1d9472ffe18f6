"""ctypes binding to the C restatement (oracle/_build/libtaxi2_oracle.so).

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# TAXI2_ORACLE_LIB: another build of the same source in _build/ (the sanitizer build, `make -C oracle san`)
LIB_PATH = HERE / "_build" / os.path.basename(os.environ.get("TAXI2_ORACLE_LIB", "libtaxi2_oracle.so"))

METRIC_CODES = {"p": 0, "p-gaps": 1, "jc": 2, "k2p": 3}


class Counts(ctypes.Structure):
    _fields_ = [("valid", ctypes.c_int32), ("ts", ctypes.c_int32),
                ("tv", ctypes.c_int32), ("gap", ctypes.c_int32)]

    def tuple(self):
        return (self.valid, self.ts, self.tv, self.gap)


class CScores(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("match", "mismatch", "open", "extend", "end_open", "end_extend")]


def build() -> Path:
    if "TAXI2_ORACLE_LIB" in os.environ:
        return LIB_PATH
    if not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "taxi2_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(LIB_PATH))
        L.t2o_align_counts.restype = ctypes.c_int32
        L.t2o_align_counts.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                       ctypes.POINTER(CScores), ctypes.POINTER(Counts),
                                       ctypes.POINTER(Counts)]
        L.t2o_prealigned_counts.restype = None
        L.t2o_prealigned_counts.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                            ctypes.c_int, ctypes.POINTER(Counts)]
        L.t2o_metric.restype = ctypes.c_double
        L.t2o_metric.argtypes = [ctypes.c_int, ctypes.POINTER(Counts)]
        L.t2o_batch.restype = ctypes.c_int
        L.t2o_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int64, ctypes.c_int, ctypes.POINTER(CScores),
                                ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int]
        _lib = L
    return _lib


def cscores(scores) -> CScores:
    s = tuple(scores)
    return CScores(*[int(v) for v in s])


def align_counts(x: str, y: str, scores):
    a, b = Counts(), Counts()
    xb, yb = x.encode("latin-1"), y.encode("latin-1")
    sc = cscores(scores)
    s = lib().t2o_align_counts(xb, len(xb), yb, len(yb), ctypes.byref(sc), ctypes.byref(a), ctypes.byref(b))
    return a.tuple(), b.tuple(), s


def prealigned_counts(x: str, y: str):
    c = Counts()
    xb, yb = x.encode("latin-1"), y.encode("latin-1")
    lib().t2o_prealigned_counts(xb, len(xb), yb, len(yb), ctypes.byref(c))
    return c.tuple()


def metric(label: str, counts) -> float:
    c = Counts(*counts)
    return lib().t2o_metric(METRIC_CODES[label], ctypes.byref(c))


def pack(seqs: list[str]) -> tuple[np.ndarray, np.ndarray]:
    enc = [s.encode("latin-1") for s in seqs]
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(e) for e in enc])
    buf = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8).copy()
    return buf, offs


def batch(seqs: list[str] | tuple[np.ndarray, np.ndarray], pa, pb, *, align: bool, scores,
          metrics=("p", "p-gaps", "jc", "k2p"), threads: int | None = None):
    """Per pair (a, b): out[k, 0, m] = metric of (a, b), out[k, 1, m] = metric of (b, a)."""
    buf, offs = pack(seqs) if isinstance(seqs, list) else seqs
    pa = np.ascontiguousarray(pa, dtype=np.int64)
    pb = np.ascontiguousarray(pb, dtype=np.int64)
    codes = np.array([METRIC_CODES[m] for m in metrics], dtype=np.int32)
    out = np.empty((len(pa), 2, len(codes)), dtype=np.float64)
    sc = np.empty(len(pa), dtype=np.int32)
    cs = cscores(scores)
    threads = threads or os.cpu_count() or 1
    lib().t2o_batch(buf.ctypes.data, offs.ctypes.data, pa.ctypes.data, pb.ctypes.data, len(pa),
                    1 if align else 0, ctypes.byref(cs), codes.ctypes.data, len(codes),
                    out.ctypes.data, sc.ctypes.data, int(threads))
    return out, sc
