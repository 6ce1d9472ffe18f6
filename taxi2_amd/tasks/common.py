"""Shared pieces of the GPU-backed tasks: Results, progress reporting, output formatting."""

from __future__ import annotations

from pathlib import Path
from typing import Callable, NamedTuple

import numpy as np


class Results(NamedTuple):
    output_directory: Path
    seconds_taken: float


def console_report(caption, index, total):
    """``versus_all.py:25-30`` progress printer."""
    if caption == "Finalizing...":
        print(f"\rCalculating... {total}/{total} = {100:.2f}%", end="")
        print("\nFinalizing...")
    else:
        print(f"\rCalculating... {index}/{total} = {100 * index / total:.2f}%", end="")


def create_parents(path: Path) -> None:
    if path.suffix:
        path = path.parent
    path.mkdir(parents=True, exist_ok=True)


def format_values(vals: np.ndarray, fmt: str, missing: str) -> np.ndarray:
    """Format f64 distances with the reference's ``formatter.format(d)``; NaN/inf -> missing.

    Vectorised through numpy's %-formatting, which applies Python's own float formatting per
    element, so '{:.4f}' and '%.4f' give identical text (incl. '-0.0000')."""
    out = np.full(vals.shape, missing, dtype=object)
    ok = np.isfinite(vals)
    if ok.any():
        pct = _brace_to_percent(fmt)
        if pct is not None:
            out[ok] = np.char.mod(pct, vals[ok]).astype(object)
        else:
            out[ok] = [fmt.format(float(v)) for v in vals[ok]]
    return out


def fixed_decimals(fmt: str) -> int | None:
    """N for a "{:.Nf}" / "{:f}" formatter (the forms the GPU text formatter reproduces)."""
    import re

    m = re.fullmatch(r"\{:(?:\.(\d+))?f\}", fmt)
    if not m:
        return None
    n = int(m.group(1)) if m.group(1) is not None else 6
    return n if n <= 17 else None


def gpu_text_ok(vals: np.ndarray, decimals: int | None) -> bool:
    """True when taxi2_format_rows can format every finite value exactly."""
    if decimals is None:
        return False
    fin = vals[np.isfinite(vals)]
    return fin.size == 0 or float(np.max(np.abs(fin))) * 10.0 ** decimals < 2.0 ** 62


def write_rows_gpu(fh, eng, vals, row_pre: list, col_pre, decimals: int, missing: str,
                   max_values: int = 1 << 23, stream: int | None = None) -> None:
    """Stream writer text (linear when col_pre is given, matrix otherwise) to the binary file
    ``fh`` in row chunks of about ``max_values`` values (``vals`` on the host, or a CUDA tensor
    formatted where it is, ordered on ``stream``)."""
    per_row = max(1, int(np.prod(tuple(vals.shape[1:]))))
    step = max(1, max_values // per_row)
    for r0 in range(0, vals.shape[0], step):
        r1 = min(vals.shape[0], r0 + step)
        kw = {"stream": stream} if stream is not None else {}
        fh.write(eng.format_rows(vals[r0:r1], row_pre[r0:r1], col_pre, decimals=decimals, missing=missing, view=True,
                                 **kw))


def _brace_to_percent(fmt: str) -> str | None:
    import re

    m = re.fullmatch(r"\{:(\.\d+)?([feEgG])\}", fmt)
    if not m:
        return None
    return "%" + (m.group(1) or "") + m.group(2)


def report(progress: Callable | None, caption: str, index: int, total: int) -> None:
    if progress is not None:
        progress(caption, index, total)


def seq_key(s) -> tuple:
    """Full-tuple identity used by the diagonal rule (versus_all.py:549 ``x != y``)."""
    return (s.id, s.seq, tuple(sorted(s.extras.items())) if s.extras else ())


def full_tuple_groups(seqs) -> list:
    """Indices of identical full tuples (seq_key), groups in first-appearance order.  Equal tuples
    have equal ids, so a sequence whose id occurs once is its own group without hashing its
    sequence (N = 200 000 x 1 000 bp: 0.5 s of string hashing otherwise)."""
    import gc
    from collections import Counter

    ids = [s.id for s in seqs]
    cnt = Counter(ids)
    # (N small lists: the cyclic collector would run several times over them while they are built)
    enabled = gc.isenabled()
    gc.disable()
    try:
        if len(cnt) == len(ids):
            return [[i] for i in range(len(ids))]
        groups: dict = {}
        for i, s in enumerate(seqs):
            groups.setdefault(seq_key(s) if cnt[ids[i]] > 1 else (i,), []).append(i)
        return list(groups.values())
    finally:
        if enabled:
            gc.enable()
