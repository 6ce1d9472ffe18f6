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
