#!/usr/bin/env python3
"""Writer text throughput: GPU formatter (taxi2_format_rows) vs the numpy/Python path, on an
N x N x M distance table (N = 2000, M = 3, '{:.4f}', 'NA'), linear (WithExtras-shaped rows)."""

from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    from taxi2_amd._native import Engine
    from taxi2_amd.tasks.common import format_values, write_rows_gpu

    n, M = 2000, 3
    D = np.random.default_rng(0).random((n, n, M)) * 0.3
    D[::7, ::5, 1] = np.nan
    pre = [f"seq{i}\tvoucher{i}\torganism {i}" for i in range(n)]
    eng = Engine(0)
    eng.format_rows(D[:2], pre[:2], pre, decimals=4)  # warm-up
    t0 = time.perf_counter()
    with open("/tmp/lin_gpu.tsv", "wb") as fh:
        write_rows_gpu(fh, eng, D, pre, pre, 4, "NA")
    t_gpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    text = format_values(D, "{:.4f}", "NA")
    with open("/tmp/lin_py.tsv", "w") as fh:
        for i in range(n):
            fh.write("\n".join("\t".join((pre[i], pre[j], *text[i, j])) for j in range(n)) + "\n")
    t_py = time.perf_counter() - t0
    same = Path("/tmp/lin_gpu.tsv").read_bytes() == Path("/tmp/lin_py.tsv").read_bytes()
    size = Path("/tmp/lin_gpu.tsv").stat().st_size
    print(json.dumps({"workload": f"linear writer text, {n}x{n}x{M} values", "bytes": size,
                      "gpu_seconds": t_gpu, "python_seconds": t_py, "speedup": t_py / t_gpu,
                      "gpu_MB_per_s": size / t_gpu / 1e6, "identical": same}))


if __name__ == "__main__":
    main()
