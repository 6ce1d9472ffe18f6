#!/usr/bin/env python3
"""NCD throughput: raw-mode ncd_pairs (both orders: 6 compressed streams per unordered pair) on
1 000 bp synthetic family sequences, vs the CPU (Python zlib, one core) on a sample."""

from __future__ import annotations

import json
import sys
import time
import zlib
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    import torch  # noqa: F401  (HIP runtime load order, see _native.Engine)

    from taxi2_amd._native import Engine, tri_pairs
    from taxi2_amd.synth import family_sequences

    n = 400
    seqs = family_sequences(n, 1000, 0x7A12)
    eng = Engine(0)
    st = eng.upload(seqs, align=False)
    a, b = tri_pairs(n)
    eng.ncd_pairs(st, st, a[:64], b[:64], aligned=False, both=True)
    t0 = time.perf_counter()
    got = eng.ncd_pairs(st, st, a, b, aligned=False, both=True)
    dt = time.perf_counter() - t0
    S = 300
    t1 = time.perf_counter()
    for k in range(S):
        x, y = seqs[a[k]].encode(), seqs[b[k]].encode()
        c1, c2 = len(zlib.compress(x)), len(zlib.compress(y))
        for u, v in ((x, y), (y, x)):
            c12 = len(zlib.compress(u + v))
            _ = (c12 - min(c1, c2)) / max(c1, c2)
    cpu = S / (time.perf_counter() - t1)
    print(json.dumps({"workload": f"NCD raw, {len(a)} unordered pairs x 2 orders, 1 000 bp", "gpu_pairs_per_s": len(a) / dt,
                      "gpu_seconds": dt, "cpu_pairs_per_s_1core": cpu, "finite": bool(np.isfinite(got).all())}))


if __name__ == "__main__":
    main()
