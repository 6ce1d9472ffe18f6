#!/usr/bin/env python3
"""Ragged lengths: the packed aligner on sequences of random length (chains of consecutive pairs
break when no sequence is shared, see at_swap in alignt_kernel.hpp).  Times a triangle block and a
query x reference rectangle on device buffers; prints one JSON line each.

usage: python tools/bench_ragged.py [--lo 850] [--hi 1000] [--nseq 4000] [--batch 131072]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def packed(n: int, lo: int, hi: int, seed: int):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, size=n)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    buf = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=int(offs[-1]))]
    return np.concatenate([buf, np.zeros(1, np.uint8)]), offs


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lo", type=int, default=850)
    ap.add_argument("--hi", type=int, default=1000)
    ap.add_argument("--nseq", type=int, default=4000)
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from taxi2_amd._native import Engine

    eng = Engine(0)
    metrics = ("p", "p-gaps", "jc", "k2p")
    stream = torch.cuda.current_stream().cuda_stream
    buf, offs = packed(args.nseq, args.lo, args.hi, 0x5EED)
    st = eng.upload_packed(buf, offs, align=True)
    B = args.batch
    out = torch.empty((B, 2, 4), dtype=torch.float64, device="cuda")
    sc = torch.empty((B,), dtype=torch.int32, device="cuda")
    eng.all_pairs_dev(st, 0, B, metrics, out.data_ptr(), None, sc.data_ptr(), stream)
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(args.reps):
        t0 = time.perf_counter()
        eng.all_pairs_dev(st, 0, B, metrics, out.data_ptr(), None, sc.data_ptr(), stream)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(json.dumps({"shape": "triangle", "lens": [args.lo, args.hi], "pairs": B, "pairs_per_s": B / best}), flush=True)
    # rectangle: 64 queries x nseq references (query-major, one query against all references)
    qb, qo = packed(64, args.lo, args.hi, 0x0BE)
    qs = eng.upload_packed(qb, qo, align=True)
    R = args.nseq
    eng.rect_pairs(qs, st, 0, 64, metrics, None)  # host outputs (includes the copy back)
    best = 1e30
    for _ in range(args.reps):
        t0 = time.perf_counter()
        eng.rect_pairs(qs, st, 0, 64, metrics, None)
        best = min(best, time.perf_counter() - t0)
    print(json.dumps({"shape": "rectangle", "lens": [args.lo, args.hi], "pairs": 64 * R, "pairs_per_s": 64 * R / best}),
          flush=True)
    qs.free()
    st.free()


if __name__ == "__main__":
    main()
