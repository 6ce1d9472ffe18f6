#!/usr/bin/env python3
"""Secondary workloads of BASELINE.json on one MI355X (bench.py keeps the headline config 3).

  config2: versusAll, pre-aligned p / jc / k2p.  samples/Taxi2test1_ca9000.tab is missing from the
           reference; stand-in = 9 000 synthetic pre-aligned 600-column rows
           (lowercase acgt, 2 % '-' runs, 0.5 % 'n'), the full 4.05e7-pair space.
  config5: versusAll pre-aligned p / jc / k2p at FULL size on one GPU: N = 200 000 synthetic
           1 000-column rows (seed 0x7A14), all 2.0e10 unordered pairs in 2^26-pair blocks whose
           outputs are overwritten in HBM (the multi-GPU task streams such blocks to rank 0, §6).
  config4: versusReference, align + p (closest reference per query, extras p-gaps / jc / k2p for
           the argmin pair), Q x R with R = 10 000 references of 650 bp (seed 0x7A13 generator);
           a Q slice is timed and pairs/s = Q_slice x R / time (the full 1e6 x 1e4 job scales
           linearly in Q).

Prints one JSON line per workload.  Inputs are uploaded before timing; outputs stay on the GPU
(config2) or come back as the closest-pair vectors (config4, what the task consumes).
usage: python tools/bench_configs.py [--config2] [--config4] [--config5] [--q-slice 1024]
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


def prealigned_rows(n: int, L: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    from bench_secondary import prealigned_rows as rows

    return rows(n, L, seed)


def config2(eng, steps: int) -> dict:
    import torch

    n, L = 9000, 600
    buf, offs = prealigned_rows(n, L, 0x7A12)
    st = eng.upload_packed(buf, offs, align=False)
    total = n * (n - 1) // 2
    metrics = ("p", "jc", "k2p")
    B = 1 << 22
    out = torch.empty((B, len(metrics)), dtype=torch.float64, device="cuda")
    stream = torch.cuda.Stream()
    eng.all_pairs_dev(st, 0, min(B, total), metrics, out.data_ptr(), None, None, stream.cuda_stream)
    stream.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for k0 in range(0, total, B):
            c = min(B, total - k0)
            eng.all_pairs_dev(st, k0, c, metrics, out.data_ptr(), None, None, stream.cuda_stream)
    stream.synchronize()
    dt = (time.perf_counter() - t0) / steps
    bp = 2 * ((L + 3) // 4) + 8 * len(metrics)
    return {"workload": "config2 stand-in: versusAll 9 000 x 600 pre-aligned, p/jc/k2p, full pair space",
            "pairs": total, "seconds": dt, "pairs_per_s": total / dt,
            "algorithmic_GBps": total * bp / dt / 1e9, "hbm_frac": total * bp / dt / 8e12}


def config5(eng) -> dict:
    import torch

    n, L = 200_000, 1000
    buf, offs = prealigned_rows(n, L, 0x7A14)
    st = eng.upload_packed(buf, offs, align=False)
    del buf
    total = n * (n - 1) // 2
    metrics = ("p", "jc", "k2p")
    B = 1 << 26
    out = torch.empty((B, len(metrics)), dtype=torch.float64, device="cuda")
    stream = torch.cuda.Stream()
    eng.all_pairs_dev(st, 0, B, metrics, out.data_ptr(), None, None, stream.cuda_stream)
    stream.synchronize()
    t0 = time.perf_counter()
    for k0 in range(0, total, B):
        c = min(B, total - k0)
        eng.all_pairs_dev(st, k0, c, metrics, out.data_ptr(), None, None, stream.cuda_stream)
    stream.synchronize()
    dt = time.perf_counter() - t0
    bp = 2 * ((L + 3) // 4) + 8 * len(metrics)
    return {"workload": "config5 pre-aligned at full size: versusAll 200 000 x 1 000 pre-aligned, p/jc/k2p, "
                        "all unordered pairs on ONE GPU (outputs overwritten per 2^26-pair block)",
            "pairs": total, "seconds": dt, "pairs_per_s": total / dt,
            "algorithmic_GBps": total * bp / dt / 1e9, "hbm_frac": total * bp / dt / 8e12}


def config4(eng, q_slice: int, steps: int) -> dict:
    from taxi2_amd.synth import family_sequences

    R, L = 10_000, 650
    refs = family_sequences(R, L, 0x7A13)
    qs = family_sequences(q_slice, L, 0x7A13 + 1)
    sq = eng.upload(qs, align=True)
    sr = eng.upload(refs, align=True)
    extras = ("p-gaps", "jc", "k2p")
    eng.closest(sq, sr, 0, min(8, q_slice), "p", extras)
    t0 = time.perf_counter()
    for _ in range(steps):
        idx, d, ex, _ = eng.closest(sq, sr, 0, q_slice, "p", extras)
    dt = (time.perf_counter() - t0) / steps
    pairs = q_slice * R
    return {"workload": f"config4 slice: versusReference {q_slice} queries x {R} refs x {L} bp, Gotoh align + p, "
                        f"closest + extras on the GPU", "pairs": pairs, "seconds": dt, "pairs_per_s": pairs / dt,
            "gcups": pairs * L * L / dt / 1e9, "full_job_hours_1gpu": 1e10 / (pairs / dt) / 3600}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config2", action="store_true")
    ap.add_argument("--config4", action="store_true")
    ap.add_argument("--config5", action="store_true")
    ap.add_argument("--q-slice", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    if not (args.config2 or args.config4 or args.config5):
        args.config2 = args.config4 = True
    import torch  # noqa: F401  -- before the engine: torch's bundled HIP runtime must load first

    from taxi2_amd._native import Engine

    eng = Engine(0)
    if args.config2:
        print(json.dumps(config2(eng, args.steps)), flush=True)
    if args.config4:
        print(json.dumps(config4(eng, args.q_slice, args.steps)), flush=True)
    if args.config5:
        print(json.dumps(config5(eng)), flush=True)


if __name__ == "__main__":
    main()
