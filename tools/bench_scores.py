#!/usr/bin/env python3
"""Aligned pairs/s of the config-3 workload (50 000 x 1 000 bp, the bench's generator and pair
blocks) under other alignment scores than TaxI2's default (align.py:20-27): a generic Gotoh set
(the packed aligner's non-default variant: per-column extend constants, sign-digit trace) and a
linear set (open == extend: the NW kernels).  Same metrics as bench.py, HIP events on the launch
stream; not the headline (bench.py), a map of what other scores cost.

usage: python tools/bench_scores.py [--batch 131072] [--steps 3] > profiles/r3/bench_scores.json
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

SETS = {
    "default": (1, -1, -8, -1, -1, -1),
    "generic": (2, -3, -5, -2, -1, -1),
    "generic1": (2, -3, -5, -2, -3, -2),  # one extend: the best-open fill
    "linear": (1, -1, -2, -2, -2, -2),
}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from bench import METRICS, N_SEQS, SEED, SEQ_LEN
    from taxi2_amd._native import Engine
    from taxi2_amd.synth import family_packed

    buf, offs = family_packed(N_SEQS, SEQ_LEN, SEED)
    eng = Engine(0)
    st = eng.upload_packed(buf, offs, align=True)
    B, M = args.batch, len(METRICS)
    out = torch.empty((B, 2, M), dtype=torch.float64, device="cuda")
    stream = torch.cuda.Stream()
    for name, sc in SETS.items():
        eng.all_pairs_dev(st, 0, B, METRICS, out.data_ptr(), sc, None, stream.cuda_stream)  # warm-up
        stream.synchronize()
        ms = 0.0
        for s in range(args.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            eng.all_pairs_dev(st, (s + 1) * B, B, METRICS, out.data_ptr(), sc, None, stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            ms += e0.elapsed_time(e1)
        print(json.dumps({"scores": name, "values": sc, "pairs": B * args.steps, "kernel_s": ms / 1e3,
                          "pairs_per_s": B * args.steps / (ms / 1e3)}), flush=True)


if __name__ == "__main__":
    main()
