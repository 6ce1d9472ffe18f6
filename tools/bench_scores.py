#!/usr/bin/env python3
"""Aligned pairs/s of the config-3 workload (50 000 x 1 000 bp, the bench's generator and pair
blocks) under other alignment scores than TaxI2's default (align.py:20-27): a generic Gotoh set
(the packed aligner's non-default variant: per-column extend constants, sign-digit trace), one-extend
sets (round 6: the row-shared k_alignr, and the same set forced onto k_alignt2) and a linear set (open == extend: the NW kernels).  Same metrics as bench.py, HIP events on the launch
stream; not the headline (bench.py), a map of what other scores cost.

usage: python tools/bench_scores.py [--batch 131072] [--steps 3] > profiles/r3/bench_scores.json
"""

from __future__ import annotations

import argparse
import json
import os
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

SETS = {
    "default": (1, -1, -8, -1, -1, -1),
    "generic": (2, -3, -5, -2, -1, -1),
    "generic1": (2, -3, -5, -2, -3, -2),  # one extend: k_alignr (round 6)
    "generic1_alignt2": (2, -3, -5, -2, -3, -2),  # the same set on k_alignt2 (rounds 3-5)
    "small1": (1, -2, -4, -1, -2, -1),  # other one-extend sets (k_alignr)
    "equal_opens": (3, -1, -6, -2, -6, -2),
    "free_ends": (5, -4, -10, -3, -3, -3),
    "linear": (1, -1, -2, -2, -2, -2),
}
ENV = {"generic1_alignt2": {"TAXI2_NO_ALIGNR_GEN": "1"}}


def _stderr_of(fn) -> str:
    """What the C library writes to fd 2 while fn runs."""
    import tempfile

    sys.stderr.flush()
    saved = os.dup(2)
    with tempfile.TemporaryFile(mode="w+b") as tf:
        os.dup2(tf.fileno(), 2)
        try:
            fn()
        finally:
            os.dup2(saved, 2)
            os.close(saved)
        tf.seek(0)
        return tf.read().decode(errors="replace")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 19)  # bench.py's block
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--sets", default=os.environ.get("BENCH_SCORE_SETS", ",".join(SETS)), help="comma-separated subset of the score sets")
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

    for name in re.split(r"[,+]", args.sets):
        sc = SETS[name]
        for k in ("TAXI2_NO_ALIGNR_GEN",):
            os.environ.pop(k, None)
        os.environ.update(ENV.get(name, {}))
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
        # one more (untimed) launch with the band statistics: kernel and pairs requeued to the full trace
        os.environ["TAXI2_AT_BAND_STATS"] = "1"
        err = _stderr_of(lambda: (eng.all_pairs_dev(st, 0, B, METRICS, out.data_ptr(), sc, None, stream.cuda_stream),
                                  stream.synchronize()))
        os.environ.pop("TAXI2_AT_BAND_STATS", None)
        q = re.findall(r"band: (k_\w+)<[^>]*> band \d+: (\d+) of", err)
        print(json.dumps({"scores": name, "values": sc, "pairs": B * args.steps, "kernel_s": ms / 1e3,
                          "pairs_per_s": B * args.steps / (ms / 1e3), "kernel": sorted({k for k, _ in q}),
                          "requeued": sum(int(n) for _, n in q)}), flush=True)


if __name__ == "__main__":
    main()
