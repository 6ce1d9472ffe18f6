#!/usr/bin/env python3
"""Debug helper: the packed aligner against the forward-carry kernels (TAXI2_NO_ALIGNT=1) on the
random-bucket inputs of tests/test_gpu_parity.py, several repetitions, printing every pair whose
score or metrics differ (pair, lengths, both values).  No oracle: the forward-carry path is the
reference here.

usage: python tools/debug_at2.py [--bucket 900 1024] [--scores default] [--reps 3]
"""

from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bucket", type=int, nargs="+", default=[900, 1024], help="lo hi [lo hi ...], in order")
    ap.add_argument("--scores", default="default")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--host", action="store_true", help="host-buffer entry point instead of device buffers")
    args = ap.parse_args()
    import torch

    torch.cuda.init()  # before the library's own HIP context
    from taxi2_amd._native import Engine

    eng = Engine(0)
    bl = args.bucket
    for lo, hi in zip(bl[0::2], bl[1::2]):
        print(f"### bucket {lo} {hi}", flush=True)
        one(eng, lo, hi, args, torch)


def dev_run(eng, st, total, METRICS, sc, torch):
    # device outputs pre-filled with a sentinel: a pair the kernel never writes shows as such
    out = torch.full((total, 2, len(METRICS)), -7.0, dtype=torch.float64, device="cuda")
    osc = torch.full((total,), 0x7FFF0000, dtype=torch.int32, device="cuda")
    eng.all_pairs_dev(st, 0, total, METRICS, out.data_ptr(), sc, osc.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got, gsc = out.cpu().numpy(), osc.cpu().numpy()
    print(f"unwritten scores {int((gsc == 0x7FFF0000).sum())}, unwritten metric slots {int((got == -7.0).sum())}",
          flush=True)
    return got, gsc


def one(eng, lo, hi, args, torch):
    from taxi2_amd._native import tri_pairs
    from tests.seqgen import mutate, random_sequences
    from tests.test_gpu_parity import METRICS, SCORE_SETS

    n = 10 if hi > 1100 else 16
    seed = hash((lo, hi, args.scores)) & 0xFFFF
    base = random_sequences(n // 2, lo, hi, seed, "ACGT", n_rate=0.02)
    seqs = base + mutate(base, seed + 1, rate=0.15)
    seqs = [s if s else "A" for s in seqs]
    sc = SCORE_SETS[args.scores]
    st = eng.upload(seqs, align=True)
    total = n * (n - 1) // 2
    a, b = tri_pairs(n)
    runs = []
    for rep in range(args.reps):  # packed runs first: no forward-carry results left in the buffers
        if args.host:  # host-buffer path (taxi2_all_pairs), as the tests call it
            runs.append(eng.all_pairs(st, 0, total, METRICS, sc, with_scores=True))
        else:
            runs.append(dev_run(eng, st, total, METRICS, sc, torch))
    os.environ["TAXI2_NO_ALIGNT"] = "1"
    ref, rsc = eng.all_pairs(st, 0, total, METRICS, sc, with_scores=True)
    del os.environ["TAXI2_NO_ALIGNT"]
    for rep, (got, gsc) in enumerate(runs):
        bad_s = np.nonzero(gsc != rsc)[0]
        bad_m = np.nonzero(~np.all(np.nan_to_num(got, nan=9.0) == np.nan_to_num(ref, nan=9.0), axis=(1, 2)))[0]
        print(f"rep {rep}: {len(bad_s)} score mismatches, {len(bad_m)} metric mismatches", flush=True)
        for p in sorted(set(bad_s.tolist()) | set(bad_m.tolist()))[:40]:
            print(f"  pair {p} ({a[p]},{b[p]}) lens {len(seqs[a[p]])},{len(seqs[b[p]])} score {gsc[p]} (0x{int(gsc[p]) & 0xffffffff:08x})"
                  f" vs {rsc[p]}  metrics {got[p].ravel().tolist()} vs {ref[p].ravel().tolist()}", flush=True)
    st.free()


if __name__ == "__main__":
    main()
