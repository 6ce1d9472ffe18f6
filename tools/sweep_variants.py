#!/usr/bin/env python3
"""A/B the aligner's kernel shapes (K columns per lane, W waves per pair, OCC waves/SIMD) in one
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Every variant's outputs are
compared bit-for-bit with the first variant's.

usage: python tools/sweep_variants.py [--batch 131072] [--rounds 3] [--len 1000] K,W,OCC ...
(K,W,OCC = single-orientation kernel shape; o:K,W,OCC = two-orientation kernel shape)
"""

from __future__ import annotations

import argparse
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--batch", type=int, default=1 << 17)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--len", type=int, default=1000)
    ap.add_argument("--nseq", type=int, default=50000)
    ap.add_argument("--scores", default="1,-1,-8,-1,-1,-1")
    ap.add_argument("--lib", default=None, help="A/B another build of the engine library")
    args = ap.parse_args()
    import torch

    from taxi2_amd import _native
    from taxi2_amd._native import Engine

    if args.lib:
        _native.LIB_PATH = Path(args.lib).resolve()
    from taxi2_amd.synth import family_packed

    metrics = ("p", "p-gaps", "jc", "k2p")
    sc = tuple(int(v) for v in args.scores.split(","))
    buf, offs = family_packed(args.nseq, args.len, 0x7A12)
    eng = Engine(0)
    st = eng.upload_packed(buf, offs, align=True)
    B = args.batch
    out = torch.empty((B, 2, 4), dtype=torch.float64, device="cuda")
    sco = torch.empty((B,), dtype=torch.int32, device="cuda")
    stream = torch.cuda.Stream()
    ref = None
    times = {v: [] for v in args.variants}
    for rnd in range(args.rounds):
        for v in args.variants:
            if v.startswith("o:"):  # two-orientation kernel
                os.environ["TAXI2_NO_ALIGN1"] = "1"
                os.environ["TAXI2_VARIANT"] = v[2:]
            else:  # single-orientation kernel (sequences <= 1023)
                os.environ.pop("TAXI2_NO_ALIGN1", None)
                os.environ["TAXI2_VARIANT1"] = v
            k0 = (rnd * 7919 * B) % (args.nseq * (args.nseq - 1) // 2 - B)
            eng.all_pairs_dev(st, k0, B, metrics, out.data_ptr(), sc, sco.data_ptr(), stream.cuda_stream)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            eng.all_pairs_dev(st, k0, B, metrics, out.data_ptr(), sc, sco.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            stream.synchronize()
            times[v].append(e0.elapsed_time(e1) / 1e3)
            if rnd == 0:
                res = (out.cpu().numpy().copy(), sco.cpu().numpy().copy())
                if ref is None:
                    ref = res
                else:
                    same = np.array_equal(res[1], ref[1]) and np.array_equal(
                        np.nan_to_num(res[0], nan=7.0), np.nan_to_num(ref[0], nan=7.0))
                    print(f"{v}: outputs identical to {args.variants[0]}: {same}", flush=True)
    for v in args.variants:
        t = np.array(times[v])
        print(f"{v:>10}  median {B / np.median(t):12.0f} pairs/s   min-time {B / t.min():12.0f} pairs/s   "
              f"GCUPS {B * args.len * args.len / np.median(t) / 1e9:8.1f}", flush=True)


if __name__ == "__main__":
    main()
