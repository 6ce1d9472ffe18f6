#!/usr/bin/env python3
"""Linear (open == extend) scores: forward-carry two-orientation kernel (k_align, default up to
4 095 bp) vs the column-tiled NW trace-and-walk kernel (k_alignlong<LIN>, TAXI2_LONG=1), same pairs,
identical outputs required.  usage: python tools/bench_linear.py [--lens 600 1000 2000]"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", type=int, nargs="+", default=[600, 1000, 2000])
    ap.add_argument("--batch", type=int, default=16384)
    args = ap.parse_args()
    import torch  # noqa: F401

    from taxi2_amd._native import Engine
    from taxi2_amd.synth import family_sequences

    eng = Engine(0)
    sc = (1, -1, -2, -2, -1, -1)
    metrics = ("p", "p-gaps", "jc", "k2p")
    for L in args.lens:
        seqs = family_sequences(400, L, 0x7A12 + L)
        st = eng.upload(seqs, align=True)
        res = {}
        outs = {}
        for name, env in (("forward_carry", {}), ("tiled_nw", {"TAXI2_LONG": "1"})):
            os.environ.pop("TAXI2_LONG", None)
            os.environ.update(env)
            eng.all_pairs(st, 0, 256, metrics, sc)
            t0 = time.perf_counter()
            outs[name] = eng.all_pairs(st, 0, args.batch, metrics, sc)
            res[name] = args.batch / (time.perf_counter() - t0)
        os.environ.pop("TAXI2_LONG", None)
        same = np.array_equal(np.nan_to_num(outs["forward_carry"], nan=9.0), np.nan_to_num(outs["tiled_nw"], nan=9.0))
        print(json.dumps({"len": L, "pairs": args.batch, "identical": bool(same),
                          **{f"{k}_pairs_per_s": v for k, v in res.items()}}), flush=True)
        st.free()


if __name__ == "__main__":
    main()
