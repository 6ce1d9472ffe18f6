#!/usr/bin/env python3
"""Long sequences: the default dispatch (packed trace-and-walk up to 2 048 columns, forward-carry
k_align1c to 4 095 bp, column-tiled k_alignlong beyond) against the forward-carry kernels
(TAXI2_NO_ALIGNT=1, <= 4 095 bp) and the column-tiled aligner forced (TAXI2_LONG=1), on the
config-3 generator, same pairs, outputs compared bit for bit.  One JSON line per length.

usage: python tools/bench_long.py [--lens 1200 1500 2000] [--batch 16384] [--nseq 4000]
"""

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


def run(eng, st, k0, batch, env, out, scores):
    import torch

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        stream = torch.cuda.current_stream()
        eng.all_pairs_dev(st, k0, batch, ("p", "p-gaps", "jc", "k2p"), out.data_ptr(), None, scores.data_ptr(),
                          stream.cuda_stream)  # warm-up (allocations)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.all_pairs_dev(st, k0, batch, ("p", "p-gaps", "jc", "k2p"), out.data_ptr(), None, scores.data_ptr(),
                          stream.cuda_stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", type=int, nargs="+", default=[1200, 1500, 2000])
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--nseq", type=int, default=4000)
    args = ap.parse_args()
    import torch

    from taxi2_amd._native import Engine
    from taxi2_amd.synth import family_packed

    eng = Engine(0)
    for L in args.lens:
        buf, offs = family_packed(args.nseq, L, 0x7A12)
        st = eng.upload_packed(buf, offs, align=True)
        B = args.batch
        outs, times = {}, {}
        envs = {"default": {}, "tiled": {"TAXI2_LONG": "1"}}
        if L <= 4095:
            envs["forward_carry"] = {"TAXI2_NO_ALIGNT": "1"}
        for name, env in envs.items():
            out = torch.empty((B, 2, 4), dtype=torch.float64, device="cuda")
            sc = torch.empty((B,), dtype=torch.int32, device="cuda")
            times[name] = run(eng, st, 0, B, env, out, sc)
            outs[name] = (out.cpu().numpy(), sc.cpu().numpy())
        ref = outs["default"]
        same = all(bool(np.array_equal(np.nan_to_num(o[0], nan=9.0), np.nan_to_num(ref[0], nan=9.0))
                        and np.array_equal(o[1], ref[1])) for o in outs.values())
        rec = {"len": L, "pairs": B, "identical": same}
        for name, t in times.items():
            rec[f"{name}_pairs_per_s"] = B / t
            rec[f"{name}_gcups"] = B * L * L / t / 1e9
        print(json.dumps(rec), flush=True)
        st.free()


if __name__ == "__main__":
    main()
