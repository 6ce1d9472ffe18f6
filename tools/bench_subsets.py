#!/usr/bin/env python3
"""Subset aggregation throughput (DistanceAggregator, versus_all.py:57-96 / 617-640) on the GPU:
taxi2_subset_aggregate_dev fed the streamed row blocks of an N x N x M value matrix, as the
streamed versusAll does (VersusAll._stream_rows).  Partitions: 2 genera, ~1 000 species, ~10 000
groups (ragged sizes), random assignment.  Values are synthetic f64 in [0, 1) with ~1 % NaN
(None), generated on the device per block outside the timed region; only the aggregator calls are
timed (HIP events on the current stream).  Exactness is covered by tests/test_gpu_subsets.py.

usage: python tools/bench_subsets.py [--n 50000] [--m 4] [--block-rows 512] > profiles/r3/bench_subsets.json
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


def main() -> None:
    import torch

    from taxi2_amd._native import Engine
    from taxi2_amd.partitions import Partition
    from taxi2_amd.tasks.subsets import SubsetAggregatorDev

    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--block-rows", type=int, default=512)
    ap.add_argument("--groups", type=int, nargs="+", default=[2, 1000, 10000])
    args = ap.parse_args()
    n, m, B = args.n, args.m, args.block_rows
    eng = Engine.default()
    dev = torch.device("cuda", eng.device)
    ids = [f"s{k}" for k in range(n)]
    rng = np.random.default_rng(5)
    gen = torch.Generator(device=dev)
    stream = torch.cuda.Stream(dev)  # a real stream: every op and both events on it
    results = []
    for g in args.groups:
        # ragged group sizes: Zipf-like weights, every group non-empty when g <= n
        w = 1.0 / np.arange(1, g + 1) ** 0.8
        lab = rng.choice(g, size=n, p=w / w.sum())
        lab[:g] = np.arange(g)
        part = Partition({i: f"grp{lab[k]}" for k, i in enumerate(ids)})
        with torch.cuda.stream(stream):
            results.append(run_one(torch, dev, gen, eng, ids, part, n, m, B, SubsetAggregatorDev))
        print(json.dumps(results[-1]), file=sys.stderr, flush=True)
        torch.cuda.empty_cache()
    print(json.dumps({"bench": "subset_aggregate_dev", "results": results}))


def run_one(torch, dev, gen, eng, ids, part, n, m, B, SubsetAggregatorDev) -> dict:
    agg = SubsetAggregatorDev(eng, ids, part, m)
    gen.manual_seed(11)
    total_ms, defined = 0.0, 0
    t_wall = time.perf_counter()
    blk = torch.empty((B, n, m), dtype=torch.float64, device=dev)
    for x0 in range(0, n, B):
        x1 = min(n, x0 + B)
        D = blk[: x1 - x0]
        D.uniform_(generator=gen)
        D.masked_fill_(D < 0.01, float("nan"))
        r = torch.arange(x1 - x0, device=dev)
        D[r, r + x0] = float("nan")  # the diagonal is None (A11)
        defined += int(torch.isfinite(D).sum())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        agg.add(D, x0, x1)
        e1.record()
        e1.synchronize()
        total_ms += e0.elapsed_time(e1)
    wall = time.perf_counter() - t_wall
    st = agg.result()
    values = n * n * m
    return ({
        "groups": len(agg.subsets), "n": n, "metrics": m, "block_rows": B, "aggregate_s": total_ms / 1e3,
        "values_per_s": values / (total_ms / 1e3), "input_GB_per_s": values * 8 / (total_ms / 1e3) / 1e9,
        "wall_s_incl_generation": wall, "state_entries": int(np.prod(st.count.shape)),
        "values_counted": int(st.count.sum()), "values_defined": defined,
    })


if __name__ == "__main__":
    main()
