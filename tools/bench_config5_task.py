#!/usr/bin/env python3
"""Config 5 through the task path: VersusAll.start() on 200 000 x 1 000 pre-aligned synthetic
sequences (BASELINE.json configs[4], the pre-aligned p / jc / k2p form SURVEY.md §8(d) asks to
run at full size), reductions only -- per-sequence closest other sequence (params.engine.row_minima)
and the genus / species subset statistics -- with per-phase wall times (params.engine.timings).

Every one of the N^2 = 4e10 ordered pairs is evaluated (the streamed pre-aligned path computes
x-major row blocks with the tiled kernel) and reduced on the GPU; nothing N^2 leaves HBM.

usage: python tools/bench_config5_task.py [--n 200000] [--len 1000] [--block-gb 2] > profiles/r3/config5_task.json
       (under torch.distributed.run with N ranks: the sharded reductions chain)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def build_task(n: int, L: int, eng, out: Path, block_gb: float, aligned: bool = False):
    from bench_secondary import build_config5_task

    return build_config5_task(n, L, eng, out, block_gb, aligned)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--len", type=int, default=1000)
    ap.add_argument("--block-gb", type=float, default=2.0)
    ap.add_argument("--aligned", action="store_true",
                    help="config-3 sequences, Gotoh alignment + p / p-gaps / jc / k2p (the aligned form of config 5)")
    args = ap.parse_args()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from taxi2_amd._native import Engine

    eng = Engine(local)
    with tempfile.TemporaryDirectory() as tmp:
        t0 = time.perf_counter()
        task, _, _ = build_task(args.n, args.len, eng, Path(tmp), args.block_gb, args.aligned)
        t_build = time.perf_counter() - t0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = task.start()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        files = sorted(str(p.relative_to(tmp)) for p in Path(tmp).rglob("*") if p.is_file())
    n = args.n
    if local == 0:
        print(json.dumps({
            "workload": (f"config5 task path: VersusAll.start() on {n} x {args.len} " +
                         ("config-3 synthetic sequences (seed 0x7A12), Gotoh align + p/p-gaps/jc/k2p"
                          if args.aligned else "pre-aligned synthetic sequences (seed 0x7A14), p/jc/k2p") +
                         " x100, reductions only: row minima + 2-genus and ~1 000-species subset statistics "
                         "(exact x-major sums)"),
            "n_seqs": n, "ordered_pairs": n * n, "unordered_pairs": n * (n - 1) // 2,
            "ranks": world, "start_seconds": wall, "results_seconds_taken": res.seconds_taken,
            "ordered_pairs_per_s": n * n / wall, "unordered_pairs_per_s": n * (n - 1) / 2 / wall,
            "phases_s": task.timings, "input_build_s": t_build, "files": files,
        }), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
