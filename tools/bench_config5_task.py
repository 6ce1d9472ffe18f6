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
    import numpy as np

    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.partitions import Partition
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll
    from tools.bench_configs import prealigned_rows

    if aligned:  # the config-3 generator: Gotoh alignment of every pair
        from taxi2_amd.synth import family_sequences

        buf = offs = None
        seqs = [Sequence(f"s{k}", s) for k, s in enumerate(family_sequences(n, L, 0x7A12))]
    else:
        buf, offs = prealigned_rows(n, L, 0x7A14)
        raw = buf[:-1].reshape(n, L)
        seqs = [Sequence(f"s{k}", raw[k].tobytes().decode()) for k in range(n)]
    rng = np.random.default_rng(0x7A15)
    t = VersusAll()
    t.engine, t.progress_handler, t.work_dir = eng, None, out
    t.input.sequences = Sequences(seqs)
    # two genera (the few-subsets case that used to serialise the sums) and ~1 000 species
    t.input.genera = Partition({s.id: "g%d" % (k % 2) for k, s in enumerate(seqs)})
    t.input.species = Partition({s.id: "sp%d" % int(rng.integers(0, 1000)) for s in seqs})
    t.params.pairs.align = aligned
    t.params.pairs.write = False
    t.params.distances.write_linear = t.params.distances.write_matricial = False
    t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.JukesCantor(),
                                  DistanceMetric.Kimura2P()]
    if aligned:
        t.params.distances.metrics.insert(1, DistanceMetric.UncorrectedWithGaps())
    t.params.format.percentage_multiply = True
    t.params.engine.stream = True
    t.params.engine.write_summary = False
    t.params.engine.row_minima = "p"
    t.params.engine.block_bytes = int(block_gb * (1 << 30))
    t.params.engine.timings = True
    return t, buf, offs


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
