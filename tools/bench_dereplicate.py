#!/usr/bin/env python3
"""Dereplicate end to end on the GPU (tasks/dereplicate.py): N COI-like sequences (~650 bp) in
clusters of near-identical variants (0-2% substitutions, a few bp trimmed), default parameters
(p-distance, similarity 0.07, aligned), timed per phase:
  distances  -- every ordered pair on the GPU (pair_matrix)
  walk       -- the native greedy walk (taxi2_dereplicate_walk)
  task       -- the whole task with its files (summary, sequences, linear + matrix distances,
                aligned_pairs.txt only with --pairs)
and, for scale, the C oracle's single-core time per aligned pair on a sample of the kept pairs
times the number of kept pairs (the reference aligns and measures exactly those, one by one)."""

from __future__ import annotations

import argparse
import json
import random
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def make(n: int, seed: int = 0):
    from taxi2_amd.sequences import Sequence

    rng = random.Random(seed)
    out = []
    while len(out) < n:
        base = "".join(rng.choice("ACGT") for _ in range(650))
        for v in range(rng.randint(1, 8)):
            s = list(base)
            for _ in range(rng.randint(0, 13)):
                s[rng.randrange(len(s))] = rng.choice("ACGT")
            a, b = rng.randint(0, 5), rng.randint(0, 5)
            out.append(Sequence(f"s{len(out)}", "".join(s[a : len(s) - b]), {"organism": f"org{len(out) % 97}"}))
    rng.shuffle(out)
    return out[:n]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--pairs", action="store_true", help="also write aligned_pairs.txt")
    ap.add_argument("--cpu-sample", type=int, default=300)
    args = ap.parse_args()

    import torch  # noqa: F401  (HIP runtime load order, see _native.Engine)

    from taxi2_amd._native import Engine, dereplicate_walk
    from taxi2_amd.align import Scores
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequences
    from taxi2_amd.tasks import Dereplicate
    from taxi2_amd.tasks.dereplicate import pair_matrix

    data = make(args.n)
    eng = Engine(0)
    scores = Scores().as_tuple()
    work = [s.normalize() for s in data]
    st = eng.upload([s.seq for s in work], align=True)
    warm = eng.upload([s.seq for s in work[:64]], align=True)
    pair_matrix(eng, warm, DistanceMetric.Uncorrected(), True, scores)
    warm.free()
    t0 = time.perf_counter()
    D = pair_matrix(eng, st, DistanceMetric.Uncorrected(), True, scores)
    t_dist = time.perf_counter() - t0
    t0 = time.perf_counter()
    w = dereplicate_walk(D, np.arange(args.n), [len(s.seq) for s in data], 0.07)
    t_walk = time.perf_counter() - t0
    st.free()
    kept = int(w.row_kept.sum())

    with tempfile.TemporaryDirectory() as tmp:
        task = Dereplicate()
        task.engine = eng
        task.progress_handler = None
        task.work_dir = Path(tmp) / "out"
        task.input = Sequences(data)
        task.params.pairs.write = args.pairs
        t0 = time.perf_counter()
        task.start()
        t_task = time.perf_counter() - t0
        sizes = {p.name: p.stat().st_size for p in Path(task.work_dir).rglob("*") if p.is_file()}

    from oracle import oracle_c

    oracle_c.build()
    rows = np.repeat(np.arange(args.n), w.row_kept)
    rng = np.random.default_rng(0)
    pick = rng.choice(kept, size=min(args.cpu_sample, kept), replace=False)
    seqs = [s.seq for s in work]
    t0 = time.perf_counter()
    oracle_c.batch(seqs, rows[pick], w.kept_cols[pick].astype(np.int64), align=True, scores=scores, metrics=("p",),
                   threads=1)
    per_pair = (time.perf_counter() - t0) / len(pick) / 2  # batch does both orientations
    print(json.dumps({
        "workload": f"Dereplicate, {args.n} x ~650 bp in near-identical clusters, p, similarity 0.07",
        "n": args.n, "ordered_pairs": args.n * (args.n - 1), "kept_pairs": kept, "summary_lines": len(w.line_idx),
        "excluded": int(w.excluded.sum()), "distances_s": t_dist, "walk_s": t_walk, "task_s": t_task,
        "aligned_pairs_written": args.pairs, "files": sizes,
        "cpu_oracle_s_per_pair_1core": per_pair, "cpu_oracle_est_s_kept_1core": per_pair * kept,
    }))


if __name__ == "__main__":
    main()
