#!/usr/bin/env python3
"""Task-level throughput with the reference's defaults: VersusAll.start() (versus_all.py:374-773,
Results.seconds_taken) on N synthetic 1 000 bp sequences (the config-3 generator), align = True,
the four default metrics, aligned_pairs.txt, linear.tsv, matricial/*.tsv and summary.tsv all ON
(versus_all.py:389-397), one GPU.  Wall time split by phase (task.timings): compute (alignment +
metrics, incl. D2H of the N x N x 4 matrix), aligned-pairs text (GPU formatter + file write), and
each writer.

By default the output files point at /dev/null (symlinks made before start()): the text is still
produced and written through the file API, only the disk is taken out (aligned_pairs.txt alone is
~2.2 KB per ordered pair: 55 GB at N = 5 000).

usage: python tools/bench_task.py [--n 5000 10000] [--files] > profiles/r3/bench_task.json
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

NULL_FILES = ("align/aligned_pairs.txt", "distances/linear.tsv", "summary.tsv", "distances/matricial/p.tsv",
              "distances/matricial/p-gaps.tsv", "distances/matricial/jc.tsv", "distances/matricial/k2p.tsv")


def run(n: int, eng, null: bool) -> dict:
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.synth import family_sequences
    from taxi2_amd.tasks import VersusAll

    seqs = [Sequence(f"seq{k}", s) for k, s in enumerate(family_sequences(n, 1000, 0x7A12))]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as tmp:
        out = Path(tmp)
        if null:
            for f in NULL_FILES:
                (out / f).parent.mkdir(parents=True, exist_ok=True)
                os.symlink("/dev/null", out / f)
        t = VersusAll()
        last = [time.perf_counter()]

        def progress(caption, index, total):  # a line every ~20 s (long runs must keep writing)
            now = time.perf_counter()
            if now - last[0] > 20.0:
                last[0] = now
                print(f"n={n}: {caption} {index}/{total}", file=sys.stderr, flush=True)

        t.engine, t.progress_handler, t.work_dir = eng, progress, out
        t.input.sequences = Sequences(seqs)
        t0 = time.perf_counter()
        res = t.start()
        wall = time.perf_counter() - t0
        sizes = {str(p.relative_to(out)): p.stat().st_size for p in out.rglob("*") if p.is_file() and not p.is_symlink()}
    pairs = n * (n - 1) // 2
    return {"n": n, "seconds": wall, "seconds_taken": res.seconds_taken, "unordered_pairs": pairs,
            "ordered_pairs": n * n, "task_pairs_per_s": pairs / wall, "phases_s": t.timings,
            "pairs_from_walks": bool(t.pairs_walked), "null_outputs": null, "file_bytes": sizes}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[5000, 10000])
    ap.add_argument("--files", action="store_true",
                    help="write real files (default: /dev/null symlinks; N = 10 000 is ~240 GB of text)")
    args = ap.parse_args()
    args.null = not args.files
    import torch  # noqa: F401  -- torch's HIP runtime first (Engine shares it)

    from taxi2_amd._native import Engine

    eng = Engine(0)
    for n in args.n:
        print(json.dumps({"workload": "VersusAll.start() with reference defaults (align, 4 metrics, aligned_pairs, "
                                      "linear, matricial, summary), config-3 generator, 1 000 bp", **run(n, eng, args.null)}),
              flush=True)


if __name__ == "__main__":
    main()
