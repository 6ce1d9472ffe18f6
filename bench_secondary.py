"""Secondary workloads bench.py measures after its headline line's timed region (one GPU, rank 0).

The headline (bench.py) is BASELINE.json's metric on config 3: the aligner over config-3 pairs with
four metrics, outputs resident in HBM.  These legs put the other numbers the driver should observe
into the same record (bench.py's ``secondary`` key), each on its own synthetic, seeded workload:

* ``task``: VersusAll.start() with the reference's defaults (versus_all.py:389-397: align, the four
  metrics, aligned_pairs.txt, linear.tsv, the matricial files, summary.tsv) on N = 5 000 config-3
  sequences, timed as the reference times it (Results.seconds_taken, versus_all.py:732-773), split by
  phase (task.timings).  The text files are written through the file API into /dev/null symlinks in
  a temporary directory (aligned_pairs.txt alone is ~55 GB at N = 5 000); their sizes are counted.
* ``config5``: VersusAll.start() on 200 000 x 1 000 pre-aligned rows (BASELINE.json configs[4], one
  GPU), p / jc / k2p x100, reductions only (row minima + 2-genus / ~1 000-species subset statistics):
  every one of the 4e10 ordered pairs evaluated and reduced on the GPU.
* ``config4``: versusReference slice, 4 096 queries x 10 000 references of 650 bp (seed 0x7A13
  generator), Gotoh align + p, closest reference + extras on the GPU (versus_reference.py:184-188,
  124-129).
* ``allmetrics``: config 3 with ALL metrics (BASELINE.json configs[2], "+ncd"): p / p-gaps / jc / k2p
  from the aligner and NCD of the aligned strings (distances.py:351-358, three zlib streams per
  ordered pair) on a block of config-3 pairs.

Every leg prints a progress line to stderr and returns a dict (or {"error": ...}: a failing leg never
takes the headline line with it).
"""

from __future__ import annotations

import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

NULL_FILES = ("align/aligned_pairs.txt", "distances/linear.tsv", "summary.tsv", "distances/matricial/p.tsv",
              "distances/matricial/p-gaps.tsv", "distances/matricial/jc.tsv", "distances/matricial/k2p.tsv")


def _log(msg: str) -> None:
    print(f"[bench secondary] {msg}", file=sys.stderr, flush=True)


def prealigned_rows(n: int, L: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """Pre-aligned synthetic rows (config 2 / 5 stand-ins): lowercase acgt from the family generator
    (substitutions only: a pre-aligned row's gaps are its '-' runs), ~2 % '-' in short runs, 0.5 % 'n'."""
    from taxi2_amd.synth import family_codes

    rng = np.random.default_rng(seed)
    codes = family_codes(n, L, seed, ancestors=64, indel_rate=0.0)
    rows = np.frombuffer(b"acgt", dtype=np.uint8)[codes].copy()
    gap = rng.random((n, L)) < 0.01
    gap |= np.roll(gap, 1, axis=1)  # short runs
    rows[gap] = ord("-")
    rows[rng.random((n, L)) < 0.005] = ord("n")
    buf = np.concatenate([rows.reshape(-1), np.zeros(1, np.uint8)])
    return buf, np.arange(n + 1, dtype=np.int64) * L


def build_config5_task(n: int, L: int, eng, out: Path, block_gb: float, aligned: bool = False):
    """VersusAll configured as config 5's reductions-only run (see module docstring); returns
    (task, packed bytes, offsets) -- the bytes are None for the aligned form."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.partitions import Partition
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

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


def leg_task(eng, n: int = 5000) -> dict:
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.synth import family_sequences
    from taxi2_amd.tasks import VersusAll

    _log(f"task: VersusAll.start() N = {n}")
    seqs = [Sequence(f"seq{k}", s) for k, s in enumerate(family_sequences(n, 1000, 0x7A12))]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as tmp:
        out = Path(tmp)
        for f in NULL_FILES:
            (out / f).parent.mkdir(parents=True, exist_ok=True)
            os.symlink("/dev/null", out / f)
        t = VersusAll()
        t.engine, t.progress_handler, t.work_dir = eng, None, out
        t.input.sequences = Sequences(seqs)
        t0 = time.perf_counter()
        res = t.start()
        wall = time.perf_counter() - t0
        files = sorted(str(p.relative_to(out)) for p in out.rglob("*") if p.is_file() or p.is_symlink())
    pairs = n * (n - 1) // 2
    ph = dict(t.timings or {})
    compute = ph.get("compute_s")
    return {
        "workload": f"VersusAll.start() with the reference's defaults (align, p/p-gaps/jc/k2p, aligned_pairs.txt, "
                    f"linear.tsv, matricial/*.tsv, summary.tsv), {n} x 1 000 bp config-3 sequences; text files "
                    f"written through /dev/null symlinks in a temporary directory",
        "n_seqs": n, "unordered_pairs": pairs, "ordered_pairs": n * n,
        "seconds_taken": res.seconds_taken, "wall_s": wall,
        "unordered_pairs_per_s": pairs / res.seconds_taken,
        "compute_unordered_pairs_per_s": pairs / compute if compute else None,
        "phases_s": ph, "pairs_from_walks": bool(t.pairs_walked), "files": files,
    }


def leg_config5(eng, n: int = 200_000, L: int = 1000) -> dict:
    import torch

    _log(f"config5: building {n} x {L} pre-aligned rows")
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as tmp:
        t0 = time.perf_counter()
        task, _, _ = build_config5_task(n, L, eng, Path(tmp), 2.0)
        t_build = time.perf_counter() - t0
        _log("config5: VersusAll.start()")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = task.start()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    return {
        "workload": f"config5 reductions: VersusAll.start() on {n} x {L} pre-aligned synthetic rows (seed 0x7A14), "
                    f"p/jc/k2p x100, row minima + 2-genus / ~1 000-species subset statistics, one GPU",
        "n_seqs": n, "ordered_pairs": n * n, "seconds_taken": res.seconds_taken, "wall_s": wall,
        "ordered_pairs_per_s": n * n / wall, "phases_s": task.timings, "input_build_s": t_build,
    }


def leg_config4(eng, q_slice: int = 4096, R: int = 10_000, L: int = 650) -> dict:
    from taxi2_amd.synth import family_sequences

    _log(f"config4: {q_slice} queries x {R} refs x {L} bp")
    refs = family_sequences(R, L, 0x7A13)
    qs = family_sequences(q_slice, L, 0x7A13 + 1)
    sq = eng.upload(qs, align=True)
    sr = eng.upload(refs, align=True)
    extras = ("p-gaps", "jc", "k2p")
    try:
        eng.closest(sq, sr, 0, min(8, q_slice), "p", extras)
        t0 = time.perf_counter()
        idx, d, ex, _ = eng.closest(sq, sr, 0, q_slice, "p", extras)
        dt = time.perf_counter() - t0
    finally:
        sq.free()
        sr.free()
    pairs = q_slice * R
    return {
        "workload": f"config4 slice: versusReference {q_slice} queries x {R} refs x {L} bp (seed 0x7A13 generator), "
                    f"Gotoh align + p, closest reference + extras p-gaps/jc/k2p on the GPU",
        "pairs": pairs, "seconds": dt, "pairs_per_s": pairs / dt, "gcups": pairs * L * L / dt / 1e9,
        "full_job_minutes_1gpu": 1e10 / (pairs / dt) / 60, "closest_found": int((idx >= 0).sum()),
    }


def leg_allmetrics(eng, seqset, n_seqs: int, count: int = 1 << 15) -> dict:
    """p / p-gaps / jc / k2p from the aligner + NCD of the aligned strings for `count` config-3
    pairs (both orientations), as VersusAll computes them."""
    import torch

    from taxi2_amd._native import tri_pairs

    _log(f"allmetrics: {count} config-3 pairs, p/p-gaps/jc/k2p + ncd")
    metrics = ("p", "p-gaps", "jc", "k2p")
    k0 = 1 << 20  # a block the headline's first steps do not time
    a, b = tri_pairs(n_seqs, k0, count)
    eng.ncd_pairs(seqset, seqset, a[:256], b[:256], aligned=True, both=True)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    four = eng.all_pairs(seqset, k0, count, metrics)
    t1 = time.perf_counter()
    ncd = eng.ncd_pairs(seqset, seqset, a, b, aligned=True, both=True)
    t2 = time.perf_counter()
    return {
        "workload": f"config3 all metrics: {count} config-3 pairs (1 000 bp), Gotoh align + p/p-gaps/jc/k2p + NCD of "
                    f"the aligned strings, both ordered pairs",
        "pairs": count, "seconds": t2 - t0, "pairs_per_s": count / (t2 - t0),
        "four_metric_s": t1 - t0, "ncd_s": t2 - t1, "ncd_share": (t2 - t1) / (t2 - t0),
        "finite": bool(np.isfinite(four).all() and np.isfinite(ncd).all()),
    }


def run_all(eng, seqset, n_seqs: int, legs=("allmetrics", "config4", "task", "config5")) -> dict:
    out = {}
    for name in legs:
        t0 = time.perf_counter()
        try:
            if name == "task":
                out[name] = leg_task(eng)
            elif name == "config5":
                out[name] = leg_config5(eng)
            elif name == "config4":
                out[name] = leg_config4(eng)
            elif name == "allmetrics":
                out[name] = leg_allmetrics(eng, seqset, n_seqs)
        except Exception as e:  # a failing leg is reported, never takes the headline with it
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        _log(f"{name} done in {time.perf_counter() - t0:.1f} s")
    return out


def main() -> None:
    """python bench_secondary.py LEG [LEG ...]: run legs alone (one JSON line each)."""
    import json

    import torch  # noqa: F401  -- torch's HIP runtime first (the engine shares it)

    from taxi2_amd._native import Engine
    from taxi2_amd.synth import family_packed

    eng = Engine(0)
    seqset = None
    for name in sys.argv[1:]:
        if name == "allmetrics" and seqset is None:
            buf, offs = family_packed(50_000, 1000, 0x7A12)
            seqset = eng.upload_packed(buf, offs, align=True)
        print(json.dumps({name: run_all(eng, seqset, 50_000, [name])[name]}), flush=True)


if __name__ == "__main__":
    main()
