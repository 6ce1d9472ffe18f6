#!/usr/bin/env python3
"""VersusAll's partition outputs at N = 2000, M = 4 ('{:.4f}', 'NA'), 200 species in 40 genera:
  summary.tsv -- GPU formatter (taxi2_format_summary) vs the handler-shaped Python writer;
  subset aggregation -- taxi2_subset_aggregate (native, x-major order) vs the Python restatement
  (oracle A11) timed on a 300-sequence slice and scaled by N^2."""

from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    import torch  # noqa: F401  (HIP runtime load order)

    from oracle import restatement as R
    from taxi2_amd._native import Engine
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence
    from taxi2_amd.tasks.subsets import aggregate, write_summary

    n, M = 2000, 4
    rng = np.random.default_rng(0)
    A = rng.random((n, n, M)) * 0.3
    A[::7, ::5, 1] = np.nan
    seqs = [Sequence(f"seq{i}", "", {"voucher": f"v{i}", "organism": f"Genus{i % 40} species{i % 200}"})
            for i in range(n)]
    species = {s.id: s.extras["organism"] for s in seqs}
    genera = {s.id: s.extras["organism"].split(" ")[0] for s in seqs}
    metrics = [DistanceMetric.Uncorrected(), DistanceMetric.UncorrectedWithGaps(), DistanceMetric.JukesCantor(),
               DistanceMetric.Kimura2P()]
    eng = Engine(0)
    write_summary(Path("/tmp/s_warm.tsv"), seqs[:4], A[:4, :4], metrics, genera, species, "{:.4f}", "NA", eng)
    t0 = time.perf_counter()
    write_summary(Path("/tmp/s_gpu.tsv"), seqs, A, metrics, genera, species, "{:.4f}", "NA", eng)
    t_gpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    write_summary(Path("/tmp/s_py.tsv"), seqs, A, metrics, genera, species, "{:.4f}", "NA", None)
    t_py = time.perf_counter() - t0
    same = Path("/tmp/s_gpu.tsv").read_bytes() == Path("/tmp/s_py.tsv").read_bytes()
    size = Path("/tmp/s_gpu.tsv").stat().st_size

    ids = [s.id for s in seqs]
    t0 = time.perf_counter()
    aggregate(A, ids, species)
    aggregate(A, ids, genera)
    t_agg = time.perf_counter() - t0
    k = 300
    sub = A[:k, :k]

    def value(i, j, m):
        v = sub[i, j, m]
        return float(v) if np.isfinite(v) else None

    t0 = time.perf_counter()
    R.subset_aggregates(ids[:k], species, value, M)
    t_ref = (time.perf_counter() - t0) * (n / k) ** 2 * 2
    print(json.dumps({
        "workload": f"summary.tsv + species/genera aggregation, N={n}, M={M}", "summary_bytes": size,
        "summary_gpu_s": t_gpu, "summary_python_s": t_py, "summary_speedup": t_py / t_gpu,
        "summary_identical": same, "aggregate_native_s_both_partitions": t_agg,
        "aggregate_python_est_s_both_partitions": t_ref,
    }))


if __name__ == "__main__":
    main()
