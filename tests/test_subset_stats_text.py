"""The engine library's host formatter of the subset statistics files (taxi2_format_subset_stats)
writes the same bytes as the Python writer (tasks/subsets.py write_subset_statistics, the
handlers' per-value text, versus_all.py:642-684): NaN / zero-count cells, -0.0, huge and tiny
values, None subset names, the default and a custom matricial template."""

from __future__ import annotations

import numpy as np
import pytest

from taxi2_amd.tasks import subsets as S


def _stats(ns: int, m: int, seed: int) -> S.SubsetStats:
    rng = np.random.default_rng(seed)
    mean = rng.random((ns, ns, m)) * 100.0
    mean[rng.random((ns, ns, m)) < 0.1] = np.nan
    mean.flat[0] = -0.0
    mean.flat[1] = 12.345
    mean.flat[2] = 1e-9
    mn, mx = mean * 0.5, mean * 2.0 + 1e6
    cnt = rng.integers(0, 5, size=(ns, ns, m)).astype(np.int64)
    names = [f"sp{k}" for k in range(ns)]
    names[1] = None
    return S.SubsetStats(names, mean, mn, mx, cnt)


def _files(root):
    return {p.relative_to(root).as_posix(): p.read_bytes() for p in sorted(root.rglob("*.tsv"))}


@pytest.mark.parametrize("template", ["{mean} ({min}-{max})", "{min}..{max} ~{mean}"])
@pytest.mark.parametrize("fmt", ["{:.4f}", "{:.2f}", "{:f}"])
def test_native_subset_statistics_text(tmp_path, monkeypatch, template, fmt):
    st = _stats(37, 3, 5)
    metrics = ["p", "jc", "k2p"]
    S.write_subset_statistics(tmp_path / "native", st, metrics, fmt, template)
    # the Python writer: no native path
    monkeypatch.setattr(S, "fixed_decimals", lambda f: None)
    S.write_subset_statistics(tmp_path / "py", st, metrics, fmt, template)
    a, b = _files(tmp_path / "native"), _files(tmp_path / "py")
    assert a.keys() == b.keys() and len(a) == 5
    for k in a:
        assert a[k] == b[k], k
