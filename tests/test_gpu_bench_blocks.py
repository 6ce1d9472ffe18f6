"""GPU parity at the headline bench's launch structure.

bench.py times 524 288-pair ``all_pairs`` blocks spread over the whole config-3 triangle
(50 000 x 1 000 bp, ``bench.step_block``).  The blocks near the triangle's end hold short rows: the
row-shared aligner's segment builder (capi.hip ``build_segments``) then makes many segments, units of
one pair (one half of every lane idle), chains cut at segment ends and the guided chain tail of the
persistent grid (alignr_kernel.hpp) -- none of which the small parity tests reach.  Here one such
block is computed on the GPU exactly as the bench launches it, and pairs sampled across it (every
segment shape: uniform samples plus the block's first and last pairs) are checked against the C
restatement: alignment scores and p / p-gaps bit-exact, jc / k2p within 1e-12
(versus_all.py:746-769 aligns every pair of the space).
"""

from __future__ import annotations

import numpy as np
import pytest

from tests.test_gpu_parity import METRICS, SCORE_SETS, assert_metrics_equal

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def config3(engine):
    import bench
    from taxi2_amd.synth import family_packed

    buf, offs = family_packed(bench.N_SEQS, bench.SEQ_LEN, bench.SEED)
    st = engine.upload_packed(buf, offs, align=True)
    yield bench, buf, offs, st
    st.free()


def _check_block(engine, oracle_c, config3, k0: int, nsample: int, seed: int):
    from taxi2_amd._native import tri_pairs

    bench, buf, offs, st = config3
    B = 1 << 19
    got, gsc = engine.all_pairs(st, k0, B, METRICS, with_scores=True)
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([np.arange(256), B - 256 + np.arange(256),
                                    rng.choice(B, size=nsample, replace=False)]))
    a, b = tri_pairs(bench.N_SEQS, k0, B)
    exp, esc = oracle_c.batch((buf, offs), a[idx], b[idx], align=True, scores=SCORE_SETS["default"],
                              metrics=METRICS, threads=ORACLE_THREADS)
    assert np.array_equal(gsc[idx], esc)
    assert_metrics_equal(got[idx], exp)
    # rows covered by the sample (the last block spans thousands of short rows)
    return len(np.unique(a[idx]))


def test_bench_last_block(engine, oracle_c, config3):
    """The bench's last timed block (step_block(steps - 1)): the end of the triangle, short rows."""
    bench = config3[0]
    total = bench.N_SEQS * (bench.N_SEQS - 1) // 2
    k0 = bench.step_block(19, 0, 1, 1 << 19, total, 20)
    assert k0 == total - (1 << 19)
    rows = _check_block(engine, oracle_c, config3, k0, 3584, 0x6B1)
    assert rows > 500


def test_bench_middle_block(engine, oracle_c, config3):
    """A block from the middle of the triangle, where row pairs straddle the block's start."""
    bench = config3[0]
    total = bench.N_SEQS * (bench.N_SEQS - 1) // 2
    k0 = bench.step_block(13, 0, 1, 1 << 19, total, 20)
    _check_block(engine, oracle_c, config3, k0, 1536, 0x6B2)
