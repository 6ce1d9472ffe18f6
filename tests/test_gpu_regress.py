"""Regression: the packed aligner (k_alignt2) must give the single-pair (oracle) result whatever
ran before it in the same process.

Round 1 saw builds of k_alignt2 that differ only in code layout (AT2_CHUNK = 16, the range-
guarded `make guard` build) give wrong scores or fault, but only after other kernel variants had
run in the process.  A kernel that reads LDS or trace memory it did not write this
launch sees what EARLIER kernels left there, which is exactly that symptom; the guard build now
poisons LDS and each chain's trace buffer so such a read fails on the first launch (AG_* codes,
alignt2_kernel.hpp).  This test replays the round-1 failing shape in one process: every other
aligner variant (forward-carry chained / unchained, two-orientation, 32-bit trace, traceback,
NCD, pre-aligned) runs first and leaves its state in LDS / the shared buffers, then the packed
kernel runs every shape (K, W) on the random buckets of test_gpu_parity.py, the 1 025-2 048
column (W = 4) shape in both the triangle and the rectangle, forced long chains, and device-
buffer launches on a caller stream, each compared with the oracle.

Reference: /root/reference/src/itaxotools/taxi2/align.py:151-157 (one pair at a time: its result
cannot depend on what was aligned before it).
"""

from __future__ import annotations

import os

import numpy as np
import pytest

from tests.seqgen import family_sequences, mutate, random_sequences
from tests.test_gpu_parity import METRICS, SCORE_SETS, assert_metrics_equal

pytestmark = pytest.mark.gpu


def _env(env: dict, fn):
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _bucket(lo: int, hi: int, n: int, seed: int) -> list[str]:
    base = random_sequences(n // 2, lo, hi, seed, "ACGT", n_rate=0.02)
    return [s if s else "A" for s in base + mutate(base, seed + 1, rate=0.15)]


def _other_kernels(engine, seqs):
    """Run every non-packed kernel on `seqs` (results discarded): they leave their LDS and the
    shared d_trace / d_work buffers in the state a later packed launch would inherit."""
    from taxi2_amd._native import tri_pairs

    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    k = len(a)
    for env in ({"TAXI2_NO_ALIGNT": "1"},                                  # k_align1c (chained forward carry)
                {"TAXI2_NO_ALIGNT": "1", "TAXI2_A1_NOCHAIN": "1"},         # k_align1
                {"TAXI2_NO_ALIGNT": "1", "TAXI2_NO_ALIGN1": "1"},          # k_align (two orientations)
                {"TAXI2_NO_PACKED": "1"}):                                 # k_alignt (32-bit trace)
        _env(env, lambda: engine.all_pairs(st, 0, k, METRICS, None))
    engine.all_pairs(st, 0, k, METRICS, SCORE_SETS["linear"])                # linear scores: k_align NW
    engine.align_strings(st, st, a[:6], b[:6], None, both=True)              # k_trace_fill / k_traceback
    engine.ncd_pairs(st, st, a[:6], b[:6])                                   # NCD kernels
    pre = engine.upload(seqs, align=False)
    engine.all_pairs(pre, 0, k, METRICS)                                     # k_prealigned
    pre.free()
    st.free()


@pytest.mark.parametrize("scores", ["default", "generic"])
def test_packed_after_other_kernels(engine, oracle_c, scores):
    from taxi2_amd._native import tri_pairs

    sc = SCORE_SETS[scores]
    _other_kernels(engine, _bucket(600, 1400, 10, 0x5EED))
    # every packed shape (K, W): 256, 512, 768, 1 024, 1 536, 2 048 columns
    for lo, hi in ((60, 250), (300, 380), (600, 760), (900, 1024), (1100, 1500), (1700, 2048)):
        n = 10 if hi > 1100 else 14
        seqs = _bucket(lo, hi, n, (lo * 7 + hi) & 0xFFFF)
        st = engine.upload(seqs, align=True)
        a, b = tri_pairs(n)
        exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
        for env in ({}, {"TAXI2_AT_CHUNK": "8"}, {"TAXI2_AT_CHUNK": "3", "TAXI2_AT_HOPS": "1"}):
            got, gsc = _env(env, lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
            assert np.array_equal(gsc, esc), (lo, hi, env)
            assert_metrics_equal(got, exp)
        st.free()
        _other_kernels(engine, seqs[:6])  # and again between shapes


def test_packed_w4_rectangle_after_other_kernels(engine, oracle_c):
    """The 2 048-column shape (four fill waves + walker) as a rectangle with references both
    shorter and longer than 9/8 of each query (rows / columns swapped within a chain)."""
    rng = np.random.default_rng(0x2048)
    fam = family_sequences(12, 2000, 0x57, ancestors=2, max_sub=0.05, indel_rate=0.02)
    seqs = [s[: 1100 + int(rng.integers(0, 900))] for s in fam]
    q, r = seqs[:4], seqs[4:] + [s[:1300] for s in seqs[:2]]
    _other_kernels(engine, seqs[:5])
    qs = engine.upload(q, align=True)
    rs = engine.upload(r, align=True)
    allseq = q + r
    pa = np.repeat(np.arange(len(q)), len(r))
    pb = np.tile(np.arange(len(r)), len(q)) + len(q)
    for name in ("default", "generic", "generic1"):
        sc = SCORE_SETS[name]
        exp, _ = oracle_c.batch(allseq, pa, pb, align=True, scores=sc)
        for env in ({}, {"TAXI2_AT_CHUNK": "5"}):
            got = _env(env, lambda: engine.rect_pairs(qs, rs, 0, len(q), METRICS, sc))
            assert_metrics_equal(got, exp[:, 0, :])
    qs.free()
    rs.free()


def test_packed_device_buffers_on_caller_stream(engine, oracle_c):
    """taxi2_all_pairs_dev on a torch stream, interleaved with host-buffer calls on the engine's
    own stream that use the same shared buffers (d_trace / d_work) and regrow them."""
    torch = pytest.importorskip("torch")
    from taxi2_amd._native import tri_pairs

    seqs = family_sequences(20, 1000, 0x7A12, ancestors=4)
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=SCORE_SETS["default"])
    stream = torch.cuda.Stream()
    for rep in range(3):
        out = torch.full((len(a), 2, len(METRICS)), -7.0, dtype=torch.float64, device="cuda")
        osc = torch.full((len(a),), 0x7FFF0000, dtype=torch.int32, device="cuda")
        engine.all_pairs_dev(st, 0, len(a), METRICS, out.data_ptr(), None, osc.data_ptr(), stream.cuda_stream)
        # host-buffer calls right behind it (no host synchronisation in between): longer sequences
        # regrow the shared trace buffer while the device-buffer launch may still be running
        longer = engine.upload(_bucket(1700, 2048, 6, rep + 1), align=True)
        engine.all_pairs(longer, 0, 15, METRICS, None)
        longer.free()
        stream.synchronize()
        assert np.array_equal(osc.cpu().numpy(), esc)
        assert_metrics_equal(out.cpu().numpy(), exp)
    st.free()
