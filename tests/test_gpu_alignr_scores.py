"""GPU parity of the row-shared aligner (alignr_kernel.hpp k_alignr) under user-set Gotoh scores.

Round 6 runs k_alignr for every score set with ONE extend for internal and end gaps whose opens are
no better than the extend (the best-open recurrences, capi.hip bopen_ok), an internal open no better
than the end open relative to the extend, and fill values inside the f16 range at the launch's
length (alignr_kernel.hpp ar_scores_ok); other sets keep k_alignt2.  Linear gaps (opens = extends)
with one extend run it too, its walker in the reference's single-matrix tie order (full trace).  Each set here: alignment
scores and metrics against the C oracle bit for bit (jc / k2p within 1e-12), the launch's kernel
named by its band statistics line, the walked strings equal to the trace kernels', and -- at sizes
the oracle would take minutes for -- the same launch through k_alignt2 (TAXI2_NO_ALIGNR_GEN=1).
Reference: /root/reference/src/itaxotools/taxi2/align.py:20-27 (the score parameters), :151-157
(one global alignment per pair).
"""

from __future__ import annotations

import os
import re

import numpy as np
import pytest

from tests.seqgen import family_sequences, mutate, random_sequences
from tests.test_gpu_alignt import _tie_heavy, _with_env
from tests.test_gpu_parity import METRICS, assert_metrics_equal

pytestmark = pytest.mark.gpu

# (ma, mi, io, ie, eo, ee)
SETS = {
    "generic1": (2, -3, -5, -2, -3, -2),     # co_i = -3, co_e = -1
    "small": (1, -2, -4, -1, -2, -1),        # co_i = -3, co_e = -1
    "equal_opens": (3, -1, -6, -2, -6, -2),  # co_i = co_e = -4
    "free_ends": (5, -4, -10, -3, -3, -3),   # co_e = 0, a large match (eqm = 11: L <= 994)
    "ties": (1, 0, -2, -1, -1, -1),          # mismatch = 0, opens one below the extend: tie-heavy
    "big": (10, -10, -10, -6, -10, -6),      # eqm = 22: k_alignr up to 497 columns only
    "end_open_worse": (2, -1, -3, -3, -12, -3),  # co_i = 0 > co_e = -9: k_alignt2
    # linear gaps with one extend: k_alignr with the single-matrix (Needleman-Wunsch) tie order
    "linear1": (1, -1, -2, -2, -2, -2),
    "linear_ties": (1, 0, -1, -1, -1, -1),
    "linear2": (2, -3, -3, -3, -3, -3),
    "linear_two_extends": (1, -1, -2, -2, -1, -1),  # ie != ee: k_align
}


def _fits16(sc, length: int) -> bool:
    """alignt2_kernel.hpp at_fits16 restated: the packed fills' 16-bit range (else the 32-bit fill)."""
    ma, mi, io, ie, eo, ee = (abs(v) for v in sc)
    p, o = max(ma, mi, ie, ee), max(io, eo)
    lo = 2 * (p * 2 * length + 2 * o + 2)
    hi = 2 * ma * length + 2 + 2 * ie * 2 * length
    return lo + 2 * o + 2 * p + 16384 + 8 < 32767 and hi + 2 * o + 2 * p + 16384 + 8 < 32767


def alignr_eligible(sc, length: int) -> bool:
    """capi.hip pick_variantr's choice restated: no linear gaps with two extends, bopen_ok (ie == ee, opens <=
    extends) and alignr_kernel.hpp ar_scores_ok.  (Past the packed queued pass's range, _fits16,
    k_alignr stores the full trace and requeues nothing.)"""
    ma, mi, io, ie, eo, ee = sc
    if sc == (1, -1, -8, -1, -1, -1):
        return True
    if io == ie and eo == ee and ie != ee:  # linear gaps, two extends: k_align (capi.hip is_linear)
        return False
    small = all(-12 <= v <= 12 for v in sc)
    eqm = ma - 2 * ie
    return ie == ee and io <= ie and eo <= ee and small and io - ie <= eo - ee and length * max(0, eqm) + 64 <= 11000


def _kernels(err: str) -> set[str]:
    return set(re.findall(r"band: (k_\w+)<", err))


def _mixed(seed: int, length: int) -> list[str]:
    return (_tie_heavy(6, length, seed) + family_sequences(8, length - 100, seed + 1, ancestors=2)
            + random_sequences(6, 1, 120, seed + 2, "ACGTN") + mutate(random_sequences(2, 40, 200, seed + 3, "AC"), 5, 0.2)
            + ["", "A", "N" * 7])


@pytest.mark.parametrize("name", list(SETS))
def test_alignr_scores_triangle(engine, oracle_c, capfd, name):
    from taxi2_amd._native import tri_pairs

    sc = SETS[name]
    length = 280 if name == "big" else 700
    seqs = _mixed(0x300 + len(name), length)
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    capfd.readouterr()
    got, gsc = _with_env({"TAXI2_AT_BAND_STATS": "1"},
                         lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    ks = _kernels(capfd.readouterr().err)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    ml = max(len(s) for s in seqs)
    if alignr_eligible(sc, ml):
        assert ks == {"k_alignr"}, ks
    else:
        assert "k_alignr" not in ks, ks
    st.free()


@pytest.mark.parametrize("name", ["generic1", "free_ends", "big"])
def test_alignr_scores_too_long_falls_back(engine, oracle_c, capfd, name):
    """The longest lengths: k_alignr up to its f16 range (generic1 at 1 024 columns), another
    aligner past it (L eqm > ~11 000): the same results either way."""
    from taxi2_amd._native import tri_pairs

    sc = SETS[name]
    length = {"generic1": 1024, "free_ends": 1010, "big": 520}[name]
    seqs = family_sequences(6, length, 0x320, ancestors=2, max_sub=0.1)
    seqs[0] = (seqs[0] * 2)[:length]
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    capfd.readouterr()
    got, gsc = _with_env({"TAXI2_AT_BAND_STATS": "1"},
                         lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    ks = _kernels(capfd.readouterr().err)
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    ml = max(len(s) for s in seqs)
    assert ("k_alignr" in ks) == alignr_eligible(sc, ml), (ks, ml)
    st.free()


@pytest.mark.parametrize("length", [900, 990])
def test_alignr_scores_full_trace_without_queue(engine, oracle_c, capfd, length):
    """free_ends at 900 / 990 bp: outside the packed queued pass's 16-bit range (at_fits16) but
    inside k_alignr's own (ar_scores_ok): band 0, the full trace, nothing requeued."""
    from taxi2_amd._native import tri_pairs
    from tests.test_gpu_band import _indel_family

    sc = SETS["free_ends"]
    seqs = [s[:length] for s in _indel_family(length, 0x370)] + _tie_heavy(5, length, 0x371) + ["", "G"]
    assert max(len(s) for s in seqs) <= length and not _fits16(sc, max(len(s) for s in seqs))
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    capfd.readouterr()
    got, gsc = _with_env({"TAXI2_AT_BAND_STATS": "1"},
                         lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    err = capfd.readouterr().err
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    assert re.search(r"band: k_alignr<\d+,\d+> band 0: 0 of", err), err
    st.free()


@pytest.mark.parametrize("name", ["generic1", "equal_opens", "ties", "linear1", "linear_ties"])
def test_alignr_scores_rectangle(engine, oracle_c, name):
    sc = SETS[name]
    q = _tie_heavy(7, 600, 0x330) + ["", "C"]
    r = family_sequences(9, 500, 0x331, ancestors=2) + random_sequences(4, 1, 90, 0x332, "ACGTN")
    qs, rs = engine.upload(q, align=True), engine.upload(r, align=True)
    pa = np.repeat(np.arange(len(q)), len(r))
    pb = np.tile(np.arange(len(r)), len(q)) + len(q)
    got = engine.rect_pairs(qs, rs, 0, len(q), METRICS, sc)
    exp, _ = oracle_c.batch(q + r, pa, pb, align=True, scores=sc)
    assert_metrics_equal(got, exp[:, 0, :])
    qs.free()
    rs.free()


@pytest.mark.parametrize("name", ["generic1", "free_ends", "linear1"])
@pytest.mark.parametrize("band", ["6", "default"])
def test_alignr_scores_narrow_band(engine, oracle_c, name, band):
    """Escapes from a narrow trace band requeue to the full-trace pass under user scores too."""
    from taxi2_amd._native import tri_pairs
    from tests.test_gpu_band import _indel_family

    sc = SETS[name]
    seqs = _indel_family(800, 0x340)
    st = engine.upload(seqs, align=True)
    a, b = tri_pairs(len(seqs))
    env = {} if band == "default" else {"TAXI2_AT_BAND": band}
    got, gsc = _with_env(env, lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    exp, esc = oracle_c.batch(seqs, a, b, align=True, scores=sc)
    assert np.array_equal(gsc, esc)
    assert_metrics_equal(got, exp)
    st.free()


@pytest.mark.parametrize("name", ["generic1", "free_ends", "ties"])
def test_alignr_scores_strings(engine, name):
    """Walked strings (both orientations) == the trace kernels' (k_trace_fill + k_traceback)."""
    sc = SETS[name]
    seqs = _tie_heavy(10, 500, 0x350) + random_sequences(12, 1, 80, 0x351, "ACGTN") + ["", "A"]
    st = engine.upload(seqs, align=True)
    n = len(seqs)
    xs = np.repeat(np.arange(n), n)
    ys = np.tile(np.arange(n), n)
    got = engine.align_strings(st, st, xs, ys, sc, both=True)
    exp = _with_env({"TAXI2_NO_WALK_STRINGS": "1"}, lambda: engine.align_strings(st, st, xs, ys, sc, both=True))
    assert got == exp
    st.free()


def test_alignr_scores_equal_alignt2_at_scale(engine):
    """A 1 000 bp family of 96 sequences (4 560 pairs) under generic1: k_alignr == k_alignt2
    (TAXI2_NO_ALIGNR_GEN=1), scores and all four metrics bit for bit."""
    from taxi2_amd._native import tri_pairs

    sc = SETS["generic1"]
    seqs = family_sequences(96, 1000, 0x360, ancestors=6)
    st = engine.upload(seqs, align=True)
    a, _ = tri_pairs(len(seqs))
    got, gsc = engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True)
    ref, rsc = _with_env({"TAXI2_NO_ALIGNR_GEN": "1"},
                         lambda: engine.all_pairs(st, 0, len(a), METRICS, sc, with_scores=True))
    assert np.array_equal(gsc, rsc)
    assert np.array_equal(np.nan_to_num(got, nan=9.0), np.nan_to_num(ref, nan=9.0))
    st.free()
    os.environ.pop("TAXI2_NO_ALIGNR_GEN", None)
