"""Writer text: the product's fixed-point formatter (format_kernels.hpp) == Python "{:.Nf}".

CPU: the formatter compiled for the host vs Python on ties, subnormals, -0.0 and random doubles.
GPU: taxi2_format_rows (linear / matrix text) vs the Python rendering of the same table.
"""

from __future__ import annotations

import ctypes
import os
import random
import shutil
import struct
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

EDGE = [0.0, -0.0, 0.5, 1.5, 2.5, 0.125, 0.375, -0.125, 0.00005, -0.00005, 0.99995, 9.99995, 1e-320,
        -1e-320, 5e-324, 123456.78905, 0.045, 1.005, 100.0, 99.99995, 0.1, 0.7]


def _values(seed: int, n: int) -> list[float]:
    rng = random.Random(seed)
    out = list(EDGE)
    for _ in range(n):
        k = rng.randrange(5)
        if k == 0:
            x = rng.random()
        elif k == 1:
            x = rng.random() * 200 - 100
        elif k == 2:
            x = struct.unpack("d", struct.pack("Q", rng.getrandbits(64)))[0]
        elif k == 3:
            x = round(rng.random(), rng.randint(1, 6)) + rng.choice([0, 5e-5, -5e-5])
        else:
            x = rng.randint(0, 100000) / 2 ** rng.randint(0, 20)
        out.append(x)
    return out


@pytest.fixture(scope="module")
def fmt_host(tmp_path_factory):
    gxx = os.environ.get("TAXI2_HOST_CXX") or shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    out = tmp_path_factory.mktemp("fmt") / "libfmt_host.so"
    subprocess.run([gxx, "-O2", "-std=c++17", "-shared", "-fPIC", *os.environ.get("TAXI2_HOST_CFLAGS", "").split(), "-o", str(out),
                    str(ROOT / "tests/native/fmt_host.cpp")], check=True)
    lib = ctypes.CDLL(str(out))
    lib.fmt_host.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_char_p]
    buf = ctypes.create_string_buffer(64)

    def f(x, n):
        length = lib.fmt_host(x, n, buf)
        return buf.raw[:length].decode()

    return f


def test_fixed_formatter_matches_python(fmt_host):
    bad = []
    for x in _values(5, 20000):
        if x != x or x in (float("inf"), float("-inf")):
            continue
        for n in (0, 1, 2, 4, 6, 9):
            if abs(x) * 10.0 ** n >= 2.0 ** 62:
                continue
            if fmt_host(x, n) != "{:.{}f}".format(x, n):
                bad.append((x, n))
    assert not bad, bad[:10]


@pytest.mark.gpu
@pytest.mark.parametrize("decimals", [0, 2, 4, 6])
def test_format_rows_gpu(engine, decimals):
    rng = np.random.default_rng(decimals)
    vals = np.array([v for v in _values(decimals, 3000) if v == v and abs(v) * 10.0 ** decimals < 2.0 ** 62])
    nrows, ncols, nm = 7, 45, 3
    V = rng.choice(vals, size=(nrows, ncols, nm))
    V[0, 0, 0], V[1, 2, 1], V[3, 4, 2] = np.nan, np.inf, -np.inf
    rows = [f"q{i}\tvoucher{i}\tNA" if i % 2 else f"q{i}\tvoucher é{i}\tx" for i in range(nrows)]
    cols = [f"r{j}\tv{j}\t{'NA' if j % 3 else 'org'}" for j in range(ncols)]

    def txt(v):
        return "{:.{}f}".format(v, decimals) if np.isfinite(v) else "NA"

    exp = "".join(rows[i] + "\t" + cols[j] + "".join("\t" + txt(V[i, j, m]) for m in range(nm)) + "\n"
                  for i in range(nrows) for j in range(ncols))
    got = engine.format_rows(V, rows, cols, decimals=decimals, missing="NA")
    assert got.decode("utf-8") == exp
    M = V[:, :, 1]
    ids = [f"id{i}" for i in range(nrows)]
    expm = "".join(ids[i] + "".join("\t" + txt(M[i, j]) for j in range(ncols)) + "\n" for i in range(nrows))
    assert engine.format_rows(M, ids, None, decimals=decimals, missing="NA").decode() == expm


@pytest.mark.gpu
@pytest.mark.parametrize("decimals", [0, 4])
def test_format_rows_dev_values(engine, decimals):
    """taxi2_format_rows_dev / taxi2_format_summary_dev (values read in HBM: a block, one metric's
    strided column of it, a row slice) == the host-value formatters byte for byte; a value too large
    for exact fixed-point text fails the call instead of printing a wrong number."""
    import torch

    from taxi2_amd._native import NativeError

    rng = np.random.default_rng(11 + decimals)
    vals = np.array([v for v in _values(decimals, 3000) if v == v and abs(v) * 10.0 ** decimals < 2.0 ** 62])
    nrows, ncols, nm = 9, 37, 4
    V = rng.choice(vals, size=(nrows, ncols, nm))
    V[0, 0, 0], V[1, 2, 1], V[3, 4, 3], V[2, 2, 2] = np.nan, np.inf, -np.inf, -0.0
    rows = [f"q{i}\tv{i}" for i in range(nrows)]
    cols = [f"r{j}\tw{j}" for j in range(ncols)]
    Vd = torch.as_tensor(V, device="cuda")
    assert engine.format_rows(Vd, rows, cols, decimals=decimals) == engine.format_rows(V, rows, cols, decimals=decimals)
    for m in range(nm):  # the matricial files: one metric of the block, stride nm
        assert (engine.format_rows(Vd[:, :, m], rows, None, decimals=decimals)
                == engine.format_rows(np.ascontiguousarray(V[:, :, m]), rows, None, decimals=decimals))
    sub = engine.format_rows(Vd[3:7], rows[3:7], cols, decimals=decimals, view=True)
    assert bytes(sub) == engine.format_rows(V[3:7], rows[3:7], cols, decimals=decimals)
    suf_r = [s for i in range(nrows) for s in (f"\tx{i}", f"\tg{i % 2}\ts{i % 3}")]
    suf_c = [s for j in range(ncols) for s in ("", f"\tg{j % 2}\ts{j % 3}")]
    rc = np.array([[i % 2, i % 3] for i in range(nrows)], dtype=np.int32)
    cc = np.array([[j % 2, j % 3] for j in range(ncols)], dtype=np.int32)
    kw = dict(has_genera=True, has_species=True, decimals=decimals)
    assert (engine.format_summary(Vd, rows, cols, suf_r, suf_c, rc, cc, **kw)
            == engine.format_summary(V, rows, cols, suf_r, suf_c, rc, cc, **kw))
    Vd[5, 6, 1] = 2.0 ** 63
    with pytest.raises(NativeError, match="too large"):
        engine.format_rows(Vd, rows, cols, decimals=decimals)
