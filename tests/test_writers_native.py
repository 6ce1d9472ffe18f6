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
