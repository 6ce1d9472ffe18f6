"""Multi-rank pair sharding + gather (world_size 2, gloo, CPU).

On GPUs each rank runs its pair block on its own MI355X and the gather is RCCL; here the
block computation is the C oracle so the partition / gather logic is exercised without a GPU.
"""

from __future__ import annotations

import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from tests.conftest import ROOT

WORKER = textwrap.dedent(
    """
    import os, sys
    import numpy as np
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from oracle import oracle_c
    from taxi2_amd._native import tri_pairs
    from taxi2_amd.sharding import distributed_all_pairs
    from taxi2_amd.synth import family_sequences

    dist.init_process_group("gloo")
    seqs = family_sequences(23, 120, 5, ancestors=3)
    n = len(seqs)

    def compute(k0, count):
        a, b = tri_pairs(n, k0, count)
        out, _ = oracle_c.batch(seqs, a, b, align=True, scores=(1, -1, -8, -1, -1, -1), threads=1)
        return out.reshape(count, -1)

    res = distributed_all_pairs(n, compute)
    np.save(os.environ["OUT"] + f".{{dist.get_rank()}}.npy", res)
    dist.destroy_process_group()
    """
)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_all_pairs(tmp_path, oracle_c):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=str(ROOT)))
    out = tmp_path / "res"
    env = dict(os.environ, OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    r0 = np.load(str(out) + ".0.npy")
    r1 = np.load(str(out) + ".1.npy")
    from taxi2_amd._native import tri_pairs
    from taxi2_amd.synth import family_sequences

    seqs = family_sequences(23, 120, 5, ancestors=3)
    a, b = tri_pairs(len(seqs))
    exp, _ = oracle_c.batch(seqs, a, b, align=True, scores=(1, -1, -8, -1, -1, -1), threads=2)
    exp = exp.reshape(len(a), -1)
    for got in (r0, r1):
        assert got.shape == exp.shape
        assert np.array_equal(np.nan_to_num(got, nan=7.0), np.nan_to_num(exp, nan=7.0))


ROWS_WORKER = textwrap.dedent(
    """
    import os, sys
    import numpy as np
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from taxi2_amd.sharding import distributed_rows

    dist.init_process_group("gloo")
    def compute(q0, q1):
        q = np.arange(q0, q1, dtype=np.float64)
        return np.stack([q, q * q, -q], axis=1)
    res = distributed_rows(37, compute)
    np.save(os.environ["OUT"] + f".{{dist.get_rank()}}.npy", res)
    dist.destroy_process_group()
    """
)


def test_two_rank_gloo_query_rows(tmp_path):
    """versusReference query sharding (contiguous blocks, all-gather): every rank gets all rows."""
    script = tmp_path / "rows.py"
    script.write_text(ROWS_WORKER.format(root=str(ROOT)))
    out = tmp_path / "rows"
    env = dict(os.environ, OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    q = np.arange(37, dtype=np.float64)
    exp = np.stack([q, q * q, -q], axis=1)
    for k in range(2):
        assert np.array_equal(np.load(str(out) + f".{k}.npy"), exp)


def test_shard_range_covers():
    from taxi2_amd.sharding import shard_range

    for n in (0, 1, 7, 100):
        for w in (1, 2, 3, 8):
            b = shard_range(n, w)
            assert b[0][0] == 0 and b[-1][1] == n and all(b[i][1] == b[i + 1][0] for i in range(w - 1))


GATHER_WORKER = textwrap.dedent(
    """
    import os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from taxi2_amd.sharding import gather_blocks, shard_range

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    rows = shard_range(23, world)
    lo, hi = rows[rank]
    loc = np.stack([np.arange(lo, hi, dtype=np.float64), -np.arange(lo, hi, dtype=np.float64)], axis=1)
    got = gather_blocks(loc, [b - a for a, b in rows], dst=0)              # numpy, to rank 0 only
    got_t = gather_blocks(torch.from_numpy(loc), [b - a for a, b in rows], dst=world - 1)  # a tensor, to the last rank
    np.save(os.environ["OUT"] + f".{{rank}}.npy", np.array([got is None, got_t is None]))
    if got is not None:
        np.save(os.environ["OUT"] + ".g0.npy", got)
    if got_t is not None:
        np.save(os.environ["OUT"] + ".gl.npy", got_t)
    dist.destroy_process_group()
    """
)


@pytest.mark.parametrize("world", [2, 3])
def test_gather_blocks_to_one_rank_gloo(tmp_path, world):
    """gather_blocks(dst=r) (the streamed path's row minima): only rank r receives the
    rank-ordered concatenation; numpy and tensor inputs alike."""
    script = tmp_path / "gather.py"
    script.write_text(GATHER_WORKER.format(root=str(ROOT)))
    out = tmp_path / "g"
    env = dict(os.environ, OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    q = np.arange(23, dtype=np.float64)
    exp = np.stack([q, -q], axis=1)
    assert np.array_equal(np.load(str(out) + ".g0.npy"), exp)
    assert np.array_equal(np.load(str(out) + ".gl.npy"), exp)
    for k in range(world):
        none0, nonel = np.load(str(out) + f".{k}.npy")
        assert none0 == (k != 0) and nonel == (k != world - 1)
