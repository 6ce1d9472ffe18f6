"""Streamed versusAll assembly (taxi2_amd/streaming.py) with 2 and 3 ranks over gloo on CPU.

Each rank fills its TriangleStore with values that name their ordered pair (counts plane: the
int64 x * n + y + 1 of orientation (x, y); ncd plane: the float x * n + y + 0.5), then rank 0
assembles every row block and checks that slot (x - x0, y) holds exactly the value of the ordered
pair (x, y), the diagonal the fill value -- for several block heights, so blocks start and end
inside and across the ranks' row ranges.  On GPUs the same code moves the blocks with RCCL
point-to-point sends over xGMI (tests/test_gpu_streaming.py).
"""

from __future__ import annotations

import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from tests.conftest import ROOT
from tests.test_sharding_gloo import free_port

WORKER = textwrap.dedent(
    """
    import os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from taxi2_amd.streaming import TriangleStore

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    bad = 0
    for n in (1, 2, 5, 17, 40):
        st = TriangleStore(n, world, rank)
        c = st.add_plane("counts", torch.int64)
        f = st.add_plane("ncd", torch.float64)
        # pairs of this rank's rows, in pair-index order
        for k in range(st.count):
            g = st.k0 + k
            a = 0
            while a + 1 < n and (a + 1) * (2 * n - a - 2) // 2 <= g:
                a += 1
            b = a + 1 + g - a * (2 * n - a - 1) // 2
            c[k, 0], c[k, 1] = a * n + b + 1, b * n + a + 1
            f[k, 0], f[k, 1] = a * n + b + 0.5, b * n + a + 0.5
        for B in (1, 3, 7, n):
            for x0 in range(0, n, B):
                x1 = min(n, x0 + B)
                blk = st.assemble(x0, x1)
                if rank != 0:
                    assert blk is None
                    continue
                for x in range(x0, x1):
                    for y in range(n):
                        cv, fv = int(blk["counts"][x - x0, y]), float(blk["ncd"][x - x0, y])
                        if x == y:
                            bad += cv != 0 or not np.isnan(fv)
                        else:
                            bad += cv != x * n + y + 1 or fv != x * n + y + 0.5
    with open(os.environ["OUT"] + f".{{rank}}", "w") as fh:
        fh.write(str(bad))
    dist.destroy_process_group()
    """
)


@pytest.mark.parametrize("world", [2, 3])
def test_streamed_blocks_over_gloo(tmp_path, world):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=str(ROOT)))
    out = tmp_path / "res"
    env = dict(os.environ, OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    for rank in range(world):
        assert (tmp_path / f"res.{rank}").read_text() == "0"


def test_block_entry_count_closed_form():
    from taxi2_amd.sharding import shard_rows
    from taxi2_amd.streaming import block_entries, block_entry_count

    for n in range(1, 13):
        for world in (1, 2, 3, 5):
            for r0, r1 in shard_rows(n, world):
                for x0 in range(n):
                    for x1 in range(x0 + 1, n + 1):
                        assert len(block_entries(n, r0, r1, x0, x1)[0]) == block_entry_count(n, r0, r1, x0, x1)


def test_store_memory_bound_config5():
    """at N = 200 000 on 8 ranks every rank's store (16 B per unordered pair) stays far
    inside one MI355X's 288 GB, and a streamed block stays at the requested size."""
    from taxi2_amd.sharding import shard_pairs
    from taxi2_amd.streaming import block_rows

    n, world = 200_000, 8
    per_rank = max(c for _, c in shard_pairs(n, world)) * 16
    assert per_rank < 45e9
    B = block_rows(n, 8 * (1 + 4), 256 << 20)
    assert B * n * 8 * 5 <= 256 << 20 and B >= 1
    assert np.isclose(sum(c for _, c in shard_pairs(n, world)), n * (n - 1) / 2)
