"""Streamed versusAll output for large N (config 5: 200 000 x 1 000 bp on 8 GPUs).

The reference never holds the N x N result: ``VersusAll.start`` pulls one ``Distance`` at a time
through a generator chain into the writers (``/root/reference/src/itaxotools/taxi2/tasks/
versus_all.py:732-773``, drained at :768-769), x-major.  This module gives the GPU path the same
bounded-memory shape without giving up the one-fill-per-unordered-pair kernels:

1. Every rank owns a contiguous row range of the upper triangle, balanced by pair count
   (``sharding.shard_rows``), and computes it into a :class:`TriangleStore` kept in ITS OWN memory
   (HBM with RCCL, host memory with gloo): per unordered pair (a, b) and orientation
   ((a, b), (b, a)) the packed column counters of ``TAXI2_METRIC_COUNTS`` (8 bytes; every metric
   is a function of them) plus, for NCD, one f64 per orientation.  Nothing is all-gathered.
2. The ordered product is then streamed to rank 0 in ROW BLOCKS [x0, x1) x [0, N), in x-major
   order: row x's entries (x, y > x) are orientation (a, b) of the pairs of row x (owned by the
   rank of row x); its entries (x, y < x) are orientation (b, a) of the pairs (y, x) of earlier rows
   (owned by the ranks of those rows).  Each rank sends rank 0 exactly the entries it owns
   (point-to-point, RCCL ``ncclSend/ncclRecv`` over xGMI or gloo), rank 0 scatters them into the
   block, and the writers consume the block before the next one is assembled.

Memory: per rank 16 B x its unordered pairs (+16 B with NCD); at N = 200 000 on 8
ranks 2.5e9 pairs -> 40 GB of the 288 GB HBM; rank 0 additionally holds one block of
B x N x 8 B counters (+ B x N x M x 8 B of metrics for the writers), B chosen for ~256 MB.
"""

from __future__ import annotations

from dataclasses import dataclass, field

from .sharding import shard_rows, tri_row_start

COUNTS_FILL = 0  # counters of a pair that has none (diagonal slots): every metric NaN


def _torch():
    import torch

    return torch


def block_entries(n: int, r0: int, r1: int, x0: int, x1: int, device=None):
    """Entries of the ordered-pair row block [x0, x1) x [0, n) owned by the rank of triangle rows
    [r0, r1), as (src, dst) int64 index tensors:

    * src indexes that rank's store viewed flat as [pair - k0][orientation] (k0 = first pair of
      row r0): 2 * (pair - k0) + 0 for (a, b), + 1 for (b, a);
    * dst indexes the block viewed flat as [x - x0][y].

    Orientation (a, b) of the pairs of rows x in [x0, x1) the rank owns gives entries (x, y > x);
    orientation (b, a) of its pairs (y, x) with y < x, x in the block, gives entries (x, y < x)."""
    torch = _torch()
    k0 = tri_row_start(r0, n)
    srcs, dsts = [], []
    # A part: own rows inside the block, every y > x
    a0, a1 = max(x0, r0), min(x1, r1)
    if a0 < a1:
        xs = torch.arange(a0, a1, dtype=torch.int64, device=device)
        lens = (n - 1 - xs).clamp(min=0)
        tot = int(lens.sum())
        if tot:
            rx = torch.repeat_interleave(xs, lens)
            first = torch.cumsum(lens, 0) - lens
            t = torch.arange(tot, dtype=torch.int64, device=device) - torch.repeat_interleave(first, lens)
            pair = rx * (2 * n - rx - 1) // 2 - k0 + t
            srcs.append(2 * pair)
            dsts.append((rx - x0) * n + rx + 1 + t)
    # B part: own rows y below the block's last row, columns x in [max(x0, y + 1), x1)
    b0, b1 = r0, min(r1, x1 - 1)
    if b0 < b1:
        ys = torch.arange(b0, b1, dtype=torch.int64, device=device)
        xst = torch.clamp(ys + 1, min=x0)
        lens = (x1 - xst).clamp(min=0)
        tot = int(lens.sum())
        if tot:
            ry = torch.repeat_interleave(ys, lens)
            rs = torch.repeat_interleave(xst, lens)
            first = torch.cumsum(lens, 0) - lens
            t = torch.arange(tot, dtype=torch.int64, device=device) - torch.repeat_interleave(first, lens)
            xcol = rs + t
            pair = ry * (2 * n - ry - 1) // 2 - k0 + (xcol - ry - 1)
            srcs.append(2 * pair + 1)
            dsts.append((xcol - x0) * n + ry)
    if not srcs:
        e = torch.empty(0, dtype=torch.int64, device=device)
        return e, e
    return torch.cat(srcs), torch.cat(dsts)


def block_entry_count(n: int, r0: int, r1: int, x0: int, x1: int) -> int:
    """len(block_entries(...)[0]) in closed form (called per rank and block: no index build)."""

    def span(lo: int, hi: int, top: int) -> int:  # sum over v in [lo, hi) of (top - v)
        return 0 if hi <= lo else (hi - lo) * top - (hi - lo) * (lo + hi - 1) // 2

    tot = span(max(x0, r0), min(x1, r1), n - 1)
    b1 = min(r1, x1 - 1)
    tot += max(0, min(b1, x0) - r0) * (x1 - x0)  # rows y < x0: every column of the block
    tot += span(max(r0, x0), b1, x1 - 1)          # rows x0 <= y: columns y + 1 .. x1 - 1
    return tot


@dataclass
class TriangleStore:
    """One rank's share of the versusAll triangle: rows [r0, r1) = pairs [k0, k0 + count), each
    plane a (count, 2) tensor [pair][orientation] on ``device``.  Planes: "counts" (int64 bit
    patterns of TAXI2_METRIC_COUNTS), optionally "ncd" (float64)."""

    n: int
    world: int
    rank: int
    device: object = None
    planes: dict = field(default_factory=dict)

    def __post_init__(self):
        self.rows = shard_rows(self.n, self.world)
        self.r0, self.r1 = self.rows[self.rank]
        self.k0 = tri_row_start(self.r0, self.n)
        self.count = tri_row_start(self.r1, self.n) - self.k0

    def add_plane(self, name: str, dtype) -> object:
        torch = _torch()
        t = torch.empty((self.count, 2), dtype=dtype, device=self.device)
        self.planes[name] = t
        return t

    # ------------------------------------------------------------------ streaming
    def assemble(self, x0: int, x1: int, group=None) -> dict | None:
        """Collective over the group: rank 0 receives the row block [x0, x1) x [0, n) of every
        plane ({name: (x1 - x0, n) tensor}; diagonal slots hold COUNTS_FILL / NaN); the other
        ranks send rank 0 the entries they own and get None."""
        torch = _torch()
        names = sorted(self.planes)
        src, dst = block_entries(self.n, self.r0, self.r1, x0, x1, self.device)
        # one message per rank: the planes' entries one after the other, as int64 bit patterns
        mine = torch.cat([self._flat(nm).index_select(0, src) for nm in names])
        if self.rank != 0:
            if mine.numel():
                import torch.distributed as dist

                dist.send(mine, dst=_global(group, 0), group=group)
            return None
        parts = [(dst, mine)]
        if self.world > 1:
            import torch.distributed as dist

            # every peer's entries in flight at once (one receive per rank, posted together: RCCL
            # groups them into one launch, so all xGMI links into rank 0 carry data concurrently)
            recvs = []
            for r in range(1, self.world):
                q0, q1 = self.rows[r]
                cnt = block_entry_count(self.n, q0, q1, x0, x1)
                if cnt == 0:
                    continue
                buf = torch.empty(cnt * len(names), dtype=torch.int64, device=self.device)
                recvs.append((r, q0, q1, buf))
            if recvs:
                if dist.get_backend(group) == "nccl":
                    ops = [dist.P2POp(dist.irecv, buf, _global(group, r), group) for r, _, _, buf in recvs]
                    reqs = dist.batch_isend_irecv(ops)
                else:
                    reqs = [dist.irecv(buf, src=_global(group, r), group=group) for r, _, _, buf in recvs]
                for q in reqs:
                    q.wait()
            for r, q0, q1, buf in recvs:
                parts.append((block_entries(self.n, q0, q1, x0, x1, self.device)[1], buf))
        out = {nm: self._blank(nm, x1 - x0) for nm in names}
        for d, buf in parts:
            per = d.numel()
            if not per:
                continue
            for i, nm in enumerate(names):
                out[nm].view(-1).view(torch.int64)[d] = buf[i * per : (i + 1) * per]
        return out

    def _flat(self, name: str):
        torch = _torch()
        t = self.planes[name]
        return t.reshape(-1).view(torch.int64)

    def _blank(self, name: str, rows: int):
        torch = _torch()
        t = self.planes[name]
        if t.dtype == torch.float64:
            return torch.full((rows, self.n), float("nan"), dtype=torch.float64, device=self.device)
        return torch.full((rows, self.n), COUNTS_FILL, dtype=t.dtype, device=self.device)


def block_rows(n: int, bytes_per_entry: int, budget: int = 256 << 20) -> int:
    """Rows per streamed block so that one block stays within ``budget`` bytes."""
    return max(1, min(max(n, 1), budget // max(1, n * bytes_per_entry)))


def _global(group, rank: int) -> int:
    if group is None:
        return rank
    import torch.distributed as dist

    return dist.get_global_rank(group, rank)
