"""bench.py's multi-GPU arithmetic with 2 ranks over gloo on CPU (the driver runs the real thing on
an 8-GPU node with RCCL): every rank's blocks are disjoint from every other rank's and step's, the
slowest rank's time is the job time (all-reduce MAX), and value = all ranks' pairs / that time."""

from __future__ import annotations

import os
import subprocess
import sys
import textwrap

from tests.conftest import ROOT
from tests.test_sharding_gloo import free_port

WORKER = textwrap.dedent(
    """
    import json, os, sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    import bench

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    total, B, steps, warm = bench.N_SEQS * (bench.N_SEQS - 1) // 2, 1 << 19, 6, 2
    mine = [bench.step_block(s, rank, world, B, total, steps) for s in range(steps)]
    got = [None] * world
    dist.all_gather_object(got, mine)
    elapsed = bench.max_over_ranks(1.0 + rank, world)    # rank 1 is the slow one
    value = bench.job_value(steps, B, world, elapsed)
    # the step pipeline on CPU: each step's result block names (rank, step); the gather of every
    # step must hold every rank's block of that step, and the line's two times are reported
    b, m = 64, 4
    pipe = bench.StepPipeline(world, b, m, torch.device("cpu"))
    out = [torch.empty((b, 2, m), dtype=torch.float64) for _ in range(2)]
    seen = []

    def kernel(k, slot):
        out[slot].fill_(1000.0 * rank + k)

    for k in range(warm + steps):
        pipe.step(k, kernel, out, None, record=k >= warm)
        g = pipe.gathered.view(world, b, 2, m)
        seen.append([float(g[r].min()) for r in range(world)] + [float(g[r].max()) for r in range(world)])
    pipe.drain()
    with open(os.environ["OUT"] + f".{{rank}}", "w") as fh:
        json.dump({{"blocks": got, "elapsed": elapsed, "value": value, "seen": seen,
                   "kernel_ms": pipe.kernel_ms(), "gather_ms": pipe.gather_ms(), "nk": len(pipe.kev),
                   "ng": len(pipe.gev)}}, fh)
    dist.destroy_process_group()
    """
)


def test_bench_two_ranks_gloo(tmp_path):
    import json

    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=str(ROOT)))
    out = tmp_path / "res"
    env = dict(os.environ, OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [json.loads((tmp_path / f"res.{k}").read_text()) for k in range(2)]
    B = 1 << 19
    total = 50_000 * 49_999 // 2
    starts = [b for blocks in res[0]["blocks"] for b in blocks]
    assert len(set(starts)) == len(starts)
    spans = sorted(starts)
    assert all(b - a >= B for a, b in zip(spans, spans[1:]))  # no two blocks overlap
    assert spans[0] == 0 and spans[-1] == total - B             # the whole triangle, first to last pair
    for rec in res:
        assert rec["elapsed"] == 2.0                        # the slower rank's time on both
        assert rec["value"] == 6 * B * 2 / 2.0              # all ranks' pairs / that time
        assert rec["nk"] == 6 and rec["ng"] == 6            # timed steps only, kernel and gather apart
        assert rec["kernel_ms"] >= 0 and rec["gather_ms"] >= 0
        for k, row in enumerate(rec["seen"]):               # step k's gather: rank r's block = 1000 r + k
            assert row == [float(k), 1000.0 + k, float(k), 1000.0 + k]


DIST_LEG_WORKER = textwrap.dedent(
    """
    import json, os, sys, time
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    import bench_secondary

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()

    class Res:
        seconds_taken = 0.25

    class Task:  # stands in for VersusAll: rank r takes 0.1 (r + 1) s, of which 0.01 (r + 1) s talking
        timings = None

        def start(self):
            time.sleep(0.1 * (rank + 1))
            self.timings = {{"comm_s": 0.01 * (rank + 1), "compute_s": 0.05 * (rank + 1), "reduce_s": 0.0}}
            return Res()

    t = Task()
    rec = bench_secondary.timed_dist_task(t.start, lambda: t.timings, world, rank)
    with open(os.environ["OUT"] + f".{{rank}}", "w") as fh:
        json.dump(rec, fh)
    dist.destroy_process_group()
    """
)


def test_dist_leg_timing_gloo(tmp_path):
    """The N > 1 leg's timing (bench_secondary.timed_dist_task, the config-5 leg bench.py runs on every
    rank when N > 1): the slowest rank's wall time on every rank, the task's comm / compute phases
    reduced to their maximum over ranks (comm reported apart from compute), rank 0's own
    seconds_taken."""
    import json

    script = tmp_path / "leg.py"
    script.write_text(DIST_LEG_WORKER.format(root=str(ROOT)))
    out = tmp_path / "leg"
    env = dict(os.environ, OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads((tmp_path / f"leg.{k}").read_text()) for k in range(2)]
    for k, rec in enumerate(recs):
        assert rec["n_ranks"] == 2
        assert 0.2 <= rec["wall_s"] < 1.5                 # rank 1's 0.2 s, on both ranks
        assert abs(rec["comm_s_max"] - 0.02) < 1e-12      # rank 1's comm
        assert abs(rec["compute_s_max"] - 0.10) < 1e-12
        assert rec["seconds_taken_rank0"] == (0.25 if k == 0 else None)
    assert recs[0]["wall_s"] == recs[1]["wall_s"]


def test_bench_dist_legs_wired():
    """bench.py runs the N > 1 legs on every rank after the timed region (before rank 0's line) and
    puts them in the line; rank 0 runs cpu_baseline at every N."""
    src = (ROOT / "bench.py").read_text()
    assert "if world > 1 and args.dist_legs:" in src and '"dist_legs": dist_legs' in src
    assert "if rank == 0 and not args.no_cpu_baseline:" in src
