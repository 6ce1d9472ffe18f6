"""GPU: the tasks under torch.distributed (2 ranks, gloo, one GPU shared) write the same files
as a single process: versusAll pair-space shards and versusReference query shards."""

from __future__ import annotations

import os
import subprocess
import sys
import textwrap

import pytest

from tests.conftest import ROOT
from tests.test_sharding_gloo import free_port

pytestmark = pytest.mark.gpu

SETUP = textwrap.dedent(
    """
    import sys
    sys.path.insert(0, {root!r})
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.synth import mutate, random_sequences
    from taxi2_amd.tasks import VersusAll, VersusReference

    def run(eng, out):
        raw = random_sequences(9, 60, 300, 71, "ACGTN", n_rate=0.02)
        seqs = [Sequence(f"s{{k}}", s, {{"v": str(k)}}) for k, s in enumerate(raw + mutate(raw[:4], 72, rate=0.1))]
        t = VersusAll()
        t.engine, t.progress_handler, t.work_dir = eng, None, out / "all"
        t.input.sequences = Sequences(seqs)
        t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.Kimura2P(), DistanceMetric.NCD()]
        t.start()
        q = random_sequences(11, 80, 250, 73, "ACGT")
        r = mutate(q[:5], 74, rate=0.2) + random_sequences(6, 80, 250, 75, "ACGT")
        v = VersusReference()
        v.engine, v.progress_handler, v.work_dir = eng, None, out / "ref"
        v.input.data = Sequences([Sequence(f"q{{k}}", s) for k, s in enumerate(q)])
        v.input.reference = Sequences([Sequence(f"r{{k}}", s) for k, s in enumerate(r)])
        v.params.pairs.write = False
        v.start()
    """
)

WORKER = SETUP + textwrap.dedent(
    """
    import os
    from pathlib import Path
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from taxi2_amd._native import Engine
    run(Engine(0), Path(os.environ["OUT"]))
    dist.barrier()
    dist.destroy_process_group()
    """
)


def test_tasks_two_ranks_match_single_process(tmp_path, engine):
    ns: dict = {}
    exec(SETUP.format(root=str(ROOT)), ns)
    ns["run"](engine, tmp_path / "single")
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=str(ROOT)))
    env = dict(os.environ, OUT=str(tmp_path / "dist"), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    files = sorted(p.relative_to(tmp_path / "single") for p in (tmp_path / "single").rglob("*") if p.is_file())
    assert files
    for f in files:
        assert (tmp_path / "dist" / f).read_bytes() == (tmp_path / "single" / f).read_bytes(), f
