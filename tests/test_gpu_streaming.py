"""GPU: the streamed versusAll path (taxi2_amd/streaming.py, config 5's output shape).

* TAXI2_METRIC_COUNTS: the packed counters of every ordered pair, turned into metrics by
  taxi2_counts_metrics_dev, equal the metrics the pair entry points write directly, bit for bit
  (and the oracle's counters).
* taxi2_subset_aggregate_dev fed row blocks equals the host aggregation over the full matrix
  (the reference's x-major summation order, versus_all.py:57-96, 617-640), bit for bit.
* VersusAll with params.engine.stream = True (row blocks of a few rows) writes files byte-
  identical to the dense path: linear / matricial / summary / subsets / aligned pairs, with
  partitions, percentage_multiply, identical duplicates (the diagonal rule), NCD, pre-aligned.
* The same under torch.distributed with 2 ranks: gloo on the one GPU of the box, and RCCL (nccl)
  when the box has two GPUs (skipped otherwise): rank 0 writes, the other rank sends its blocks.
Reference: /root/reference/src/itaxotools/taxi2/tasks/versus_all.py:732-773 (streamed drain).
"""

from __future__ import annotations

import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from tests.conftest import ROOT
from tests.seqgen import family_sequences, mutate, random_sequences
from tests.test_gpu_parity import METRICS, SCORE_SETS
from tests.test_sharding_gloo import free_port

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("align", [True, False])
def test_counts_mode_equals_direct_metrics(engine, oracle_c, align):
    import torch

    from taxi2_amd._native import tri_pairs, unpack_counts

    seqs = family_sequences(14, 700, 0x31, ancestors=3) + ["", "A", "NNNN"]
    if not align:
        seqs = random_sequences(15, 0, 200, 9, "ACGTacgtN--?")
    st = engine.upload(seqs, align=align)
    a, b = tri_pairs(len(seqs))
    k = len(a)
    direct = engine.all_pairs(st, 0, k, METRICS, SCORE_SETS["default"])
    counts = engine.all_pairs(st, 0, k, ("counts",), SCORE_SETS["default"])
    if align:
        exp, _ = oracle_c.batch(seqs, a, b, align=True, scores=SCORE_SETS["default"])
        c = unpack_counts(counts[:, :, 0])
        valid = c[..., 0]
        assert np.array_equal(np.isfinite(exp[..., 0]), valid > 0)
    dc = torch.as_tensor(counts.reshape(-1).view(np.int64)).cuda()
    for scale in (1.0, 100.0):
        out = torch.empty((dc.numel(), len(METRICS)), dtype=torch.float64, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            engine.counts_metrics_dev(dc.data_ptr(), dc.numel(), METRICS, out.data_ptr(), scale, s.cuda_stream)
        s.synchronize()
        got = out.cpu().numpy().reshape(direct.shape)
        ref = direct * 100.0 if scale != 1.0 else direct
        assert np.array_equal(np.nan_to_num(got, nan=7.0), np.nan_to_num(ref, nan=7.0))
        assert np.array_equal(np.signbit(got[got == 0]), np.signbit(ref[ref == 0]))
    st.free()


def test_subset_aggregate_dev_row_blocks(engine):
    import torch

    from taxi2_amd._native import subset_aggregate
    from taxi2_amd.tasks.subsets import SubsetAggregatorDev

    rng = np.random.default_rng(3)
    n, m = 57, 3
    A = rng.random((n, n, m)) * 30
    A[rng.random((n, n, m)) < 0.1] = np.nan
    A[rng.random((n, n, m)) < 0.05] = -0.0
    ids = [f"s{i}" for i in range(n)]
    part = {i: ("g%d" % (k % 5) if k % 7 else None) for k, i in enumerate(ids)}
    agg = SubsetAggregatorDev(engine, ids, part, m)
    Dd = torch.as_tensor(A).cuda()
    with torch.cuda.stream(torch.cuda.Stream()):
        for x0 in range(0, n, 8):
            x1 = min(n, x0 + 8)
            agg.add(Dd[x0:x1], x0, x1)
    torch.cuda.synchronize()
    st = agg.result()
    from taxi2_amd.tasks.subsets import subset_codes

    code, subsets = subset_codes(ids, part)
    host = subset_aggregate(A, code, len(subsets))
    assert np.array_equal(st.count, host.count)
    ok = host.count > 0
    for got, exp in ((st.mean, np.where(ok, host.sum / np.maximum(host.count, 1), np.nan)),
                     (st.min, np.where(ok, host.min, np.nan)), (st.max, np.where(ok, host.max, np.nan))):
        assert np.array_equal(np.nan_to_num(got, nan=-9.0), np.nan_to_num(exp, nan=-9.0))


TASK = textwrap.dedent(
    """
    import sys
    sys.path.insert(0, {root!r})
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.partitions import Partition
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.synth import mutate, random_sequences
    from taxi2_amd.tasks import VersusAll

    def run(eng, out, stream, variant):
        raw = random_sequences(11, 60, 300, 81, "ACGTN", n_rate=0.02)
        raw = raw + mutate(raw[:5], 82, rate=0.1)
        seqs = [Sequence(f"s{{k}}", s, {{"v": str(k % 3)}}) for k, s in enumerate(raw)]
        # same sequence and extras under other ids (not identical full tuples: values, not None)
        seqs.append(Sequence("dup", raw[2], {{"v": "1"}}))
        seqs.append(Sequence("dup2", raw[2], {{"v": "1"}}))
        t = VersusAll()
        t.engine, t.progress_handler, t.work_dir = eng, None, out
        t.input.sequences = Sequences(seqs)
        t.params.engine.stream = stream
        t.params.engine.block_bytes = 3 * len(seqs) * 8 * 8  # ~3 rows per block
        t.params.engine.launch_pairs = 0
        if variant == "full":
            t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.UncorrectedWithGaps(),
                                          DistanceMetric.JukesCantor(), DistanceMetric.Kimura2P(),
                                          DistanceMetric.NCD()]
            t.params.format.percentage_multiply = True
            t.input.species = Partition({{s.id: "sp%d" % (k % 4) for k, s in enumerate(seqs) if k % 5}})
            t.input.genera = Partition({{s.id: "g%d" % (k % 2) for k, s in enumerate(seqs)}})
        elif variant == "generic":
            t.params.pairs.scores = dict(match_score=2, mismatch_score=-3, internal_open_gap_score=-5,
                                         internal_extend_gap_score=-2, end_open_gap_score=-1,
                                         end_extend_gap_score=-1)
        elif variant == "prealigned":
            t.params.pairs.align = False
            t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.JukesCantor()]
        elif variant == "dupids":  # duplicate ids (handler line grouping across row blocks), %g formatter
            for k in (2, 3, 4, 9):
                seqs[k] = Sequence("same", seqs[k].seq, seqs[k].extras)
            seqs[6] = Sequence("s5", seqs[6].seq, seqs[6].extras)
            t.input.sequences = Sequences(seqs)
            t.params.format.float = "{{:.5g}}"
            t.input.genera = Partition({{s.id: "g%d" % (k % 2) for k, s in enumerate(seqs)}})
        elif variant == "reductions":  # config-5 shape: pre-aligned, no N x N text, reductions only
            t.params.pairs.align = False
            t.params.pairs.write = False
            t.params.distances.write_linear = t.params.distances.write_matricial = False
            t.params.engine.write_summary = False
            t.params.engine.row_minima = "p"
            t.params.format.percentage_multiply = True
            t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.JukesCantor(),
                                          DistanceMetric.Kimura2P()]
            t.input.species = Partition({{s.id: "sp%d" % (k % 4) for k, s in enumerate(seqs) if k % 5}})
            t.input.genera = Partition({{s.id: "g%d" % (k % 2) for k, s in enumerate(seqs)}})
        t.start()
    """
)


def _files(root):
    return sorted(p.relative_to(root) for p in root.rglob("*") if p.is_file())


@pytest.mark.parametrize("variant", ["full", "generic", "prealigned", "dupids"])
def test_streamed_task_matches_dense(tmp_path, engine, variant):
    ns: dict = {}
    exec(TASK.format(root=str(ROOT)), ns)
    ns["run"](engine, tmp_path / "dense", False, variant)
    ns["run"](engine, tmp_path / "stream", True, variant)
    files = _files(tmp_path / "dense")
    assert files and files == _files(tmp_path / "stream")
    for f in files:
        assert (tmp_path / "stream" / f).read_bytes() == (tmp_path / "dense" / f).read_bytes(), f


WORKER = TASK + textwrap.dedent(
    """
    import os
    from pathlib import Path
    import torch
    import torch.distributed as dist
    backend = os.environ["BACKEND"]
    local = int(os.environ["LOCAL_RANK"])
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    from taxi2_amd._native import Engine
    run(Engine(local if backend == "nccl" else 0), Path(os.environ["OUT"]), True, os.environ.get("VARIANT", "full"))
    dist.barrier()
    dist.destroy_process_group()
    """
)


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
@pytest.mark.parametrize("variant", ["full", "reductions"])
def test_streamed_task_two_ranks(tmp_path, engine, backend, variant):
    """2 ranks stream their row blocks to rank 0 (gloo: both ranks on this GPU, stores in host
    memory; nccl = RCCL: one rank per GPU, stores in HBM, point-to-point sends)."""
    import torch

    if backend == "nccl" and torch.cuda.device_count() < 2:
        pytest.skip("RCCL path needs two GPUs (one process per GPU); this box has one")
    ns: dict = {}
    exec(TASK.format(root=str(ROOT)), ns)
    # "reductions": the sharded pre-aligned chain (row ranges per rank, subset state passed rank to
    # rank, row minima gathered) against one rank streaming every block
    ns["run"](engine, tmp_path / "single", variant == "reductions", variant)
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=str(ROOT)))
    env = dict(os.environ, OUT=str(tmp_path / "dist"), OMP_NUM_THREADS="1", BACKEND=backend, VARIANT=variant)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    files = _files(tmp_path / "single")
    assert files and files == _files(tmp_path / "dist")
    for f in files:
        assert (tmp_path / "dist" / f).read_bytes() == (tmp_path / "single" / f).read_bytes(), f


def test_streamed_reductions_only(tmp_path, engine):
    """Reductions without the N x N text (config 5's "gather only reductions" mode): per-row minima
    and the subset aggregates, with linear / matricial / summary / aligned-pairs output off."""
    ns: dict = {}
    exec(TASK.format(root=str(ROOT)), ns)
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.partitions import Partition
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    raw = random_sequences(14, 60, 300, 91, "ACGTN", n_rate=0.02)
    raw = raw + mutate(raw[:6], 92, rate=0.05) + [raw[3]]
    seqs = Sequences([Sequence(f"s{k}", s) for k, s in enumerate(raw)])
    part = Partition({f"s{k}": "g%d" % (k % 3) for k in range(len(raw))})

    def task(out, stream):
        t = VersusAll()
        t.engine, t.progress_handler, t.work_dir = engine, None, out
        t.input.sequences = seqs
        t.input.genera = part
        t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.Kimura2P()]
        t.params.engine.stream = stream
        t.params.engine.block_bytes = 4 * len(raw) * 8 * 8
        t.params.engine.launch_pairs = 0
        if stream:
            t.params.engine.row_minima = "k2p"
            t.params.engine.write_summary = False
            t.params.distances.write_linear = False
            t.params.distances.write_matricial = False
            t.params.pairs.write = False
        t.start()
        return t

    dense = task(tmp_path / "dense", False)
    red = task(tmp_path / "red", True)
    D = dense.distances[:, :, 1]
    for i in range(len(raw)):
        row = np.where(np.isfinite(D[i]), D[i], np.inf)
        j = int(np.argmin(row))
        if not np.isfinite(row[j]):
            assert red.row_minima[0][i] == -1
        else:
            assert red.row_minima[0][i] == j and red.row_minima[1][i] == row[j]
    assert not (tmp_path / "red" / "summary.tsv").exists()
    assert not (tmp_path / "red" / "distances" / "linear.tsv").exists()
    assert (tmp_path / "red" / "distances" / "row_minima.tsv").read_text().count("\n") == len(raw) + 1
    for f in sorted((tmp_path / "dense" / "subsets").rglob("*.tsv")):
        rel = f.relative_to(tmp_path / "dense")
        assert (tmp_path / "red" / rel).read_bytes() == f.read_bytes(), rel


def test_streamed_wide_sequences_match_dense(tmp_path, engine):
    """Past 32 767 bp the streamed store keeps f64 metric planes instead of 16-bit packed counters
    (aligned pairs of ~33 kb, the column-tiled aligner)."""
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    base = random_sequences(1, 33000, 33000, 301, "ACGT")[0]
    raw = [base, mutate([base], 302, rate=0.02)[0], mutate([base], 303, rate=0.05)[0][:32900]]
    seqs = Sequences([Sequence(f"w{k}", s) for k, s in enumerate(raw)])

    def run(out, stream):
        t = VersusAll()
        t.engine, t.progress_handler, t.work_dir = engine, None, out
        t.input.sequences = seqs
        t.params.pairs.write = False
        t.params.engine.stream = stream
        t.params.engine.block_bytes = 2 * len(raw) * 8 * 8
        t.start()

    run(tmp_path / "dense", False)
    run(tmp_path / "stream", True)
    files = _files(tmp_path / "dense")
    assert files and files == _files(tmp_path / "stream")
    for f in files:
        assert (tmp_path / "stream" / f).read_bytes() == (tmp_path / "dense" / f).read_bytes(), f
