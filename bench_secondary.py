"""Secondary workloads bench.py measures after its headline line's timed region (one GPU, rank 0).

The headline (bench.py) is BASELINE.json's metric on config 3: the aligner over config-3 pairs with
four metrics, outputs resident in HBM.  These legs put the other numbers the driver should observe
into the same record (bench.py's ``secondary`` key), each on its own synthetic, seeded workload:

* ``task``: VersusAll.start() with the reference's defaults (versus_all.py:389-397: align, the four
  metrics, aligned_pairs.txt, linear.tsv, the matricial files, summary.tsv) on N = 5 000 config-3
  sequences, timed as the reference times it (Results.seconds_taken, versus_all.py:732-773), split by
  phase (task.timings).  The text files are written through the file API into /dev/null symlinks in
  a temporary directory (aligned_pairs.txt alone is ~55 GB at N = 5 000); their sizes are counted.
* ``config5``: VersusAll.start() on 200 000 x 1 000 pre-aligned rows (BASELINE.json configs[4], one
  GPU), p / jc / k2p x100, reductions only (row minima + 2-genus / ~1 000-species subset statistics):
  every one of the 4e10 ordered pairs evaluated and reduced on the GPU.
* ``config5_aligned``: config 5's aligned form on a stated subset (N = 12 000 of its generator):
  VersusAll.start() with Gotoh alignment of every pair, four metrics x100, streamed reductions.
* ``prealigned``: the pre-aligned path alone: config 2 on the ca2000 stand-in file and config 5's
  tile kernel over all 2.0e10 pairs, with its VALU-issue and traffic rooflines.
* ``config4``: versusReference slice, 4 096 queries x 10 000 references of 650 bp (seed 0x7A13
  generator), Gotoh align + p, closest reference + extras on the GPU (versus_reference.py:184-188,
  124-129).
* ``allmetrics``: config 3 with ALL metrics (BASELINE.json configs[2], "+ncd"): p / p-gaps / jc / k2p
  and NCD of the same alignment's strings (distances.py:351-358) from one fill per pair, on a block
  of config-3 pairs, split into the fill and the strings + deflate part.

Every leg prints a progress line to stderr and returns a dict (or {"error": ...}: a failing leg never
takes the headline line with it).
"""

from __future__ import annotations

import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

NULL_FILES = ("align/aligned_pairs.txt", "distances/linear.tsv", "summary.tsv", "distances/matricial/p.tsv",
              "distances/matricial/p-gaps.tsv", "distances/matricial/jc.tsv", "distances/matricial/k2p.tsv")


def _log(msg: str) -> None:
    print(f"[bench secondary] {msg}", file=sys.stderr, flush=True)


def prealigned_rows(n: int, L: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """Pre-aligned synthetic rows (config 2 / 5 stand-ins): lowercase acgt from the family generator
    (substitutions only: a pre-aligned row's gaps are its '-' runs), ~2 % '-' in short runs, 0.5 % 'n'."""
    from taxi2_amd.synth import family_codes

    rng = np.random.default_rng(seed)
    codes = family_codes(n, L, seed, ancestors=64, indel_rate=0.0)
    rows = np.frombuffer(b"acgt", dtype=np.uint8)[codes].copy()
    gap = rng.random((n, L)) < 0.01
    gap |= np.roll(gap, 1, axis=1)  # short runs
    rows[gap] = ord("-")
    rows[rng.random((n, L)) < 0.005] = ord("n")
    buf = np.concatenate([rows.reshape(-1), np.zeros(1, np.uint8)])
    return buf, np.arange(n + 1, dtype=np.int64) * L


def build_config5_task(n: int, L: int, eng, out: Path, block_gb: float, aligned: bool = False):
    """VersusAll configured as config 5's reductions-only run (see module docstring); returns
    (task, packed bytes, offsets) -- the bytes are None for the aligned form."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.partitions import Partition
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.tasks import VersusAll

    if aligned:  # config 5's generator (seed 0x7A14) with indels: Gotoh alignment of every pair
        from taxi2_amd.synth import family_sequences

        buf = offs = None
        seqs = [Sequence(f"s{k}", s) for k, s in enumerate(family_sequences(n, L, 0x7A14))]
    else:
        buf, offs = prealigned_rows(n, L, 0x7A14)
        raw = buf[:-1].reshape(n, L)
        seqs = [Sequence(f"s{k}", raw[k].tobytes().decode()) for k in range(n)]
    rng = np.random.default_rng(0x7A15)
    t = VersusAll()
    t.engine, t.progress_handler, t.work_dir = eng, None, out
    t.input.sequences = Sequences(seqs)
    # two genera (the few-subsets case that used to serialise the sums) and ~1 000 species
    t.input.genera = Partition({s.id: "g%d" % (k % 2) for k, s in enumerate(seqs)})
    t.input.species = Partition({s.id: "sp%d" % int(rng.integers(0, 1000)) for s in seqs})
    t.params.pairs.align = aligned
    t.params.pairs.write = False
    t.params.distances.write_linear = t.params.distances.write_matricial = False
    t.params.distances.metrics = [DistanceMetric.Uncorrected(), DistanceMetric.JukesCantor(),
                                  DistanceMetric.Kimura2P()]
    if aligned:
        t.params.distances.metrics.insert(1, DistanceMetric.UncorrectedWithGaps())
    t.params.format.percentage_multiply = True
    t.params.engine.stream = True
    t.params.engine.write_summary = False
    t.params.engine.row_minima = "p"
    t.params.engine.block_bytes = int(block_gb * (1 << 30))
    t.params.engine.timings = True
    return t, buf, offs


def leg_task(eng, n: int = 5000) -> dict:
    from taxi2_amd.sequences import Sequence, Sequences
    from taxi2_amd.synth import family_sequences
    from taxi2_amd.tasks import VersusAll

    _log(f"task: VersusAll.start() N = {n}")
    seqs = [Sequence(f"seq{k}", s) for k, s in enumerate(family_sequences(n, 1000, 0x7A12))]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as tmp:
        out = Path(tmp)
        for f in NULL_FILES:
            (out / f).parent.mkdir(parents=True, exist_ok=True)
            os.symlink("/dev/null", out / f)
        t = VersusAll()
        t.engine, t.progress_handler, t.work_dir = eng, None, out
        t.input.sequences = Sequences(seqs)
        t0 = time.perf_counter()
        res = t.start()
        wall = time.perf_counter() - t0
        files = sorted(str(p.relative_to(out)) for p in out.rglob("*") if p.is_file() or p.is_symlink())
    pairs = n * (n - 1) // 2
    ph = dict(t.timings or {})
    # the pipelined one-fill path: the fills' GPU time from events (the host phases overlap them)
    compute = ph.get("fill_gpu_s") or ph.get("compute_s")
    return {
        "workload": f"VersusAll.start() with the reference's defaults (align, p/p-gaps/jc/k2p, aligned_pairs.txt, "
                    f"linear.tsv, matricial/*.tsv, summary.tsv), {n} x 1 000 bp config-3 sequences; text files "
                    f"written through /dev/null symlinks in a temporary directory",
        "n_seqs": n, "unordered_pairs": pairs, "ordered_pairs": n * n,
        "seconds_taken": res.seconds_taken, "wall_s": wall,
        "unordered_pairs_per_s": pairs / res.seconds_taken,
        "compute_unordered_pairs_per_s": pairs / compute if compute else None,
        "compute_basis": "fill_gpu_s (HIP events around each block's fill)" if ph.get("fill_gpu_s") else "compute_s",
        "text_reserve_cus": int(os.environ.get("TAXI2_TEXT_RESERVE_CUS", t.params.engine.text_reserve_cus)),
        "text_pipeline": os.environ.get("TAXI2_TEXT_PIPELINE", t.params.engine.text_pipeline),
        # (the fused pipeline's transfer: 0 means its default, the copy kernel)
        "text_copy": int(os.environ.get("TAXI2_TEXT_COPY", t.params.engine.text_copy)) or (
            2 if os.environ.get("TAXI2_TEXT_PIPELINE", t.params.engine.text_pipeline) == "fused" else 0),
        "text_cu_mask": os.environ.get("TAXI2_TEXT_MASK", "1" if t.params.engine.text_cu_mask else "") not in ("", "0"),
        "phases_s": ph, "pairs_from_walks": bool(t.pairs_walked), "files": files,
    }


def leg_config5(eng, n: int = 200_000, L: int = 1000) -> dict:
    import torch

    _log(f"config5: building {n} x {L} pre-aligned rows")
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as tmp:
        t0 = time.perf_counter()
        task, _, _ = build_config5_task(n, L, eng, Path(tmp), 2.0)
        t_build = time.perf_counter() - t0
        _log("config5: VersusAll.start()")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = task.start()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    return {
        "workload": f"config5 reductions: VersusAll.start() on {n} x {L} pre-aligned synthetic rows (seed 0x7A14), "
                    f"p/jc/k2p x100, row minima + 2-genus / ~1 000-species subset statistics, one GPU",
        "n_seqs": n, "ordered_pairs": n * n, "seconds_taken": res.seconds_taken, "wall_s": wall,
        "ordered_pairs_per_s": n * n / wall, "phases_s": task.timings, "input_build_s": t_build,
    }


def timed_dist_task(start, timings, world: int, rank: int, sync=None, device=None) -> dict:
    """Time one collective task run on every rank the way bench.py times its headline: barrier and
    device sync on both sides, the slowest rank's wall time; the task's own phase times (its
    ``timings()`` dict) are reduced to their maximum over ranks, so ``comm_s`` -- the rank-to-rank
    state passing and the row-minima gather of the streamed path -- is reported apart from
    ``compute_s``."""
    import torch
    import torch.distributed as dist

    if sync:
        sync()
    dist.barrier()
    t0 = time.perf_counter()
    res = start()
    if sync:
        sync()
    local = time.perf_counter() - t0
    dist.barrier()
    ph = dict(timings() or {})
    keys = ("comm_s", "compute_s", "reduce_s")
    v = torch.tensor([local] + [float(ph.get(k, 0.0) or 0.0) for k in keys], dtype=torch.float64, device=device)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    out = {"wall_s": float(v[0]), "n_ranks": world}
    out.update({k + "_max": float(x) for k, x in zip(keys, v[1:].tolist())})
    out["seconds_taken_rank0"] = getattr(res, "seconds_taken", None) if rank == 0 else None
    return out


def leg_config5_dist(eng, world: int, rank: int, n: int = 200_000, L: int = 1000) -> dict:
    """BASELINE.json configs[4] on every GPU of the run: VersusAll.start() on 200 000 x 1 000 pre-aligned
    rows under torch.distributed (one process per GPU).  The streamed path shards the rows by rank
    (versus_all.py _stream_rows: row blocks computed on each rank's GPU, the subset statistics'
    state passed rank to rank, the row minima gathered to rank 0 -- RCCL point-to-point and gather
    over xGMI), p / jc / k2p x100, row minima + 2-genus / ~1 000-species subset statistics.  Strong
    scaling: the whole job is fixed as the ranks grow."""
    import torch

    _log(f"config5_dist: rank {rank}/{world}: building {n} x {L} pre-aligned rows")
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as tmp:
        task, _, _ = build_config5_task(n, L, eng, Path(tmp), 2.0)
        _log(f"config5_dist: rank {rank}: VersusAll.start()")
        rec = timed_dist_task(task.start, lambda: task.timings, world, rank, sync=torch.cuda.synchronize,
                              device=torch.device("cuda", torch.cuda.current_device()))
    rec.update({
        "workload": f"config5 on {world} GPUs: VersusAll.start() on {n} x {L} pre-aligned synthetic rows (seed "
                    f"0x7A14), p/jc/k2p x100, row minima + 2-genus / ~1 000-species subset statistics, rows "
                    f"sharded by rank, statistics state passed rank to rank, row minima gathered to rank 0",
        "n_seqs": n, "ordered_pairs": n * n, "ordered_pairs_per_s": n * n / rec["wall_s"], "scaling": "strong",
    })
    return rec


def leg_config5_aligned(eng, n: int = 12_000, L: int = 1000) -> dict:
    """Config 5's aligned (NW / Gotoh) form on a stated subset ("Run NW on a stated
    tile subset"): VersusAll.start() on N = 12 000 sequences of the config-5 generator (seed 0x7A14,
    1 000 bp, with indels), Gotoh align + p / p-gaps / jc / k2p x100, the streamed path's reductions
    (row minima + 2-genus / ~1 000-species subset statistics), no N x N text -- 1.44e8 ordered pairs,
    0.36 % of the full 200 000 job, which extrapolates linearly in pairs (the triangle store and the
    block assembly are per pair)."""
    import torch

    _log(f"config5_aligned: VersusAll.start() N = {n} x {L} bp, align + 4 metrics, reductions only")
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as tmp:
        task, _, _ = build_config5_task(n, L, eng, Path(tmp), 2.0, aligned=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = task.start()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    pairs = n * (n - 1) // 2
    full = 200_000 * 199_999 // 2
    return {
        "workload": f"config5 aligned subset: VersusAll.start() on {n} x {L} bp config-5-generator sequences "
                    f"(seed 0x7A14), Gotoh align + p/p-gaps/jc/k2p x100, row minima + 2-genus / ~1 000-species "
                    f"subset statistics (streamed reductions, no N x N text), one GPU",
        "n_seqs": n, "unordered_pairs": pairs, "seconds_taken": res.seconds_taken, "wall_s": wall,
        "unordered_pairs_per_s": pairs / wall, "phases_s": task.timings,
        "full_job_200k_hours_1gpu": full / (pairs / wall) / 3600,
        "full_job_200k_minutes_8gpu": full / (pairs / wall) / 8 / 60,
    }


PREALIGNED_CEILING_JSON = ROOT / "profiles" / "prealigned_ceiling.json"


def leg_prealigned(eng) -> dict:
    """The pre-aligned path (params.pairs.align = False, versus_all.py:546-552 on the raw rows):
    config 2 on BASELINE.md's stand-in file (samples/Taxi2test1_ca2000.tab, 1 999 rows, the full
    pair space, p / jc / k2p) and config 5's tile kernel alone over all 2.0e10 unordered pairs of
    200 000 x 1 000 synthetic rows (2^26-pair launches, outputs overwritten in HBM), kernel time from
    HIP events on the launch stream.  With profiles/prealigned_ceiling.json (tools/tile_ceiling.py:
    the tile kernel's PMC VALU count per pair-word and its instruction mix priced with the measured
    issue costs) the kernel's VALU-issue fraction and its real-traffic fraction are attached."""
    import json

    import torch

    from taxi2_amd.sequences import SequenceHandler, Sequences

    _log("prealigned: config2 (ca2000 stand-in) and config5's tile kernel at full size")
    out = {}
    path = ROOT / "tests" / "golden" / "samples" / "Taxi2test1_ca2000.tab"
    # TAXI2_PREALIGNED_PARTS=config5: the tile kernel alone (a PMC pass of just its launches)
    parts = os.environ.get("TAXI2_PREALIGNED_PARTS", "config2,config5").split(",")
    if path.exists() and "config2" in parts:
        seqs = [x.seq for x in Sequences.fromPath(path, SequenceHandler.Tabfile, idHeader="seqid",
                                                   seqHeader="sequence")]
        st = eng.upload(seqs, align=False)
        n = len(seqs)
        total = n * (n - 1) // 2
        o = torch.empty((total, 3), dtype=torch.float64, device="cuda")
        stream = torch.cuda.Stream()
        eng.all_pairs_dev(st, 0, total, ("p", "jc", "k2p"), o.data_ptr(), None, None, stream.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record(stream)
        for _ in range(reps):
            eng.all_pairs_dev(st, 0, total, ("p", "jc", "k2p"), o.data_ptr(), None, None, stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        dt = e0.elapsed_time(e1) * 1e-3 / reps
        st.free()
        del o
        out["config2_ca2000"] = {
            "workload": f"config 2 stand-in: samples/Taxi2test1_ca2000.tab ({n} rows, 416-618 columns), pre-aligned "
                        f"p/jc/k2p over all {total} unordered pairs, outputs in HBM",
            "pairs": total, "seconds": dt, "pairs_per_s": total / dt}
    n, L = 200_000, 1000
    buf, offs = prealigned_rows(n, L, 0x7A14)
    st = eng.upload_packed(buf, offs, align=False)
    del buf
    total = n * (n - 1) // 2
    B = 1 << 26
    o = torch.empty((B, 3), dtype=torch.float64, device="cuda")
    stream = torch.cuda.Stream()
    eng.all_pairs_dev(st, 0, B, ("p", "jc", "k2p"), o.data_ptr(), None, None, stream.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    launches = 0
    for k0 in range(0, total, B):
        eng.all_pairs_dev(st, k0, min(B, total - k0), ("p", "jc", "k2p"), o.data_ptr(), None, None, stream.cuda_stream)
        launches += 1
    e1.record(stream)
    e1.synchronize()
    dt = e0.elapsed_time(e1) * 1e-3
    st.free()
    words = (L + 31) // 32
    rec = {"workload": f"config 5 pre-aligned, tile kernel alone: {n} x {L} synthetic rows (seed 0x7A14), p/jc/k2p, "
                       f"all {total} unordered pairs in {launches} launches of 2^26, outputs overwritten in HBM",
           "pairs": total, "seconds": dt, "pairs_per_s": total / dt, "ms_per_launch": dt * 1e3 / launches,
           "pair_words_per_s": total * words / dt, "output_GBps": total * 24 / dt / 1e9}
    if PREALIGNED_CEILING_JSON.exists():
        c = json.loads(PREALIGNED_CEILING_JSON.read_text())
        instr_rate = total * words * c["valu_instr_per_pair_word"] / dt  # wave-instructions / s
        ach = instr_rate / (1024 * c["clock_ghz"] * 1e9)
        rec["compute_roofline"] = {
            "bound": "valu-issue", "unit": "wave64 VALU instructions per SIMD-cycle", "achieved": ach,
            "peak": c["ceiling_instr_per_simd_clk"], "frac": ach / c["ceiling_instr_per_simd_clk"],
            "full_rate_peak": 1 / 2.28, "frac_of_full_rate": ach * 2.28, "source": c["source"]}
        if c.get("hbm_bytes_per_pair"):
            gbps = c["hbm_bytes_per_pair"] * total / dt / 1e9
            rec["traffic_roofline"] = {"bound": "hbm", "achieved": gbps, "peak": 8000.0, "unit": "GB/s",
                                       "frac": gbps / 8000.0, "bytes_per_pair": c["hbm_bytes_per_pair"]}
    out["config5_tile"] = rec
    return out


def leg_config4(eng, q_slice: int = 4096, R: int = 10_000, L: int = 650) -> dict:
    from taxi2_amd.synth import family_sequences

    _log(f"config4: {q_slice} queries x {R} refs x {L} bp")
    refs = family_sequences(R, L, 0x7A13)
    qs = family_sequences(q_slice, L, 0x7A13 + 1)
    sq = eng.upload(qs, align=True)
    sr = eng.upload(refs, align=True)
    extras = ("p-gaps", "jc", "k2p")
    try:
        eng.closest(sq, sr, 0, min(8, q_slice), "p", extras)
        t0 = time.perf_counter()
        idx, d, ex, _ = eng.closest(sq, sr, 0, q_slice, "p", extras)
        dt = time.perf_counter() - t0
    finally:
        sq.free()
        sr.free()
    pairs = q_slice * R
    return {
        "workload": f"config4 slice: versusReference {q_slice} queries x {R} refs x {L} bp (seed 0x7A13 generator), "
                    f"Gotoh align + p, closest reference + extras p-gaps/jc/k2p on the GPU",
        "pairs": pairs, "seconds": dt, "pairs_per_s": pairs / dt, "gcups": pairs * L * L / dt / 1e9,
        "full_job_minutes_1gpu": 1e10 / (pairs / dt) / 60, "closest_found": int((idx >= 0).sum()),
    }


def leg_allmetrics(eng, seqset, n_seqs: int, count: int = 1 << 17) -> dict:
    """p / p-gaps / jc / k2p AND NCD for `count` config-3 pairs (both orientations) from ONE fill per
    pair, as VersusAll computes them (versus_all.py:546-552: one alignment per ordered pair feeds every
    metric): taxi2_all_pairs_dev with the five metrics -- the walkers write both orientations' aligned
    strings into HBM slots, NCD deflates them there (distances.py:351-358).  Timed with HIP events on
    the launch stream, outputs resident in HBM; the four-metric launch of the same block beside it
    splits the time into the fill and the strings + deflate part."""
    import torch

    from taxi2_amd._native import tri_pairs

    _log(f"allmetrics: {count} config-3 pairs, p/p-gaps/jc/k2p + ncd, one fill per pair")
    four, five = ("p", "p-gaps", "jc", "k2p"), ("p", "p-gaps", "jc", "k2p", "ncd")
    k0 = 1 << 20  # a block the headline's first steps do not time
    stream = torch.cuda.Stream()
    out = torch.empty((count, 2, 5), dtype=torch.float64, device="cuda")

    def timed(metrics, n) -> float:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.all_pairs_dev(seqset, k0, n, metrics, out.data_ptr(), None, None, stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3

    timed(five, 4096)  # warm: scratch, LDS attributes
    t0 = time.perf_counter()
    t_all = timed(five, count)
    wall = time.perf_counter() - t0
    vals = out.cpu().numpy()
    t_four = timed(four, count)
    # deflate input of the block, from a sample of the same pairs' strings (tri_strings_dev): per pair
    # C(x0), C(y0), C(x0 + y0), C(y1 + x1), and C(y1), C(x1) only when the (b, a) alignment differs
    S = min(count, 8192)
    cap = 2 * 1000 + 1
    sx = torch.empty((S, 2, cap), dtype=torch.uint8, device="cuda")
    sy = torch.empty((S, 2, cap), dtype=torch.uint8, device="cuda")
    sl = torch.empty((S, 2), dtype=torch.int32, device="cuda")
    eng.tri_strings_dev(seqset, k0, S, (), None, cap, sx.data_ptr(), sy.data_ptr(), sl.data_ptr(), None,
                        stream.cuda_stream)
    stream.synchronize()
    a, b = tri_pairs(n_seqs, k0, S)
    hx, hy, hl = sx.cpu().numpy(), sy.cpu().numpy(), sl.cpu().numpy()
    end = 2000  # 1 000 bp each
    dup = 0
    nbytes = 0
    for k in range(S):
        L0, L1 = int(hl[k, 0]), int(hl[k, 1])
        same = L0 == L1 and np.array_equal(hx[k, 0, end - L0:end], hx[k, 1, end - L1:end]) and \
            np.array_equal(hy[k, 0, end - L0:end], hy[k, 1, end - L1:end])
        dup += same
        nbytes += 4 * L0 + 2 * L1 + (0 if same else 2 * L1)
    deflate_bytes = nbytes * count / S
    return {
        "workload": f"config3 all metrics: {count} config-3 pairs (1 000 bp) from pair {k0}, Gotoh align + "
                    f"p/p-gaps/jc/k2p + NCD of the same alignment's strings, both ordered pairs, one fill per "
                    f"pair (taxi2_all_pairs_dev), outputs in HBM",
        "pairs": count, "seconds": t_all, "wall_s": wall, "pairs_per_s": count / t_all,
        "four_metric_s": t_four, "strings_and_ncd_s": t_all - t_four, "ncd_share": (t_all - t_four) / t_all,
        "deflate_input_bytes": deflate_bytes, "deflate_input_gb_per_s": deflate_bytes / (t_all - t_four) / 1e9,
        "same_alignment_both_orders": dup / S,
        "finite": bool(np.isfinite(vals).all()),
    }


def run_all(eng, seqset, n_seqs: int,
            legs=("allmetrics", "config4", "task", "config5", "config5_aligned", "prealigned")) -> dict:
    out = {}
    for name in legs:
        t0 = time.perf_counter()
        try:
            if name == "task":
                out[name] = leg_task(eng)
            elif name == "config5":
                out[name] = leg_config5(eng)
            elif name == "config5_aligned":
                out[name] = leg_config5_aligned(eng)
            elif name == "prealigned":
                out[name] = leg_prealigned(eng)
            elif name == "config4":
                out[name] = leg_config4(eng)
            elif name == "allmetrics":
                out[name] = leg_allmetrics(eng, seqset, n_seqs)
        except Exception as e:  # a failing leg is reported, never takes the headline with it
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        _log(f"{name} done in {time.perf_counter() - t0:.1f} s")
    return out


def main() -> None:
    """python bench_secondary.py LEG [LEG ...]: run legs alone (one JSON line each)."""
    import json

    import torch  # noqa: F401  -- torch's HIP runtime first (the engine shares it)

    from taxi2_amd._native import Engine
    from taxi2_amd.synth import family_packed

    eng = Engine(0)
    seqset = None
    for name in sys.argv[1:]:
        if name == "allmetrics" and seqset is None:
            buf, offs = family_packed(50_000, 1000, 0x7A12)
            seqset = eng.upload_packed(buf, offs, align=True)
        print(json.dumps({name: run_all(eng, seqset, 50_000, [name])[name]}), flush=True)


if __name__ == "__main__":
    main()
