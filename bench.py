#!/usr/bin/env python3
"""Headline benchmark: aligned pairs/sec for versusAll at 1 000 bp (BASELINE.json metric).

Workload (BASELINE.json configs[2]): 50 000 synthetic 1 000 bp
sequences (seed 0x7A12, 64 ancestors, substitutions U(0, 0.20) ts:tv 2:1, 1 % indel pairs),
versusAll pair space N(N-1)/2 = 1.25e9 unordered pairs, every pair globally aligned (Gotoh,
default TaxI2 scores) and measured with p, p-gaps, jc, k2p for BOTH ordered pairs -- exactly
the work VersusAll.start() does per pair (versus_all.py:746-752).

A step = one block of `--batch` consecutive unordered pairs per GPU (shards of the pair space;
weak scaling: per-GPU work is fixed as N grows), results written to device memory, then (N > 1)
gathered to every rank with an RCCL all-gather over xGMI.  Inputs are resident in HBM before
the timed region.  value = pairs processed by all ranks / max-over-ranks wall time.

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "aligned pairs/sec (versusAll, 1 000 bp) at 1/2/4/8 MI355X; % HBM roofline"
METRICS = ("p", "p-gaps", "jc", "k2p")
N_SEQS = 50_000
SEQ_LEN = 1000
SEED = 0x7A12
HBM_PEAK_GBS = 8000.0               # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_SIMDS = 256 * 4                   # 256 CUs x 4 SIMDs
# The aligner's compute roofline is the VALU issue rate of ITS instruction mix, not a nominal
# lane-op peak: tools/valu_peak (profiles/r2/valu_peak.txt) measures 2.28 SIMD-cycles per wave64
# instruction for 32-bit add / logic / mov and the VOP2 16-bit ops, but 4.09 for every v_pk_* op,
# max / min / shifts and every 3-source VOP3 (v_perm, v_bfi, v_med3, ...), which is most of the
# fill.  tools/issue_ceiling.py weights the measured costs by the kernel's step-loop instruction
# histogram (gfx950 ISA) and combines them with the rocprofv3 PMC pass of the same build
# (SQ_INSTS_VALU, GRBM_GUI_ACTIVE) into this file; the bench reads it for the roofline.
COMPUTE_CEILING_JSON = ROOT / "profiles" / "compute_ceiling.json"
def b_pair(L: int, M: int) -> int:
    """SURVEY.md §8(d) canonical algorithmic bytes per unordered pair: 2 * ceil(L/4) + 8 * M."""
    return 2 * math.ceil(L / 4) + 8 * M


def step_block(step: int, rank: int, world: int, batch: int, total_pairs: int, nsteps: int = 1) -> int:
    """First pair of the block rank `rank` runs at timed step `step` (0 .. nsteps - 1; warmup steps
    reuse them): the nsteps x world blocks (weak scaling: `batch` pairs per rank and step) are spread
    evenly over the whole config-3 triangle, first pair to last, so that the timed steps sample its
    long rows (the start) and its short ones (the end, where the row-shared aligner's units pair
    fewer rows) alike -- versus_all.py:746-769 aligns every pair of the space."""
    T = nsteps * world
    i = (step % max(1, nsteps)) * world + rank
    return 0 if T <= 1 else (i * (total_pairs - batch)) // (T - 1)


class StepPipeline:
    """The bench's steps with N > 1's all-gather of each step's result block (north_star: RCCL
    all-gather of distance-matrix row blocks over xGMI) on a stream of its own, ordered after the
    step's kernel by an event, so that step k's gather overlaps step k + 1's kernel (double-buffered
    results: step k + 1 writes the other slot; step k + 2 waits for step k's gather before it
    rewrites slot k % 2).  Kernel and gather times are measured separately with events on their own
    streams (report gather time separately from kernel time).  On CPU (gloo, the
    tests) the same code runs with no streams and wall-clock timing."""

    def __init__(self, world: int, batch: int, m: int, device):
        import torch

        self.world, self.device = world, device
        self.cuda = device.type == "cuda"
        self.gstream = torch.cuda.Stream(device) if self.cuda and world > 1 else None
        self.gathered = (torch.empty((world * batch, 2, m), dtype=torch.float64, device=device)
                         if world > 1 else None)
        self.done = [None, None]  # per slot: the event after its last gather
        self.kev, self.gev = [], []

    def _event(self):
        import torch

        return torch.cuda.Event(enable_timing=True) if self.cuda else time.perf_counter

    def _mark(self, stream):
        if self.cuda:
            import torch

            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            return e
        return time.perf_counter()

    @staticmethod
    def _ms(a, b) -> float:
        return a.elapsed_time(b) if not isinstance(a, float) else (b - a) * 1e3

    def step(self, k: int, kernel, out: list, stream, record: bool) -> None:
        import torch.distributed as dist

        slot = k % 2
        if self.cuda and self.done[slot] is not None:
            stream.wait_event(self.done[slot])  # the gather of step k - 2 has read this slot
        e0 = self._mark(stream)
        kernel(k, slot)
        e1 = self._mark(stream)
        if record:
            self.kev.append((e0, e1))
        if self.world <= 1:
            return
        if self.cuda:
            import torch

            self.gstream.wait_event(e1)
            with torch.cuda.stream(self.gstream):
                g0 = self._mark(self.gstream)
                dist.all_gather_into_tensor(self.gathered, out[slot])
                g1 = self._mark(self.gstream)
            self.done[slot] = g1
        else:
            g0 = self._mark(None)
            dist.all_gather_into_tensor(self.gathered, out[slot])
            g1 = self._mark(None)
        if record:
            self.gev.append((g0, g1))

    def drain(self) -> None:
        if self.cuda and self.gstream is not None:
            import torch

            torch.cuda.current_stream(self.device).wait_stream(self.gstream)
            self.gstream.synchronize()

    def kernel_ms(self) -> float:
        return float(np.mean([self._ms(a, b) for a, b in self.kev])) if self.kev else float("nan")

    def gather_ms(self) -> float | None:
        return float(np.mean([self._ms(a, b) for a, b in self.gev])) if self.gev else None


def max_over_ranks(elapsed: float, world: int, device=None) -> float:
    """The slowest rank's wall time (all-reduce MAX; RCCL on GPUs, gloo in tests)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_value(steps: int, batch: int, world: int, elapsed: float) -> float:
    """Whole-job throughput: the pairs every rank processed / the slowest rank's time."""
    return steps * batch * world / elapsed


def parse() -> argparse.Namespace:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1 << 19, help="unordered pairs per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=8192,
                    help="pairs timed on the host oracle on all host threads (~6 s on 16 threads)")
    ap.add_argument("--cpu-sample-1t", type=int, default=512,
                    help="pairs timed on ONE host thread, the reference's serial loop shape (~6 s)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all host cores (max 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"))
    ap.add_argument("--secondary", default="allmetrics,config4,task,config5,config5_aligned,prealigned",
                    help="secondary legs after the headline (one GPU only; bench_secondary.py); '' = none")
    ap.add_argument("--dist-legs", default="config5",
                    help="legs every rank runs together after the headline when N > 1 (config5: BASELINE "
                         "configs[4] sharded over the ranks); '' = none")
    ap.add_argument("--dist-timeout", type=float, default=900.0,
                    help="seconds the N > 1 legs may take before they are reported as timed out")
    return ap.parse_args()


def main() -> None:
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus > 1 needs torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from taxi2_amd._native import Engine
    from taxi2_amd.synth import family_packed

    # ---- inputs resident in HBM before timing (every rank packs the same seeded set)
    buf, offs = family_packed(N_SEQS, SEQ_LEN, SEED)
    eng = Engine(local)
    seqset = eng.upload_packed(buf, offs, align=True)
    total_pairs = N_SEQS * (N_SEQS - 1) // 2
    B = int(args.batch)
    M = len(METRICS)
    # two result slots: step k's kernel writes slot k % 2 while step k - 1's all-gather (N > 1) still
    # reads the other one on the gather stream
    out = [torch.empty((B, 2, M), dtype=torch.float64, device="cuda") for _ in range(2)]
    scores = torch.empty((B,), dtype=torch.int32, device="cuda")
    stream = torch.cuda.Stream()  # a real stream handle: the kernel and its HIP events share it
    torch.cuda.set_stream(stream)
    pipe = StepPipeline(world, B, M, torch.device("cuda", local))

    def kernel(step: int, slot: int) -> None:
        eng.all_pairs_dev(seqset, step_block(step, rank, world, B, total_pairs, args.steps), B, METRICS,
                          out[slot].data_ptr(), None, scores.data_ptr(), stream.cuda_stream)

    for w in range(args.warmup):
        pipe.step(w, kernel, out, stream, record=False)
    pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        pipe.step(s, kernel, out, stream, record=True)
    pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, "cuda")

    kern_ms, gather_ms = pipe.kernel_ms(), pipe.gather_ms()
    value = job_value(args.steps, B, world, elapsed)
    bp = b_pair(SEQ_LEN, M)
    achieved_gbs = B * bp / (kern_ms * 1e-3) / 1e9
    traffic = None
    tj = Path(args.traffic_json)
    if tj.exists():
        try:
            rec = json.loads(tj.read_text())
            if rec.get("batch") == B and rec.get("workload") == "config3":
                traffic = rec.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    cells = float(SEQ_LEN) * SEQ_LEN
    gcups = B * cells / (kern_ms * 1e-3) / 1e9
    compute = compute_roofline(gcups)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:  # rank 0 at every N (after the timed region)
        cpu = cpu_baseline(args, buf, offs, eng, seqset,
                           [step_block(k, 0, world, B, total_pairs, args.steps) for k in range(args.steps)])
    secondary = None
    legs = [x for x in args.secondary.split(",") if x]
    if rank == 0 and world == 1 and legs:  # after the timed region, outside the headline
        import bench_secondary

        del out, scores
        torch.cuda.empty_cache()
        secondary = bench_secondary.run_all(eng, seqset, N_SEQS, legs)
    dist_legs = None
    if world > 1 and args.dist_legs:  # every rank, after the timed region and the CPU baseline
        dist_legs = run_dist_legs(args, eng, world, rank)
    from taxi2_amd._native import build_info

    build = build_info()

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # the fill computes in packed int16 halves (two DP cells per 32-bit register), admitted
            # only when every DP difference fits int16 (at_fits16): exact, not reduced precision
            "dtype": "int16x2 (packed, range-checked exact)",
            "data": "synthetic",
            "config": {
                "workload": "config3: versusAll 50 000 x 1 000 bp synthetic, Gotoh align (default "
                            "TaxI2 scores) + p/p-gaps/jc/k2p for both ordered pairs",
                "n_seqs": N_SEQS,
                "seq_len": SEQ_LEN,
                "pairs_per_step_per_gpu": B,
                "pair_space": total_pairs,
                "parallelism": f"pair-space shards x{world}" + (" + RCCL all-gather" if world > 1 else ""),
                "blocks": f"{args.steps} x {world} blocks spread evenly over the whole triangle (first to last pair)",
            },
            "kernel_ms": kern_ms,
            "gather_ms": gather_ms,
            "full_job_eta_s": total_pairs / value,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "bytes_per_pair": bp,
                "kernel_ms": kern_ms,
            },
            "compute_roofline": compute,
            "ceilings": ceilings(value / world, traffic, B, compute),
            "cpu_baseline": cpu,
            "secondary": secondary,
            "dist_legs": dist_legs,
            "build": build,
            "assumptions": [
                "Biopython 1.85's tie order among equal-scoring alignments is restated (end state M>Ix>Iy, "
                "each backward step the first tied predecessor; (y, x) = Ix/Iy swapped), not pinned: every "
                "reference alignment vector accepts all tied optima (DESIGN.md §2)",
                "the workload is the config-3 generator (synthetic, seeded); no reference number exists "
                "(BASELINE.json published = {})",
            ],
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        if dist_legs and dist_legs.get("timed_out"):
            # a collective left hanging: the line is out, leave without the group's teardown
            sys.stdout.flush()
            os._exit(0)
        dist.destroy_process_group()


def run_dist_legs(args, eng, world: int, rank: int) -> dict:
    """The N > 1 legs (bench_secondary.py leg_config5_dist), on every rank, in a worker thread with a
    deadline: a collective that never completes is reported as timed out instead of holding the
    headline line back (the ranks then exit without the process group's teardown)."""
    import threading

    import bench_secondary

    out: dict = {}

    def work():
        for name in [x for x in args.dist_legs.split(",") if x]:
            try:
                if name == "config5":
                    out[name] = bench_secondary.leg_config5_dist(eng, world, rank)
                else:
                    out[name] = {"error": f"unknown distributed leg {name}"}
            except Exception as e:  # a failing leg never takes the headline line with it
                out[name] = {"error": f"{type(e).__name__}: {e}"}

    th = threading.Thread(target=work, daemon=True)
    th.start()
    th.join(args.dist_timeout)
    if th.is_alive():
        out["timed_out"] = True
    return out


NORTH_STAR_PER_GPU = 1e8 / 8          # BASELINE.json north_star: >= 1e8 aligned pairs/s on 8 x MI355X
HBM_MEASURED_GBS = 6290.0             # measured achievable HBM bandwidth (MI355X_MICROARCH.md)


def ceilings(per_gpu: float, traffic: float | None, batch: int, compute: dict | None) -> dict:
    """What the kernel's own limits imply in the metric's unit (pairs/s per GPU): the VALU issue
    ceilings at today's measured instructions per cell (the kernel's mix, and every instruction at
    the full VOP2 rate), the HBM cap of today's measured bytes per pair (trace stream + walker
    fetches, PMC) at the measured achievable bandwidth, and the share of north_star's per-GPU rate."""
    out = {"north_star_per_gpu": NORTH_STAR_PER_GPU, "share_of_north_star_per_gpu": per_gpu / NORTH_STAR_PER_GPU}
    if compute:
        c = json.loads(COMPUTE_CEILING_JSON.read_text())
        cells = float(SEQ_LEN) * SEQ_LEN
        rate = N_SIMDS * c["clock_ghz"] * 1e9 / (c["valu_instr_per_cell"] * cells)  # pairs/s per instr/SIMD-clk
        out["valu_mix_ceiling_pairs_per_s"] = c["ceiling_instr_per_simd_clk"] * rate
        out["valu_full_rate_ceiling_pairs_per_s"] = rate / c.get("full_rate_cycles", 2.28)
        out["valu_instr_per_cell"] = c["valu_instr_per_cell"]
    if traffic:
        bpp = traffic / batch
        out["hbm_bytes_per_pair"] = bpp
        out["hbm_cap_pairs_per_s"] = HBM_MEASURED_GBS * 1e9 / bpp
    return out


def compute_roofline(gcups: float) -> dict | None:
    """VALU issue roofline of the timed kernel (see COMPUTE_CEILING_JSON): the ceiling is the
    issue rate of the kernel's measured instruction mix; achieved = the live GCUPS x the PMC
    instructions per cell, per SIMD-cycle at the PMC pass's clock."""
    if not COMPUTE_CEILING_JSON.exists():
        return None
    c = json.loads(COMPUTE_CEILING_JSON.read_text())
    if c.get("workload") != "config3":
        return None
    instr_per_cell = c["valu_instr_per_cell"]          # SQ_INSTS_VALU / useful cells (PMC)
    clock = c["clock_ghz"] * 1e9                          # GRBM_GUI_ACTIVE / 8 / kernel time (PMC)
    achieved = gcups * 1e9 * instr_per_cell / (N_SIMDS * clock)  # wave-instructions per SIMD-cycle
    peak = c["ceiling_instr_per_simd_clk"]
    full = 1.0 / c.get("full_rate_cycles", 2.28)  # every instruction at the full VOP2 rate
    return {
        "bound": "valu-issue",
        "unit": "wave64 VALU instructions per SIMD-cycle",
        "achieved": achieved,
        "peak": peak,
        "frac": achieved / peak,
        "full_rate_peak": full,
        "frac_of_full_rate": achieved / full,
        "full_rate_share_of_mix": c.get("full_rate_share"),
        "gcups": gcups,
        "ops_per_cell": instr_per_cell * 64,
        "source": c["source"],
    }


def cpu_baseline(args, buf, offs, eng, seqset, blocks):
    """Oracle (C restatement, kind "port") on pairs sampled from the timed blocks themselves (the
    same share of every block, seeded offsets), on all host cores and on ONE core (the reference's
    serial per-pair loop, versus_all.py:746-769).  The GPU check recomputes each timed block with
    the bench's own launch (all 524 288 pairs, the same segments, chains and grid) and compares the
    sampled pairs' metrics with the oracle's."""
    from oracle import oracle_c
    from taxi2_amd._native import tri_pairs

    B = int(args.batch)
    S = int(args.cpu_sample)
    per = max(1, S // len(blocks))
    rng = np.random.default_rng(0x7A12)
    picks = [(k0, np.sort(rng.choice(B, size=per, replace=False))) for k0 in blocks]
    pa, pb = [], []
    for k0, off in picks:
        a, b = tri_pairs(N_SEQS, k0, B)
        pa.append(a[off])
        pb.append(b[off])
    pa, pb = np.concatenate(pa), np.concatenate(pb)

    def timed(n: int, threads: int):
        t0 = time.perf_counter()
        exp, _ = oracle_c.batch((buf, offs), pa[:n], pb[:n], align=True, scores=(1, -1, -8, -1, -1, -1),
                                metrics=METRICS, threads=threads)
        return exp, time.perf_counter() - t0

    threads = args.cpu_threads or min(os.cpu_count() or 1, 16)
    S = len(pa)
    exp, dt = timed(S, threads)
    # one thread: every len(blocks)-th sample (the same blocks, fewer pairs)
    S1 = min(int(args.cpu_sample_1t), S)
    sel1 = np.linspace(0, S - 1, S1).astype(np.int64)
    t0 = time.perf_counter()
    oracle_c.batch((buf, offs), pa[sel1], pb[sel1], align=True, scores=(1, -1, -8, -1, -1, -1),
                   metrics=METRICS, threads=1)
    dt1 = time.perf_counter() - t0
    got = np.concatenate([eng.all_pairs(seqset, k0, B, METRICS)[off] for k0, off in picks])
    fin = np.isfinite(exp)
    same = bool(np.array_equal(np.isfinite(got), fin)
                and np.all(np.abs(got[fin] - exp[fin]) <= 1e-12)
                and np.array_equal(got[:, :, :2][fin[:, :, :2]], exp[:, :, :2][fin[:, :, :2]]))
    return {
        "value": S / dt,
        "unit": "pairs/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{S} pairs: {per} seeded random pairs of each of the {len(blocks)} timed {B}-pair blocks "
                  f"(first block at pair {blocks[0]}, last at {blocks[-1]}), C restatement (oracle/taxi2_oracle.c, "
                  f"gcc -O2) on {threads} host threads; GPU==CPU on the sample (each block recomputed with the "
                  f"bench's own launch; p/p-gaps exact, jc/k2p within 1e-12): {same}",
        "gpu_equals_cpu": same,
        "single_thread": {
            "value": S1 / dt1,
            "unit": "pairs/s",
            "cores": 1,
            "sample": f"{S1} of the same sampled pairs on one host thread (the reference's serial loop "
                      f"shape, versus_all.py:746-769)",
        },
    }


if __name__ == "__main__":
    main()
