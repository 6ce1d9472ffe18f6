#!/usr/bin/env python3
"""VALU issue roofline of one kernel: its step-loop instruction mix (gfx950 ISA) priced with the
measured per-instruction issue costs (tools/valu_peak -> profiles/r2/valu_peak.txt), combined with
the rocprofv3 PMC pass of the same build into profiles/compute_ceiling.json (read by bench.py).

usage:
  make -C taxi2_amd/csrc asm        # /tmp/taxi2_asm/capi-hip-amdgcn-amd-amdhsa-gfx950.s
  python tools/issue_ceiling.py /tmp/taxi2_asm/capi-hip-amdgcn-amd-amdhsa-gfx950.s \\
      'k_alignt2ILi8ELi2ELb1ELi6E' profiles/r2/pmc_valu_alignt2.csv --batch 524288 --cells 1e6

Method.
* Loops = backward branches to a label above them; the fill step loops are those with a 16-byte
  global store (the trace) and at least 150 VALU instructions; within them, instructions are split
  into basic blocks and a block is HOT when it is reached on the straight path of the step (no
  s_cbranch_execz / s_cbranch_vccz jumps over it): the cold blocks (a pair's first row, a row byte
  other than A/C/G/T, the owner of column nB on a pair's last row) run once per pair or never.
* The trace block (byte packing + the 16-byte store, behind the band's lane mask) runs only on
  the steps where some lane of the wave meets the stored strip: it is priced with weight
  band_store_fraction(); with the out-of-band skip (split_skip) the whole trace-forming cell
  block has that weight and the no-trace cell block the rest (the fraction of (fill wave, step) pairs of a config-3 chain with a lane
  in the strip; 1.0 with --band 0).
* Each VALU opcode (suffixes _e32 / _e64 / _dpp / _sdwa stripped) gets the SIMD cycles per wave64
  instruction measured at 8 waves per SIMD in valu_peak.txt; an opcode the microbenchmark does
  not list gets the cost of its class (v_pk_* and 3-source VOP3 4.09, v_cmp / v_cndmask, other
  VOP2 ops as measured for their nearest listed relative, see CLASS_RULES) and is reported.
* ceiling = 1 / (mean cycles per hot VALU instruction)  [wave-instructions per SIMD-cycle];
  achieved = SQ_INSTS_VALU / (1 024 SIMDs x GRBM_GUI_ACTIVE / 8)  (PMC, same build and workload).
"""

from __future__ import annotations

import argparse
import csv
import json
import re
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

# fallbacks for opcodes valu_peak does not list: (regex, listed opcode whose cost applies)
CLASS_RULES = [
    (r"^v_pk_", "v_pk_add_u16"),
    (r"^v_(med3|max3|min3)_", "v_med3_i32"),
    (r"^v_(perm|bfi|alignbit|alignbyte|bfe|lshl_add|add_lshl|and_or|or3|xad|lshl_or|add3|mad|mbcnt)", "v_perm_b32"),
    (r"^v_(max|min)_(i32|u32|f32)", "v_max_i32"),
    (r"^v_(lshlrev|lshrrev|ashrrev)_b32", "v_lshlrev_b32"),
    (r"^v_(lshlrev|lshrrev|ashrrev)_b16", "v_add_u16"),
    (r"^v_(max|min)_(i16|u16|f16)", "v_max_i16"),
    (r"^v_(add|sub|subrev)_(u16|i16|f16)", "v_add_u16"),
    (r"^v_(add|sub|subrev)(_co)?(_ci)?_u32", "v_add_u32"),
    (r"^v_(and|or|xor|not)_b32", "v_and_b32"),
    (r"^v_(mov|readfirstlane|readlane|writelane)_b32", "v_mov_b32"),
    (r"^v_cvt_", "v_cvt_f32_i32"),
    (r"^v_cmp", "v_max_i32"),         # not measured: priced as a half-rate op (upper bound on cost)
    (r"^v_cndmask", "v_max_i32"),     # the vcc-form microbenchmark is hazard-bound (22.8 cyc): not used
    (r"^v_mul_", "v_mul_u32_u24"),
]


def valu_costs(path: Path) -> dict[str, float]:
    costs = {}
    for line in path.read_text().splitlines():
        m = re.match(r"^(v_\w+)\s+.*w8:\s+([\d.]+) cyc", line)
        if m:
            costs[m.group(1)] = float(m.group(2))
    return costs


def base_op(op: str) -> str:
    return re.sub(r"_(e32|e64|dpp|sdwa)$", "", op)


def price(op: str, costs: dict[str, float], unlisted: Counter) -> float:
    b = base_op(op)
    if b in costs and not b.startswith("v_cndmask"):
        return costs[b]
    for rx, ref in CLASS_RULES:
        if re.match(rx, b):
            unlisted[b] += 1
            return costs[ref]
    unlisted[b] += 1
    return max(costs.values())


def step_loops(lines: list[str]) -> list[tuple[int, int]]:
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(lines):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            a = labels[m.group(1)]
            body = lines[a:i + 1]
            nv = sum(1 for x in body if re.match(r"^\s+v_", x))
            if nv >= 150 and any("global_store_dwordx4" in x for x in body):
                loops.append((a, i))
    # innermost only: drop a loop that contains another
    return [lp for lp in loops if not any(o != lp and lp[0] <= o[0] and o[1] <= lp[1] for o in loops)]


def hot_instructions(body: list[str]) -> tuple[list[str], list[str]]:
    """Instructions of the blocks on the straight path: a forward s_cbranch_exec/vcc z jump marks
    everything up to its target label as a conditional (cold) block -- except the block holding
    the trace store, returned separately (second list)."""
    out, store, skip_to, block = [], [], None, []
    for l in body:
        lab = re.match(r"^(\.LBB\w+):", l)
        if lab and skip_to == lab.group(1):
            if any(op.startswith("global_store_dwordx4") for op in block):
                store.extend(block)
            skip_to, block = None, []
            continue
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        m = re.match(r"s_cbranch_(execz|vccz|vccnz|execnz|scc0|scc1)$", t[0])
        if m and skip_to is None and len(t) > 1:
            skip_to = t[1]
            continue
        if skip_to is None:
            out.append(t[0])
        else:
            block.append(t[0])
    return out, store


def split_skip(body: list[str], kernel: list[str], a: int):
    """The out-of-band skip (alignt2_kernel.hpp A2_SKIP_OUT_OF_BAND): a wave-uniform
    `s_cbranch_scc0/scc1 L` to an out-of-line stub (outside the loop) that `s_branch`es back to the
    in-line no-trace cells; the fall-through is the trace-forming cells + store, which end with
    `s_cbranch_execnz J` over the no-trace cells to the common tail at J.  Returns
    (prefix, trace_variant, no_trace_variant, tail) instruction-line lists, or None without it."""
    labels = {}
    for i, l in enumerate(kernel):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_cbranch_scc[01]\s+(\.LBB\w+)", l)
        if not m or m.group(1) not in labels:
            continue
        out = labels[m.group(1)]
        if a <= out < a + len(body):
            continue
        stub = []
        for l2 in kernel[out + 1:]:
            mb = re.match(r"^\s+s_branch\s+(\.LBB\w+)", l2)
            if mb:
                back = mb.group(1)
                break
            stub.append(l2)
        else:
            return None
        b = next((k for k, x in enumerate(body) if x.startswith(back + ":")), None)
        if b is None:  # an scc branch out of the loop that is not the skip's stub
            continue
        mj = next((re.match(r"^\s+s_cbranch_execnz\s+(\.LBB\w+)", x) for x in reversed(body[i:b])
                   if re.match(r"^\s+s_cbranch_execnz", x)), None)
        if mj is None:
            return None
        j = next((k for k, x in enumerate(body) if x.startswith(mj.group(1) + ":")), None)
        if j is None:
            return None
        return body[:i], body[i + 1:b], stub + body[b:j], body[j:]
    return None


def band_store_fraction(L: int, K: int, W: int, band: int, pairs: int) -> float:
    """Fraction of (fill wave, step) pairs of one chain (`pairs` pairs of L x L per stream, both
    streams alike) in which some lane's column block meets the stored strip of its row
    (alignt2_kernel.hpp a2_band_blocks with nA = nB = L)."""
    import numpy as np

    if band <= 0:
        return 1.0
    rows = pairs * L
    steps = rows + 63
    lanes = np.arange(64)
    hit = 0
    for w in range(W):
        t = 64 * w + lanes
        for st in range(steps):
            g = st - lanes
            ok = (g >= 0) & (g < rows)
            i = g % L + 1
            lo = (np.maximum(1, i - band) - 1) // K
            hi = (np.minimum(L, i + band) - 1) // K
            hit += bool(np.any(ok & (t >= lo) & (t <= hi)))
    return hit / (W * steps)


def pmc(path: Path, kernel_pat: str) -> dict[str, float]:
    tot: dict[str, float] = Counter()
    for r in csv.DictReader(open(path)):
        if re.search(kernel_pat, r["Kernel_Name"]):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            tot["_t0"] = float(r["Start_Timestamp"])
            tot["_t1"] = float(r["End_Timestamp"])
    return tot


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="mangled-name fragment, e.g. k_alignt2ILi8ELi2ELb1ELi6E")
    ap.add_argument("pmc_csv")
    ap.add_argument("--kernel-regex", default=r"k_alignt2<8, 2, true, 6>")
    ap.add_argument("--costs", default=str(ROOT / "profiles/r2/valu_peak.txt"))
    ap.add_argument("--batch", type=int, default=524288)
    ap.add_argument("--cells", type=float, default=1e6, help="useful DP cells per pair")
    ap.add_argument("--out", default=str(ROOT / "profiles/compute_ceiling.json"))
    ap.add_argument("--band", type=int, default=95, help="trace band of the run (capi.hip default at 1 000 bp)")
    ap.add_argument("--shape", default="1000,8,2,4", help="L,K,W,pairs per stream of the profiled chains")
    args = ap.parse_args()

    costs = valu_costs(Path(args.costs))
    lines = open(args.asm).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\w*{args.kernel}\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    unlisted: Counter = Counter()
    loops = []
    hot_all: Counter = Counter()
    L, K, W, P = (int(x) for x in args.shape.split(","))
    f = band_store_fraction(L, K, W, args.band, P)
    for a, b in step_loops(body):
        sk = split_skip(body[a:b + 1], body, a)
        if sk is None:  # one variant: hot blocks weight 1, the trace store block weight f
            hot, store = hot_instructions(body[a:b + 1])
            segs = [(hot, 1.0), (store, f)]
            skip_valu = 0
        else:  # prefix + tail weight 1; trace cells + store weight f; no-trace cells weight 1 - f
            pre, tr, nt, tail = sk
            h_pre, s_pre = hot_instructions(pre)
            h_tr, s_tr = hot_instructions(tr)
            h_nt, _ = hot_instructions(nt)
            h_tl, s_tl = hot_instructions(tail)
            hot = h_pre + h_tl
            store = s_pre + h_tr + s_tr + s_tl
            segs = [(hot, 1.0), (store, f), (h_nt, 1.0 - f)]
            skip_valu = sum(1 for op in h_nt if op.startswith("v_"))
        segs = [([op for op in ops if op.startswith("v_")], wgt) for ops, wgt in segs]
        hist = Counter(base_op(op) for op in segs[0][0])
        shist = Counter(base_op(op) for op in segs[1][0])
        cyc = sum(wgt * sum(price(op, costs, unlisted) for op in ops) for ops, wgt in segs)
        n = sum(wgt * len(ops) for ops, wgt in segs)
        loops.append({"lines": [start + a + 1, start + b + 1], "hot_valu": len(segs[0][0]),
                      "trace_block_valu": len(segs[1][0]), "trace_block_weight": f,
                      "no_trace_block_valu": skip_valu, "no_trace_block_weight": (1.0 - f) if skip_valu else 0.0,
                      "cycles": cyc, "mean_cyc": cyc / max(1e-9, n),
                      "histogram": dict(hist.most_common()), "trace_block_histogram": dict(shist.most_common())})
        for ops, wgt in segs:
            for op in ops:
                hot_all[base_op(op)] += wgt
    n_all = sum(hot_all.values())
    cyc_all = sum(price(op, costs, Counter()) * c for op, c in hot_all.items())
    mean_cyc = cyc_all / n_all
    p = pmc(Path(args.pmc_csv), args.kernel_regex)
    insts = p["SQ_INSTS_VALU"]
    xcd_cycles = p["GRBM_GUI_ACTIVE"] / 8.0
    secs = (p["_t1"] - p["_t0"]) * 1e-9
    achieved = insts / (1024 * xcd_cycles)
    rec = {
        "workload": "config3",
        "kernel": args.kernel_regex,
        "batch": args.batch,
        "valu_instr_per_cell": insts / (args.batch * args.cells),
        "clock_ghz": xcd_cycles / secs / 1e9,
        "pmc_instr_per_simd_clk": achieved,
        "mean_issue_cycles_per_valu": mean_cyc,
        "ceiling_instr_per_simd_clk": 1.0 / mean_cyc,
        "pmc_frac_of_ceiling": achieved * mean_cyc,
        "full_rate_share": sum(c for op, c in hot_all.items() if price(op, costs, Counter()) < 3.0) / n_all,
        "full_rate_cycles": costs.get("v_add_u32", 2.28),  # the full-rate (VOP2 32-bit) issue cost
        "trace_band": args.band,
        "trace_block_weight": f,
        "step_loops": loops,
        "priced_by_class": dict(unlisted),
        "source": f"{Path(args.pmc_csv).relative_to(ROOT) if Path(args.pmc_csv).is_absolute() else args.pmc_csv} "
                  f"(SQ_INSTS_VALU, GRBM_GUI_ACTIVE); {Path(args.costs).name} (measured issue cycles); "
                  f"step-loop ISA of {args.kernel} (tools/issue_ceiling.py)",
    }
    Path(args.out).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps({k: v for k, v in rec.items() if k != "step_loops"}, indent=1))
    for lp in loops:
        print(lp["lines"], lp["hot_valu"], round(lp["mean_cyc"], 3), list(lp["histogram"].items())[:12])


if __name__ == "__main__":
    main()
