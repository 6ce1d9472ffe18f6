#!/usr/bin/env python3
"""VALU issue roofline of the pre-aligned tile kernel (prealigned_kernel.hpp k_prealigned_tile): the
instruction mix of its word loop (gfx950 ISA) priced with the measured per-instruction issue costs
(tools/valu_peak -> profiles/r5/valu_peak.txt, which adds v_bcnt, v_bitop3 and the f64 ops; as tools/issue_ceiling.py does for the aligner),
combined with rocprofv3 PMC passes of the bench's `prealigned` leg (config 5's tile launches alone,
TAXI2_PREALIGNED_PARTS=config5) into profiles/prealigned_ceiling.json, which bench_secondary.py's
leg reads for its compute_roofline / traffic_roofline.

usage:
  make -C taxi2_amd/csrc asm
  python tools/tile_ceiling.py /tmp/taxi2_asm/capi-hip-amdgcn-amd-amdhsa-gfx950.s \\
      --valu gpurun_out/T/pmcsec_prealigned_valu/.../run_counter_collection.csv \\
      [--fetch ...csv --write ...csv] --pairs 19999900000 --words 32

The word loop = the innermost backward branch of the kernel whose body holds the LDS operand reads
(ds_read_b96 / b128) and the popcounts (v_bcnt); ceiling = 1 / (mean issue cycles of its VALU
instructions) [wave-instructions per SIMD-cycle]; achieved (bench) = the PMC's SQ_INSTS_VALU per
pair-word x pair-words per second / (1 024 SIMDs x clock).
"""

from __future__ import annotations

import argparse
import csv
import json
import re
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from issue_ceiling import price, valu_costs  # noqa: E402


def kernel_lines(lines: list[str], frag: str) -> list[str]:
    a = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\w*{frag}\w*:", l))
    b = next(i for i in range(a + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[a:b]


def word_loop(body: list[str]) -> list[str]:
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\w+):", l))}
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = body[labels[m.group(1)]:i + 1]
            if any("v_bcnt" in x for x in seg) and any("ds_read_b" in x for x in seg):
                loops.append((labels[m.group(1)], i))
    inner = [lp for lp in loops if not any(o != lp and lp[0] <= o[0] and o[1] <= lp[1] for o in loops)]
    a, b = max(inner, key=lambda lp: lp[1] - lp[0])
    return body[a:b + 1]


def pmc_sum(path: Path, pat: str) -> tuple[Counter, float, int]:
    tot, dur, seen = Counter(), 0.0, set()
    for r in csv.DictReader(open(path)):
        if re.search(pat, r["Kernel_Name"]):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            key = (r.get("Dispatch_Id"), r["Start_Timestamp"])
            if key not in seen:
                seen.add(key)
                dur += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return tot, dur, len(seen)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="k_prealigned_tileILi0ELb0E", help="mangled-name fragment")
    ap.add_argument("--kernel-regex", default=r"k_prealigned_tile<0, false>")
    ap.add_argument("--valu", required=True, help="PMC csv of the valu set")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--pairs", type=float, required=True, help="unordered pairs over the profiled launches")
    ap.add_argument("--words", type=int, required=True, help="32-column plane words per pair")
    ap.add_argument("--costs", default=str(ROOT / "profiles/r5/valu_peak.txt"))
    ap.add_argument("--out", default=str(ROOT / "profiles/prealigned_ceiling.json"))
    a = ap.parse_args()
    costs = valu_costs(Path(a.costs))
    loop = word_loop(kernel_lines(Path(a.asm).read_text().splitlines(), a.kernel))
    ops = [m.group(1) for l in loop if (m := re.match(r"^\s+(v_\w+)", l))]
    unlisted: Counter = Counter()
    cyc = [price(o, costs, unlisted) for o in ops]
    hist = Counter(re.sub(r"_(e32|e64|dpp|sdwa)$", "", o) for o in ops)
    mean = sum(cyc) / len(cyc)
    v, dur, nd = pmc_sum(Path(a.valu), a.kernel_regex)
    pair_words = a.pairs * a.words
    clock = v["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-9) / 1e9  # GRBM counts per XCD (8)
    ach = v["SQ_INSTS_VALU"] / (1024 * v["GRBM_GUI_ACTIVE"] / 8)
    rec = {
        "workload": "config5 tile kernel", "kernel": a.kernel_regex, "dispatches": nd,
        "pairs": a.pairs, "words_per_pair": a.words,
        "valu_instr_per_pair_word": v["SQ_INSTS_VALU"] / pair_words,
        "clock_ghz": clock, "pmc_kernel_s": dur * 1e-9,
        "pmc_instr_per_simd_clk": ach, "wait_over_active": v["SQ_WAIT_INST_ANY"] / max(1.0, v["SQ_ACTIVE_INST_ANY"]),
        "word_loop_valu": len(ops), "word_loop_mean_issue_cycles": mean,
        "ceiling_instr_per_simd_clk": 1.0 / mean, "pmc_frac_of_ceiling": ach * mean,
        "word_loop_histogram": dict(hist.most_common()), "priced_by_class": dict(unlisted),
        "source": f"{Path(a.valu).name} + {a.kernel} word loop of {Path(a.asm).name}",
    }
    hbm = 0.0
    if a.fetch:
        f, _, _ = pmc_sum(Path(a.fetch), a.kernel_regex)
        rec["fetch_bytes"] = f["FETCH_SIZE"] * 1024 * 2  # KB; gfx950 tallies half of each 128-B request
        hbm += rec["fetch_bytes"]
    if a.write:
        w, _, _ = pmc_sum(Path(a.write), a.kernel_regex)
        rec["write_bytes"] = w["WRITE_SIZE"] * 1024
        hbm += rec["write_bytes"]
    if a.fetch and a.write:
        rec["hbm_bytes_per_pair"] = hbm / a.pairs
    Path(a.out).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
