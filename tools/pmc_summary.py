#!/usr/bin/env python3
"""Summarise a tools/profile_r1.sh run into profiles/: kernel stats + per-launch HBM traffic.

usage: python tools/pmc_summary.py gpurun_out/prof_a1 profiles/r1 --tag align1

Writes <dst>/kernel_stats_<tag>.csv, <dst>/pmc_{valu,fetch,write}_<tag>.csv, <dst>/bench_<tag>.json
and profiles/pmc_traffic.json (read by bench.py for roofline.traffic): FETCH_SIZE + WRITE_SIZE (KB,
separate rocprofv3 --pmc passes over one bench launch) summed over the path's kernels, x 1024.
"""

from __future__ import annotations

import argparse
import csv
import json
import shutil
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def counters(path: Path) -> dict[str, dict[str, float]]:
    out: dict[str, dict[str, float]] = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        out[name][r["Counter_Name"]] = out[name].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--batch", type=int, default=524288)
    ap.add_argument("--band", type=int, default=95, help="trace band of the profiled run")
    args = ap.parse_args()
    src, dst = Path(args.src), Path(args.dst)
    dst.mkdir(parents=True, exist_ok=True)
    shutil.copy(src / "trace/run_kernel_stats.csv", dst / f"kernel_stats_{args.tag}.csv")
    for k in ("valu", "fetch", "write"):
        shutil.copy(src / f"pmc_{k}/run_counter_collection.csv", dst / f"pmc_{k}_{args.tag}.csv")
    shutil.copy(src / "bench.json", dst / f"bench_{args.tag}.json")
    fetch = counters(src / "pmc_fetch/run_counter_collection.csv")
    write = counters(src / "pmc_write/run_counter_collection.csv")
    kernels = sorted(set(fetch) | set(write))
    per = {k: {"fetch_kb": fetch.get(k, {}).get("FETCH_SIZE", 0.0), "write_kb": write.get(k, {}).get("WRITE_SIZE", 0.0)}
           for k in kernels}
    # gfx950: FETCH_SIZE tallies each 128-B request as 64 B (MI355X_MICROARCH.md HBM section): x 2
    total_kb = sum(2.0 * v["fetch_kb"] + v["write_kb"] for v in per.values())
    rec = {
        "workload": "config3",
        "batch": args.batch,
        "kernels": per,
        "hbm_bytes_per_launch": total_kb * 1024.0,
        "source": f"{dst.relative_to(ROOT) if dst.is_absolute() else dst}/pmc_fetch_{args.tag}.csv, pmc_write_{args.tag}.csv",
        "note": "WRITE_SIZE (KB) x 1024: exact for the 16-B-per-lane trace stores (MI355X_MICROARCH.md HBM "
                "section). FETCH_SIZE (KB) x 1024 x 2: gfx950 tallies each 128-B request as 64 B (same section); "
                "the walker's reads are single-byte gathers whose lines this counts once each.  Separate "
                "rocprofv3 --pmc passes over one launch of bench.py --steps 1 --warmup 0.",
        "trace_band": args.band,
    }
    (ROOT / "profiles/pmc_traffic.json").write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
