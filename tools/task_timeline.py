"""Fill-stream timeline of a task trace (rocprofv3 --kernel-trace CSV, e.g. gpu_run.sh sectrace:task):
per k_alignr launch its duration, the idle gap before it on the fill's queue, and the time other
kernels overlapped it; then the span before the first and after the last fill.

    python tools/task_timeline.py gpurun_out/TAG/sectrace_task/run_kernel_trace.csv
"""

from __future__ import annotations

import csv
import sys


def main(path: str) -> None:
    tr = list(csv.DictReader(open(path)))
    for r in tr:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = min(r["s"] for r in tr)
    t1 = max(r["e"] for r in tr)
    fills = sorted((r for r in tr if "k_alignr" in r["Kernel_Name"]), key=lambda r: r["s"])
    prev = None
    busy = gaps = 0.0
    for f in fills:
        ov = {}
        for r in tr:
            if r is f:
                continue
            a, b = max(r["s"], f["s"]), min(r["e"], f["e"])
            if b > a:
                name = r["Kernel_Name"].split("(")[0].split("::")[-1][:20]
                ov[name] = ov.get(name, 0.0) + (b - a) / 1e6
        gap = (f["s"] - prev) / 1e6 if prev is not None else 0.0
        dur = (f["e"] - f["s"]) / 1e6
        busy += dur
        gaps += gap
        print(f"fill {(f['s'] - t0) / 1e6:9.1f} ms  dur {dur:7.1f}  gap {gap:7.1f}  overlapped "
              + ", ".join(f"{k} {v:.0f}" for k, v in sorted(ov.items(), key=lambda kv: -kv[1]) if v >= 1))
        prev = f["e"]
    print(f"fills {busy:.1f} ms, gaps between fills {gaps:.1f} ms, before the first "
          f"{(fills[0]['s'] - t0) / 1e6:.1f} ms, after the last {(t1 - fills[-1]['e']) / 1e6:.1f} ms, "
          f"trace span {(t1 - t0) / 1e6:.1f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
