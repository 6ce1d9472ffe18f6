#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a gfx950 .s file (make -C taxi2_amd/csrc asm).

usage: python tools/loop_stats.py /tmp/taxi2_asm/capi-hip-amdgcn-amd-amdhsa-gfx950.s 'k_alignILi8ELi2ELb0ELb1ELi2E' [min_valu]

Prints the six smallest loops with at least min_valu (100) VALU instructions.

A loop is a backward branch `s_cbranch_* / s_branch .LBB_x` to a label above it; the body is every
line from the label to the branch.  Counts: VALU (v_*), of which compares (v_cmp*), v_cndmask,
SALU (s_* minus branches / waitcnt / barrier), exec-mask writes, branches, LDS and DPP ops.
"""

from __future__ import annotations

import re
import sys
from collections import Counter


def main() -> None:
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\w*{pat}\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i, m.group(1)))
    min_valu = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    shown = 0
    for a, b, name in sorted(loops, key=lambda t: t[1] - t[0]):
        c = Counter()
        for l in body[a:b + 1]:
            t = l.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            op = t[0]
            if op.startswith("v_"):
                c["valu"] += 1
                if op.startswith("v_cmp"):
                    c["v_cmp"] += 1
                elif op.startswith("v_cndmask"):
                    c["v_cndmask"] += 1
                if "dpp" in l or "row_" in l or "wave_" in l:
                    c["dpp"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith("s_cbranch") or op == "s_branch":
                c["branch"] += 1
            elif op.startswith("s_"):
                if op in ("s_waitcnt", "s_barrier", "s_nop"):
                    c[op] += 1
                else:
                    c["salu"] += 1
                    if "exec" in l:
                        c["exec_write"] += 1
            elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
                c["vmem"] += 1
        if c["valu"] < min_valu or shown >= 6:
            continue
        shown += 1
        print(f"{name}: lines {a + start + 1}-{b + start + 1}  " + "  ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
