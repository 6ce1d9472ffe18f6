#!/usr/bin/env python3
"""Condensed view of the packed aligner's fill step loops in a gfx950 .s file: per loop the VALU
count, the scratch (spill) and vmcnt waits, and the non-VALU instructions in order.
usage: python tools/step_isa.py /tmp/isa/at2.s [--kernel k_alignt2ILi8ELi2ELb1ELi6E] [--show]"""
from __future__ import annotations

import argparse
import collections
import re


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="k_alignt2ILi8ELi2ELb1ELi6E")
    ap.add_argument("--show", action="store_true")
    a = ap.parse_args()
    text = open(a.asm).read()
    m = re.search(r"^(_Z\w*" + a.kernel + r"\w*):", text, re.M)
    body = text[m.start(): text.index(".Lfunc_end", m.start())].splitlines()
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
    for i, l in enumerate(body):
        mm = re.search(r"s_branch (\.LBB\w+)|s_cbranch_\w+ (\.LBB\w+)", l)
        if not mm:
            continue
        tgt = mm.group(1) or mm.group(2)
        if tgt in labels and labels[tgt] < i:
            seg = body[labels[tgt]: i + 1]
            if not any("global_store_dwordx4" in s for s in seg):
                continue
            ops = [s.strip().split()[0] for s in seg if s.strip() and not s.strip().startswith((";", "."))]
            valu = sum(o.startswith("v_") for o in ops)
            c = collections.Counter(o for o in ops if not o.startswith("v_"))
            waits0 = sum(1 for s in seg if "vmcnt(0)" in s)
            print(f"loop {tgt} lines {labels[tgt]}-{i}: {valu} VALU, scratch {sum(v for k, v in c.items() if 'scratch' in k)}, "
                  f"vmcnt(0) waits {waits0}, lds {sum(v for k, v in c.items() if k.startswith('ds_'))}")
            if a.show:
                nv = 0
                for s in seg:
                    t = s.strip()
                    if not t or t.startswith(";"):
                        continue
                    if t.startswith("v_"):
                        nv += 1
                        continue
                    if nv:
                        print(f"    [{nv} valu]")
                        nv = 0
                    print("  " + t[:100])


if __name__ == "__main__":
    main()
