#!/usr/bin/env python3
"""SGPR spill traffic inside a kernel's Newton passes, from the device assembly.

The compiler spills SGPRs it cannot keep into VGPR lanes (v_writelane_b32) and reloads them with
v_readlane_b32: VALU instructions.  This counts them per basic block of one kernel and reports the ones in
the Newton blocks (the blocks that hold the patch arithmetic: at least --min-valu VALU instructions and at
least one v_div_fmas / v_sqrt), so "are there reloads inside the pass loop" has a number.
usage: hipcc ... --cuda-device-only -S csrc/device/trace.hip -o trace.s
       python scripts/isa_spills.py trace.s [--kernel k_traceILi2ELb0ELb0E]
"""
from __future__ import annotations

import argparse
import re
from collections import Counter


def kernel_body(lines, pat):
    start = None
    for k, ln in enumerate(lines):
        if start is None and re.match(rf"^_Z\S*{pat}\S*:", ln):
            start = k
        elif start is not None and ln.startswith(".Lfunc_end"):
            return lines[start:k]
    raise SystemExit(f"kernel {pat} not found")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="k_traceILi2ELb0ELb0E")
    ap.add_argument("--min-valu", type=int, default=60)
    ap.add_argument("--blocks", action="store_true", help="list every heavy block")
    a = ap.parse_args()
    body = kernel_body(open(a.asm).read().splitlines(), a.kernel)
    blocks, cur = [], {"label": "entry", "ins": []}
    for ln in body:
        s = ln.strip()
        if re.match(r"^\.LBB\S+:", s):
            blocks.append(cur)
            cur = {"label": s.split(":")[0], "ins": []}
        elif s and not s.startswith((";", ".")):
            cur["ins"].append(s.split()[0])
    blocks.append(cur)
    tot = Counter()
    newton = Counter()
    nblocks = 0
    for b in blocks:
        c = Counter(b["ins"])
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        tot.update(c)
        if valu >= a.min_valu and any(k.startswith(("v_div_fmas", "v_sqrt")) for k in c):
            nblocks += 1
            newton.update(c)
    def row(c):
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        return {"valu": valu, "v_readlane": c["v_readlane_b32"], "v_writelane": c["v_writelane_b32"],
                "s_load": sum(v for k, v in c.items() if k.startswith("s_load")),
                "scratch": sum(v for k, v in c.items() if k.startswith("scratch_"))}
    print({"kernel": a.kernel, "whole_kernel": row(tot)})
    print({"newton_blocks": nblocks, **row(newton)})
    if a.blocks:  # every heavy block: the unrolled Newton iterations are the 170-330-VALU blocks with 3 v_div_fmas
        for b in blocks:
            c = Counter(b["ins"])
            valu = sum(v for k, v in c.items() if k.startswith("v_"))
            if valu >= a.min_valu or c["v_readlane_b32"] or c["v_writelane_b32"]:
                print(f'  {b["label"]:>12}  valu {valu:4d}  div_fmas {c["v_div_fmas_f32"]}  sqrt {c["v_sqrt_f32"]}  '
                      f'readlane {c["v_readlane_b32"]}  writelane {c["v_writelane_b32"]}')


if __name__ == "__main__":
    main()
