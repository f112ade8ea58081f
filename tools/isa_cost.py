#!/usr/bin/env python3
"""Weighted VALU issue cost of a kernel's instruction stream (gfx950 rates
measured by tools/probes/valu_rate.hip: VOP1/VOP2/VOPC e32 encodings issue one
wave64 instruction per 2 cycles, VOP3 encodings per 4; 64-bit ops and
v_mad_u64_u32 counted 8).  usage: isa_cost.py file.s kernel_symbol_substring"""
import re
import sys
from collections import Counter


def kernel_lines(path, sym):
    lines = open(path).read().splitlines()
    out, on = [], False
    for ln in lines:
        if not on and re.match(r"^_Z\w*" + re.escape(sym) + r"\w*:", ln):
            on = True
            continue
        if on:
            out.append(ln)
            if "s_endpgm" in ln:
                break
    return out


def cost(op):
    if op.startswith("v_"):
        if any(x in op for x in ("_u64", "_b64", "_i64", "_f64")):
            return 8
        if op.endswith("_e32") or op.startswith("v_cmp") and op.endswith("_e32") or op in ("v_readfirstlane_b32", "v_nop"):
            return 2
        return 4
    return 0


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, sym)
    blocks, cur = {}, "entry"
    blocks[cur] = Counter()
    for ln in lines:
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):", ln)
        if m:
            cur = m.group(1)
            blocks.setdefault(cur, Counter())
            continue
        m = re.match(r"^\s+([a-z_0-9]+)", ln)
        if m:
            blocks[cur][m.group(1)] += 1
    tot = Counter()
    for b, c in blocks.items():
        v = sum(n for op, n in c.items() if op.startswith("v_"))
        cyc = sum(cost(op) * n for op, n in c.items())
        s = sum(n for op, n in c.items() if op.startswith("s_"))
        if v or s:
            print(f"{b:14s} valu {v:5d} salu {s:4d} valu_cycles {cyc:6d}")
        tot.update(c)
    print("total valu", sum(n for op, n in tot.items() if op.startswith("v_")),
          "cycles", sum(cost(op) * n for op, n in tot.items()))


if __name__ == "__main__":
    main()
