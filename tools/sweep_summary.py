#!/usr/bin/env python3
"""Print a compact table of a tools/sweep.py log (variant bits decoded)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "mode" not in d:
        print(d)
        continue
    v = d["var"]
    tags = []
    if v & 128:
        tags.append("W%d" % ((v >> 8) & 7))
    if v & 32:
        tags.append("rs")
    for bit, name in ((2048, "w4"), (4096, "pair"), (8192, "t64"), (16384, "t256sorted"), (32768, "t128sorted"), (1 << 17, "grouped"), (1 << 18, "over3"), (1, "sa"), (8, "nohash"), (64, "cached")):
        if v & bit:
            tags.append(name)
    print(f"{d['config']} {d['mode']:>10} {v:6d} {'+'.join(tags) or 'wg':<18} {d['ms_median']:.4f} {d['hbm_frac']:.4f}")
