#!/usr/bin/env python3
"""Pivot a tools/sweep.py log: one row per (config, mode), one column per variant (median ms), best marked."""
import json
import sys

rows, cols = {}, []
for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "mode" not in d:
        continue
    v = "%d:%d:%d" % (d["grid_cap"], d["sort"], d["var"])
    if v not in cols:
        cols.append(v)
    rows.setdefault((d["config"], d["mode"]), {})[v] = d["ms_median"]
print("%-6s %-14s" % ("cfg", "mode") + "".join("%12s" % c for c in cols))
for (c, m), r in rows.items():
    best = min(r.values())
    print("%-6s %-14s" % (c, m) + "".join("%11.4f%s" % (r[k], "*" if r[k] == best else " ") if k in r else "%12s" % "-"
                                         for k in cols))
