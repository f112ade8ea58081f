#!/usr/bin/env python3
"""Summarise rocprofv3 outputs per kernel.

    python tools/pmc_summary.py <dir-or-csv> [...]

For *_counter_collection.csv files: mean of every counter per kernel name
(one value per dispatch = sum over the counter's instances). For
*_kernel_stats.csv: prints calls / mean ns. HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads half the bytes of a wide
coalesced stream on gfx950, so hbm_read = 2 x FETCH_SIZE x 1024;
hbm_write = WRITE_SIZE x 1024.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(nc_hash_kernel(?:_rs)?)<(\d+), (true|false), (\d+)>", name)
    if m:
        return f"{m.group(1)}<mode={m.group(2)},sort={m.group(3)},var={m.group(4)}>"
    m = re.search(r"(nc_hash_kernel_wr)<(\d+), ([-\d, ]+)>", name)
    if m:
        return f"{m.group(1)}<mode={m.group(2)},{m.group(3).replace(' ', '')}>"
    return name.replace("void (anonymous namespace)::", "").split("(")[0][:80]


def counters(path):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            key = (r.get("Kernel_Name", ""), r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            names[key] = r.get("Kernel_Name", "")
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(list))
    for key, cs in per.items():
        for c, v in cs.items():
            agg[short(names[key])][c].append(v)
    res = {}
    for k, cs in agg.items():
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k]["_dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in res[k]:
            res[k]["hbm_read_bytes_corrected"] = 2.0 * res[k]["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in res[k]:
            res[k]["hbm_write_bytes"] = res[k]["WRITE_SIZE"] * 1024.0
    return res


def main():
    paths = []
    for a in sys.argv[1:]:
        if os.path.isdir(a):
            paths += glob.glob(os.path.join(a, "**", "*.csv"), recursive=True)
        else:
            paths.append(a)
    for p in sorted(paths):
        if p.endswith("counter_collection.csv"):
            print(json.dumps({"file": p, "kernels": counters(p)}, indent=1))
        elif p.endswith("kernel_stats.csv"):
            with open(p) as f:
                for r in csv.DictReader(f):
                    print(f"{p}: {short(r['Name'])} calls={r['Calls']} avg_ns={float(r['AverageNs']):.0f}")


if __name__ == "__main__":
    main()
