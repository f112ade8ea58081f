#!/usr/bin/env python3
"""Summarise tools/gpu_c4_tlb.sh runs: for each keys placement (k0-k3, in
the order tools/c4_placement.py --grid --keys-only launches them: 4 checks,
then 3 warm-up + ITERS timed launches per placement) the median duration and
counters of the timed launches, from rocprofv3's per-pass databases.

    python tools/c4_mode_pmc.py gpurun_out/r06_c4tlb gpurun_out/r06_c4tlb2 ... > profiles/x.json
"""
import collections
import glob
import json
import os
import sqlite3
import statistics
import sys

ITERS, WARM = 5, 3


def one_pass(db_path):
    db = sqlite3.connect(db_path)
    cols = [r[1] for r in db.execute("pragma table_info(counters_collection)")]
    ci = {c: j for j, c in enumerate(cols)}
    d = collections.OrderedDict()
    for r in db.execute("select * from counters_collection"):
        e = d.setdefault(r[ci["dispatch_id"]], {"kernel": r[ci["kernel_name"]],
                                                 "dur_ms": (r[ci["end"]] - r[ci["start"]]) / 1e6})
        e[r[ci["counter_name"]]] = r[ci["value"]]
    hk = [v for v in d.values() if "nc_bytes_direct" in v["kernel"]][-4 * (WARM + ITERS):]
    out = {}
    for g in range(4):
        blk = hk[g * (WARM + ITERS) + WARM:(g + 1) * (WARM + ITERS)]
        out[f"k{g}"] = {k: round(statistics.median(b[k] for b in blk), 4) for k in blk[0] if k != "kernel"}
    return out


def main():
    res = {"what": "C4 shard fnv1a_64, the same keys in four device allocations of one process "
                   "(tools/c4_placement.py --grid --keys-only); per placement the median of 5 launches "
                   "under each rocprofv3 --pmc pass (tools/gpu_c4_tlb.sh)", "runs": []}
    for d in sys.argv[1:]:
        run = {"run": os.path.basename(d.rstrip("/"))}
        plain = os.path.join(d, "plain.json")
        if os.path.exists(plain):
            run["plain"] = json.loads(open(plain).read().strip().splitlines()[-1])
        for db in sorted(glob.glob(os.path.join(d, "pmc*", "*.db"))):
            run[os.path.basename(os.path.dirname(db))] = one_pass(db)
        res["runs"].append(run)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
