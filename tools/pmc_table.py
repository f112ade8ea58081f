#!/usr/bin/env python3
"""Average per-dispatch counter values of the hash kernels in rocprofv3 csv dirs."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    agg = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "nc_hash_kernel" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    print(d, {k: f"{agg[k] / n[k]:.4g}" for k in sorted(agg)})
