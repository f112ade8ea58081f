#!/usr/bin/env python3
"""Per replay point of a rocprofv3 --kernel-trace --hip-trace run of
tools/nc_c5_replay (tools/gpu_c5_trace.sh): GPU occupancy (idle / one op /
two or more ops at once), kernel time per batch, and the host thread's HIP
API time per batch.

    python3 tools/c5_trace_summary.py gpurun_out/<tag>/trace > profiles/<file>.json
"""
import collections
import csv
import json
import os
import sys

POINTS = ["copy depth 1", "copy depth 2", "copy depth 4", "zero-copy depth 1", "zero-copy depth 2", "zero-copy depth 4"]


def main():
    d = sys.argv[1]
    K = list(csv.DictReader(open(os.path.join(d, "c5_kernel_trace.csv"))))
    A = list(csv.DictReader(open(os.path.join(d, "c5_hip_api_trace.csv"))))
    for r in K:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    K.sort(key=lambda r: r["s"])
    segs = [[K[0]]]
    for a, b in zip(K, K[1:]):  # the replay points are > 2 ms apart
        if b["s"] - a["e"] > 2_000_000:
            segs.append([])
        segs[-1].append(b)
    segs = [s for s in segs if sum("nc_hash" in r["Kernel_Name"] for r in s) > 100]
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in A)
    out = []
    for name, s in zip(POINTS, segs):
        t0, t1 = s[0]["s"], s[-1]["e"]
        span = t1 - t0
        kern = [r for r in s if "nc_hash" in r["Kernel_Name"]]
        ev = sorted([(r["s"], 1) for r in s] + [(r["e"], -1) for r in s])
        cur, last, busy = 0, t0, collections.Counter()
        for t, dd in ev:
            busy[cur] += t - last
            cur += dd
            last = t
        apit = collections.Counter()
        for a0, a1, f in api:
            if a0 >= t0 and a1 <= t1:
                apit[f] += a1 - a0
        nb = len(kern)
        out.append({"point": name, "batches": nb, "us_per_batch": round(span / nb / 1e3, 2),
                    "kernel_us": round(sum(r["e"] - r["s"] for r in kern) / nb / 1e3, 2),
                    "gpu_idle": round(busy[0] / span, 3), "gpu_one_op": round(busy[1] / span, 3),
                    "gpu_two_or_more_ops": round(sum(v for k, v in busy.items() if k >= 2) / span, 3),
                    "host_api_us_per_batch": {f: round(apit[f] / nb / 1e3, 2) for f in
                                              ("hipLaunchKernel", "hipMemcpyAsync", "hipEventRecord", "hipEventQuery",
                                               "hipEventSynchronize") if apit[f]},
                    "host_thread_in_hip_api": round(sum(apit.values()) / span, 3)})
    print(json.dumps({"source": "rocprofv3 --kernel-trace --hip-trace -- tools/nc_c5_replay 0.05 (tools/gpu_c5_trace.sh)",
                      "points": out}, indent=1))


if __name__ == "__main__":
    main()
