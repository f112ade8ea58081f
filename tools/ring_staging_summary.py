#!/usr/bin/env python3
"""Collect tools/gpu_r6_bar.sh runs (the batch ring's staging and
write-through A/Bs) into one record: per run and
configuration, the C5 replay's host-per-key rows, its ring rows (1024-thread
lanes, depth <= 8) and the depth-1 timeline.

    python tools/ring_staging_summary.py > profiles/r06x_ring_staging.json
"""
import glob
import json
import os

RUNS = [
    ("r06x_bar", "first cut: device staging for every ring ('device') against host staging ('host'); "
                 "plain stores + release"),
    ("r06y_parts", "DROPPED: a lane of a 1-2 lane ring split over 4 / 2 workgroups (parts): hash 1.68 -> 1.24 us, "
                   "but every part fetched the whole image (0.80 -> 1.72 us); submit -> done 6.33 -> 7.16 us"),
    ("r06za_sort", "DROPPED: an in-LDS counting sort of each batch by key length, longest first: hash 1.80 -> "
                   "1.28 us, the sort ~0.68 us (counted in dev_fetch)"),
    ("r06zb_wt", "write-through 4-byte hash stores (sc0 sc1) and no system-scope release (wt1) against plain "
                 "stores + release (wt0), sort on / off"),
    ("r06zc_wt4", "KEPT: hashes to LDS, then 16-byte write-through stores, no release (wt1) against wt0; "
                  "host staging with wt1"),
    ("r06zd_acq", "DROPPED: sc0 sc1 fetch loads with no acquire fence (acq0) against the acquire (acq1), "
                  "alternated twice on one box: no difference (a box slow at BAR stores and uncached reads)"),
    ("r06ze_pairs", "device staging (default for one lane) against host staging, alternated twice on one box"),
    ("r06zm_copy", "KEPT: the staging copy into BAR memory as 64-byte AVX-512 stores (default) against 32-byte "
                   "AVX2 stores and glibc memcpy, alternated twice on one box"),
    ("r06zo_deep", "DROPPED: the worker's byte readers two steps ahead (QStream kDeep, deep1) against one (deep0), "
                   "alternated twice on one box: the hash phase stays 1.88 us"),
    ("r06zq_spread", "DROPPED: a batch's keys spread over all sixteen waves (x1) against the first ten (x0), "
                     "alternated twice on one box: hash 2.32-2.36 us against 1.92; the timeline also reports the "
                     "shader clock over the hash phase and wave 0's own share"),
]


def main():
    out = {"what": "the batch ring at small depth (DESIGN.md §6.2.1): tools/gpu_r6_bar.sh, one fresh MI355X box "
                   "per run; rows from tools/nc_c5_replay (1024-thread lanes, depth <= 8)",
           "runs": []}
    out["bar_probe"] = []
    for probe in ("gpurun_out/bar_probe2.jsonl", "gpurun_out/bar_probe3.jsonl"):  # attributes + ping-pong; copies
        if os.path.exists(probe):
            out["bar_probe"] += [json.loads(l) for l in open(probe) if l.startswith("{")]
    for name, what in RUNS:
        d = f"gpurun_out/{name}"
        if not os.path.isdir(d):
            continue
        run = {"run": name, "what": what, "configs": {}}
        for f in sorted(glob.glob(f"{d}/c5_*.jsonl")):
            tag = os.path.basename(f)[3:-6]
            keep = []
            for r in (json.loads(l) for l in open(f) if l.startswith("{")):
                if r["point"] == "host_per_key":
                    keep.append({"host_per_key_mkeys_s": r["mkeys_s"], "us_per_mbuf": r["us_per_mbuf"]})
                elif r["point"] == "gpu" and r["path"].startswith("ring") and r["threads"] == 1024 and r["depth"] <= 8:
                    keep.append({k: r.get(k) for k in ("staging", "depth", "lanes", "submit_to_done_us", "mkeys_s",
                                                       "mismatches")})
            tlf = f"{d}/timeline_{tag}.jsonl"
            tl = [json.loads(l) for l in open(tlf) if l.startswith("{")] if os.path.exists(tlf) else []
            run["configs"][tag] = {"c5": keep, "timeline": [x for x in tl if x.get("point") == "ring_timeline"]}
        lines = open(f"{d}/tests.log").read().strip().splitlines()
        run["gpu_tests"] = lines[-1].strip("= ") if lines else None
        out["runs"].append(run)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
