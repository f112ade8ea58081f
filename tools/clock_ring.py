#!/usr/bin/env python3
"""Shader clock while the batch ring serves one batch at a time (DESIGN.md
§6.2, the C5 crossover): the clock sampler of tools/clock_probe.py
(nc_gpuhash_probe_clock_sampler, s_memtime against s_memrealtime every
20 us) runs in this process while `tools/nc_c5_replay SECONDS timeline`
(depth 1, one lane, the worker's own stamps) runs as a child process; then
the same with the replay's full depth sweep, and idle.

    python3 tools/clock_ring.py [--out gpurun_out/clock_ring.json]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--samples", type=int, default=20000)
    ap.add_argument("--gap", type=int, default=2000, help="100 MHz ticks between samples (20 us)")
    args = ap.parse_args()
    import torch

    from twemproxy_amd import _lib as L

    dev = torch.device("cuda", 0)
    exe = os.path.join(HERE, "tools", "nc_c5_replay")
    res = {"gap_us": args.gap / 100.0, "samples": args.samples}

    def sample(label, child_args=None):
        buf = torch.zeros(2 * args.samples, dtype=torch.int64, device=dev)
        s_samp = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        proc = None
        if child_args:
            proc = subprocess.Popen([exe, *child_args], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
            time.sleep(0.3)  # the child's set-up (context, ring launch) before the window opens
        L.check(L.lib().nc_gpuhash_probe_clock_sampler(buf.data_ptr(), args.samples, args.gap, s_samp.cuda_stream),
                "nc_gpuhash_probe_clock_sampler")
        s_samp.synchronize()
        out = proc.communicate(timeout=120)[0] if proc else ""
        a = buf.cpu().numpy().astype(np.int64)
        dc, dr = np.diff(a[0::2]), np.diff(a[1::2])
        mhz = np.sort(dc[dr > 0] / dr[dr > 0] * 100.0)
        rec = {"mhz_median": round(float(np.median(mhz)), 1), "mhz_p10": round(float(mhz[int(0.1 * (mhz.size - 1))]), 1),
               "mhz_p90": round(float(mhz[int(0.9 * (mhz.size - 1))]), 1),
               "window_ms": round(float((a[-1] - a[1]) / 1e5), 2)}
        if child_args:
            rec["child"] = " ".join(child_args)
            rec["child_rows"] = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")][:40]
        res[label] = rec
        print(label, json.dumps({k: v for k, v in rec.items() if k != "child_rows"}), flush=True)

    sample("idle")
    sample("ring depth 1 (timeline)", ["1.5", "timeline"])
    sample("c5 replay sweep", ["0.3"])
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
