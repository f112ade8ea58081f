#!/usr/bin/env python3
"""Shader clock under each kernel ("measure the clock
question"): one sampler wave (nc_gpuhash_probe_clock_sampler) records
(s_memtime, s_memrealtime) every 20 us while the workload's kernel runs back
to back on another stream, so the clock the CUs actually ran at is
d(memtime) / d(realtime) x 100 MHz per interval. Workloads: idle, C2
fnv1a_64 (HBM-bound), C2 md5, C3 md5, C4 shard md5 (VALU-bound), and the
compute-only md5 probe (tools/probes/md5_rate, the ceiling bench.py quotes,
which stamps its own clock; its last row runs after 300 ms of sustained
load).

    python3 tools/clock_probe.py [--out gpurun_out/clock.json]
"""
from __future__ import annotations

import argparse
import ctypes
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
    ap.add_argument("--samples", type=int, default=6000)
    ap.add_argument("--gap", type=int, default=2000, help="100 MHz ticks between samples (20 us)")
    args = ap.parse_args()
    import torch

    import twemproxy_amd as t
    from twemproxy_amd import _lib as L

    dev = torch.device("cuda", 0)
    lib = L.lib()
    res = {"gap_us": args.gap / 100.0, "samples": args.samples}

    def sample(label, launch=None, child=None):
        buf = torch.zeros(2 * args.samples, dtype=torch.int64, device=dev)
        s_samp = torch.cuda.Stream(device=dev)
        s_work = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        L.check(lib.nc_gpuhash_probe_clock_sampler(buf.data_ptr(), args.samples, args.gap, s_samp.cuda_stream),
                "nc_gpuhash_probe_clock_sampler")
        done_ev = torch.cuda.Event()
        done_ev.record(s_samp)
        launches = 0
        proc = subprocess.Popen([child], stdout=subprocess.DEVNULL) if child else None
        t0 = time.perf_counter()
        while not done_ev.query():
            if launch is not None:
                with torch.cuda.stream(s_work):
                    for _ in range(4):
                        launch(s_work)
                        launches += 1
                s_work.synchronize()
            else:
                time.sleep(0.002)
            if time.perf_counter() - t0 > 5:
                break
        if proc is not None:
            proc.wait(timeout=120)
        torch.cuda.synchronize()
        a = buf.cpu().numpy().astype(np.int64)
        c, r = a[0::2], a[1::2]
        dc, dr = np.diff(c), np.diff(r)
        ok = dr > 0
        mhz = dc[ok] / dr[ok] * 100.0
        # the middle 80 % of the window (the work stream ramps in and out)
        lo, hi = int(0.1 * mhz.size), int(0.9 * mhz.size)
        mid = np.sort(mhz[lo:hi]) if hi > lo else np.sort(mhz)
        rec = {"launches": launches, "mhz_median": round(float(np.median(mid)), 1),
               "mhz_p10": round(float(mid[int(0.1 * (mid.size - 1))]), 1),
               "mhz_p90": round(float(mid[int(0.9 * (mid.size - 1))]), 1),
               "mhz_mean": round(float(mid.mean()), 1),
               "window_ms": round(float((r[-1] - r[0]) / 1e5), 2)}
        res[label] = rec
        print(label, json.dumps(rec), flush=True)

    sample("idle")
    c2 = t.CONFIGS["C2"]["spec"]
    keys, off = t.synth_device(c2, 0, 1 << 26, device=dev)
    kb = int(off[-1].item())
    shape = c2.shape(kb)
    out = torch.empty(1 << 26, dtype=torch.int32, device=dev)
    for mode in ("fnv1a_64", "md5"):
        sample(f"C2 {mode}", lambda s, m=mode: t.hash_batch_device(m, keys, off, out, stream=s, shape=shape,
                                                                   key_end=kb))
    del keys, off
    torch.cuda.empty_cache()
    c3 = t.CONFIGS["C3"]["spec"]
    keys, off = t.synth_device(c3, 0, 1 << 26, device=dev)
    kb = int(off[-1].item())
    shape = c3.shape(kb)
    for mode in ("fnv1a_64", "md5"):
        sample(f"C3 {mode}", lambda s, m=mode: t.hash_batch_device(m, keys, off, out, stream=s, shape=shape,
                                                                   key_end=kb))
    del keys, off, out
    torch.cuda.empty_cache()
    c4 = t.CONFIGS["C4"]["spec"]
    keys, off = t.synth_device(c4, 0, 1 << 25, device=dev)
    kb = int(off[-1].item())
    shape = c4.shape(kb)
    out = torch.empty(1 << 25, dtype=torch.int32, device=dev)
    for mode in ("md5", "crc32"):
        sample(f"C4 {mode}", lambda s, m=mode: t.hash_batch_device(m, keys, off, out, stream=s, shape=shape,
                                                                   key_end=kb))
    del keys, off, out
    torch.cuda.empty_cache()
    exe = os.path.join(HERE, "tools", "probes", "md5_rate")
    if os.path.exists(exe):  # the compute-only ceiling stamps its own clock (clock_mhz per row)
        rows = [json.loads(ln) for ln in subprocess.run([exe], capture_output=True, text=True, timeout=120,
                                                        check=True).stdout.splitlines() if ln.startswith("{")]
        res["md5_rate"] = [r for r in rows if "form" in r]
        for r in res["md5_rate"]:
            print("md5_rate", json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
