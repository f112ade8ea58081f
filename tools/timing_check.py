#!/usr/bin/env python3
"""Why bench.py's per-launch time differs from tools/sweep.py's: the same C2/C3
launches timed (a) by nc_gpuhash_time_device (C loop between two hipEvents),
(b) bench-style (Python loop between torch events), (c) (b) after a long warm-up."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import twemproxy_amd as t

    for cfg in ("C2", "C3"):
        spec = t.CONFIGS[cfg]["spec"]
        keys, off = t.synth_device(spec, 0, 1 << 26)
        kb = int(off[-1].item())
        shape = spec.shape(kb)
        out = torch.empty(1 << 26, dtype=torch.int32, device="cuda")
        res = {"config": cfg}

        def pyloop(n):
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(n):
                t.hash_batch_device("fnv1a_64", keys, off, out, stream=st, shape=shape)
            e1.record(st)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / n

        res["py_cold"] = round(pyloop(20), 4)
        res["c_loop"] = round(t.time_batch_device("fnv1a_64", keys, off, out, 20, shape=shape), 4)
        res["py_after"] = round(pyloop(20), 4)
        t0 = time.time()
        while time.time() - t0 < 2.0:
            t.time_batch_device("fnv1a_64", keys, off, out, 50, shape=shape)
        res["py_warm"] = round(pyloop(20), 4)
        res["c_warm"] = round(t.time_batch_device("fnv1a_64", keys, off, out, 20, shape=shape), 4)
        res["py_warm200"] = round(pyloop(200), 4)
        print(json.dumps(res), flush=True)
        del keys, off, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
