#!/usr/bin/env python3
"""Where the host batch path's time goes: one C5 batch of N keys through the
context (submit+wait) under each pipeline, next to the device-resident kernel
time of the same batch and the host packing cost."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import twemproxy_amd as t
    from twemproxy_amd import _lib as L

    spec = t.CONFIGS["C5"]["spec"]
    for n in (798, 8192, 1 << 20):
        k, o = t.synth_host(spec, 0, n)
        kd, od = torch.from_numpy(k).cuda(), torch.from_numpy(o.astype(np.int64)).cuda()
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        shape = t.shape_of(o)
        res = {"nkeys": n, "key_bytes": int(o[-1])}
        for var in (0, 32, 65536):
            L.lib().nc_gpuhash_set_tuning(0, 0, var)
            res[f"kernel_ms_var{var}"] = round(t.time_batch_device("fnv1a_64", kd, od, out, 50, shape=shape), 4)
            for zc in (0, 1 << 40):
                with t.Context(max_keys=n, max_key_bytes=int(o[-1]), nslots=1, zero_copy_bytes=zc) as ctx:
                    for _ in range(3):
                        tk, _o = ctx.submit("fnv1a_64", k, o)
                        ctx.wait(tk)
                    reps = 20
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        tk, _o = ctx.submit("fnv1a_64", k, o)
                        ctx.wait(tk)
                    res[f"ctx_us_var{var}_zc{int(zc > 0)}"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)
        t0 = time.perf_counter()
        for _ in range(20):
            np.copyto(np.empty_like(k), k)
        res["host_memcpy_keys_us"] = round((time.perf_counter() - t0) / 20 * 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
