#!/usr/bin/env python3
"""C4 shard fnv1a_64 (the policy's two-lines-per-round kernel) with the same
keys at different device placements, in one process: the leg runs 1.41-1.44
ms on some boxes and 1.53-1.54 on others with the same kernel (DESIGN.md
§5.1); this asks whether where the 8 GiB lands moves it.

    python tools/c4_placement.py [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mode", default="fnv1a_64")
    ap.add_argument("--extra", type=int, default=0, help="more plain 8 GiB copies after the others")
    ap.add_argument("--spacer-gib", type=int, default=0, help="hold this much device memory before synthesising the keys")
    ap.add_argument("--contig-only", action="store_true",
                    help="only the synthesised keys and a copy in hipExtMallocWithFlags(hipDeviceMallocContiguous) memory")
    ap.add_argument("--grid", action="store_true", help="4 key placements x 4 offset placements")
    ap.add_argument("--keys-only", action="store_true", help="with --grid: the 4 key placements, one offsets buffer "
                    "(for a PMC pass: 4 checks, then per placement 3 warm-up + ITERS timed launches, in order)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import twemproxy_amd as t

    spec, n = t.CONFIGS["C4"]["spec"], 1 << 25
    spacer = torch.empty(args.spacer_gib << 30, dtype=torch.uint8, device="cuda") if args.spacer_gib else None
    keys, off = t.synth_device(spec, 0, n)
    del spacer
    kb = int(off[-1].item())
    shape = spec.shape(kb)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ref = t.hash_batch_device(args.mode, keys, off, shape=shape, key_end=kb).cpu().numpy()
    nbytes = keys.numel()
    places = {"synth": keys}
    if args.contig_only:
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(4))
        assert rc == 0, f"hipExtMallocWithFlags contiguous: {rc}"
        torch.cuda.synchronize()
        rc = hip.hipMemcpy(p, ctypes.c_void_p(keys.data_ptr()), ctypes.c_size_t(nbytes), ctypes.c_int(3))
        assert rc == 0, f"hipMemcpy: {rc}"

        class Raw:  # what time_batch_device reads of a key buffer: its device address
            def __init__(self, ptr):
                self.ptr = ptr

            def data_ptr(self):
                return self.ptr

        raw = Raw(p.value)
        res = {"synth": [], "contiguous": []}
        for _ in range(args.rounds):
            for name, k in (("synth", keys), ("contiguous", raw)):
                t.time_batch_device(args.mode, k, off, out, 3, shape=shape)
                res[name].append(t.time_batch_device(args.mode, k, off, out, args.iters, shape=shape))
        print(json.dumps({"mode": args.mode, "config": "C4S", "ms_median": {k: round(statistics.median(v), 4) for k, v in res.items()},
                          "ms_min": {k: round(min(v), 4) for k, v in res.items()},
                          "ptr_hex": {"synth": hex(keys.data_ptr()), "contiguous": hex(p.value)}}), flush=True)
        hip.hipFree(p)
        return
    if args.grid:
        # keys x offsets placements: which of the two buffers (or the pair)
        # decides the mode
        kp = {"k0": keys}
        op = {"o0": off}
        for i in (1, 2, 3):
            b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            b.copy_(keys)
            kp[f"k{i}"] = b
            if args.keys_only:
                continue
            o = torch.empty(off.numel() + (i << 14), dtype=off.dtype, device="cuda")[i << 14:]
            o.copy_(off)
            op[f"o{i}"] = o
        torch.cuda.synchronize()
        res, chk = {}, {}
        for kn, k in kp.items():
            for on, o in op.items():
                got = t.hash_batch_device(args.mode, k, o, shape=shape, key_end=kb).cpu().numpy()
                chk[f"{kn}{on}"] = "ok" if np.array_equal(got, ref) else "DIFF"
                res[f"{kn}{on}"] = []
        for _ in range(args.rounds):
            for kn, k in kp.items():
                for on, o in op.items():
                    t.time_batch_device(args.mode, k, o, out, 3, shape=shape)
                    res[f"{kn}{on}"].append(t.time_batch_device(args.mode, k, o, out, args.iters, shape=shape))
        print(json.dumps({"mode": args.mode, "config": "C4S", "grid": "keys k0-k3 x offsets o0-o3",
                          "ms_median": {k: round(statistics.median(v), 4) for k, v in res.items()},
                          "check": "ok" if all(v == "ok" for v in chk.values()) else chk,
                          "keys_ptr": {k: hex(v.data_ptr()) for k, v in kp.items()},
                          "offs_ptr": {k: hex(v.data_ptr()) for k, v in op.items()}}), flush=True)
        return
    fresh = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    fresh.copy_(keys)
    places["fresh"] = fresh
    for sh in (64 << 10, 1 << 20, 2 << 20):
        b = torch.empty(nbytes + sh, dtype=torch.uint8, device="cuda")[sh:]
        b.copy_(keys)
        places[f"offset_{sh >> 10}k"] = b
    dummy = torch.empty(32 << 30, dtype=torch.uint8, device="cuda")
    high = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    high.copy_(keys)
    places["after_32g"] = high
    for i in range(args.extra):
        b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        b.copy_(keys)
        places[f"extra_{i}"] = b
    torch.cuda.synchronize()
    res = {k: [] for k in places}
    chk = {}
    for name, k in places.items():
        got = t.hash_batch_device(args.mode, k, off, shape=shape, key_end=kb).cpu().numpy()
        chk[name] = "ok" if np.array_equal(got, ref) else "DIFF"
    for _ in range(args.rounds):
        for name, k in places.items():
            t.time_batch_device(args.mode, k, off, out, 3, shape=shape)
            res[name].append(t.time_batch_device(args.mode, k, off, out, args.iters, shape=shape))
    print(json.dumps({"mode": args.mode, "config": "C4S", "ms_median": {k: round(statistics.median(v), 4) for k, v in res.items()},
                      "ms_min": {k: round(min(v), 4) for k, v in res.items()}, "check": chk,
                      "ptr_hex": {k: hex(v.data_ptr()) for k, v in places.items()},
                      "ptr_mod_1g_mib": {k: (v.data_ptr() % (1 << 30)) >> 20 for k, v in places.items()}}), flush=True)
    del dummy


if __name__ == "__main__":
    main()
