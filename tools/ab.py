#!/usr/bin/env python3
"""In-process A/B of launch variants with correctness checks.

    python tools/ab.py --configs C2,C3,C4S --modes md5 --variants 0,16512,262176 [--rounds 3 --iters 10]

Configs: C1..C5, C4S = one GPU's C4 shard (2^25 x 256 B),
F<len> fixed length (about 2 GiB), U<lo>-<hi> uniform lengths. Variant 0 is
the shape policy; others are nc_gpuhash_set_tuning variant bits, "v:g" the
same with grid cap g (workgroup pipelines). For every
(config, mode) the outputs of each variant are compared with the first
variant's, key for key, and 512 sampled keys with the per-key host symbols.
Prints one JSON line per (config, mode, variant): median / min kernel ms
(hipEvents), Gkeys/s and the algorithmic HBM fraction. --lib times another
build of the library (e.g. an older commit's) in this process.
"""
import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def config(t, name, nkeys):
    if name == "C4S":
        return t.CONFIGS["C4"]["spec"], min(nkeys, 1 << 25)
    if name in t.CONFIGS:
        return t.CONFIGS[name]["spec"], min(nkeys, t.CONFIGS[name]["nkeys"])
    if name.startswith("F"):
        ln = int(name[1:])
        return t.SynthSpec.fixed(7, ln), min(nkeys, (1 << 31) // ln)
    lo, hi = (int(x) for x in name[1:].split("-"))
    return t.SynthSpec.uniform(8, lo, hi), min(nkeys, (1 << 32) // (lo + hi))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="md5")
    ap.add_argument("--configs", default="C2,C3")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--nkeys", type=int, default=1 << 26)
    ap.add_argument("--spinup", type=float, default=0.0, help="seconds of untimed launches before each timing")
    ap.add_argument("--lib", default="", help="another build of libnc_gpuhash.so (same-box A/B of builds)")
    args = ap.parse_args()

    import numpy as np
    import torch

    from twemproxy_amd import _lib as L

    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import twemproxy_amd as t

    # "v" or "v:g": variant bits v with grid cap g (nc_gpuhash_set_tuning)
    variants = args.variants.split(",")
    tune = {v: (int(v.split(":")[1]) if ":" in v else 0, int(v.split(":")[0])) for v in variants}
    rng = np.random.default_rng(1)
    for cfg in args.configs.split(","):
        spec, n = config(t, cfg, args.nkeys)
        keys, off = t.synth_device(spec, 0, n)
        kb = int(off[-1].item())
        shape = spec.shape(kb)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        sample = np.sort(rng.integers(0, n, size=512))
        host = {}
        for i in sample:
            kh, oh = t.synth_host(spec, int(i), 1)
            host[int(i)] = kh[: int(oh[-1])].tobytes()
        modes = t.HASH_NAMES if args.modes == "all" else args.modes.split(",")
        for mode in modes:
            ref = None
            res = {v: [] for v in variants}
            ok = {}
            for v in variants:
                L.lib().nc_gpuhash_set_tuning(tune[v][0], 0, tune[v][1])
                out.fill_(0)
                t.hash_batch_device(mode, keys, off, out, shape=shape, key_end=kb)
                torch.cuda.synchronize()
                h = out.cpu().numpy().view(np.uint32).copy()
                if ref is None:
                    ref = h
                    bad = sum(int(h[i]) != t.hash_key(mode, host[int(i)]) for i in sample)
                    ok[v] = f"host-sample mismatches {bad}"
                else:
                    diff = np.flatnonzero(h != ref)
                    ok[v] = "same" if diff.size == 0 else f"DIFF {diff.size} first {int(diff[0])}"
            if args.spinup > 0:  # clocks ramp up under load (bench.py SPINUP_S): untimed launches first
                t_end = time.perf_counter() + args.spinup
                while time.perf_counter() < t_end:
                    t.time_batch_device(mode, keys, off, out, 10, shape=shape)
            for _ in range(args.rounds):
                for v in variants:
                    L.lib().nc_gpuhash_set_tuning(tune[v][0], 0, tune[v][1])
                    t.time_batch_device(mode, keys, off, out, 3, shape=shape)
                    res[v].append(t.time_batch_device(mode, keys, off, out, args.iters, shape=shape))
            for v in variants:
                med = statistics.median(res[v])
                alg = kb + 12.0 * n
                print(json.dumps({"lib": os.path.basename(L.LIB_PATH), "config": cfg, "mode": mode, "var": v, "nkeys": n, "key_bytes": kb,
                                  "ms_median": round(med, 4), "ms_min": round(min(res[v]), 4),
                                  "gkeys_s": round(n / med / 1e6, 2), "hbm_frac": round(alg / med / 1e6 / 8000.0, 4),
                                  "check": ok[v]}), flush=True)
        del keys, off, out
        torch.cuda.empty_cache()
    L.lib().nc_gpuhash_set_tuning(0, 0, 0)


if __name__ == "__main__":
    main()
