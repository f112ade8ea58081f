#!/usr/bin/env python3
"""A/B sweep of launch variants and modes in ONE process (interleaved rounds).

    python tools/sweep.py [--modes fnv1a_64,md5] [--configs C2,C3] [--rounds 3] [--iters 20]
                          [--variants 0:0:0,0:1:1]

variant = grid_cap:sort:var (var bit 0 = shift-add FNV multiply). Configs: C1..C5, F<len> (fixed),
U<lo>-<hi> (uniform lengths). Prints one JSON line per (config, mode, variant) with
the median / min kernel ms (hipEvents over `iters` launches) and the
algorithmic HBM fraction (sum(len + 12) per launch / time / 8 TB/s).
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
    ap.add_argument("--modes", default="fnv1a_64")
    ap.add_argument("--configs", default="C2,C3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="0:0:0,0:1:0,0:0:1,0:1:1")
    ap.add_argument("--nkeys", type=int, default=1 << 26)
    args = ap.parse_args()

    import torch

    import twemproxy_amd as t
    from twemproxy_amd import _lib as L

    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    for cfg in args.configs.split(","):
        if cfg in t.CONFIGS:
            spec = t.CONFIGS[cfg]["spec"]
            n = min(args.nkeys, t.CONFIGS[cfg]["nkeys"])
        elif cfg.startswith("F"):  # F<len>: fixed-length keys, about 2 GiB of key bytes
            ln = int(cfg[1:])
            spec = t.SynthSpec.fixed(7, ln)
            n = min(args.nkeys, (1 << 31) // ln)
        else:  # U<lo>-<hi>: uniform lengths
            lo, hi = (int(x) for x in cfg[1:].split("-"))
            spec = t.SynthSpec.uniform(8, lo, hi)
            n = min(args.nkeys, (1 << 32) // (lo + hi))
        keys, off = t.synth_device(spec, 0, n)
        kb = int(off[-1].item())
        shape = spec.shape(kb)  # var 0 = the auto policy for this shape; 65536 = the workgroup pipeline
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        rd = [t.probe_read_gbs(keys, args.iters) for _ in range(args.rounds)]
        rdn = [t.probe_read_gbs(keys, args.iters, nt=True) for _ in range(args.rounds)]
        print(json.dumps({"config": cfg, "probe_read_gbs": round(statistics.median(rd), 1),
                          "probe_read_nt_gbs": round(statistics.median(rdn), 1),
                          "bytes": int(keys.numel())}), flush=True)
        modes = t.HASH_NAMES if args.modes == "all" else args.modes.split(",")
        for mode in modes:
            res = {v: [] for v in variants}
            for _ in range(args.rounds):
                for v in variants:
                    L.lib().nc_gpuhash_set_tuning(v[0], v[1], v[2])
                    t.hash_batch_device(mode, keys, off, out, shape=shape)
                    res[v].append(t.time_batch_device(mode, keys, off, out, args.iters, shape=shape))
            for v in variants:
                med = statistics.median(res[v])
                alg = kb + 12.0 * n
                print(json.dumps({"config": cfg, "mode": mode, "grid_cap": v[0], "sort": v[1], "var": v[2], "nkeys": n,
                                  "key_bytes": kb, "ms_median": round(med, 4), "ms_min": round(min(res[v]), 4),
                                  "gkeys_s": round(n / med / 1e6, 2), "alg_gbs": round(alg / med / 1e6, 1),
                                  "hbm_frac": round(alg / med / 1e6 / 8000.0, 4)}), flush=True)
        del keys, off, out
        torch.cuda.empty_cache()
    L.lib().nc_gpuhash_set_tuning(0, 0, 0)


if __name__ == "__main__":
    main()
