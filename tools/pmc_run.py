#!/usr/bin/env python3
"""Minimal driver for rocprofv3 counter passes: generate one synthetic
workload on the device and launch one hash mode `--iters` times.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/x -o pmc --output-format csv -- \
        python3 tools/pmc_run.py --config C3 --mode fnv1a_64 --variant 0:0:0 --iters 10
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--mode", default="fnv1a_64")
    ap.add_argument("--variant", default="0:0:0", help="grid_cap:sort:var")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--nkeys", type=int, default=0)
    ap.add_argument("--lib", default="", help="another build of libnc_gpuhash.so (A/B builds)")
    args = ap.parse_args()

    import torch

    from twemproxy_amd import _lib as L

    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import twemproxy_amd as t

    if args.config == "C4S":  # one GPU's C4 shard, as bench.py's c4_shard leg
        cfg = {"spec": t.CONFIGS["C4"]["spec"], "nkeys": 1 << 25}
    else:
        cfg = t.CONFIGS[args.config]
    n = args.nkeys or cfg["nkeys"]
    keys, off = t.synth_device(cfg["spec"], 0, n)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    g, s, v = (int(x) for x in args.variant.split(":"))
    L.lib().nc_gpuhash_set_tuning(g, s, v)
    kb = int(off[-1].item())
    shape = cfg["spec"].shape(kb)  # as bench.py: the auto policy's pipeline
    for mode in args.mode.split(","):
        for _ in range(args.iters):
            if mode in ("probe_read", "probe_read_nt"):  # FETCH_SIZE calibration: a known byte count
                t.probe_read_gbs(keys, 1, nt=mode.endswith("_nt"))
            elif mode == "server_idx":  # bench.py's fused leg: fnv1a_64 + ketama over 8 x 160 points
                import numpy as np

                rng = np.random.default_rng(9)
                cvals = np.sort(rng.integers(0, 1 << 32, size=8 * 160, dtype=np.uint64)).astype(np.uint32)
                cidx = rng.integers(0, 8, size=cvals.size).astype(np.uint32)
                cont = t.continuum_device(cidx, cvals)
                t.server_idx_device("fnv1a_64", "ketama", keys, off, cont, 8, out=out, shape=shape, key_end=kb)
            else:
                t.hash_batch_device(mode, keys, off, out, shape=shape, key_end=kb)
    torch.cuda.synchronize()
    print(f"{args.config} {args.mode} {args.variant} n={n} key_bytes={int(off[-1].item())}")


if __name__ == "__main__":
    main()
