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
    args = ap.parse_args()

    import torch

    import twemproxy_amd as t
    from twemproxy_amd import _lib as L

    cfg = t.CONFIGS[args.config]
    n = args.nkeys or cfg["nkeys"]
    keys, off = t.synth_device(cfg["spec"], 0, n)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    g, s, v = (int(x) for x in args.variant.split(":"))
    L.lib().nc_gpuhash_set_tuning(g, s, v)
    shape = cfg["spec"].shape(int(off[-1].item()))  # as bench.py: the auto policy's pipeline
    for mode in args.mode.split(","):
        for _ in range(args.iters):
            t.hash_batch_device(mode, keys, off, out, shape=shape)
    torch.cuda.synchronize()
    print(f"{args.config} {args.mode} {args.variant} n={n} key_bytes={int(off[-1].item())}")


if __name__ == "__main__":
    main()
