#!/usr/bin/env python3
"""In-process A/B of the fused server_pool_idx pipelines (wave ring vs
workgroup) with a key-for-key comparison between them.

    python tools/ab_sidx.py --configs C2,C3 --modes fnv1a_64,md5 --tags none,{}
"""
import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

PIPES = {"policy": 0, "ring": 1 << 28, "workgroup": 1 << 29, "grouped": 1 << 30, "grouped3": (1 << 30) | (2 << 21),
         "grouped1": (1 << 30) | (1 << 21), "grouped_lut16": (1 << 30) | (1 << 24), "grouped_lut12": (1 << 30) | (1 << 23), "grouped512": (1 << 30) | (1 << 26),
         "workgroup_bkt": (1 << 29) | (1 << 25), "grouped_bkt": (1 << 30) | (1 << 25),
         "grouped3_bkt": (1 << 30) | (2 << 21) | (1 << 25),
         # ketama pools of <= 1280 points: the packed LDS continuum (512-key tiles, 3 sets by default, or 8),
         # and the 5-byte one it replaces (bit 27)
         "grouped8": (1 << 30) | (3 << 21), "grouped_5b": (1 << 30) | (1 << 27),
         # DIAGNOSTIC (fnv1a_64, packed continuum): no hash_tag code / no search (outputs are hashes) / neither
         "diag_notag": (1 << 30) | (1 << 19), "diag_nosearch": (1 << 30) | (2 << 19),
         "diag_bare": (1 << 30) | (3 << 19), "diag_bare_noprologue": (1 << 30) | (3 << 19) | (1 << 26),
         # the plain hash of the same keys (hash_device, its own policy)
         "plain_hash": None}
GRIDS = {}  # name -> grid cap (--grids: workgroup pipeline at these caps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2")
    ap.add_argument("--modes", default="fnv1a_64")
    ap.add_argument("--dists", default="ketama,modula")
    ap.add_argument("--tags", default="none")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--spinup", type=float, default=0.5, help="seconds of untimed launches before each entry "
                    "(device clocks ramp up under load, as bench.py's SPINUP_S)")
    ap.add_argument("--grids", default="", help="comma-separated grid caps for extra workgroup entries")
    ap.add_argument("--gs-grids", default="", help="comma-separated grid caps for extra grouped-pipeline entries")
    ap.add_argument("--pipes", default="", help="comma-separated subset of the pipeline names")
    ap.add_argument("--lib", default="", help="another build of libnc_gpuhash.so (same-box A/B of builds)")
    args = ap.parse_args()
    if args.pipes:
        for k in [k for k in PIPES if k not in args.pipes.split(",")]:
            del PIPES[k]
    for g in filter(None, args.grids.split(",")):
        PIPES[f"workgroup_g{g}"] = 1 << 29
        GRIDS[f"workgroup_g{g}"] = int(g)
    for g in filter(None, args.gs_grids.split(",")):  # the grouped pipeline (packed continuum) at a grid cap
        PIPES[f"grouped_g{g}"] = 1 << 30
        GRIDS[f"grouped_g{g}"] = int(g)

    import numpy as np
    import torch

    from twemproxy_amd import _lib as L

    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import twemproxy_amd as t

    rng = np.random.default_rng(9)
    cvals = np.sort(rng.integers(0, 1 << 32, size=8 * 160, dtype=np.uint64)).astype(np.uint32)
    cidx = rng.integers(0, 8, size=cvals.size).astype(np.uint32)
    conts = {"ketama": t.continuum_device(cidx, cvals), "modula": t.continuum_device(np.arange(8, dtype=np.uint32))}
    for cfg in args.configs.split(","):
        spec, n = t.CONFIGS[cfg]["spec"], t.CONFIGS[cfg]["nkeys"]
        keys, off = t.synth_device(spec, 0, n)
        kb = int(off[-1].item())
        shape = spec.shape(kb)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        for mode in args.modes.split(","):
            for dist in args.dists.split(","):
                for tag in args.tags.split(","):
                    tg = None if tag == "none" else tag.encode()

                    def launch_sidx():
                        t.server_idx_device(mode, dist, keys, off, conts[dist], 8, hash_tag=tg, out=out,
                                            shape=shape, key_end=kb)

                    def launch_hash():
                        t.hash_batch_device(mode, keys, off, out, shape=shape, key_end=kb)
                    ref, res = None, {}
                    for name, v in PIPES.items():
                        launch = launch_hash if v is None else launch_sidx
                        L.lib().nc_gpuhash_set_tuning(GRIDS.get(name, 0), 0, v or 0)
                        out.fill_(-1)
                        launch()
                        torch.cuda.synchronize()
                        h = out.cpu().numpy().copy()
                        if ref is None:
                            ref = h
                            chk = "ref"
                        else:
                            d = np.flatnonzero(h != ref)
                            chk = "same" if d.size == 0 else f"DIFF {d.size} first {int(d[0])}"
                        ms = []
                        t_end = time.perf_counter() + args.spinup
                        while time.perf_counter() < t_end:
                            for _ in range(10):
                                launch()
                            torch.cuda.synchronize()
                        for _ in range(args.rounds):
                            for _ in range(3):
                                launch()
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record()
                            for _ in range(args.iters):
                                launch()
                            e1.record()
                            torch.cuda.synchronize()
                            ms.append(e0.elapsed_time(e1) / args.iters)
                        res[name] = (round(statistics.median(ms), 4), chk)
                    L.lib().nc_gpuhash_set_tuning(0, 0, 0)
                    alg = kb + 12.0 * n
                    print(json.dumps({"lib": os.path.basename(L.LIB_PATH), "config": cfg, "mode": mode, "dist": dist, "tag": tag,
                                      "ms": {k: v[0] for k, v in res.items()},
                                      "frac": {k: round(alg / v[0] / 1e6 / 8000.0, 4) for k, v in res.items()},
                                      "check": {k: v[1] for k, v in res.items()}}), flush=True)
        del keys, off, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
