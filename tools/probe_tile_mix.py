#!/usr/bin/env python3
"""is the C2 ceiling (the read+write mix probe, one nt
16-B store per 128 B read, 5.51-5.56 TB/s) a property of that probe's store
pattern? The grouped pipeline stores 2 KiB contiguous per 512-key tile
(~14 KiB read). nc_gpuhash_probe_tile_mix streams 2.2 GB in that shape:
16 KiB read + 2 KiB stored per tile (11 % writes, the old probe's ratio),
512-thread workgroups at the kernel's grid (six resident sets of four per
CU = 6,144) or fewer, tiles grid-strided one at a time, in runs of four
consecutive tiles, and with each run's 8 KiB of outputs stored at once from
LDS (deferred). Three interleaved rounds beside the old mix and nt read
probes; GB/s counts bytes read + written.

    python tools/probe_tile_mix.py [--flavours [--rounds 3]]

--flavours: the kernel's shape (and the deferred 8 KiB-run shape) with the
output stores as nt (the kernels'), plain, sc1 and sc0 sc1 (write-through),
beside the read-only tile."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flavours", action="store_true")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch

    import twemproxy_amd as t
    from twemproxy_amd import _lib as L

    lib = L.lib()
    nbytes = 2200 * 1000 * 1000 // 16384 * 16384
    buf = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    out = torch.empty(nbytes // 4, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(65536, dtype=torch.int32, device="cuda")
    cus = torch.cuda.get_device_properties(0).multi_processor_count

    def tile_mix(rd, wr, run, grid, defer, iters=20, sf=0):
        ms = ctypes.c_float(0.0)
        L.check(lib.nc_gpuhash_probe_tile_mix(buf.data_ptr(), nbytes, out.data_ptr(), out.numel(), rd, wr, run, grid,
                                              int(defer) | (sf << 4), sink.data_ptr(), None, iters,
                                              ctypes.byref(ms)),
                "nc_gpuhash_probe_tile_mix")
        ntiles = nbytes // rd
        return (ntiles * (rd + wr)) / (ms.value * 1e-3) / 1e9

    shapes = [("tile16k_2k_run1_g6x", 16384, 2048, 1, 24 * cus, False),
              ("tile16k_2k_run1_g3x", 16384, 2048, 1, 12 * cus, False),
              ("tile16k_2k_run4_g6x", 16384, 2048, 4, 24 * cus, False),
              ("tile16k_2k_run4_defer_g6x", 16384, 2048, 4, 24 * cus, True),
              ("tile16k_2k_run4_defer_g3x", 16384, 2048, 4, 12 * cus, True),
              ("tile8k_1k_run8_defer_g6x", 8192, 1024, 8, 24 * cus, True),
              ("tile16k_0_run1_g6x", 16384, 0, 1, 24 * cus, False)]
    if args.flavours:
        # the store flavour of the kernel's shape: nt (the kernels'), plain, sc1, sc0 sc1
        for r in range(args.rounds):
            row = {"round": r, "shape": "tile16k_2k_run1_g6x / tile8k_1k_run8_defer_g6x",
                   "read_only_gbs": round(tile_mix(16384, 0, 1, 24 * cus, False), 1)}
            for sf, name in enumerate(("nt", "plain", "sc1", "sc0sc1")):
                row[name] = round(tile_mix(16384, 2048, 1, 24 * cus, False, sf=sf), 1)
                row[name + "_run8_defer"] = round(tile_mix(8192, 1024, 8, 24 * cus, True, sf=sf), 1)
            print(json.dumps(row), flush=True)
        return
    for s in shapes:
        tile_mix(*s[1:], iters=3)
    t.probe_mix_gbs(buf, 3)
    for r in range(3):
        row = {"round": r, "bytes": nbytes, "read_nt_gbs": round(t.probe_read_gbs(buf, 20, nt=True), 1),
               "mix_gbs": round(t.probe_mix_gbs(buf, 20), 1)}
        for s in shapes:
            row[s[0]] = round(tile_mix(*s[1:]), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
