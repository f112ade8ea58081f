#!/usr/bin/env python3
"""Locate where a launch variant disagrees with variant 0: for each
mismatching tile print its block, step index j (= tile // grid), span and
which lanes differ.   python tools/diag_variant.py C2 fnv1a_64 0:0:224 1536 [nkeys]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ranges(lanes):
    out, st = [], None
    prev = None
    for x in list(lanes) + [None]:
        if st is None:
            st = prev = x
        elif x is not None and x == prev + 1:
            prev = x
        else:
            out.append(f"{st}-{prev}")
            st = prev = x
    return ",".join(out)


def main():
    cfg, mode, var, grid = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    import numpy as np
    import torch

    import twemproxy_amd as t
    from twemproxy_amd import _lib as L

    n = int(sys.argv[5]) if len(sys.argv) > 5 else t.CONFIGS[cfg]["nkeys"]
    keys, off = t.synth_device(t.CONFIGS[cfg]["spec"], 0, n)
    ref = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    L.lib().nc_gpuhash_set_tuning(grid, 0, 0)
    t.hash_batch_device(mode, keys, off, ref)
    g, s, v = (int(x) for x in var.split(":"))
    L.lib().nc_gpuhash_set_tuning(grid, s, v)
    torch.cuda.synchronize()
    t0 = time.time()
    t.hash_batch_device(mode, keys, off, out)
    torch.cuda.synchronize()
    print(f"n={n} grid={grid} var={var} wall={(time.time()-t0)*1e3:.1f} ms", flush=True)
    bad = (ref != out).nonzero().flatten().cpu().numpy()
    print(f"mismatches={bad.size}")
    if bad.size == 0:
        return
    o = off.cpu().numpy()
    r_np = ref.cpu().numpy()
    o_np = out.cpu().numpy()
    order = np.argsort(r_np, kind="stable")
    srt = r_np[order]
    vals = o_np[bad[:2000]]
    pos = np.searchsorted(srt, vals)
    pos = np.minimum(pos, srt.size - 1)
    hit = srt[pos] == vals
    print(f"bad values == -1 (never stored): {(vals == -1).sum()} of {vals.size}; "
          f"equal to another key's hash: {hit.sum()}")
    for b_, v_, h_, p_ in list(zip(bad[:2000], vals, hit, pos))[:12]:
        other = int(order[p_]) if h_ else -1
        d = other - int(b_) if h_ else 0
        print(f"  key {b_} (tile {b_ // 256} lane {b_ % 256}) got {v_ & 0xffffffff:#010x} "
              f"{'= hash of key %d (delta %d, tiles %+d)' % (other, d, other // 256 - b_ // 256) if h_ else ''}")
    tiles = np.unique(bad // 256)
    ntiles = (n + 255) // 256
    print(f"bad tiles={tiles.size} of {ntiles}; steps per block={ntiles / grid:.2f}")
    for tl in tiles[:40]:
        lanes = bad[(bad // 256) == tl] % 256
        k0, k1 = tl * 256, min(tl * 256 + 256, n)
        span = int(o[k1] - (o[k0] & ~15))
        j = tl // grid
        nsteps = (ntiles - 1 - tl % grid) // grid + 1
        print(f"tile {tl} block {tl % grid} j={j} j%6={j % 6} nsteps={nsteps} span={span} "
              f"lanes={lanes.size} ranges={ranges(lanes)}")
    js = (tiles // grid)
    print("j histogram (mod 6):", np.bincount(js % 6, minlength=6).tolist())
    print("j values:", np.unique(js)[:30].tolist())


if __name__ == "__main__":
    main()
