"""Debug helper for the wave-sorted pipeline: compare variant outputs with
the policy on C2 keys and summarize the mismatching keys."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import twemproxy_amd as t
from twemproxy_amd import _lib as L

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
var = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
spec = t.CONFIGS["C2"]["spec"]
kd, od = t.synth_device(spec, 0, n)
L.lib().nc_gpuhash_set_tuning(0, 0, 0)
ref = t.hash_batch_device("fnv1a_64", kd, od).cpu().numpy().view(np.uint32)
L.lib().nc_gpuhash_set_tuning(0, 0, var)
got = t.hash_batch_device("fnv1a_64", kd, od).cpu().numpy().view(np.uint32)
L.lib().nc_gpuhash_set_tuning(0, 0, 0)
bad = np.flatnonzero(ref != got)
off = od.cpu().numpy()
lens = np.diff(off)
print("n", n, "bad", bad.size)
print("first", bad[:20].tolist())
print("idx mod 256 hist", np.bincount(bad % 256, minlength=256).nonzero()[0][:40].tolist())
print("tiles with bad", np.unique(bad // 256).size, "of", (n + 255) // 256)
print("bad lens", np.bincount(lens[bad], minlength=65).nonzero()[0].tolist())
tb = bad // 256
for tile in np.unique(tb)[:5]:
    k = np.arange(tile * 256, min(n, tile * 256 + 256))
    span = off[k[-1] + 1] - off[k[0]]
    print("tile", int(tile), "span", int(span), "bad in tile", (bad[tb == tile] % 256).tolist(),
          "lens", lens[bad[tb == tile]].tolist(), "maxlen tile", int(lens[k].max()))
