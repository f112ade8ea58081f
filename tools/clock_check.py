import sys, os, json
sys.path.insert(0, os.getcwd())
import torch, numpy as np
import bench, twemproxy_amd as t
dev = torch.device("cuda", 0)
for cfg in ("C3", "C2", "C3"):
    spec = t.CONFIGS[cfg]["spec"]
    k, o = t.synth_device(spec, 0, 1 << 26, device=dev)
    kb = int(o[-1].item()); sh = spec.shape(kb)
    out = torch.empty(1 << 26, dtype=torch.int32, device=dev)
    for mode in ("md5", "fnv1a_64", "md5"):
        r = bench.clock_under(t, torch, lambda st: t.hash_batch_device(mode, k, o, out, stream=st, shape=sh, key_end=kb))
        print(cfg, mode, r, flush=True)
    del k, o, out; torch.cuda.empty_cache()
