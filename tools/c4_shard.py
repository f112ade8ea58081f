#!/usr/bin/env python3
"""One GPU's shard of BASELINE.json configs[3] (C4: md5 + crc32 over 2^28
256-byte keys across 8 GPUs = 2^25 keys, 8 GiB per GPU), device-resident,
through the shape policy: kernel ms (hipEvents over `iters` launches), Gkeys/s
and the HBM roofline fraction; sampled keys checked against the per-key host
symbols (the reference's hash_t prototypes)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import twemproxy_amd as t

    spec = t.CONFIGS["C4"]["spec"]
    n = int(sys.argv[1]) if len(sys.argv) > 1 else t.CONFIGS["C4"]["nkeys"] // 8
    keys, off = t.synth_device(spec, 0, n)
    kb = int(off[-1].item())
    shape = spec.shape(kb)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    alg = kb + 12.0 * n
    for mode in ("md5", "crc32", "fnv1a_64"):
        t.hash_batch_device(mode, keys, off, out, shape=shape)
        torch.cuda.synchronize()
        print(f"# {mode} first launch ok", file=sys.stderr, flush=True)
        for _ in range(3):
            t.time_batch_device(mode, keys, off, out, 5, shape=shape)  # clock ramp
        ms = t.time_batch_device(mode, keys, off, out, 10, shape=shape)
        h = out.cpu().numpy().view(np.uint32)
        rng = np.random.default_rng(4)
        bad = 0
        for i in rng.integers(0, n, size=256):
            kh, oh = t.synth_host(spec, int(i), 1)
            bad += int(h[i]) != t.hash_key(mode, kh[: int(oh[-1])].tobytes())
        print(json.dumps({"workload": f"C4 shard: {n} x 256 B keys (2^25 = one of 8 GPUs)", "mode": mode,
                          "variant": t.pick_variant(mode, n, shape), "kernel_ms": round(ms, 4),
                          "gkeys_s": round(n / ms / 1e6, 2), "gb_s_hashed": round(kb / ms / 1e6, 1),
                          "hbm_frac": round(alg / ms / 1e6 / 8000.0, 4), "sample_mismatches": bad}), flush=True)


if __name__ == "__main__":
    main()
