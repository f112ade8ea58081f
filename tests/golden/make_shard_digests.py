#!/usr/bin/env python3
"""Per-rank digests of the multi-GPU bench legs, from the REAL reference.

Run in the build container (where /root/reference exists):

    make -C oracle ref && python tests/golden/make_shard_digests.py

bench.py --gpus N gives every rank one shard of an N-shard batch: rank 0
generates N x n_per_rank keys of a config (C2, C3: 2^26 per rank; C4: 2^25
x 256 B per rank) and scatters byte-balanced contiguous ranges
(twemproxy_amd/shard.py plan_bounds). This script hashes the same N x
n_per_rank keys with the reference's own src/hashkit (oracle/_ref, compiled
from /root/reference; threads over byte-balanced ranges) for N = 8 — the
batches at N = 1, 2, 4 are its prefixes, since the generator is counter-based
— cuts them with the same plan_bounds rule for N = 1, 2, 4, 8, and writes
per (config, mode, N, rank) the key range and the sha256 of the reference's
u32 outputs over it: tests/golden/shard_digests.json (data only). bench.py
checks every rank against it outside the timed region; the -m gpu test
test_shard_setup_n8 checks the N = 8 root set-up on one GPU.

    python tests/golden/make_shard_digests.py --small

adds (or refreshes) only the "small" section: the same records at the
reduced sizes of SMALL (keys per rank), which the one-GPU multi-rank
rehearsal of bench.py (tests/test_gpu_bench_dist.py) runs at, so that its
per-rank parity reads "ok" rather than "unpinned".
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)

from tests.golden.make_golden import load_ref, ref_batch  # noqa: E402
from twemproxy_amd import hashkit as hk  # noqa: E402  (input generator only)
from twemproxy_amd.shard import plan_bounds  # noqa: E402

NS = (1, 2, 4, 8)
LEGS = {  # config -> (keys per rank, modes bench.py times on it)
    "C2": (1 << 26, ("fnv1a_64", "md5")),
    "C3": (1 << 26, ("fnv1a_64", "crc32", "md5")),
    "C4": (1 << 25, ("md5", "crc32", "fnv1a_64")),
}
SMALL = {"C2": (1 << 16,), "C3": (1 << 16,), "C4": (1 << 12,)}
CHUNK_BYTES = 1 << 30


def offsets_all(spec, n: int) -> np.ndarray:
    import ctypes

    from twemproxy_amd import _lib as L

    off = np.empty(n + 1, dtype=np.uint64)
    cs = spec.c()
    L.check(L.lib().nc_synth_offsets_host(ctypes.byref(cs), 0, n, off.ctypes.data), "nc_synth_offsets_host")
    return off


def main() -> None:
    path = os.path.join(HERE, "shard_digests.json")
    if "--small" in sys.argv[1:]:
        res = json.load(open(path))
        res["small"] = {cfg: {str(n): entry(load_ref(), cfg, n, LEGS[cfg][1], 1, time.time()) for n in ns}
                        for cfg, ns in SMALL.items()}
        with open(path, "w") as f:
            json.dump(res, f, indent=1)
        return
    ref = load_ref()
    threads = min(os.cpu_count() or 1, 16)
    t0 = time.time()
    res = {"source": "oracle/_ref (reference src/hashkit compiled from /root/reference), "
                     "tests/golden/make_shard_digests.py",
           "rule": "twemproxy_amd/shard.py plan_bounds over the N x n_per_rank batch (keys from index 0)",
           "configs": {cfg: entry(ref, cfg, per_rank, modes, threads, t0) for cfg, (per_rank, modes) in LEGS.items()}}
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(f"done in {time.time() - t0:.0f}s")


def entry(ref, cfg: str, per_rank: int, modes, threads: int, t0: float) -> dict:
    """per (N, rank): key range, byte range and sha256 of the reference's
    outputs, for the N x per_rank batch of cfg"""
    spec = hk.CONFIGS[cfg]["spec"]
    ntot = per_rank * max(NS)
    off = offsets_all(spec, ntot)
    outs = {m: np.empty(ntot, dtype=np.uint32) for m in modes}
    mean = max(1, int(off[-1]) // ntot)
    step = max(1 << 16, CHUNK_BYTES // mean)
    for k0 in range(0, ntot, step):
        n = min(step, ntot - k0)
        kb, ob = hk.synth_host(spec, k0, n)
        for m in modes:
            outs[m][k0: k0 + n] = ref_batch(ref, hk.HASH_NAMES.index(m), kb, ob, threads)
        del kb, ob
        print(f"  {cfg}: {k0 + n}/{ntot} keys, {time.time() - t0:.0f}s", flush=True)
    rec = {"spec": spec.__dict__, "n_per_rank": per_rank, "N": {}}
    for N in NS:
        n = per_rank * N
        kb_ = plan_bounds(torch.from_numpy(off[: n + 1].view(np.int64)), N).tolist()
        ranks = []
        for r in range(N):
            lo, hi = kb_[r], kb_[r + 1]
            ranks.append({"keys": [lo, hi], "bytes": [int(off[lo]), int(off[hi])],
                          **{m: hashlib.sha256(outs[m][lo:hi].tobytes()).hexdigest() for m in modes}})
        rec["N"][str(N)] = ranks
    return rec


if __name__ == "__main__":
    main()
