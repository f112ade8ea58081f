"""Multi-rank sharding on CPU (gloo, world_size 2 and 3): byte-balanced bounds,
the root scatter, and that the shards' hashes reassemble to the full batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import twemproxy_amd as t
from twemproxy_amd.shard import plan_bounds, scatter_shards


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, spec_args, n, q, msg=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if msg:  # small message cap: every shard goes as many pieces
            import twemproxy_amd.shard as sh

            sh.MAX_MSG_BYTES = msg
        from tests.oracle_lib import Oracle

        spec = t.SynthSpec(*spec_args)
        keys_np, off_np = t.synth_host(spec, 0, n)
        keys = torch.from_numpy(keys_np) if rank == 0 else None
        off = torch.from_numpy(off_np.astype(np.int64)) if rank == 0 else None
        lk, lo, first = scatter_shards(keys, off, torch.device("cpu"))
        lo_np = lo.numpy().astype(np.uint64)
        oracle = Oracle()
        mine = oracle.batch(6, lk.numpy(), lo_np, threads=1)
        full = oracle.batch(6, keys_np, off_np, threads=1)
        ok = np.array_equal(mine, full[first: first + lo_np.size - 1])
        # pad after the shard's last key is zero and present
        ok &= lk.numel() == int(lo_np[-1]) + t.NC_GPUHASH_PAD
        q.put((rank, bool(ok), first, lo_np.size - 1, int(lo_np[-1])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("msg", [None, 777], ids=["whole", "pieces777"])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("spec_args,n", [((2, t.hashkit.SYNTH_ZIPF, 8, 57), 20000),
                                         ((6, t.hashkit.SYNTH_UNIFORM, 0, 600), 3000)])
def test_scatter_and_hash_shards(world, spec_args, n, msg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, spec_args, n, q, msg)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), res
    # contiguous cover of [0, n), byte-balanced
    starts = [r[2] for r in res]
    counts = [r[3] for r in res]
    assert starts[0] == 0 and sum(counts) == n
    assert all(starts[i] + counts[i] == starts[i + 1] for i in range(world - 1))
    bytes_ = [r[4] for r in res]
    assert max(bytes_) - min(bytes_) <= 2 * 600


def test_plan_bounds_matches_c_shard_bounds():
    for spec in (t.SynthSpec.zipf(2), t.SynthSpec.uniform(6, 0, 600), t.SynthSpec.fixed(3, 32)):
        _, off = t.synth_host(spec, 0, 12345)
        for g in (1, 2, 3, 4, 5, 8):
            want = t.shard_bounds(off, g).astype(np.int64)
            got = plan_bounds(torch.from_numpy(off.astype(np.int64)), g).numpy()
            np.testing.assert_array_equal(got, want)
    off = np.zeros(9, dtype=np.int64)
    np.testing.assert_array_equal(plan_bounds(torch.from_numpy(off), 4).numpy(),
                                  t.shard_bounds(off.astype(np.uint64), 4).astype(np.int64))


def test_small_shard_digests_pin_the_oracle():
    """The reduced-size per-rank digests (from the compiled reference, the
    multi-rank rehearsal's parity check) agree with the restatement's hashes
    over the same plan_bounds cut, and bench.py finds them by size and N."""
    import hashlib
    import json

    import bench
    from tests.oracle_lib import Oracle

    oracle = Oracle()
    small = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "shard_digests.json")))["small"]
    assert set(small) == {"C2", "C3", "C4"}
    for cfg, by_n in small.items():
        spec = t.CONFIGS[cfg]["spec"]
        for n_s, rec in by_n.items():
            per = int(n_s)
            for world, ranks in rec["N"].items():
                w = int(world)
                keys, off = t.synth_host(spec, 0, per * w)
                kb = plan_bounds(torch.from_numpy(off.astype(np.int64)), w).tolist()
                assert [r["keys"] for r in ranks] == [[kb[i], kb[i + 1]] for i in range(w)]
                assert bench.digest_ranks(cfg, per, w) == ranks
                for mode in ("fnv1a_64", "md5", "crc32"):
                    if mode not in ranks[0]:
                        continue
                    h = oracle.batch(t.mode_of(mode), keys, off, threads=2)
                    for i, r in enumerate(ranks):
                        got = hashlib.sha256(h[kb[i]: kb[i + 1]].tobytes()).hexdigest()
                        assert got == r[mode], (cfg, per, w, i, mode)
    assert bench.digest_ranks("C2", 1 << 26, 8) is not None  # the full-size records stay reachable
    assert bench.digest_ranks("C2", 12345, 2) is None
