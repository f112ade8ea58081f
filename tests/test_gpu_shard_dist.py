"""Multi-rank sharding with the HIP kernel doing the hashing: world_size 2
over gloo on the one GPU of the test box (both ranks on cuda:0). Rank 0
scatters byte-balanced key ranges (twemproxy_amd.shard.scatter_shards, the
code bench.py --gpus N runs over RCCL), every rank copies its shard to the
device and hashes it with nc_gpuhash (fnv1a_64, md5, crc32), and the shards'
hashes must reassemble to the oracle's hashes of the full batch."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import twemproxy_amd as t

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, spec_args, n, q):
    import torch
    import torch.distributed as dist

    from twemproxy_amd.shard import scatter_shards

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.oracle_lib import Oracle

        spec = t.SynthSpec(*spec_args)
        keys_np, off_np = t.synth_host(spec, 0, n)
        keys = torch.from_numpy(keys_np) if rank == 0 else None
        off = torch.from_numpy(off_np.astype(np.int64)) if rank == 0 else None
        lk, lo, first = scatter_shards(keys, off, torch.device("cpu"))
        kd, od = lk.cuda(), lo.cuda()
        oracle = Oracle()
        ok = True
        for mode in ("fnv1a_64", "md5", "crc32"):
            out = t.hash_batch_device(mode, kd, od)
            torch.cuda.synchronize()
            mine = out.cpu().numpy().view(np.uint32)
            full = oracle.batch(t.mode_of(mode), keys_np, off_np, threads=1)
            ok &= bool(np.array_equal(mine, full[first: first + lo.numel() - 1]))
        q.put((rank, ok, first, lo.numel() - 1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("spec_args,n", [((2, t.hashkit.SYNTH_ZIPF, 8, 57), 50000),
                                         ((6, t.hashkit.SYNTH_UNIFORM, 0, 600), 4000)])
def test_shards_hashed_by_the_kernel(gpu, spec_args, n):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, spec_args, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), res
    assert res[0][2] == 0 and res[0][3] + res[1][3] == n and res[1][2] == res[0][3]
