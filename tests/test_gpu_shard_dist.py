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


def _shard_setup(cfg: str, modes):
    """Rank 0's N = 8 set-up of bench.py --gpus 8 on one GPU: the whole
    8 x n_per_rank batch of `cfg` generated on the device (C4: 2^28 x 256 B =
    64 GiB + 2 GiB of offsets), plan_bounds, then every rank's shard cut and
    copied the way scatter_shards hands it over (shard_of, the root's local
    copy, offsets rebased to 0), hashed with the shape the bench passes,
    against the compiled reference's per-rank digests
    (tests/golden/shard_digests.json)."""
    import hashlib
    import json

    import torch

    from twemproxy_amd.shard import plan_bounds, shard_of

    dg = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "shard_digests.json")))["configs"][cfg]
    spec = t.CONFIGS[cfg]["spec"]
    world = 8
    fk, fo = t.synth_device(spec, 0, dg["n_per_rank"] * world)
    kb = plan_bounds(fo, world)
    bb = fo[kb]
    kb, bb = kb.tolist(), bb.tolist()
    assert [[kb[r], kb[r + 1]] for r in range(world)] == [x["keys"] for x in dg["N"]["8"]]
    assert [[bb[r], bb[r + 1]] for r in range(world)] == [x["bytes"] for x in dg["N"]["8"]]
    for r in range(world):
        ks, os_ = shard_of(fk, fo, kb, bb, r)
        lk = torch.zeros(ks.numel() + t.NC_GPUHASH_PAD, dtype=torch.uint8, device="cuda")
        lk[: ks.numel()].copy_(ks)
        lo = os_ - bb[r]
        nk = lo.numel() - 1
        out = torch.empty(nk, dtype=torch.int32, device="cuda")
        shape = spec.shape(ks.numel())
        for mode in modes:
            t.hash_batch_device(mode, lk, lo, out, shape=shape, key_end=ks.numel())
            torch.cuda.synchronize()
            got = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
            assert got == dg["N"]["8"][r][mode], (cfg, mode, r)
        del lk, lo, out
    del fk, fo
    torch.cuda.empty_cache()


def test_shard_setup_n8_c4(gpu):
    _shard_setup("C4", ("md5", "crc32", "fnv1a_64"))


def test_shard_setup_n8_c2(gpu):
    _shard_setup("C2", ("fnv1a_64", "md5"))


def test_shard_setup_n8_c3(gpu):
    _shard_setup("C3", ("fnv1a_64", "crc32", "md5"))
