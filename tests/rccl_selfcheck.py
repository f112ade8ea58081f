"""RCCL (the ``nccl`` backend on ROCm) on one GPU, world size 1: every call
bench.py and shard.py make on the 8-GPU node, with device tensors, so the
transport has carried bytes before the driver's scaling run.

- ``init_process_group("nccl", device_id=...)`` as bench.py does;
- ``batch_isend_irecv`` of ``shard._pieces()``-cut device buffers (a self
  send and receive per piece: ``NC_SCATTER_MAX_MSG_BYTES`` is set small by the
  caller so offsets and keys go as several pieces, paired in order as in
  ``scatter_shards``' rounds);
- ``scatter_shards`` at world size 1 (broadcast of the bounds, the root's own
  shard);
- ``bench.max_over_ranks`` / ``sum_over_ranks`` (CUDA-tensor ``all_reduce``),
  ``barrier`` and ``all_gather_object`` (the per-rank parity gather).

Run as a fresh process (tests/test_gpu_rccl.py) before anything else touches
the GPU; prints one JSON line and exits 0 when every byte round-tripped.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main() -> int:
    import torch
    import torch.distributed as dist

    port = int(sys.argv[1])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"

    import bench
    from twemproxy_amd import shard

    g = torch.Generator(device="cpu").manual_seed(5)
    n = 40_003
    lens = torch.randint(0, 65, (n,), generator=g)
    off = torch.zeros(n + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(lens, 0)
    keys = torch.randint(0, 256, (int(off[-1]),), generator=g, dtype=torch.uint8)
    off_d, keys_d = off.to(dev), keys.to(dev)

    # the scatter's wire pattern, to self: piece j of the offsets and keys in
    # round j, each round one grouped batch_isend_irecv
    got_off, got_keys = torch.empty_like(off_d), torch.empty_like(keys_d)
    sends = shard._pieces(off_d) + shard._pieces(keys_d)
    recvs = shard._pieces(got_off) + shard._pieces(got_keys)
    assert len(sends) == len(recvs) >= 4, (len(sends), shard.MAX_MSG_BYTES)
    for s, r in zip(sends, recvs):
        ops = [dist.P2POp(dist.isend, s, 0), dist.P2POp(dist.irecv, r, 0)]
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    torch.cuda.synchronize()
    p2p_ok = torch.equal(got_off, off_d) and torch.equal(got_keys, keys_d)

    lk, lo, first = shard.scatter_shards(keys_d, off_d, dev)
    scatter_ok = first == 0 and torch.equal(lo, off_d) and torch.equal(lk[: keys_d.numel()], keys_d)

    bench.COMM_DEV = "cuda"
    mx = bench.max_over_ranks(torch, 1.25, True)
    sm = bench.sum_over_ranks(torch, 2.5, True)
    dist.barrier()
    gathered = [None]
    dist.all_gather_object(gathered, {"rank": 0, "parity": "ok"})
    coll_ok = mx == 1.25 and sm == 2.5 and gathered == [{"rank": 0, "parity": "ok"}]
    dist.destroy_process_group()
    ok = p2p_ok and scatter_ok and coll_ok
    print(json.dumps({"backend": "nccl", "pieces": len(sends), "piece_bytes": shard.MAX_MSG_BYTES,
                      "p2p_bytes": int(off_d.numel() * 8 + keys_d.numel()), "p2p": p2p_ok, "scatter": scatter_ok,
                      "collectives": coll_ok, "ok": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
