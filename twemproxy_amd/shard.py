"""Multi-GPU sharding of a key batch.

Keys are independent, so a batch splits into contiguous, byte-balanced key
ranges — one per rank — and each rank hashes its range with no exchange. The
only collective is the ingest scatter from a root rank: RCCL has no
variable-size scatter, so the root issues grouped point-to-point sends (one
``ncclSend`` per peer inside a group, i.e. ``torch.distributed.
batch_isend_irecv`` on the ``nccl`` backend), which use the root's direct xGMI
links to all peers in parallel. The same code runs on the ``gloo`` backend:
with CPU tensors for the CPU tests, and staged through host memory when the
tensors live on a GPU (bench.py --backend gloo --same-device: every rank on
cuda:0, the one-GPU rehearsal of the multi-GPU bench).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ._lib import NC_GPUHASH_PAD

# Largest single point-to-point message of the scatter: a C4 shard is 8 GiB;
# it goes as 1 GiB pieces (one round per piece, see scatter_shards), so no
# count or size inside the transport ever approaches 2^31 elements.
MAX_MSG_BYTES = int(os.environ.get("NC_SCATTER_MAX_MSG_BYTES", 1 << 30))  # smaller in the rehearsal tests


def plan_bounds(offsets: torch.Tensor, nshards: int) -> torch.Tensor:
    """Key bounds (nshards + 1, int64) splitting offsets' bytes evenly.

    Cut g is the first key whose start offset is >= g/nshards of the bytes —
    the same lower-bound rule as nc_gpuhash_shard_bounds (host C); computed
    with searchsorted on whatever device `offsets` lives on.
    """
    n = offsets.numel() - 1
    base = offsets[0]
    total = offsets[-1] - base
    g = torch.arange(1, nshards, device=offsets.device, dtype=torch.int64)
    if int(total) == 0:
        cuts = (g * n) // nshards
    else:
        # total * g / nshards without int64 overflow for multi-GiB batches
        q, r = total // nshards, total % nshards
        targets = base + q * g + (r * g) // nshards
        cuts = torch.searchsorted(offsets[:n].contiguous(), targets, right=False)
        cuts = torch.cummax(cuts, 0).values
    zero = torch.zeros(1, dtype=torch.int64, device=offsets.device)
    end = torch.full((1,), n, dtype=torch.int64, device=offsets.device)
    return torch.cat([zero, cuts.to(torch.int64), end])


def _pieces(t: torch.Tensor, max_bytes: int | None = None):
    """A 1-D tensor as contiguous views of at most max_bytes (MAX_MSG_BYTES)
    each; both ends cut it the same way, so sends and receives pair up in
    order."""
    step = max(1, (max_bytes or MAX_MSG_BYTES) // max(1, t.element_size()))
    return [t[i: i + step] for i in range(0, t.numel(), step)]


def shard_of(keys: torch.Tensor, offsets: torch.Tensor, kb, bb, r: int):
    """Rank r's shard as the root holds it: views of the key bytes
    [bb[r], bb[r+1]) and offsets [kb[r], kb[r+1]] of the full batch (not yet
    rebased). Used for the root's own shard and for the sends."""
    return keys[bb[r]: bb[r + 1]], offsets[kb[r]: kb[r + 1] + 1]


def _host_staged(group) -> bool:
    """gloo moves only CPU tensors point to point: device shards are staged
    through host memory (the one-GPU rehearsal of the RCCL path, where every
    rank shares cuda:0)."""
    return dist.get_backend(group) == "gloo"


def scatter_shards(keys: torch.Tensor | None, offsets: torch.Tensor | None, device: torch.device,
                   root: int = 0, group=None, pad: int = NC_GPUHASH_PAD):
    """Scatter byte-balanced key ranges from `root` to every rank.

    keys/offsets: the full batch on the root (uint8 bytes, int64 offsets),
    ignored elsewhere. Returns (local_keys uint8 padded by `pad`,
    local_offsets int64 rebased to 0, first_key_index) on `device`.

    The sends go in ROUNDS: round j holds piece j (at most MAX_MSG_BYTES) of
    every peer's shard, offsets first, one grouped batch_isend_irecv per round.
    A round keeps all of the root's xGMI links busy at once (one message per
    peer), while no group ever holds more than world - 1 operations — a C4
    shard at N = 8 is 9 rounds of 7 one-GiB sends, not one group of 63. Both
    ends derive the same piece lists from the broadcast bounds, so sends and
    receives pair up in order.
    """
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    staged = _host_staged(group)
    comm_dev = torch.device("cpu") if staged else device
    meta = torch.zeros(2 * (world + 1), dtype=torch.int64, device=comm_dev)
    if rank == root:
        kb = plan_bounds(offsets, world)
        bb = offsets[kb]
        meta.copy_(torch.cat([kb, bb]).to(comm_dev))
    dist.broadcast(meta, src=root, group=group)
    kb = meta[: world + 1].tolist()
    bb = meta[world + 1:].tolist()
    klo, khi, blo, bhi = kb[rank], kb[rank + 1], bb[rank], bb[rank + 1]

    local_keys = torch.zeros(bhi - blo + pad, dtype=torch.uint8, device=device)
    local_off = torch.empty(khi - klo + 1, dtype=torch.int64, device=device)
    if rank == root:
        pieces = {}
        for r in range(world):
            ks, os_ = shard_of(keys, offsets, kb, bb, r)
            if r == root:
                local_keys[: bhi - blo].copy_(ks)
                local_off.copy_(os_)
            else:
                pieces[r] = _pieces(os_) + _pieces(ks)
        rounds = max((len(p) for p in pieces.values()), default=0)
        for j in range(rounds):
            ops = [dist.P2POp(dist.isend, p[j].cpu() if staged else p[j], r, group)
                   for r, p in pieces.items() if j < len(p)]
            for req in dist.batch_isend_irecv(ops):
                req.wait()
    else:
        for dst in _pieces(local_off) + _pieces(local_keys[: bhi - blo]):
            buf = torch.empty(dst.numel(), dtype=dst.dtype) if staged and dst.device.type != "cpu" else dst
            for req in dist.batch_isend_irecv([dist.P2POp(dist.irecv, buf, root, group)]):
                req.wait()
            if buf is not dst:
                dst.copy_(buf)
    local_off -= blo
    return local_keys, local_off, klo
