"""Python mirror of twemproxy's hashkit interface over the MI355X batched hasher.

Names follow the reference: the 12 modes of HASH_CODEC
(src/hashkit/nc_hashkit.h:24-36), ``conf_set_hash`` (src/nc_conf.c:1738-1764)
for the per-pool ``hash:`` selector, ``hash_<name>`` per-key functions.
Batched calls go through the C ABI (libnc_gpuhash.so) into the gfx950
kernels; they raise ``NcError`` when no GPU is usable instead of falling back.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Iterable, Sequence

import numpy as np

from . import _lib as L

# HASH_CODEC order == hash_type_t values (src/hashkit/nc_hashkit.h:24-48).
HASH_NAMES = (
    "one_at_a_time", "md5", "crc16", "crc32", "crc32a", "fnv1_64",
    "fnv1a_64", "fnv1_32", "fnv1a_32", "hsieh", "murmur", "jenkins",
)
HASH_DEFAULT = "fnv1a_64"  # CONF_DEFAULT_HASH, src/nc_conf.h:44
NMODES = len(HASH_NAMES)

# DIST_CODEC (src/hashkit/nc_hashkit.h:38-41)
DIST_NAMES = ("ketama", "modula", "random")


def conf_set_hash(value: str | bytes) -> int:
    """``hash:`` string -> hash_type_t, through the C selector.

    Raises ValueError("is not a valid hash") like conf_set_hash's error string.
    """
    raw = value.encode() if isinstance(value, str) else bytes(value)
    mode = L.lib().nc_gpuhash_mode_from_name(raw, len(raw))
    if mode < 0:
        raise ValueError(f"'{raw.decode(errors='replace')}' is not a valid hash")
    return mode


def mode_of(hash_: int | str) -> int:
    if isinstance(hash_, int):
        if not 0 <= hash_ < NMODES:
            raise ValueError(f"hash mode {hash_} out of range")
        return hash_
    return conf_set_hash(hash_)


def hash_key(hash_: int | str, key: bytes) -> int:
    """Per-key host hash through the link-compatible ``hash_<name>`` symbol."""
    name = HASH_NAMES[mode_of(hash_)]
    return int(getattr(L.lib(), "hash_" + name)(key, len(key)))


def ketama_hash(key: bytes, alignment: int) -> int:
    return int(L.lib().ketama_hash(key, len(key), alignment))


def md5_signature(key: bytes) -> bytes:
    buf = ctypes.create_string_buffer(16)
    L.lib().md5_signature(key, len(key), buf)
    return buf.raw


# ---------------------------------------------------------------- CSR helpers


def pack_keys(keys: Sequence[bytes], pad: int = L.NC_GPUHASH_PAD) -> tuple[np.ndarray, np.ndarray]:
    """List of keys -> (uint8 byte stream padded by `pad`, uint64 offsets[n+1])."""
    lens = np.fromiter((len(k) for k in keys), dtype=np.uint64, count=len(keys))
    offsets = np.zeros(len(keys) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    buf = np.zeros(int(offsets[-1]) + pad, dtype=np.uint8)
    if len(keys):
        buf[: int(offsets[-1])] = np.frombuffer(b"".join(keys), dtype=np.uint8)
    return buf, offsets


def shard_bounds(offsets: np.ndarray, nshards: int) -> np.ndarray:
    """Byte-balanced contiguous key ranges (nc_gpuhash_shard_bounds)."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.zeros(nshards + 1, dtype=np.uint64)
    L.check(
        L.lib().nc_gpuhash_shard_bounds(offsets.ctypes.data, n, nshards, out.ctypes.data),
        "nc_gpuhash_shard_bounds",
    )
    return out


def device_count() -> int:
    return int(L.lib().nc_gpuhash_device_count())


# ---------------------------------------------------------------- batches


def _stream_handle(stream) -> int | None:
    if stream is None:
        import torch

        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _shape_arg(shape):
    """(key_bytes, min_len, max_len) -> pointer to struct nc_gpuhash_shape, or None."""
    if shape is None:
        return None
    return ctypes.byref(L.NcShape(int(shape[0]), int(shape[1]), int(shape[2])))


def shape_of(offsets: np.ndarray) -> tuple[int, int, int]:
    """Batch shape (key_bytes, min_len, max_len) of a host offset CSR."""
    off = np.asarray(offsets, dtype=np.uint64)
    if off.size < 2:
        return 0, 0, 0
    lens = np.diff(off)
    return int(off[-1] - off[0]), int(lens.min()), int(lens.max())


def pick_variant(hash_: int | str, nkeys: int, shape=None) -> int:
    """The launch variant the auto policy picks (nc_gpuhash_pick_variant)."""
    v = L.lib().nc_gpuhash_pick_variant(mode_of(hash_), nkeys, _shape_arg(shape))
    if v < 0:
        raise L.NcError(ctypes.get_errno(), "nc_gpuhash_pick_variant")
    return v


def _check_batch(keys, offsets, key_end=None, stream=None) -> None:
    """Argument checks of the device-resident entry points: uint8 keys, int64
    offsets, both contiguous CUDA tensors, and a key buffer readable
    NC_GPUHASH_PAD bytes past offsets[-1] (the kernels' vector reads run up to
    that far). `key_end` is offsets[-1] as the packer knows it. When it is None
    the value is read back from the device ON THE LAUNCH STREAM `stream`, so it
    is ordered after whatever wrote the offsets there: one synchronising copy,
    which makes the call block until that stream reaches it. Pass key_end to
    keep the launch asynchronous."""
    import torch

    if keys.dtype != torch.uint8 or offsets.dtype != torch.int64:
        raise TypeError("keys must be uint8 and offsets int64")
    if not (keys.is_contiguous() and offsets.is_contiguous()):
        raise ValueError("keys and offsets must be contiguous")
    if offsets.dim() != 1 or offsets.numel() < 1:
        raise ValueError("offsets must be a 1-D tensor of n+1 entries")
    if offsets.numel() > 1 and key_end is not None:
        _check_key_room(keys.numel(), int(key_end))
    if not (keys.is_cuda and offsets.is_cuda):
        raise ValueError("device entry points need CUDA (HIP) tensors")
    if offsets.numel() > 1 and key_end is None:
        _check_key_room(keys.numel(), _read_last(offsets, stream))


def _torch_stream(stream, device):
    """The torch stream object of a launch-stream argument (None = current)."""
    import torch

    if stream is None:
        return torch.cuda.current_stream(device)
    if isinstance(stream, int):
        return torch.cuda.ExternalStream(stream, device=device)
    return stream


def _read_last(offsets, stream) -> int:
    """offsets[-1] read back on the launch stream (ordered after its writers)."""
    import torch

    with torch.cuda.stream(_torch_stream(stream, offsets.device)):
        return int(offsets[-1].item())


def _check_key_room(nbytes: int, end: int) -> None:
    if end < 0 or nbytes < end + L.NC_GPUHASH_PAD:
        raise ValueError(f"keys holds {nbytes} bytes; offsets[-1] = {end} needs "
                         f"{end + L.NC_GPUHASH_PAD} (NC_GPUHASH_PAD readable bytes past the last key)")


def hash_batch_device(hash_: int | str, keys, offsets, out=None, stream=None, shape=None, key_end=None):
    """Device-resident batch on torch tensors.

    keys: uint8 CUDA tensor readable NC_GPUHASH_PAD bytes past offsets[-1];
    offsets: int64 CUDA tensor of n+1 non-decreasing offsets;
    out: int32 CUDA tensor of n (allocated if None; the bits are the u32 hash).
    shape: optional (key_bytes, min_len, max_len) the packer knows, used only
    to pick the kernel pipeline (nc_gpuhash_batch_device_shaped).
    key_end: offsets[-1] if the caller knows it (else it is read back from
    the device once, to check the key buffer's size).
    Enqueued on `stream` (default: torch's current stream).
    """
    import torch

    mode = mode_of(hash_)
    n = offsets.numel() - 1
    _check_batch(keys, offsets, key_end, stream)
    if out is None:
        out = torch.empty(max(n, 0), dtype=torch.int32, device=keys.device)
    elif out.dtype != torch.int32 or not out.is_cuda or not out.is_contiguous() or out.numel() < n:
        raise ValueError("out must be a contiguous int32 CUDA tensor of at least n entries")
    L.check(
        L.lib().nc_gpuhash_batch_device_shaped(
            mode, keys.data_ptr(), offsets.data_ptr(), n, out.data_ptr(), _shape_arg(shape), _stream_handle(stream)
        ),
        "nc_gpuhash_batch_device_shaped",
    )
    return out


def continuum_device(indices, values=None, device="cuda"):
    """A pool's continuum (struct continuum {index, value}, src/nc_server.h:64-67)
    as the int32 (n, 2) device tensor server_idx_device takes; modula
    continua carry value 0 (src/hashkit/nc_modula.c:128-129)."""
    import torch

    idx = np.ascontiguousarray(indices, dtype=np.uint32)
    val = np.zeros_like(idx) if values is None else np.ascontiguousarray(values, dtype=np.uint32)
    pairs = np.stack([idx, val], axis=1).view(np.int32)
    return torch.from_numpy(np.ascontiguousarray(pairs)).to(device)


def ketama_build_device(names: Sequence[bytes], weights: Sequence[int], live: Sequence[bool] | None = None,
                        device="cuda", stream=None):
    """ketama_update (src/hashkit/nc_ketama.c:58-219) on the device: the pool's
    continuum as the int32 (n, 2) {index, value} tensor server_idx_device takes."""
    import torch

    n = len(names)
    if live is not None and len(live) != n:
        raise ValueError("live must have one flag per server")
    nlive = n if live is None else int(sum(bool(x) for x in live))
    cap = (nlive + 10) * 160  # the reference's allocation (KETAMA_CONTINUUM_ADDITION, nc_ketama.c:132-133)
    cont = torch.empty((cap, 2), dtype=torch.int32, device=device)
    lv = None if live is None else (ctypes.c_uint8 * n)(*[1 if x else 0 for x in live])
    cnt = ctypes.c_uint32(0)
    L.check(
        L.lib().nc_gpuhash_ketama_build_device(
            (ctypes.c_char_p * n)(*names), (ctypes.c_uint32 * n)(*[len(x) for x in names]),
            (ctypes.c_uint32 * n)(*weights), lv, n, cont.data_ptr(), cap, ctypes.byref(cnt), _stream_handle(stream),
        ),
        "nc_gpuhash_ketama_build_device",
    )
    return cont[: cnt.value].clone()


def server_idx_device(hash_: int | str, dist: int | str, keys, offsets, continuum, nserver: int,
                      hash_tag: bytes | None = None, out=None, stream=None, shape=None, key_end=None):
    """Fused server_pool_idx (src/nc_server.c:647-700) for a device-resident
    batch: hash_tag trimming, the pool's hash, then ketama/modula dispatch over
    `continuum` (continuum_device()). Returns the int32 server index per key."""
    import torch

    mode = mode_of(hash_)
    d = DIST_NAMES.index(dist) if isinstance(dist, str) else int(dist)
    n = offsets.numel() - 1
    if hash_tag is not None and len(hash_tag) != 2:
        raise ValueError("hash_tag is two bytes (conf_set_hash_tag)")
    _check_batch(keys, offsets, key_end, stream)
    if continuum.dtype != torch.int32 or not continuum.is_cuda or not continuum.is_contiguous():
        raise ValueError("continuum must be a contiguous int32 CUDA tensor (continuum_device())")
    if out is None:
        out = torch.empty(max(n, 0), dtype=torch.int32, device=keys.device)
    L.check(
        L.lib().nc_gpuhash_server_idx_device(
            mode, d, keys.data_ptr(), offsets.data_ptr(), n, continuum.data_ptr(), continuum.shape[0], nserver,
            hash_tag, _shape_arg(shape), out.data_ptr(), _stream_handle(stream),
        ),
        "nc_gpuhash_server_idx_device",
    )
    return out


MC_OK, MC_EINVAL, MC_EKEYLEN, MC_EUNSUPPORTED = 0, -1, -2, -3  # NC_GPUHASH_MC_*


def _check_stream(stream) -> None:
    """The parsers read `stream` on the device: it must be a contiguous uint8
    CUDA tensor (a host tensor's pointer would be dereferenced by a kernel)."""
    import torch

    if not isinstance(stream, torch.Tensor) or stream.dtype != torch.uint8:
        raise TypeError("stream must be a uint8 tensor")
    if not stream.is_cuda:
        raise ValueError("stream must be a CUDA (HIP) tensor")
    if not stream.is_contiguous():
        raise ValueError("stream must be contiguous")


class McParser:
    """Key extraction on the device from pipelined memcache retrieval requests
    (nc_gpuhash_mc_parse_device; memcache_parse_req, src/proto/nc_memcache.c)."""

    def __init__(self, max_bytes: int, max_reqs: int, max_keys: int):
        self._lib = L.lib()
        self._h = self._lib.nc_gpuhash_mc_parser_create(max_bytes, max_reqs, max_keys)
        if not self._h:
            raise L.NcError(ctypes.get_errno(), "nc_gpuhash_mc_parser_create failed")
        self.max_keys, self.max_reqs, self.max_bytes = max_keys, max_reqs, max_bytes

    def close(self) -> None:
        if self._h:
            self._lib.nc_gpuhash_mc_parser_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def parse(self, stream, stream_handle=None):
        """stream: uint8 CUDA tensor of requests. Returns (keys uint8 padded,
        offsets int64 (nkeys+1), key_req int32, req_status int32, result dict);
        keys/offsets feed hash_batch_device / server_idx_device directly."""
        import torch

        _check_stream(stream)
        dev = stream.device
        nbytes = stream.numel()
        keys = torch.empty(nbytes + L.NC_GPUHASH_PAD, dtype=torch.uint8, device=dev)
        off = torch.empty(self.max_keys + 1, dtype=torch.int64, device=dev)
        kreq = torch.empty(self.max_keys, dtype=torch.int32, device=dev)
        status = torch.empty(self.max_reqs, dtype=torch.int32, device=dev)
        res = L.NcMcResult()
        L.check(
            self._lib.nc_gpuhash_mc_parse_device(
                self._h, stream.data_ptr(), nbytes, keys.data_ptr(), off.data_ptr(), kreq.data_ptr(),
                status.data_ptr(), ctypes.byref(res), _stream_handle(stream_handle),
            ),
            "nc_gpuhash_mc_parse_device",
        )
        nk, nr = int(res.nkeys), int(res.nreqs)
        info = {"nreqs": nr, "nkeys": nk, "first_error": int(res.first_error), "consumed": int(res.consumed)}
        return keys, off[: nk + 1], kreq[:nk], status[:nr], info


class RedisParser(McParser):
    """Key extraction on the device from pipelined redis (RESP) requests of the
    arg0/arg1/argn/argx/argkvx classes (nc_gpuhash_redis_parse_device;
    redis_parse_req, src/proto/nc_redis.c:460-1900)."""

    def __init__(self, max_bytes: int, max_reqs: int, max_keys: int, max_key_len: int = 16336):
        self._lib = L.lib()
        self._h = self._lib.nc_gpuhash_redis_parser_create(max_bytes, max_reqs, max_keys)
        if not self._h:
            raise L.NcError(ctypes.get_errno(), "nc_gpuhash_redis_parser_create failed")
        self.max_keys, self.max_reqs, self.max_bytes = max_keys, max_reqs, max_bytes
        self.max_key_len = max_key_len  # mbuf_data_size(): 16 KiB mbuf less its header (src/nc_mbuf.c)

    def close(self) -> None:
        if self._h:
            self._lib.nc_gpuhash_redis_parser_destroy(self._h)
            self._h = None

    def parse(self, stream, stream_handle=None):
        """As McParser.parse, with NC_GPUHASH_REDIS_* statuses."""
        import torch

        _check_stream(stream)
        dev = stream.device
        nbytes = stream.numel()
        keys = torch.empty(nbytes + L.NC_GPUHASH_PAD, dtype=torch.uint8, device=dev)
        off = torch.empty(self.max_keys + 1, dtype=torch.int64, device=dev)
        kreq = torch.empty(self.max_keys, dtype=torch.int32, device=dev)
        # max_reqs + 1: a failing request after max_reqs ok ones has a status too
        status = torch.empty(self.max_reqs + 1, dtype=torch.int32, device=dev)
        res = L.NcRedisResult()
        L.check(
            self._lib.nc_gpuhash_redis_parse_device(
                self._h, stream.data_ptr(), nbytes, self.max_key_len, keys.data_ptr(), off.data_ptr(),
                kreq.data_ptr(), status.data_ptr(), ctypes.byref(res), _stream_handle(stream_handle),
            ),
            "nc_gpuhash_redis_parse_device",
        )
        nk, nr = int(res.nkeys), int(res.nreqs)
        info = {"nreqs": nr, "nkeys": nk, "first_error": int(res.first_error), "consumed": int(res.consumed)}
        return keys, off[: nk + 1], kreq[:nk], status[:nr], info


def time_batch_device(hash_: int | str, keys, offsets, out, iters: int, stream=None, shape=None) -> float:
    """Mean ms per launch over `iters` launches, timed by hipEvents on the launch stream."""
    mode = mode_of(hash_)
    ms = ctypes.c_float(0.0)
    L.check(
        L.lib().nc_gpuhash_time_device_shaped(
            mode, keys.data_ptr(), offsets.data_ptr(), offsets.numel() - 1, out.data_ptr(),
            _shape_arg(shape), _stream_handle(stream), iters, ctypes.byref(ms),
        ),
        "nc_gpuhash_time_device_shaped",
    )
    return float(ms.value)


def probe_read_gbs(buf, iters: int = 20, stream=None, nt: bool = False) -> float:
    """Same-run HBM read ceiling: GB/s of a STREAM-style 16-byte read over the
    uint8 CUDA tensor `buf` (nc_gpuhash_probe_read, or _nt for non-temporal loads)."""
    import torch

    nbytes = (buf.numel() // 16) * 16
    sink = torch.zeros(65536, dtype=torch.int32, device=buf.device)
    ms = ctypes.c_float(0.0)
    name = "nc_gpuhash_probe_read_nt" if nt else "nc_gpuhash_probe_read"
    L.check(getattr(L.lib(), name)(buf.data_ptr(), nbytes, sink.data_ptr(), _stream_handle(stream), iters,
                                   ctypes.byref(ms)), name)
    return nbytes / (ms.value * 1e-3) / 1e9


def probe_mix_gbs(buf, iters: int = 20, stream=None, policy: int = 0) -> float:
    """Same-run ceiling for a hash kernel's traffic mix: GB/s (bytes read +
    written) of the nt 16-byte read of `buf` with one streaming 16-byte store
    per 128 bytes read (nc_gpuhash_probe_mix; policy bit 0 / 1: default-policy
    loads / stores)."""
    import torch

    nbytes = (buf.numel() // 16) * 16
    wbytes = -(-nbytes // 32768) * 4096
    wout = torch.empty(wbytes, dtype=torch.uint8, device=buf.device)
    sink = torch.zeros(65536, dtype=torch.int32, device=buf.device)
    ms = ctypes.c_float(0.0)
    L.check(L.lib().nc_gpuhash_probe_mix(buf.data_ptr(), nbytes, wout.data_ptr(), wbytes, sink.data_ptr(),
                                         _stream_handle(stream), policy, iters, ctypes.byref(ms)),
            "nc_gpuhash_probe_mix")
    return (nbytes + nbytes // 8) / (ms.value * 1e-3) / 1e9


def hash_batch_host(hash_: int | str, keys: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """Synchronous host batch (nc_hashkit_batch): pinned copy -> GPU -> copy back."""
    mode = mode_of(hash_)
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.empty(n, dtype=np.uint32)
    L.check(
        L.lib().nc_hashkit_batch(mode, keys.ctypes.data, offsets.ctypes.data, n, out.ctypes.data),
        "nc_hashkit_batch",
    )
    return out


def hash_keys(hash_: int | str, keys: Sequence[bytes]) -> list[int]:
    """Batch-hash a list of keys on the GPU (host round trip)."""
    buf, off = pack_keys(keys)
    return [int(x) for x in hash_batch_host(hash_, buf, off)]


class Context:
    """nc_gpuhash_ctx: pinned, multi-slot asynchronous host batches."""

    def __init__(self, device: int = 0, max_keys: int = 65536, max_key_bytes: int = 1 << 22, nslots: int = 2,
                 zero_copy_bytes: int | None = None):
        self._lib = L.lib()
        handle = self._lib.nc_gpuhash_ctx_create(device, max_keys, max_key_bytes, nslots)
        if not handle:
            err = ctypes.get_errno()
            raise L.NcError(err, "nc_gpuhash_ctx_create failed")
        self._h = handle
        self._keep: dict[int, tuple] = {}
        if zero_copy_bytes is not None:  # None: the library default (1 MiB)
            self.set_zero_copy(zero_copy_bytes)

    def set_zero_copy(self, max_key_bytes: int) -> None:
        """Batches up to max_key_bytes skip the H2D/D2H copies (nc_gpuhash_ctx_set_zero_copy)."""
        L.check(self._lib.nc_gpuhash_ctx_set_zero_copy(self._h, max_key_bytes), "nc_gpuhash_ctx_set_zero_copy")

    def close(self) -> None:
        if self._h:
            self._lib.nc_gpuhash_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def submit(self, hash_: int | str, keys: np.ndarray, offsets: np.ndarray) -> tuple[int, np.ndarray]:
        """Returns (ticket, out); `out` is valid once poll()/wait() says NC_OK."""
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        out = np.empty(n, dtype=np.uint32)
        ticket = ctypes.c_int(-1)
        rc = self._lib.nc_gpuhash_submit(
            self._h, mode_of(hash_), keys.ctypes.data, offsets.ctypes.data, n, out.ctypes.data, ctypes.byref(ticket)
        )
        if rc == L.NC_EAGAIN:
            raise BlockingIOError("all context slots busy")
        L.check(rc, "nc_gpuhash_submit")
        self._keep[ticket.value] = (out,)
        return ticket.value, out

    def submit_spans(self, hash_: int | str, buf: np.ndarray, spans: Sequence[tuple[int, int]]) -> tuple[int, np.ndarray]:
        """Spans are (start, end) byte offsets into `buf` (keypos-style borrowed keys)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        base = buf.ctypes.data
        arr = (L.NcKeySpan * max(len(spans), 1))()
        for i, (s, e) in enumerate(spans):
            if not 0 <= s <= e <= buf.size:  # [s, e) is copied out of buf before the call returns
                raise ValueError(f"span {i} ({s}, {e}) is not inside the {buf.size}-byte buffer")
            arr[i].start = base + s
            arr[i].end = base + e
        out = np.empty(len(spans), dtype=np.uint32)
        ticket = ctypes.c_int(-1)
        rc = self._lib.nc_gpuhash_submit_spans(
            self._h, mode_of(hash_), arr, len(spans), out.ctypes.data, ctypes.byref(ticket)
        )
        if rc == L.NC_EAGAIN:
            raise BlockingIOError("all context slots busy")
        L.check(rc, "nc_gpuhash_submit_spans")
        self._keep[ticket.value] = (out,)
        return ticket.value, out

    def poll(self, ticket: int) -> bool:
        rc = self._lib.nc_gpuhash_poll(self._h, ticket)
        if rc == L.NC_EAGAIN:
            return False
        L.check(rc, "nc_gpuhash_poll")
        self._keep.pop(ticket, None)
        return True

    def wait(self, ticket: int) -> None:
        L.check(self._lib.nc_gpuhash_wait(self._h, ticket), "nc_gpuhash_wait")
        self._keep.pop(ticket, None)


class Ring:
    """nc_gpuhash_ring: small batches (one mbuf's keys) served by one resident
    launch, one workgroup per lane (batch n on lane n % lanes), polling mapped
    host memory — no HIP call per batch (include/nc_gpuhash.h 3d). Tickets
    complete in order within a lane; poll each one. Thread-safe (the ring's
    mutex)."""

    def __init__(self, device: int = 0, nslots: int = 4, max_keys: int = 4095, max_key_bytes: int = 32768,
                 lanes: int = 0, threads: int = 0):
        self._lib = L.lib()
        handle = self._lib.nc_gpuhash_ring_create_ex(device, nslots, max_keys, max_key_bytes, lanes, threads)
        if not handle:
            raise L.NcError(ctypes.get_errno(), "nc_gpuhash_ring_create failed")
        self._h = handle
        self._keep: dict[int, tuple] = {}

    @property
    def lanes(self) -> int:
        return int(self._lib.nc_gpuhash_ring_lanes(self._h))

    @property
    def staging(self) -> str:
        """where batches are staged: "device" (HBM written through the PCIe
        BAR) or "host" (mapped host memory)"""
        return "device" if self._lib.nc_gpuhash_ring_debug_staging(self._h) == 1 else "host"

    def debug_start_seq(self, seq: int) -> None:
        """number this (fresh) ring's batches from `seq` (tests of the ticket wrap)"""
        L.check(self._lib.nc_gpuhash_ring_debug_start_seq(self._h, seq), "nc_gpuhash_ring_debug_start_seq")

    def debug_hold(self, hold: bool) -> None:
        """while held, no worker is launched: submitted batches stay pending"""
        L.check(self._lib.nc_gpuhash_ring_debug_hold(self._h, int(hold)), "nc_gpuhash_ring_debug_hold")

    def close(self) -> None:
        if self._h:
            self._lib.nc_gpuhash_ring_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def launches(self) -> int:
        """worker launches so far (the first submit's, and relaunches after idle)"""
        return int(self._lib.nc_gpuhash_ring_launches(self._h))

    def submit_spans(self, hash_: int | str, buf: np.ndarray, spans: Sequence[tuple[int, int]]) -> tuple[int, np.ndarray]:
        """Spans are (start, end) byte offsets into `buf`; returns (ticket, out),
        `out` valid once poll()/wait() says so."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        base = buf.ctypes.data
        arr = (L.NcKeySpan * max(len(spans), 1))()
        for i, (s, e) in enumerate(spans):
            if not 0 <= s <= e <= buf.size:  # [s, e) is copied out of buf before the call returns
                raise ValueError(f"span {i} ({s}, {e}) is not inside the {buf.size}-byte buffer")
            arr[i].start = base + s
            arr[i].end = base + e
        out = np.empty(len(spans), dtype=np.uint32)
        ticket = ctypes.c_int(-1)
        rc = self._lib.nc_gpuhash_ring_submit_spans(self._h, mode_of(hash_), arr, len(spans), out.ctypes.data,
                                                    ctypes.byref(ticket))
        if rc == L.NC_EAGAIN:
            raise BlockingIOError("the next ring slot's batch is still in flight")
        L.check(rc, "nc_gpuhash_ring_submit_spans")
        self._keep[ticket.value] = (out,)
        return ticket.value, out

    def poll(self, ticket: int) -> bool:
        rc = self._lib.nc_gpuhash_ring_poll(self._h, ticket)
        if rc == L.NC_EAGAIN:
            return False
        L.check(rc, "nc_gpuhash_ring_poll")
        self._keep.pop(ticket, None)
        return True

    def wait(self, ticket: int) -> None:
        L.check(self._lib.nc_gpuhash_ring_wait(self._h, ticket), "nc_gpuhash_ring_wait")
        self._keep.pop(ticket, None)

    def forget(self, ticket: int) -> None:
        """nc_gpuhash_ring_forget: the batch runs on, its hashes are never
        copied into the ticket's output array"""
        L.check(self._lib.nc_gpuhash_ring_forget(self._h, ticket), "nc_gpuhash_ring_forget")
        self._keep.pop(ticket, None)


class Pipe:
    """nc_gpuhash_pipe: whole host batches from caller-pinned memory, chunked
    H2D / kernel / D2H on three streams, no repacking (the large-batch host
    path, SURVEY.md §8d end to end)."""

    def __init__(self, device: int = 0, chunk_keys: int = 1 << 22, chunk_bytes: int = 1 << 26, depth: int = 3):
        self._lib = L.lib()
        self._h = self._lib.nc_gpuhash_pipe_create(device, chunk_keys, chunk_bytes, depth)
        if not self._h:
            raise L.NcError(ctypes.get_errno(), "nc_gpuhash_pipe_create failed")

    def close(self) -> None:
        if self._h:
            self._lib.nc_gpuhash_pipe_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def hash(self, hash_: int | str, keys, offsets, out, nkeys: int | None = None, shape=None) -> None:
        """keys / offsets / out: pinned host tensors (torch pin_memory) or
        addresses of pinned memory; uint8 keys readable NC_GPUHASH_PAD bytes
        past offsets[nkeys], int64/uint64 offsets, int32/uint32 out. Blocks
        until every hash is in `out`.

        Tensor arguments are checked (_check_pinned_batch) before any copy
        starts. A raw address is the caller's promise: nothing behind it can
        be checked, and `nkeys` must then be given."""
        def addr(x):
            return x if isinstance(x, int) else x.data_ptr()

        nkeys = _check_pinned_batch(keys, offsets, out, nkeys)
        L.check(self._lib.nc_gpuhash_batch_pinned(self._h, mode_of(hash_), addr(keys), addr(offsets), nkeys,
                                                   addr(out), _shape_arg(shape), 0),
                "nc_gpuhash_batch_pinned")


def _check_pinned_batch(keys, offsets, out, nkeys: int | None) -> int:
    """Argument checks of Pipe.hash (nc_gpuhash_batch_pinned DMAs
    offsets[nkeys] + NC_GPUHASH_PAD bytes from `keys` and 4 * nkeys bytes into
    `out`, so a short tensor would be read or written past its end): dtypes,
    contiguity, sizes, then page-locked host memory. Returns nkeys."""
    import torch

    def tensor(x, name, dtypes):
        if isinstance(x, int):
            return None
        if x.dtype not in dtypes:
            raise TypeError(f"{name} must be {' or '.join(str(d) for d in dtypes)}, not {x.dtype}")
        if x.device.type != "cpu" or not x.is_contiguous() or x.dim() != 1:
            raise ValueError(f"{name} must be a contiguous 1-D host tensor")
        return x

    u64 = getattr(torch, "uint64", torch.int64)
    u32 = getattr(torch, "uint32", torch.int32)
    k = tensor(keys, "keys", (torch.uint8,))
    o = tensor(offsets, "offsets", (torch.int64, u64))
    w = tensor(out, "out", (torch.int32, u32))
    if nkeys is None:
        if o is None:
            raise ValueError("nkeys is required when offsets is a raw address")
        nkeys = o.numel() - 1
    if nkeys < 0 or (o is not None and o.numel() < nkeys + 1):
        raise ValueError(f"offsets holds {None if o is None else o.numel()} entries; {nkeys} keys need {nkeys + 1}")
    if w is not None and w.numel() < nkeys:
        raise ValueError(f"out holds {w.numel()} hashes; {nkeys} keys need {nkeys}")
    if k is not None and nkeys > 0:
        if o is not None:
            end = int(o[nkeys].item())
        else:
            end = ctypes.c_uint64.from_address(offsets + 8 * nkeys).value
        _check_key_room(k.numel(), end)
    for x, name in ((k, "keys"), (o, "offsets"), (w, "out")):
        if x is not None and x.numel() and not x.is_pinned():
            raise ValueError(f"{name} must be page-locked (pin_memory() or nc_gpuhash_host_register)")
    return nkeys


def host_register(ptr: int, nbytes: int) -> None:
    """Page-lock and map an existing host range (nc_gpuhash_host_register)."""
    L.check(L.lib().nc_gpuhash_host_register(ptr, nbytes), "nc_gpuhash_host_register")


def host_unregister(ptr: int) -> None:
    L.check(L.lib().nc_gpuhash_host_unregister(ptr), "nc_gpuhash_host_unregister")


# ---------------------------------------------------------------- synthetic keys

SYNTH_FIXED, SYNTH_ZIPF, SYNTH_UNIFORM = 0, 1, 2
BYTES_FULL, BYTES_PRINTABLE = 0, 1


@dataclass(frozen=True)
class SynthSpec:
    """Synthetic key set of SURVEY.md §8d (include/nc_gpuhash_synth.h)."""

    seed: int
    len_dist: int = SYNTH_FIXED
    len_a: int = 16
    len_b: int = 16
    charset: int = BYTES_FULL
    zipf_s: float = 1.0

    def c(self) -> L.NcSynthSpec:
        return L.NcSynthSpec(self.seed, self.len_dist, self.len_a, self.len_b, self.charset, self.zipf_s)

    def len_range(self) -> tuple[int, int]:
        """(shortest, longest) key length the generator can produce."""
        if self.len_dist == SYNTH_ZIPF:
            return self.len_a, self.len_a - 1 + self.len_b
        return self.len_a, self.len_b

    def shape(self, key_bytes: int) -> tuple[int, int, int]:
        """Batch shape (key_bytes, min_len, max_len) for hash_batch_device(shape=...)."""
        lo, hi = self.len_range()
        return int(key_bytes), lo, hi

    @staticmethod
    def fixed(seed: int, length: int, charset: int = BYTES_FULL) -> "SynthSpec":
        return SynthSpec(seed, SYNTH_FIXED, length, length, charset)

    @staticmethod
    def zipf(seed: int, lmin: int = 8, nvals: int = 57, s: float = 1.0, charset: int = BYTES_FULL) -> "SynthSpec":
        """len = lmin - 1 + r, r in [1, nvals], P(r) ~ 1/r^s (C2: 8..64 B)."""
        return SynthSpec(seed, SYNTH_ZIPF, lmin, nvals, charset, s)

    @staticmethod
    def uniform(seed: int, lo: int, hi: int, charset: int = BYTES_FULL) -> "SynthSpec":
        return SynthSpec(seed, SYNTH_UNIFORM, lo, hi, charset)


# Configurations of BASELINE.json / SURVEY.md §8d.
CONFIGS = {
    "C1": dict(spec=SynthSpec.fixed(1, 16), nkeys=1 << 20, modes=("fnv1a_64",)),
    "C2": dict(spec=SynthSpec.zipf(2), nkeys=1 << 26, modes=("fnv1a_64",)),
    "C3": dict(spec=SynthSpec.fixed(3, 32), nkeys=1 << 26, modes=HASH_NAMES),
    "C4": dict(spec=SynthSpec.fixed(4, 256), nkeys=1 << 28, modes=("md5", "crc32")),
    "C5": dict(spec=SynthSpec.zipf(5, charset=BYTES_PRINTABLE), nkeys=64 * 128, modes=("fnv1a_64",)),
}


def synth_host(spec: SynthSpec, first: int, n: int, pad: int = L.NC_GPUHASH_PAD) -> tuple[np.ndarray, np.ndarray]:
    """Keys [first, first+n) on the host: (uint8 bytes padded, uint64 offsets from 0)."""
    lib = L.lib()
    cs = spec.c()
    off = np.empty(n + 1, dtype=np.uint64)
    L.check(lib.nc_synth_offsets_host(ctypes.byref(cs), first, n, off.ctypes.data), "nc_synth_offsets_host")
    buf = np.zeros(int(off[-1]) + pad, dtype=np.uint8)
    L.check(lib.nc_synth_fill_host(ctypes.byref(cs), first, n, off.ctypes.data, buf.ctypes.data), "nc_synth_fill_host")
    return buf, off


def synth_device(spec: SynthSpec, first: int, n: int, device="cuda", pad: int = L.NC_GPUHASH_PAD, stream=None):
    """Keys [first, first+n) generated on the GPU: (uint8 tensor padded, int64 offsets tensor)."""
    import torch

    lib = L.lib()
    cs = spec.c()
    off = torch.empty(n + 1, dtype=torch.int64, device=device)
    st = _stream_handle(stream)
    L.check(lib.nc_synth_offsets_device(ctypes.byref(cs), first, n, off.data_ptr(), st), "nc_synth_offsets_device")
    total = int(off[-1].item())
    keys = torch.zeros(total + pad, dtype=torch.uint8, device=device)
    L.check(lib.nc_synth_fill_device(ctypes.byref(cs), first, n, off.data_ptr(), keys.data_ptr(), st),
            "nc_synth_fill_device")
    return keys, off


def iter_modes(modes: Iterable[int | str]) -> list[int]:
    return [mode_of(m) for m in modes]
