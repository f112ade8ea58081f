"""ctypes binding of libnc_gpuhash.so (include/nc_gpuhash.h, include/nc_gpuhash_synth.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
twemproxy_amd/csrc``). Loading fails loudly when it is missing: there is no
Python or CPU fallback for the batched path.
"""
from __future__ import annotations

import ctypes
import os
import threading

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnc_gpuhash.so")

NC_OK, NC_ERROR, NC_EAGAIN, NC_ENOMEM = 0, -1, -2, -3
NC_GPUHASH_PAD = 32

_lock = threading.Lock()
_lib = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)


class NcSynthSpec(ctypes.Structure):
    """struct nc_synth_spec (include/nc_gpuhash_synth.h)."""

    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("len_dist", ctypes.c_int32),
        ("len_a", ctypes.c_uint32),
        ("len_b", ctypes.c_uint32),
        ("charset", ctypes.c_int32),
        ("zipf_s", ctypes.c_double),
    ]


class NcShape(ctypes.Structure):
    """struct nc_gpuhash_shape (include/nc_gpuhash.h): what the packer knows about a batch."""

    _fields_ = [("key_bytes", ctypes.c_uint64), ("min_len", ctypes.c_uint32), ("max_len", ctypes.c_uint32)]


class NcMcResult(ctypes.Structure):
    """struct nc_gpuhash_mc_result (include/nc_gpuhash.h)."""

    _fields_ = [("nreqs", ctypes.c_uint64), ("nkeys", ctypes.c_uint64), ("first_error", ctypes.c_uint64),
                ("consumed", ctypes.c_uint64)]


class NcRedisResult(ctypes.Structure):
    """struct nc_gpuhash_redis_result (include/nc_gpuhash.h)."""

    _fields_ = [("nreqs", ctypes.c_uint64), ("nkeys", ctypes.c_uint64), ("first_error", ctypes.c_uint64),
                ("consumed", ctypes.c_uint64)]


class NcKeySpan(ctypes.Structure):
    """struct nc_keyspan — the shape of twemproxy's struct keypos (src/nc_message.h:232-235)."""

    _fields_ = [("start", ctypes.c_void_p), ("end", ctypes.c_void_p)]


# name -> (restype, argtypes); every symbol include/*.h declares.
SIGNATURES = {
    # per-key, src/hashkit/nc_hashkit.h:57-69
    "hash_one_at_a_time": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "md5_signature": (None, [ctypes.c_char_p, ctypes.c_uint, ctypes.c_char_p]),
    "hash_md5": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_crc16": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_crc32": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_crc32a": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_fnv1_64": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_fnv1a_64": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_fnv1_32": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_fnv1a_32": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_hsieh": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_jenkins": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "hash_murmur": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t]),
    "ketama_hash": (ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]),
    # selector
    "nc_gpuhash_mode_from_name": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "nc_gpuhash_mode_name": (ctypes.c_char_p, [ctypes.c_int]),
    # batches
    "nc_gpuhash_batch_device": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "nc_gpuhash_batch_device_shaped": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.POINTER(NcShape),
         ctypes.c_void_p],
    ),
    "nc_gpuhash_server_idx_device": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(NcShape), ctypes.c_void_p,
         ctypes.c_void_p],
    ),
    "nc_gpuhash_ketama_build_device": (
        ctypes.c_int,
        [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
         ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
         ctypes.c_void_p],
    ),
    "nc_gpuhash_mc_parser_create": (ctypes.c_void_p, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
    "nc_gpuhash_mc_parser_destroy": (None, [ctypes.c_void_p]),
    "nc_gpuhash_redis_parser_create": (ctypes.c_void_p, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
    "nc_gpuhash_redis_parser_destroy": (None, [ctypes.c_void_p]),
    "nc_gpuhash_redis_parse_device": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(NcRedisResult), ctypes.c_void_p],
    ),
    "nc_gpuhash_mc_parse_device": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.POINTER(NcMcResult), ctypes.c_void_p],
    ),
    "nc_gpuhash_pick_variant": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(NcShape)]),
    "nc_gpuhash_time_device_shaped": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.POINTER(NcShape),
         ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float)],
    ),
    "nc_gpuhash_time_device": (
        ctypes.c_int,
        [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_int, ctypes.POINTER(ctypes.c_float)],
    ),
    "nc_gpuhash_set_tuning": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "nc_gpuhash_ring_create": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "nc_gpuhash_ring_destroy": (None, [ctypes.c_void_p]),
    "nc_gpuhash_ring_submit_spans": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)],
    ),
    "nc_gpuhash_ring_poll": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "nc_gpuhash_ring_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "nc_gpuhash_ring_forget": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "nc_gpuhash_probe_tile_mix": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_float)]),
    "nc_gpuhash_probe_clock_sampler": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                                      ctypes.c_void_p]),
    "nc_gpuhash_ring_limits": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "nc_gpuhash_ring_launches": (ctypes.c_uint64, [ctypes.c_void_p]),
    "nc_gpuhash_ring_create_ex": (
        ctypes.c_void_p,
        [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32],
    ),
    "nc_gpuhash_ring_lanes": (ctypes.c_uint32, [ctypes.c_void_p]),
    "nc_gpuhash_ring_debug_staging": (ctypes.c_int, [ctypes.c_void_p]),
    "nc_gpuhash_ring_debug_start_seq": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "nc_gpuhash_ring_debug_hold": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "nc_gpuhash_ring_debug_timeline": (
        ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]),
    "nc_gpuhash_frag_plan": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "nc_gpuhash_ctx_create": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
    "nc_gpuhash_ctx_destroy": (None, [ctypes.c_void_p]),
    "nc_gpuhash_ctx_set_zero_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "nc_gpuhash_submit": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
         ctypes.POINTER(ctypes.c_int)],
    ),
    "nc_gpuhash_submit_spans": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(NcKeySpan), ctypes.c_uint32, ctypes.c_void_p,
         ctypes.POINTER(ctypes.c_int)],
    ),
    "nc_gpuhash_poll": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "nc_gpuhash_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "nc_hashkit_batch": (
        ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    ),
    # whole batches from caller-pinned memory
    "nc_gpuhash_pipe_create": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]),
    "nc_gpuhash_pipe_destroy": (None, [ctypes.c_void_p]),
    "nc_gpuhash_batch_pinned": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
         ctypes.POINTER(NcShape), ctypes.c_int],
    ),
    "nc_gpuhash_host_register": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "nc_gpuhash_host_unregister": (ctypes.c_int, [ctypes.c_void_p]),
    # sharding / info
    "nc_gpuhash_shard_bounds": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]),
    "nc_gpuhash_device_count": (ctypes.c_int, []),
    "nc_gpuhash_version": (ctypes.c_char_p, []),
    # diagnostics (include/nc_gpuhash_probe.h)
    "nc_gpuhash_probe_read": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.POINTER(ctypes.c_float)],
    ),
    "nc_gpuhash_probe_read_nt": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.POINTER(ctypes.c_float)],
    ),
    "nc_gpuhash_probe_mix": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)],
    ),
    # synthetic generator
    "nc_synth_lengths_host": (
        ctypes.c_int, [ctypes.POINTER(NcSynthSpec), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    ),
    "nc_synth_offsets_host": (
        ctypes.c_int, [ctypes.POINTER(NcSynthSpec), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    ),
    "nc_synth_fill_host": (
        ctypes.c_int,
        [ctypes.POINTER(NcSynthSpec), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "nc_synth_offsets_device": (
        ctypes.c_int,
        [ctypes.POINTER(NcSynthSpec), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p],
    ),
    "nc_synth_fill_device": (
        ctypes.c_int,
        [ctypes.POINTER(NcSynthSpec), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p],
    ),
}


class NcError(OSError):
    """A C-ABI call returned NC_ERROR / NC_ENOMEM / NC_EAGAIN."""


def lib() -> ctypes.CDLL:
    """Load libnc_gpuhash.so once; raise if it has not been built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(the batched hasher has no CPU fallback)"
                )
            # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's).
            # Load it first so this process has ONE HIP runtime, shared by torch
            # and libnc_gpuhash.so; if ours came first, torch's HIP init fails.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            handle = ctypes.CDLL(LIB_PATH, use_errno=True)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
        return _lib


def check(rc: int, what: str) -> None:
    """Raise NcError for a non-NC_OK status, with the C errno."""
    if rc != NC_OK:
        err = ctypes.get_errno()
        raise NcError(err, f"{what} failed: rstatus {rc} ({os.strerror(err) if err else 'no errno'})")
