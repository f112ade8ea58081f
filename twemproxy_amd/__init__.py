"""twemproxy_amd — MI355X-native batched key hashing, a drop-in for twemproxy's src/hashkit.

The product is the C-ABI library ``libnc_gpuhash.so`` (include/nc_gpuhash.h):
hand-written gfx950 HIP kernels for the 12 hashkit modes behind a C host layer.
This package is the Python mirror of the reference interface used by the
tests and the benchmark.
"""
from ._lib import LIB_PATH, NC_EAGAIN, NC_ENOMEM, NC_ERROR, NC_GPUHASH_PAD, NC_OK, NcError, lib
from .hashkit import (
    BYTES_FULL,
    BYTES_PRINTABLE,
    CONFIGS,
    DIST_NAMES,
    HASH_DEFAULT,
    HASH_NAMES,
    NMODES,
    Context,
    McParser,
    Pipe,
    RedisParser,
    Ring,
    SynthSpec,
    conf_set_hash,
    continuum_device,
    device_count,
    hash_batch_device,
    hash_batch_host,
    hash_key,
    hash_keys,
    host_register,
    host_unregister,
    ketama_hash,
    ketama_build_device,
    md5_signature,
    mode_of,
    pack_keys,
    pick_variant,
    probe_mix_gbs,
    probe_read_gbs,
    server_idx_device,
    shape_of,
    shard_bounds,
    synth_device,
    synth_host,
    time_batch_device,
)

__all__ = [
    "LIB_PATH", "NC_EAGAIN", "NC_ENOMEM", "NC_ERROR", "NC_GPUHASH_PAD", "NC_OK", "NcError", "lib",
    "BYTES_FULL", "BYTES_PRINTABLE", "CONFIGS", "DIST_NAMES", "HASH_DEFAULT", "HASH_NAMES", "NMODES",
    "Context", "SynthSpec", "conf_set_hash", "device_count", "hash_batch_device", "hash_batch_host",
    "hash_key", "hash_keys", "ketama_hash", "md5_signature", "mode_of", "pack_keys", "pick_variant", "probe_mix_gbs", "probe_read_gbs", "server_idx_device", "shape_of", "shard_bounds", "continuum_device", "ketama_build_device", "McParser", "RedisParser",
    "synth_device", "synth_host", "time_batch_device", "Pipe", "Ring", "host_register", "host_unregister",
]
