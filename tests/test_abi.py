"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/*.h declares, and its host logic (selector, per-key link-compat
symbols, shard planning, synthetic generator) behaves like the reference."""
import ctypes
import errno
import os
import re

import numpy as np
import pytest

import twemproxy_amd as t
from twemproxy_amd import _lib as L

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def declared_functions():
    names = set()
    for h in ("nc_gpuhash.h", "nc_gpuhash_synth.h", "nc_gpuhash_probe.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, flags=re.M):
            if m.group(1) not in ("defined",):
                names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(L.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 35
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes binding covers exactly the declared surface
    assert names == set(L.SIGNATURES), names ^ set(L.SIGNATURES)


def test_library_has_gfx950_code_object():
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"nc_hash_kernel" in blob


def test_selector_matches_conf_set_hash():
    for m, name in enumerate(t.HASH_NAMES):
        assert t.conf_set_hash(name) == m
        assert L.lib().nc_gpuhash_mode_name(m).decode() == name
    assert t.conf_set_hash(t.HASH_DEFAULT) == 6
    for bad in ("", "fnv1a", "FNV1A_64", "fnv1a_64 ", "md5\0"):
        with pytest.raises(ValueError, match="is not a valid hash"):
            t.conf_set_hash(bad)
    assert L.lib().nc_gpuhash_mode_name(12) is None
    assert L.lib().nc_gpuhash_mode_name(-1) is None


def test_per_key_symbols_match_golden_corpus(corpus):
    keys, offsets, expected = corpus
    raw = keys.tobytes()
    for m, name in enumerate(t.HASH_NAMES):
        fn = getattr(L.lib(), "hash_" + name)
        got = [fn(raw[offsets[i]:offsets[i + 1]], int(offsets[i + 1] - offsets[i])) for i in range(offsets.size - 1)]
        np.testing.assert_array_equal(np.array(got, dtype=np.uint32), expected[m], err_msg=name)


def test_per_key_symbols_kats(kat):
    for name, want in kat["apple"].items():
        assert t.hash_key(name, b"apple") == want
    assert t.ketama_hash(b"server1-8", 0) == kat["ketama_server1-8"]["0"]
    assert t.ketama_hash(b"server1-8", 3) == kat["ketama_server1-8"]["3"]
    import hashlib

    for k in (b"", b"a", b"x" * 55, b"y" * 56, b"z" * 64, b"q" * 200):
        assert t.md5_signature(k) == hashlib.md5(k).digest()


def test_shard_bounds_byte_balanced():
    rng = np.random.default_rng(0)
    lens = rng.integers(0, 300, size=10001).astype(np.uint64)
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    for g in (1, 2, 3, 4, 7, 8):
        b = t.shard_bounds(off, g)
        assert b[0] == 0 and b[-1] == lens.size and np.all(np.diff(b.astype(np.int64)) >= 0)
        shard_bytes = off[b[1:]] - off[b[:-1]]
        assert shard_bytes.max() - shard_bytes.min() <= 2 * 300
        # each cut is the lower bound of its byte quantile
        for i in range(1, g):
            target = off[-1] * i // g
            assert off[b[i]] >= target and (b[i] == 0 or off[b[i] - 1] < target)


def test_shard_bounds_degenerate():
    off = np.zeros(11, dtype=np.uint64)  # ten empty keys
    np.testing.assert_array_equal(t.shard_bounds(off, 4), [0, 2, 5, 7, 10])
    off = np.array([0], dtype=np.uint64)  # no keys
    np.testing.assert_array_equal(t.shard_bounds(off, 3), [0, 0, 0, 0])


def test_synth_host_is_shard_invariant():
    spec = t.SynthSpec.zipf(2)
    kb, ob = t.synth_host(spec, 0, 5000)
    k2, o2 = t.synth_host(spec, 1234, 1000)
    np.testing.assert_array_equal(np.diff(o2), np.diff(ob)[1234:2234])
    np.testing.assert_array_equal(k2[: int(o2[-1])], kb[int(ob[1234]): int(ob[2234])])
    lens = np.diff(ob)
    assert lens.min() >= 8 and lens.max() <= 64
    assert 17.0 < lens.mean() < 22.0  # mean ~19.3 B
    kp, op = t.synth_host(t.SynthSpec.fixed(5, 40, t.BYTES_PRINTABLE), 0, 100)
    body = kp[: int(op[-1])]
    assert body.min() >= 0x21 and body.max() <= 0x7E


def test_synth_rejects_bad_spec():
    with pytest.raises(t.NcError):
        t.synth_host(t.SynthSpec(1, 1, 8, 200), 0, 10)  # zipf range > 64
    with pytest.raises(t.NcError):
        t.synth_host(t.SynthSpec(1, 7, 8, 8), 0, 10)  # unknown distribution


@pytest.mark.skipif(t.device_count() > 0, reason="checks the no-GPU failure mode")
def test_batched_path_fails_loudly_without_gpu():
    keys, off = t.pack_keys([b"apple"])
    with pytest.raises(t.NcError) as ei:
        t.hash_batch_host("fnv1a_64", keys, off)
    assert ei.value.errno == errno.ENODEV
    with pytest.raises(t.NcError):
        t.Context()
    rc = L.lib().nc_gpuhash_batch_device(99, None, None, 1, None, None)
    assert rc == L.NC_ERROR and ctypes.get_errno() == errno.EINVAL


def test_auto_policy_choices():
    """Shape-driven pipeline choice (host logic): md5 always on
    the direct per-lane block pipeline (its LDS-DMA line image from 64-byte
    keys); the byte-serial modes on the direct pipeline for long keys (the
    fnvs in eight-wave workgroups) and the crcs for fixed short keys (tiles
    interleaved over the grid, 32 per wave, for both; crc32 / crc32a and
    one_at_a_time on fixed 20-32 B keys through the eight-wave short-key
    kernel); the register-staged workgroup pipeline when the
    shape is unknown; oversubscribed workgroup grids (and length grouping) for
    varying lengths; the wave ring for fixed 20-40 B fnv-like keys; the
    grouped workgroup pipeline (one length quartile per wave) on C2-like
    shapes."""
    WG, RS, RING5, RING4 = 1 << 16, 32, 128 | (3 << 8), 128
    SORTED, OVER = 1 << 17, 1 << 18
    DIRECT, DIRECT_LDS, IL32 = 1 << 19, 4 << 20, (8 | 2) << 20
    GSORT, CS, TK512, ISSUE = 1 << 25, 1 << 27, 1 << 26, 1 << 28
    n = 1 << 26
    assert t.pick_variant("fnv1a_64", n) == RS
    PADTAB = 1 << 15  # md5: padding selectors from the LDS table
    FULL = 1 << 12  # md5: whole-line output stores (round 6)
    assert t.pick_variant("md5", n) == DIRECT | PADTAB | FULL  # unknown shape
    # C2 (Zipf 8-64 B, mean 19.3)
    for name in ("fnv1a_64", "fnv1_64", "fnv1_32", "fnv1a_32"):  # six resident sets
        assert t.pick_variant(name, n, (19 * n, 8, 64)) == GSORT | CS | TK512, name
    assert t.pick_variant("murmur", n, (19 * n, 8, 64)) == GSORT | CS | TK512 | (2 << 21)  # three
    for name in ("crc16", "hsieh", "jenkins"):
        assert t.pick_variant(name, n, (19 * n, 8, 64)) == GSORT | CS, name
    assert t.pick_variant("crc32", n, (19 * n, 8, 64)) == WG | OVER
    assert t.pick_variant("one_at_a_time", n, (19 * n, 8, 64)) == GSORT | CS | TK512 | ISSUE
    assert t.pick_variant("one_at_a_time", n, (21 * n, 8, 64)) == GSORT | CS | TK512 | ISSUE
    assert t.pick_variant("md5", n, (19 * n, 8, 64)) == DIRECT | PADTAB | FULL
    # uniform 8-64 B (mean 36)
    assert t.pick_variant("fnv1a_64", n, (36 * n, 8, 64)) == RS
    assert t.pick_variant("md5", n, (36 * n, 8, 64)) == DIRECT | PADTAB | FULL
    assert t.pick_variant("crc32a", n, (36 * n, 8, 64)) == RS | OVER
    # C3 (fixed 32 B)
    for name in ("fnv1_64", "fnv1a_64", "fnv1_32", "fnv1a_32", "hsieh"):
        assert t.pick_variant(name, n, (32 * n, 32, 32)) == RING5, name
    SHORT = 1 << 11  # the short-key kernel (eight waves per CU); bits 20-21 depth, 22-23 the crc tables
    assert t.pick_variant("crc16", n, (32 * n, 32, 32)) == DIRECT | SHORT | (1 << 12)  # sixteen waves per CU
    assert t.pick_variant("jenkins", n, (32 * n, 32, 32)) == DIRECT | SHORT | (1 << 12)  # sixteen waves (round 6)
    for name in ("crc32", "crc32a"):  # three tiles in flight, slicing-by-8
        assert t.pick_variant(name, n, (32 * n, 32, 32)) == DIRECT | SHORT | (2 << 20) | (1 << 22), name
    assert t.pick_variant("one_at_a_time", n, (32 * n, 32, 32)) == DIRECT | SHORT | (2 << 20)
    assert t.pick_variant("murmur", n, (32 * n, 32, 32)) == DIRECT | SHORT | (1 << 20)  # one tile in flight
    assert t.pick_variant("murmur", n, (36 * n, 36, 36)) == RING5  # longer than 32 B
    assert t.pick_variant("crc32", n, (36 * n, 36, 36)) == DIRECT | IL32  # longer than 32 B
    assert t.pick_variant("jenkins", n, (36 * n, 36, 36)) == RS
    assert t.pick_variant("md5", n, (32 * n, 32, 32)) == DIRECT | PADTAB | FULL
    # short fixed, long keys (C4)
    assert t.pick_variant("fnv1a_64", n, (8 * n, 8, 8)) == WG
    assert t.pick_variant("md5", n, (16 * n, 16, 16)) == DIRECT | PADTAB | FULL
    for name in ("crc32", "one_at_a_time", "crc16"):
        assert t.pick_variant(name, n >> 3, (256 * (n >> 3), 256, 256)) == DIRECT | DIRECT_LDS | IL32, name
    for name in ("fnv1a_64", "fnv1_32"):  # eight-wave workgroups, one per CU, rounds of two lines
        assert t.pick_variant(name, n >> 3, (256 * (n >> 3), 256, 256)) == DIRECT | DIRECT_LDS | IL32 | (1 << 12) | (1 << 10), name
        assert t.pick_variant(name, n >> 3, (128 * (n >> 3), 128, 128)) == DIRECT | DIRECT_LDS | IL32 | (1 << 12), name
    assert t.pick_variant("md5", n >> 3, (256 * (n >> 3), 256, 256)) == DIRECT | DIRECT_LDS | (8 << 20)
    assert t.pick_variant("md5", n >> 3, (128 * (n >> 3), 128, 128)) == DIRECT | DIRECT_LDS | (8 << 20)
    assert t.pick_variant("murmur", n >> 3, (256 * (n >> 3), 256, 256)) == RING4
    assert t.pick_variant("hsieh", 1000, (100000, 100, 100)) == RING5
    assert t.pick_variant("fnv1a_64", 0, (0, 0, 0)) == RS
    assert L.lib().nc_gpuhash_pick_variant(12, n, None) == -1


def test_server_idx_argument_errors():
    """nc_gpuhash_server_idx_device argument checks (no device work): invalid
    mode / DIST_RANDOM / zero servers are EINVAL; an empty batch is NC_OK."""
    f = L.lib().nc_gpuhash_server_idx_device
    for mode, dist, nserver in ((12, 0, 2), (-1, 0, 2), (6, 2, 2), (6, 3, 2), (6, 0, 0)):
        ctypes.set_errno(0)
        assert f(mode, dist, None, None, 5, None, 0, nserver, None, None, None, None) == L.NC_ERROR
        assert ctypes.get_errno() == errno.EINVAL
    assert f(6, 0, None, None, 0, None, 0, 2, None, None, None, None) == L.NC_OK


def test_ketama_build_argument_errors():
    """nc_gpuhash_ketama_build_device host-side checks (no device work)."""
    f = L.lib().nc_gpuhash_ketama_build_device
    names = (ctypes.c_char_p * 2)(b"a:1", b"b:2")
    lens = (ctypes.c_uint32 * 2)(3, 3)
    cnt = ctypes.c_uint32(7)
    ctypes.set_errno(0)
    assert f(names, lens, (ctypes.c_uint32 * 2)(1, 0), None, 2, None, 0, ctypes.byref(cnt), None) == L.NC_ERROR
    assert ctypes.get_errno() == errno.EINVAL
    # every server ejected: an empty continuum, as "no live servers" (nc_ketama.c:111-116)
    dead = (ctypes.c_uint8 * 2)(0, 0)
    assert f(names, lens, (ctypes.c_uint32 * 2)(1, 1), dead, 2, None, 0, ctypes.byref(cnt), None) == L.NC_OK
    assert cnt.value == 0
    # more points than cap: NC_ENOMEM before any device work
    assert f(names, lens, (ctypes.c_uint32 * 2)(1, 1), None, 2, None, 10, ctypes.byref(cnt), None) == L.NC_ENOMEM


def test_mc_parser_argument_errors():
    lib = L.lib()
    for args in ((0, 1, 1), (1, 0, 1), (1, 1, 0), (1 << 31, 1, 1)):
        ctypes.set_errno(0)
        assert not lib.nc_gpuhash_mc_parser_create(*args)
        assert ctypes.get_errno() == errno.EINVAL
    assert lib.nc_gpuhash_mc_parse_device(None, None, 0, None, None, None, None, None, None) == L.NC_ERROR


def test_redis_parser_argument_errors():
    lib = L.lib()
    for args in ((0, 1, 1), (1, 0, 1), (1, 1, 0), (1 << 31, 1, 1), (1, 1 << 31, 1), (1, 1, 1 << 31)):
        ctypes.set_errno(0)
        assert not lib.nc_gpuhash_redis_parser_create(*args)
        assert ctypes.get_errno() == errno.EINVAL
    assert lib.nc_gpuhash_redis_parse_device(None, None, 0, 16336, None, None, None, None, None, None) == L.NC_ERROR


def test_device_entry_points_check_their_arguments():
    """The Python mirror rejects what would fault or misread on the device
    before any call reaches the C ABI (host tensors, wrong dtypes, a key buffer
    without NC_GPUHASH_PAD readable bytes past offsets[-1])."""
    import torch

    keys = torch.zeros(64, dtype=torch.uint8)
    off = torch.tensor([0, 8, 16], dtype=torch.int64)
    with pytest.raises(ValueError, match="CUDA"):
        t.hash_batch_device("fnv1a_64", keys, off)
    with pytest.raises(TypeError):
        t.hash_batch_device("fnv1a_64", keys.int(), off)
    from twemproxy_amd.hashkit import _check_stream

    # 40 bytes of keys cannot hold offsets[-1] = 16 plus NC_GPUHASH_PAD = 32 readable bytes
    with pytest.raises(ValueError, match="NC_GPUHASH_PAD"):
        t.hash_batch_device("fnv1a_64", torch.zeros(40, dtype=torch.uint8), off, key_end=16)
    with pytest.raises(ValueError, match="NC_GPUHASH_PAD"):
        t.server_idx_device("fnv1a_64", "ketama", torch.zeros(47, dtype=torch.uint8), off,
                            torch.zeros((4, 2), dtype=torch.int32), 2, key_end=16)
    with pytest.raises(ValueError, match="CUDA"):  # enough room: then residency is the error
        t.hash_batch_device("fnv1a_64", torch.zeros(48, dtype=torch.uint8), off, key_end=16)
    with pytest.raises(ValueError, match="CUDA"):
        _check_stream(torch.zeros(8, dtype=torch.uint8))
    with pytest.raises(TypeError):
        _check_stream(torch.zeros(8, dtype=torch.int16))


def test_pipe_hash_checks_its_arguments():
    """Pipe.hash's checks (_check_pinned_batch) run before any DMA: a short
    `out`, a key buffer without NC_GPUHASH_PAD, wrong dtypes, too few offsets,
    a missing nkeys beside raw addresses, and unpinned tensors all raise."""
    import torch

    from twemproxy_amd.hashkit import _check_pinned_batch

    keys_np, off_np = t.pack_keys([b"a", b"bb", b"ccc"])
    keys = torch.from_numpy(keys_np)
    off = torch.from_numpy(off_np.astype(np.int64))
    out = torch.empty(3, dtype=torch.int32)
    with pytest.raises(ValueError, match="out holds 2"):
        _check_pinned_batch(keys, off, out[:2], None)
    with pytest.raises(ValueError, match="NC_GPUHASH_PAD"):
        _check_pinned_batch(keys[: 6 + L.NC_GPUHASH_PAD - 1], off, out, None)
    with pytest.raises(TypeError):
        _check_pinned_batch(keys, off.to(torch.int32), out, None)
    with pytest.raises(TypeError):
        _check_pinned_batch(keys.to(torch.int8), off, out, None)
    with pytest.raises(ValueError, match="4 keys need 5"):
        _check_pinned_batch(keys, off, out, 4)
    with pytest.raises(ValueError, match="nkeys is required"):
        _check_pinned_batch(keys, off_np.ctypes.data, out, None)
    with pytest.raises(ValueError, match="contiguous"):
        _check_pinned_batch(keys, off, torch.empty(6, dtype=torch.int32)[::2], None)
    # the raw-address offsets are read to size the key check
    with pytest.raises(ValueError, match="NC_GPUHASH_PAD"):
        _check_pinned_batch(keys[:8], off_np.ctypes.data, out, 3)
    # everything right but the memory is not page-locked (no GPU here to pin it)
    with pytest.raises(ValueError, match="page-locked"):
        _check_pinned_batch(keys, off, out, None)
    # raw addresses alone: the caller's promise, nothing to check
    assert _check_pinned_batch(keys_np.ctypes.data, off_np.ctypes.data, 0, 3) == 3


def test_ring_without_gpu_and_bad_limits():
    """nc_gpuhash_ring_create: EINVAL past its limits (slots, 4095 keys,
    32 KiB of key bytes), ENODEV without a GPU"""
    lib = L.lib()
    for args in ((0, 0, 100, 1000), (0, 4, 4096, 1000), (0, 4, 100, 32769), (0, 4, 0, 1000)):
        assert not lib.nc_gpuhash_ring_create(*args)
        assert ctypes.get_errno() == errno.EINVAL
    if t.device_count() == 0:
        assert not lib.nc_gpuhash_ring_create(0, 4, 100, 1000)
        assert ctypes.get_errno() == errno.ENODEV
