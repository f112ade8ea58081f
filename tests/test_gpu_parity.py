"""Bit-exact parity of the gfx950 kernels (through the C ABI) with the reference
hashkit: golden KATs/corpus/full-size digests from the compiled reference, the
CPU oracle on the same seeded inputs, and size-independent properties at the
BASELINE.json sizes. All u32 outputs must match exactly."""
import hashlib

import numpy as np
import pytest

import twemproxy_amd as t
from twemproxy_amd import _lib as L

pytestmark = pytest.mark.gpu

MODES = list(range(12))


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def to_dev(keys: np.ndarray, off: np.ndarray, shift: int = 0):
    """Upload a padded key buffer (optionally `shift` bytes into the allocation)."""
    import torch

    buf = torch.zeros(keys.size + shift + 64, dtype=torch.uint8, device="cuda")
    buf[shift: shift + keys.size] = torch.from_numpy(keys).cuda()
    return buf[shift:], torch.from_numpy(off.astype(np.int64)).cuda()


def gpu_hash(mode, keys_d, off_d):
    out = t.hash_batch_device(mode, keys_d, off_d)
    import torch

    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


@pytest.fixture(params=[(0, 1, 0), (0, 0, 0), (0, 0, 65536), (37, 1, 1), (0, 0, 1), (5, 1, 65536),
                        (0, 0, 1 << 17), (0, 0, 32), (0, 1, 32), (11, 1, 33), (9, 0, 32), (0, 0, 64), (0, 1, 64),
                        (0, 0, 96), (7, 1, 96), (0, 0, 128), (37, 0, 129), (0, 0, 384), (5, 0, 640),
                        (0, 0, 896), (0, 0, 192), (0, 0, 2432 | 4096), (3, 0, 3968 | 4096), (0, 0, 2176),
                        (0, 0, 10624), (0, 0, 16512), (7, 0, 16512 | 2048 | 768), (0, 0, 16512 | 1792),
                        (0, 0, 65536 | (1 << 18)), (0, 1, 32 | (1 << 18)), (0, 0, 1 << 19),
                        (0, 0, (1 << 19) | (4 << 20)), (0, 0, (1 << 19) | (10 << 20)),
                        (0, 0, (1 << 19) | (14 << 20)), (0, 0, 1 << 24), (0, 0, (1 << 24) | (9 << 20)),
                        (0, 0, 1 << 25), (37, 0, 1 << 25), (0, 0, (1 << 25) | (1 << 21)),
                        (0, 0, (1 << 25) | (1 << 23)), (11, 0, (1 << 25) | (1 << 23) | (2 << 21)),
                        (0, 0, (1 << 25) | (1 << 27)), (0, 0, (1 << 25) | (1 << 27) | (1 << 26)),
                        (13, 0, (1 << 25) | (1 << 27) | (1 << 26))],
                ids=["persistent+sort", "auto", "workgroup", "grid37+sort+shiftadd", "shiftadd", "grid5+sort",
                     "sorted_bit", "regstage", "regstage+sort", "grid11+regstage+sort+shiftadd", "grid9+regstage",
                     "cached", "cached+sort", "regstage+cached", "grid7+regstage+cached+sort", "wavering",
                     "grid37+wavering+shiftadd", "wavering_4_1_2", "grid5+wavering_4_3_5", "wavering_5_2_3",
                     "wavering+cached", "wavering_w4_pair", "grid3+wavering_3_1_2_w4_pair", "wavering_w4",
                     "wavering_t64_w4", "wavering_t256_sorted", "grid7+wavering_t256_sorted_w4_6_2_3",
                     "wavering_t256_sorted_5_1_2", "workgroup_over3", "regstage+sort+over3", "direct",
                     "direct_lines", "direct_il32", "direct_lines_il32", "wsort", "wsort_il4",
                     "gsort", "grid37+gsort", "gsort_1set", "gsort_d3", "grid11+gsort_d3_3sets", "gsort_cs", "gsort512",
                     "grid13+gsort512"])
def tuning(request):
    grid, sort, var = request.param
    L.lib().nc_gpuhash_set_tuning(grid, sort, var)
    yield request.param
    L.lib().nc_gpuhash_set_tuning(0, 0, 0)


def test_kats(gpu, kat):
    keys, off = t.pack_keys([b"apple"])
    kd, od = to_dev(keys, off)
    for m, name in enumerate(t.HASH_NAMES):
        assert int(gpu_hash(m, kd, od)[0]) == kat["apple"][name], name
    pattern = bytes(((i * 131 + 7) & 0xFF) for i in range(512))
    lens = sorted(int(n) for n in kat["pattern_table"])
    keys, off = t.pack_keys([pattern[:n] for n in lens])
    kd, od = to_dev(keys, off)
    for m in MODES:
        got = gpu_hash(m, kd, od)
        want = [kat["pattern_table"][str(n)][m] for n in lens]
        assert got.tolist() == want, t.HASH_NAMES[m]


def test_golden_corpus(gpu, corpus, tuning):
    keys, off, expected = corpus
    kd, od = to_dev(keys, off)
    for m in MODES:
        np.testing.assert_array_equal(gpu_hash(m, kd, od), expected[m], err_msg=t.HASH_NAMES[m])


@pytest.mark.parametrize("shift", [1, 3, 5, 7, 9, 15])
def test_misaligned_key_buffer(gpu, corpus, shift):
    keys, off, expected = corpus
    kd, od = to_dev(keys, off, shift)
    for m in MODES:
        np.testing.assert_array_equal(gpu_hash(m, kd, od), expected[m], err_msg=f"{t.HASH_NAMES[m]} shift {shift}")


@pytest.mark.parametrize("var", [0, 128])
def test_offsets_not_starting_at_zero(gpu, oracle, corpus, var):
    keys, off, expected = corpus
    kd, od = to_dev(keys, off)
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        # absolute offsets into the same key buffer; lo = 101 leaves the offsets
        # pointer 8-byte aligned only (the wave ring then hands over)
        for lo, hi in ((100, 700), (101, 1000), (0, 1)):
            sub = od[lo: hi + 1]
            for m in MODES:
                np.testing.assert_array_equal(gpu_hash(m, kd, sub), expected[m][lo:hi])
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


def test_edge_batches(gpu, oracle):
    import torch

    # empty batch: no launch, no error
    kd, od = to_dev(np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    out = torch.empty(0, dtype=torch.int32, device="cuda")
    t.hash_batch_device("fnv1a_64", kd, od, out)
    # all-empty keys, a single key, one key of every byte value
    for keyset in ([b""] * 1000, [b"\xff"], [bytes([b]) for b in range(256)], [bytes(range(256)) * 3]):
        keys, off = t.pack_keys(keyset)
        kd, od = to_dev(keys, off)
        for m in MODES:
            want = [oracle.hash(m, k) for k in keyset]
            assert gpu_hash(m, kd, od).tolist() == want, t.HASH_NAMES[m]


def test_ragged_tile_boundaries(gpu, oracle):
    # batch sizes around the 256-key tile, lengths crossing 4/8/12/16/64 boundaries
    rng = np.random.default_rng(7)
    for n in (1, 255, 256, 257, 511, 513, 4097):
        keyset = [rng.integers(0, 256, size=int(rng.choice([0, 1, 3, 4, 7, 8, 12, 13, 55, 56, 63, 64, 65, 129])),
                               dtype=np.uint8).tobytes() for _ in range(n)]
        keys, off = t.pack_keys(keyset)
        kd, od = to_dev(keys, off)
        for m in MODES:
            np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off), err_msg=f"n={n}")


@pytest.mark.parametrize("lo,hi,n", [(0, 2000, 3000), (4000, 16336, 300)])
def test_long_keys_global_path(gpu, oracle, tuning, lo, hi, n):
    """Slabs beyond the LDS budget take the global-memory reader; 16,336 B is the
    largest redis key in a default 16 KiB mbuf (src/nc_mbuf.c:271)."""
    keys, off = t.synth_host(t.SynthSpec.uniform(11, lo, hi), 0, n)
    kd, od = to_dev(keys, off)
    for m in MODES:
        np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off), err_msg=t.HASH_NAMES[m])


@pytest.mark.parametrize("spec", [t.SynthSpec.fixed(21, 8), t.SynthSpec.fixed(22, 16), t.SynthSpec.fixed(23, 32),
                                  t.SynthSpec.fixed(24, 40), t.SynthSpec.fixed(25, 64), t.SynthSpec.fixed(26, 128),
                                  t.SynthSpec.fixed(27, 256), t.SynthSpec.zipf(28), t.SynthSpec.uniform(29, 8, 64),
                                  t.SynthSpec.uniform(30, 60, 300), t.SynthSpec.uniform(31, 0, 3)],
                         ids=lambda s: f"d{s.len_dist}_{s.len_a}_{s.len_b}")
def test_auto_policy_by_shape(gpu, oracle, spec):
    """Every pipeline the shape-driven policy can pick, against the oracle, with
    ragged last tiles; the same keys without a shape agree too."""
    for n in (4099, 70001):
        keys, off = t.synth_host(spec, 5, n)
        kd, od = to_dev(keys, off)
        shape = t.shape_of(off)
        for m in MODES:
            want = oracle.batch(m, keys, off)
            got = t.hash_batch_device(m, kd, od, shape=shape)
            import torch

            torch.cuda.synchronize()
            np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want,
                                          err_msg=f"{t.HASH_NAMES[m]} var {t.pick_variant(m, n, shape)}")
            np.testing.assert_array_equal(gpu_hash(m, kd, od), want, err_msg=t.HASH_NAMES[m])


def test_synth_device_matches_host(gpu):
    for spec in (t.SynthSpec.zipf(2), t.SynthSpec.fixed(3, 32), t.SynthSpec.uniform(6, 0, 600),
                 t.SynthSpec.zipf(5, charset=t.BYTES_PRINTABLE)):
        kh, oh = t.synth_host(spec, 777, 20000)
        kd, od = t.synth_device(spec, 777, 20000)
        np.testing.assert_array_equal(od.cpu().numpy().astype(np.uint64), oh)
        np.testing.assert_array_equal(kd.cpu().numpy()[: int(oh[-1])], kh[: int(oh[-1])])


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3", "C5", "UNI_0_600", "C4_prefix_2^20"])
def test_full_size_digests(gpu, digests, cfg):
    """Full BASELINE.json sizes (C2/C3: 2^26 keys) generated on the device and
    compared with the reference's own output digests."""
    import torch

    d = digests[cfg]
    spec = t.SynthSpec(**d["spec"])
    kd, od = t.synth_device(spec, 0, d["nkeys"])
    assert int(od[-1].item()) == d["key_bytes"]
    assert sha(od.cpu().numpy().astype(np.uint64)) == d["sha256_offsets"]
    out = torch.empty(d["nkeys"], dtype=torch.int32, device="cuda")
    for name, want in d["modes"].items():
        # with the shape the generator knows: the auto policy's pipeline at full size
        t.hash_batch_device(name, kd, od, out, shape=spec.shape(d["key_bytes"]))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert got[:8].tolist() == want["head"], f"{cfg} {name}"
        assert sha(got) == want["sha256"], f"{cfg} {name}"
    del kd, od, out
    torch.cuda.empty_cache()


def test_c4_shape_slices_are_independent(gpu, oracle):
    """C4 shape (256-B keys): any sub-range hashed as its own batch gives the
    same values as inside the full batch, and sampled keys match the oracle."""
    import torch

    spec = t.SynthSpec.fixed(4, 256)
    n = 1 << 22  # 1 GiB of keys
    kd, od = t.synth_device(spec, 0, n)
    rng = np.random.default_rng(3)
    for name in ("md5", "crc32"):
        full = t.hash_batch_device(name, kd, od, shape=spec.shape(256 * n))
        torch.cuda.synchronize()
        fh = full.cpu().numpy().view(np.uint32)
        for _ in range(4):
            a = int(rng.integers(0, n - 5000))
            b = a + int(rng.integers(1, 5000))
            part = t.hash_batch_device(name, kd, od[a: b + 1].contiguous())
            torch.cuda.synchronize()
            np.testing.assert_array_equal(part.cpu().numpy().view(np.uint32), fh[a:b])
        idx = rng.integers(0, n, size=512)
        keys, off = t.synth_host(spec, 0, 1)  # layout check only
        for i in idx:
            kh, oh = t.synth_host(spec, int(i), 1)
            assert int(fh[i]) == oracle.hash(t.HASH_NAMES.index(name), kh[: int(oh[-1])].tobytes())
    del kd, od
    torch.cuda.empty_cache()


def test_sort_and_grid_variants_agree_full_size(gpu):
    """Length-class sorting and grid-stride walking are permutations of the work
    only: every variant must produce identical outputs on C2 (Zipf)."""
    import torch

    kd, od = t.synth_device(t.CONFIGS["C2"]["spec"], 0, 1 << 24)
    ref = None
    for grid, sort, var in ((0, 1, 0), (0, 0, 0), (2048, 1, 1), (4096, 0, 1), (1, 0, 0), (0, 0, 65536),
                            (0, 1, 65536), (3, 1, 1), (0, 0, 1 << 17), (7, 0, 2176), (0, 0, 32), (0, 1, 32), (5, 1, 33), (13, 1, 32), (1024, 0, 32),
                            (1536, 0, 32), (2048, 1, 32), (0, 0, 64), (0, 1, 64), (0, 0, 96), (1536, 1, 96),
                            (0, 0, 128), (1, 0, 128), (7, 0, 384), (0, 0, 640), (2048, 0, 896), (0, 0, 129),
                            (0, 0, 192), (0, 0, 1 << 24), (0, 0, (1 << 24) | (2 << 20)), (0, 0, (1 << 24) | (8 << 20)),
                            (0, 0, 1 << 25), (1, 0, 1 << 25), (4096, 0, 1 << 25), (0, 0, (1 << 25) | (3 << 21)),
                            (0, 0, (1 << 25) | (1 << 23)), (1, 0, (1 << 25) | (1 << 23)),
                            (777, 0, (1 << 25) | (1 << 23)), (0, 0, (1 << 25) | (1 << 27)),
                            (0, 0, (1 << 25) | (1 << 23) | (1 << 27)), (0, 0, (1 << 25) | (1 << 27) | (1 << 26)),
                            (1, 0, (1 << 25) | (1 << 27) | (1 << 26))):
        L.lib().nc_gpuhash_set_tuning(grid, sort, var)
        out = t.hash_batch_device("fnv1a_64", kd, od)
        torch.cuda.synchronize()
        h = sha(out.cpu().numpy())
        ref = ref or h
        assert h == ref, (grid, sort, var)
    L.lib().nc_gpuhash_set_tuning(0, 0, 0)


def test_key_buffers_beyond_4gib(gpu):
    """4.25 GiB of 256-B keys (offsets past 2^31 and 2^32; C4's shard is 8 GiB):
    every pipeline and the fused server_idx, sampled keys around both marks
    against the per-key host symbols. (A signed readfirstlane once sign-
    extended the ring's tile bounds past 2 GiB.)"""
    import torch

    spec = t.SynthSpec.fixed(4, 256)
    n = (1 << 24) + (1 << 20)
    kd, od = t.synth_device(spec, 0, n)
    rng = np.random.default_rng(5)
    sample = sorted({0, n - 1} | {(1 << 23) + d for d in (-1, 0, 1)} | {(1 << 24) + d for d in (-1, 0, 1)} |
                    {int(x) for x in rng.integers(0, n, size=24)})
    host = {i: t.synth_host(spec, i, 1)[0][:256].tobytes() for i in sample}
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    try:
        for var in (0, 65536, 32, 128, 896, 2176, 1 << 19, (1 << 19) | (4 << 20), (1 << 19) | (14 << 20),
                    (1 << 19) | (8 << 20), 1 << 24, 1 << 25, (1 << 19) | (14 << 20) | (1 << 12) | (1 << 10)):
            L.lib().nc_gpuhash_set_tuning(0, 0, var)
            for name in ("md5", "crc32", "fnv1a_64"):
                t.hash_batch_device(name, kd, od, out, shape=spec.shape(256 * n))
                torch.cuda.synchronize()
                h = out.cpu().numpy().view(np.uint32)
                for i in sample:
                    assert int(h[i]) == t.hash_key(name, host[i]), (var, name, i)
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)
    cont = t.continuum_device(np.arange(8, dtype=np.uint32) % 4, np.arange(8, dtype=np.uint32) << 29)
    for shape in (None, spec.shape(256 * n)):
        got = t.server_idx_device("fnv1a_64", "ketama", kd, od, cont, 4, shape=shape)
        torch.cuda.synchronize()
        g = got.cpu().numpy().view(np.uint32)
        vals = np.arange(8, dtype=np.uint32) << 29
        for i in sample:
            hv = t.hash_key("fnv1a_64", host[i])
            p = int(np.searchsorted(vals, hv, side="left")) % 8
            assert int(g[i]) == p % 4, (shape, i)
    del kd, od, out
    torch.cuda.empty_cache()


def test_short_keys_beyond_4gib(gpu):
    """4.25 GiB of 32-byte keys (offsets past 2^31 and 2^32) through the
    short-key kernel as the policy picks it (crc32, crc16, one_at_a_time,
    murmur) and with its other shapes: sampled keys around both marks against
    the per-key host symbols."""
    import torch

    spec = t.SynthSpec.fixed(6, 32)
    n = (1 << 27) + (1 << 23)
    kd, od = t.synth_device(spec, 0, n)
    rng = np.random.default_rng(6)
    sample = sorted({0, n - 1} | {(1 << 26) + d for d in (-1, 0, 1)} | {(1 << 27) + d for d in (-1, 0, 1)} |
                    {int(x) for x in rng.integers(0, n, size=24)})
    host = {i: t.synth_host(spec, i, 1)[0][:32].tobytes() for i in sample}
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    short = (1 << 19) | (1 << 11)
    try:
        for var in (0, short, short | (1 << 20) | (1 << 22), short | (2 << 20) | (2 << 22), short | (1 << 12)):
            L.lib().nc_gpuhash_set_tuning(0, 0, var)
            for name in ("crc32", "crc16", "one_at_a_time", "murmur", "jenkins"):
                t.hash_batch_device(name, kd, od, out, shape=spec.shape(32 * n))
                torch.cuda.synchronize()
                h = out.cpu().numpy().view(np.uint32)
                for i in sample:
                    assert int(h[i]) == t.hash_key(name, host[i]), (var, name, i)
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)
    del kd, od, out
    torch.cuda.empty_cache()


def test_c4_full_shard(gpu, digests):
    """One GPU's whole C4 shard (BASELINE configs[3]: keys [0, 2^25) of the
    2^28 x 256 B set, 8 GiB, offsets past 2^31, 2^32 and 2^33): md5 and crc32
    (the C4 modes) and fnv1a_64 through the auto policy (the direct line-image
    pipelines) and the direct register path; the first 2^20 hashes against
    the reference's digest of the C4 prefix, sampled keys around every 2 GiB
    mark and at random against the per-key host symbols."""
    import torch

    d = digests["C4_prefix_2^20"]
    spec = t.SynthSpec(**d["spec"])
    n = 1 << 25
    kd, od = t.synth_device(spec, 0, n)
    assert int(od[-1].item()) == 256 * n
    rng = np.random.default_rng(25)
    marks = [(1 << 23) * j for j in range(1, 5)]  # 2, 4, 6, 8 GiB
    sample = sorted({0, n - 1} | {m + e for m in marks for e in (-1, 0, 1) if 0 <= m + e < n} |
                    {int(x) for x in rng.integers(0, n, size=64)})
    host = {i: t.synth_host(spec, i, 1)[0][:256].tobytes() for i in sample}
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    try:
        for var in (0, 1 << 19):
            L.lib().nc_gpuhash_set_tuning(0, 0, var)
            for name in ("md5", "crc32", "fnv1a_64"):
                out.fill_(0)
                t.hash_batch_device(name, kd, od, out, shape=spec.shape(256 * n))
                torch.cuda.synchronize()
                h = out.cpu().numpy().view(np.uint32)
                if name in d["modes"]:
                    assert h[:8].tolist() == d["modes"][name]["head"], (var, name)
                    assert sha(h[: d["nkeys"]]) == d["modes"][name]["sha256"], (var, name)
                for i in sample:
                    assert int(h[i]) == t.hash_key(name, host[i]), (var, name, i)
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)
    del kd, od, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("var", [16512, 16512 | 2048 | 768, 16512 | 1792, 128, 2176, 10624, 32896, 32896 | 2048])
def test_wave_ring_ragged_tiles(gpu, oracle, var):
    """Wave-ring shapes (incl. 256-key length-sorted rounds) on batch sizes
    around their 64/128/256-key tiles, Zipf keys, misaligned key buffer,
    against the oracle (fnv1a_64 and md5 take every shape, the other modes the
    plain ring)."""
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        for n in (1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 513, 1025, 4097):
            keys, off = t.synth_host(t.SynthSpec.zipf(60 + n % 7), 3, n)
            kd, od = to_dev(keys, off, shift=5)
            for m in (1, 6, 3, 10, 2, 4):
                np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off),
                                              err_msg=f"var={var} n={n} mode={m}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("var", [128 | 2048, 128 | 2048 | (1 << 12), 128 | 2048 | (2 << 12), 128 | 2048 | (3 << 12)],
                         ids=["p5x7", "p5x6", "p5x4", "p4x8"])
def test_wave_ring_crc_sliced(gpu, oracle, var):
    """crc16 / crc32 / crc32a on the wave ring with slicing-by-16 tables shared
    by the workgroup's waves (variant bit 11, bits 12-13 the ring), on ragged
    batch sizes, fixed 32-byte keys (C3's shape), Zipf and uniform lengths
    (every tail length; tiles too long for a slab slot take the global-memory
    reader), misaligned key buffers, against the oracle."""
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        for n, spec in ((1, t.SynthSpec.uniform(70, 0, 40)), (129, t.SynthSpec.fixed(71, 32)),
                        (4097, t.SynthSpec.fixed(72, 32)), (1025, t.SynthSpec.zipf(73)),
                        (3000, t.SynthSpec.uniform(74, 0, 40)), (2000, t.SynthSpec.uniform(75, 0, 300)),
                        (777, t.SynthSpec.fixed(76, 17)), (513, t.SynthSpec.fixed(77, 2))):
            keys, off = t.synth_host(spec, 3, n)
            for shift in (0, 9):
                kd, od = to_dev(keys, off, shift=shift)
                for m in (2, 3, 4):
                    np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off),
                                                  err_msg=f"var={var} n={n} spec={spec} mode={m} shift={shift}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("depth_bits,slice_bits,w16", [(0, 0, 0), (1, 1, 0), (2, 2, 0), (0, 3, 0), (0, 0, 1), (2, 1, 1)],
                         ids=["ahead2-s4", "ahead1-s8", "ahead3-s16", "ahead2-s4r32", "ahead2-s4-w16", "ahead3-s8-w16"])
def test_direct_short_keys(gpu, oracle, depth_bits, slice_bits, w16):
    """The short-key kernel (variant bit 11 with the direct
    pipeline: keys of at most 16 or 32 bytes by the caller's shape, eight
    waves per CU on a persistent grid, 1-3 tiles in flight per wave) on
    ragged batch sizes (fewer tiles than waves, a partial last tile) and
    misaligned buffers, and with a shape that understates the longest key
    (from that tile on, the slow loop from global memory), against the
    oracle, for the byte modes and the word modes (hsieh, murmur, jenkins).
    The crcs by slicing-by-4, -8 and -16 tables (variant bits 22-23;
    by-4 also in 32 copies); eight or sixteen waves per CU (bit 12)."""
    var = (1 << 19) | (1 << 11) | (depth_bits << 20) | (slice_bits << 22) | (w16 << 12)
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    import torch

    try:
        cases = [(1, t.SynthSpec.fixed(80, 32), None), (65, t.SynthSpec.fixed(81, 32), None),
                 (70001, t.SynthSpec.fixed(82, 32), None), (4097, t.SynthSpec.fixed(83, 16), None),
                 (3001, t.SynthSpec.fixed(84, 17), None), (5000, t.SynthSpec.uniform(85, 0, 32), None),
                 (2049, t.SynthSpec.uniform(86, 0, 16), None), (1 << 20, t.SynthSpec.fixed(89, 32), None),
                 (9000, t.SynthSpec.uniform(87, 0, 100), 32),  # the shape says <= 32: wrong for many tiles
                 (300000, t.SynthSpec.uniform(90, 0, 40), 32),  # wrong in a few tiles of a long batch
                 (3000, t.SynthSpec.uniform(88, 10, 40), 16)]  # says <= 16
        for n, spec, claim in cases:
            keys, off = t.synth_host(spec, 3, n)
            lens = np.diff(off)
            hi = int(lens.max()) if claim is None else claim
            for shift in (0, 7):
                kd, od = to_dev(keys, off, shift=shift)
                for m in (0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11):
                    got = t.hash_batch_device(m, kd, od, shape=(int(off[-1]), int(lens.min()), hi))
                    torch.cuda.synchronize()
                    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), oracle.batch(m, keys, off),
                                                  err_msg=f"var={var} n={n} spec={spec} claim={claim} mode={m}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("var", [1 << 19, (1 << 19) | (4 << 20), (1 << 19) | (8 << 20), (1 << 19) | (10 << 20),
                                 (1 << 19) | (11 << 20), (1 << 19) | (14 << 20), (1 << 19) | (9 << 20),
                                 (1 << 19) | (14 << 20) | (1 << 12), (1 << 19) | (10 << 20) | (1 << 13),
                                 (1 << 19) | (14 << 20) | (1 << 13), (1 << 19) | (1 << 13), (1 << 19) | (1 << 15),
                                 (1 << 19) | (8 << 20) | (1 << 15), (1 << 19) | (14 << 20) | (1 << 12) | (1 << 10)],
                         ids=["direct", "lines", "il16", "il32", "il64", "lines_il32", "il8", "lines_il32_w8",
                              "il32_s8", "lines_il32_s8", "direct_s8", "direct_padtab", "il16_padtab",
                              "pairs_il32_w8"])
def test_direct_ragged_tiles(gpu, oracle, var):
    """The direct per-lane pipelines (md5 and the byte-serial modes; the other
    modes take their default pipeline), consecutive or grid-interleaved tiles
    per wave, the byte modes' eight-wave line-image workgroups (bit 12), the
    crcs' slicing-by-8 tables (bit 13), md5's LDS padding selectors (bit 15),
    the eight-wave line image in rounds of two lines (bit 10), on
    batch sizes around the 64-key tile and the per-workgroup tile
    count, with empty keys, one-block, multi-block and padding-only-block keys,
    a misaligned key buffer, against the oracle."""
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        for n, spec in ((1, t.SynthSpec.uniform(40, 0, 3)), (63, t.SynthSpec.zipf(41)), (64, t.SynthSpec.fixed(42, 32)),
                        (65, t.SynthSpec.uniform(43, 0, 300)), (129, t.SynthSpec.uniform(44, 50, 70)),
                        (4097, t.SynthSpec.zipf(45)), (70001, t.SynthSpec.uniform(46, 0, 200)),
                        (70001, t.SynthSpec.fixed(47, 256)), (4097, t.SynthSpec.fixed(48, 16)),
                        (70001, t.SynthSpec.fixed(49, 32)), (3000, t.SynthSpec.uniform(50, 0, 16)),
                        (5000, t.SynthSpec.fixed(51, 20)), (4096, t.SynthSpec.fixed(52, 28))):
            keys, off = t.synth_host(spec, 3, n)
            kd, od = to_dev(keys, off, shift=3)
            for m in MODES:
                np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off),
                                              err_msg=f"var={var} n={n} spec={spec} mode={t.HASH_NAMES[m]}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("var", [1 << 24, (1 << 24) | (1 << 20), (1 << 24) | (2 << 20), (1 << 24) | (3 << 20),
                                 (1 << 24) | (8 << 20), (1 << 24) | (11 << 20)],
                         ids=["wsort8", "wsort4", "wsort16", "wsort32", "wsort8_il", "wsort32_il"])
def test_wsort_ragged_tiles(gpu, oracle, var):
    """The wave-sorted pipeline (fnv x4 and one_at_a_time; the other modes take
    their default pipeline) on batch sizes around its 256-key tile and the
    per-wave tile count, with empty keys, Zipf and uniform lengths, tiles that
    overflow the 6 KiB slab (the global fallback, alone and mixed with slab
    tiles), a misaligned key buffer, against the oracle."""
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        for n, spec in ((1, t.SynthSpec.uniform(50, 0, 3)), (63, t.SynthSpec.zipf(51)), (255, t.SynthSpec.zipf(52)),
                        (256, t.SynthSpec.fixed(53, 24)), (257, t.SynthSpec.uniform(54, 0, 64)),
                        (1023, t.SynthSpec.uniform(55, 0, 48)), (4097, t.SynthSpec.zipf(56)),
                        (9000, t.SynthSpec.uniform(57, 0, 60)), (70001, t.SynthSpec.zipf(58)),
                        (3000, t.SynthSpec.uniform(59, 0, 300)), (2049, t.SynthSpec.fixed(60, 25)),
                        (600, t.SynthSpec.uniform(61, 0, 2000))):
            keys, off = t.synth_host(spec, 3, n)
            kd, od = to_dev(keys, off, shift=7)
            for m in MODES:
                np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off),
                                              err_msg=f"var={var} n={n} spec={spec} mode={t.HASH_NAMES[m]}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("var", [0, (1 << 19) | (1 << 15) | (1 << 12), (1 << 19) | (1 << 15) | (1 << 12) | (1 << 14)],
                         ids=["policy", "fullline_s64", "fullline_generic"])
def test_md5_short_key_form(gpu, oracle, var):
    """md5's S64 form (round 6: the caller's shape says no key exceeds 64
    bytes, so every key is one data block and the rounds keep no chaining
    state) on ragged batches of Zipf / uniform keys with empty keys, 55- to
    64-byte keys (their tail blocks) and a misaligned buffer; and with shapes
    that understate the longest key (a wave meeting a longer key leaves the
    fast loop and runs the generic rounds from that tile: early in short
    batches, late in a long one), against the oracle. Bit 14 turns the form
    off (the generic rounds on the same shapes)."""
    import torch

    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        cases = [(1, t.SynthSpec.zipf(70), None), (63, t.SynthSpec.zipf(71), None), (64, t.SynthSpec.zipf(72), None),
                 (65, t.SynthSpec.uniform(73, 0, 64), None), (4097, t.SynthSpec.zipf(74), None),
                 (70001, t.SynthSpec.uniform(75, 50, 64), None), (70001, t.SynthSpec.zipf(76), None),
                 (9000, t.SynthSpec.uniform(77, 0, 100), 64),   # the shape says <= 64: wrong in most tiles
                 (300000, t.SynthSpec.uniform(78, 0, 66), 64),  # wrong in a few tiles of a long batch
                 (5000, t.SynthSpec.uniform(79, 60, 200), 64)]  # wrong from the first tile
        for n, spec, claim in cases:
            keys, off = t.synth_host(spec, 3, n)
            lens = np.diff(off)
            hi = int(lens.max()) if claim is None else claim
            for shift in (0, 5):
                kd, od = to_dev(keys, off, shift=shift)
                got = t.hash_batch_device(1, kd, od, shape=(int(off[-1]), int(lens.min()), hi))
                torch.cuda.synchronize()
                np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), oracle.batch(1, keys, off),
                                              err_msg=f"var={var} n={n} spec={spec} claim={claim} shift={shift}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("fl", [16, 20, 24, 32, 40, 48])
def test_md5_fixed_length_specialisation(gpu, oracle, fl):
    """md5's fixed-length instantiations (picked by a shape whose min == max)
    on batches around the 64-key tile, misaligned, and with the shape
    claiming fixed lengths while some tiles hold other lengths (each tile
    checks its keys and takes the generic path), against the oracle; the
    generic path (variant bit 26) on the same keys."""
    rng = np.random.default_rng(fl)
    for n in (1, 63, 64, 65, 1000, 4097):
        keys, off = t.synth_host(t.SynthSpec.fixed(70 + fl, fl), 3, n)
        lens = np.full(n, fl)
        if n >= 64:  # a few odd lengths in a few tiles
            for i in rng.choice(n, size=3, replace=False):
                lens[i] = int(rng.integers(0, 120))
            blob = keys[: off[-1]].tobytes()
            parts, pos = [], 0
            for ln in lens:
                parts.append((blob * 3)[pos: pos + int(ln)])
                pos += fl
            keys, off = t.pack_keys(parts)
        kd, od = to_dev(keys, off, shift=5)
        want = oracle.batch(1, keys, off)
        for var in (0, (1 << 19) | (1 << 26), (1 << 19) | (1 << 15)):
            L.lib().nc_gpuhash_set_tuning(0, 0, var)
            try:
                got = t.hash_batch_device("md5", kd, od, shape=(int(off[-1]), fl, fl))
                import torch

                torch.cuda.synchronize()
                np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want,
                                              err_msg=f"fl={fl} n={n} var={var}")
            finally:
                L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("var", [1 << 24, (1 << 24) | (1 << 20)], ids=["wsort8", "wsort4"])
def test_wsort_round_of_long_keys(gpu, oracle, var):
    """A sorted round made only of class-63 keys (63+ bytes, unordered within
    the class): tiles of 192 short keys plus 64 keys of 63-90 bytes, which
    fit the 6 KiB slab, so the fourth round's shortest key is not at lane 0
    (Lmin must be a wave minimum there), against the oracle."""
    rng = np.random.default_rng(63)
    parts = []
    for _ in range(48):  # 48 tiles of 256 keys
        lens = np.concatenate([rng.integers(0, 8, size=192), rng.integers(63, 91, size=64)])
        rng.shuffle(lens)
        parts += [rng.integers(0, 256, size=int(ln), dtype=np.uint8).tobytes() for ln in lens]
    keys, off = t.pack_keys(parts)
    kd, od = to_dev(keys, off, shift=9)
    L.lib().nc_gpuhash_set_tuning(0, 0, var)
    try:
        for m in (0, 5, 6, 7, 8):
            np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off),
                                          err_msg=f"var={var} mode={t.HASH_NAMES[m]}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("tune", [(0, 1 << 25), (0, (1 << 25) | (1 << 21)), (3, 1 << 25), (1, (1 << 25) | (3 << 21)),
                                  (0, (1 << 25) | (1 << 23)), (2, (1 << 25) | (1 << 23)),
                                  (0, (1 << 25) | (1 << 23) | (1 << 21)), (0, (1 << 25) | (1 << 27)),
                                  (5, (1 << 25) | (1 << 23) | (1 << 27)), (0, (1 << 25) | (1 << 27) | (1 << 26)),
                                  (2, (1 << 25) | (1 << 27) | (1 << 26) | (1 << 21))],
                         ids=["gsort6", "gsort1", "grid3", "grid1_8sets", "d3", "d3_grid2", "d3_1set", "cs", "d3_cs_grid5",
                              "tk512", "tk512_grid2"])
def test_gsort_ragged_tiles(gpu, oracle, tune):
    """The grouped workgroup pipeline (variant bit 25: offsets by LDS-DMA two
    tiles ahead, wave 0 sorting the next tile, each wave one length quartile)
    on batch sizes around its 256-key tile, empty keys, Zipf / uniform /
    fixed lengths, tiles whose slab overflows its 6 KiB buffer (the global
    path, alone and mixed), a misaligned key buffer and offsets not starting
    at 0, every mode, against the oracle."""
    grid, var = tune
    L.lib().nc_gpuhash_set_tuning(grid, 0, var)
    try:
        for n, spec in ((1, t.SynthSpec.uniform(80, 0, 3)), (2, t.SynthSpec.fixed(81, 0)), (63, t.SynthSpec.zipf(82)),
                        (255, t.SynthSpec.zipf(83)), (256, t.SynthSpec.fixed(84, 24)),
                        (257, t.SynthSpec.uniform(85, 0, 64)), (513, t.SynthSpec.zipf(86)),
                        (4097, t.SynthSpec.zipf(87)), (9000, t.SynthSpec.uniform(88, 0, 60)),
                        (70001, t.SynthSpec.zipf(89)), (3000, t.SynthSpec.uniform(90, 0, 300)),
                        (600, t.SynthSpec.uniform(91, 0, 2000)), (2049, t.SynthSpec.fixed(92, 25))):
            keys, off = t.synth_host(spec, 3, n)
            kd, od = to_dev(keys, off, shift=5)
            for m in MODES:
                np.testing.assert_array_equal(gpu_hash(m, kd, od), oracle.batch(m, keys, off),
                                              err_msg=f"tune={tune} n={n} spec={spec} mode={t.HASH_NAMES[m]}")
            if n > 1:  # a sub-batch whose offsets do not start at 0
                kd2, od2 = kd, od[1:].contiguous()
                np.testing.assert_array_equal(gpu_hash(6, kd2, od2), oracle.batch(6, keys, off)[1:],
                                              err_msg=f"tune={tune} n={n} offset base")
                import torch  # an output buffer that is only 4-byte aligned

                ob = torch.zeros(n + 1, dtype=torch.int32, device="cuda")
                t.hash_batch_device(6, kd, od, out=ob[1:])
                torch.cuda.synchronize()
                np.testing.assert_array_equal(ob[1:].cpu().numpy().view(np.uint32), oracle.batch(6, keys, off),
                                              err_msg=f"tune={tune} n={n} misaligned out")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


def test_virtual_key_base(gpu, oracle):
    """A batch whose offsets start far from 0 and whose key pointer is
    therefore not itself readable (keys - offsets[0] of a chunk of a larger
    CSR, as nc_gpuhash_batch_pinned hands its chunks to the kernels): every
    pipeline must only touch bytes inside [keys + offsets[0], keys +
    offsets[n] + NC_GPUHASH_PAD). The base is moved 1 TiB below the buffer."""
    import ctypes

    import torch

    shift = 1 << 40
    for n, spec in ((3000, t.SynthSpec.uniform(93, 0, 700)), (5000, t.SynthSpec.zipf(94)),
                    (4096, t.SynthSpec.fixed(95, 32)), (300, t.SynthSpec.fixed(96, 256))):
        keys, off = t.synth_host(spec, 0, n)
        kd = torch.from_numpy(keys).cuda()
        od = torch.from_numpy(off.astype(np.int64) + shift).cuda()
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        shape = L.NcShape(int(off[-1]), *spec.len_range())
        for var in (0, 65536, 32, 128, 896, 1 << 19, (1 << 19) | (4 << 20), (1 << 19) | (14 << 20), 1 << 24,
                    1 << 25, (1 << 25) | (1 << 23), (1 << 25) | (1 << 27), (1 << 25) | (1 << 27) | (1 << 26)):
            L.lib().nc_gpuhash_set_tuning(0, 0, var)
            try:
                for m in MODES:
                    L.check(L.lib().nc_gpuhash_batch_device_shaped(m, kd.data_ptr() - shift, od.data_ptr(), n,
                                                                  out.data_ptr(), ctypes.byref(shape), None),
                            "nc_gpuhash_batch_device_shaped")
                    torch.cuda.synchronize()
                    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), oracle.batch(m, keys, off),
                                                  err_msg=f"var={var} n={n} mode={t.HASH_NAMES[m]}")
            finally:
                L.lib().nc_gpuhash_set_tuning(0, 0, 0)
