"""Fused server_pool_idx on the device through the C ABI
(nc_gpuhash_server_idx_device), against the oracle's restatement of
server_pool_idx (src/nc_server.c:647-700) over continua the compiled reference
built (tests/golden/dist.json: ketama_update / modula_update output)."""
import numpy as np
import pytest

import twemproxy_amd as t

pytestmark = pytest.mark.gpu

MODES = list(range(12))


def to_dev(keys: np.ndarray, off: np.ndarray, shift: int = 0):
    import torch

    buf = torch.zeros(keys.size + shift + 64, dtype=torch.uint8, device="cuda")
    buf[shift: shift + keys.size] = torch.from_numpy(keys).cuda()
    return buf[shift:], torch.from_numpy(off.astype(np.int64)).cuda()


def tagged_keyset(rng, n):
    """Printable keys, some with {hash tags}: proper, empty {}, unclosed, reversed, repeated."""
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789:_-", dtype=np.uint8)
    out = [b"", b"{}", b"{", b"}", b"}{", b"{a}", b"x{ab}y", b"{{a}}", b"a{b{c}d}e", b"{x}{y}", b"user:{42}:name"]
    while len(out) < n:
        body = rng.choice(alpha, size=int(rng.integers(0, 40))).tobytes()
        r = rng.random()
        if r < 0.4 and len(body) > 2:
            i = int(rng.integers(0, len(body) - 1))
            j = int(rng.integers(i, len(body)))
            body = body[:i] + b"{" + body[i:j] + b"}" + body[j:]
        elif r < 0.5:
            body = body + b"{" + body[:3]
        out.append(body)
    return out


def pools(dist_fixture):
    for p in dist_fixture["pools"]:
        yield p, len(p["names"])


@pytest.mark.parametrize("pipe", [0, 1 << 28, 1 << 29, 1 << 30], ids=["policy", "ring", "workgroup", "grouped"])
@pytest.mark.parametrize("wide", [False, True], ids=["narrow", "wide"])
@pytest.mark.parametrize("tag", [None, b"{}", b"::"], ids=["notag", "braces", "colons"])
def test_server_idx_matches_oracle(gpu, oracle, dist_fixture, tag, wide, pipe):
    import torch

    from twemproxy_amd import _lib as L

    L.lib().nc_gpuhash_set_tuning(0, 0, pipe)  # bit 28: wave ring, bit 29: workgroup pipeline
    try:
        _server_idx_vs_oracle(torch, oracle, dist_fixture, tag, wide)
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


def _server_idx_vs_oracle(torch, oracle, dist_fixture, tag, wide):
    rng = np.random.default_rng(17)
    keyset = tagged_keyset(rng, 5000)
    keys, off = t.pack_keys(keyset)
    kd, od = to_dev(keys, off, shift=3)
    # the shape only picks the ring's slab size: claim 21 B/key for the wide one
    shape = (21 * (off.size - 1), 0, 64) if wide else None
    for p, nserver in pools(dist_fixture):
        kvals = np.array(p["ketama"]["values"], np.uint32)
        kidx = np.array(p["ketama"]["indices"], np.uint32)
        midx = np.array(p["modula"]["indices"], np.uint32)
        conts = {"ketama": (t.continuum_device(kidx, kvals), kvals, kidx),
                 "modula": (t.continuum_device(midx), None, midx)}
        for dist, (cd, vals, idx) in conts.items():
            for m in MODES:
                got = t.server_idx_device(m, dist, kd, od, cd, nserver, hash_tag=tag, shape=shape)
                torch.cuda.synchronize()
                want = oracle.server_idx_batch(m, t.DIST_NAMES.index(dist), vals, idx, nserver, tag, keys, off)
                np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want,
                                              err_msg=f"{dist} {t.HASH_NAMES[m]} nserver={nserver} tag={tag}")


def test_single_server_pool_is_all_zero(gpu):
    import torch

    keys, off = t.pack_keys([b"a", b"bb", b""] * 100)
    kd, od = to_dev(keys, off)
    cd = t.continuum_device(np.zeros(160, np.uint32), np.arange(160, dtype=np.uint32))
    out = torch.full((300,), 7, dtype=torch.int32, device="cuda")
    t.server_idx_device("fnv1a_64", "ketama", kd, od, cd, 1, out=out)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tolist() == [0] * 300


def test_random_dist_is_refused(gpu):
    keys, off = t.pack_keys([b"a"])
    kd, od = to_dev(keys, off)
    cd = t.continuum_device(np.zeros(1, np.uint32))
    with pytest.raises(t.NcError):
        t.server_idx_device("fnv1a_64", "random", kd, od, cd, 2)


def test_large_continuum_two_pass(gpu, oracle):
    """A ketama continuum beyond the LDS budget (300 servers x 160 points x 8 B
    = 375 KiB) takes the hash-then-dispatch pair of launches."""
    import torch

    names = [f"10.0.{i // 250}.{i % 250}:11211".encode() for i in range(300)]
    vals, idx = oracle.ketama_build(names, [1] * len(names))
    assert vals.size * 8 > 160 * 1024
    keys, off = t.synth_host(t.SynthSpec.zipf(5, charset=t.BYTES_PRINTABLE), 0, 50000)
    kd, od = to_dev(keys, off)
    cd = t.continuum_device(idx, vals)
    for m, shape in ((6, None), (1, t.shape_of(off)), (3, (30 * 50000, 0, 64))):
        got = t.server_idx_device(m, "ketama", kd, od, cd, len(names), hash_tag=b"{}", shape=shape)
        torch.cuda.synchronize()
        want = oracle.server_idx_batch(m, 0, vals, idx, len(names), b"{}", keys, off)
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want)


def test_server_idx_full_size_consistent_with_hash(gpu, dist_fixture):
    """C2 shape at 2^24 keys: the fused kernel equals the hash kernel followed
    by ketama_dispatch (a lower bound over the continuum values, wrapping)."""
    import torch

    p = dist_fixture["pools"][1]
    kvals = np.array(p["ketama"]["values"], np.uint32)
    kidx = np.array(p["ketama"]["indices"], np.uint32)
    kd, od = t.synth_device(t.CONFIGS["C2"]["spec"], 0, 1 << 24)
    cd = t.continuum_device(kidx, kvals)
    got = t.server_idx_device("fnv1a_64", "ketama", kd, od, cd, len(p["names"]))
    h = t.hash_batch_device("fnv1a_64", kd, od)
    torch.cuda.synchronize()
    hv = h.cpu().numpy().view(np.uint32)
    pos = np.searchsorted(kvals, hv, side="left")
    pos[pos == kvals.size] = 0
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), kidx[pos])
    midx = np.array(p["modula"]["indices"], np.uint32)
    got = t.server_idx_device("fnv1a_64", "modula", kd, od, t.continuum_device(midx), len(p["names"]))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), midx[hv % midx.size])


def test_ketama_build_matches_reference(gpu, dist_fixture):
    """ketama_update on the device reproduces the continua the compiled
    reference built (values and indices, in order)."""
    for p in dist_fixture["pools"]:
        names = [n.encode() for n in p["names"]]
        cont = t.ketama_build_device(names, p["weights"]).cpu().numpy().view(np.uint32)
        assert cont[:, 1].tolist() == p["ketama"]["values"], p["names"][:2]
        assert cont[:, 0].tolist() == p["ketama"]["indices"], p["names"][:2]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ketama_build_weights_and_ejection(gpu, oracle, seed):
    """Random weights, long and odd names, ejected servers: against the
    oracle's restatement of ketama_update (parity with the reference pinned
    for all-live pools by the test above)."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 40))
    names = [(b"h" * int(rng.integers(1, 300)) if i % 7 == 3 else f"10.1.{i}.{seed}:1121{i % 10}".encode())
             for i in range(n)]
    weights = [int(w) for w in rng.integers(1, 9, size=n)]
    live = [bool(x) for x in rng.random(n) > 0.25]
    live[0] = True
    for lv in (None, live):
        vals, idx = oracle.ketama_build(names, weights, lv)
        cont = t.ketama_build_device(names, weights, lv).cpu().numpy().view(np.uint32)
        np.testing.assert_array_equal(cont[:, 1], vals)
        np.testing.assert_array_equal(cont[:, 0], idx)


def test_device_continuum_end_to_end(gpu, oracle):
    """Continuum built on the device, then the fused server_pool_idx over it."""
    import torch

    names = [f"cache-{i}.example:11211".encode() for i in range(12)]
    weights = [1, 2, 1, 3, 1, 1, 2, 1, 1, 1, 4, 1]
    cd = t.ketama_build_device(names, weights)
    vals, idx = oracle.ketama_build(names, weights)
    keys, off = t.synth_host(t.SynthSpec.zipf(5, charset=t.BYTES_PRINTABLE), 0, 30000)
    kd, od = to_dev(keys, off)
    got = t.server_idx_device("md5", "ketama", kd, od, cd, len(names), hash_tag=b"{}")
    torch.cuda.synchronize()
    want = oracle.server_idx_batch(1, 0, vals, idx, len(names), b"{}", keys, off)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("pipe", [0, 1 << 28, 1 << 29, 1 << 30], ids=["policy", "ring", "workgroup", "grouped"])
@pytest.mark.parametrize("tag", [b"::", b"()", b"$$", b"{}", b"ab", b"\x00\x01"], ids=["colons", "parens", "dollars",
                                                                                      "braces", "ab", "nul01"])
def test_hash_tag_neighbour_bytes(gpu, oracle, dist_fixture, tag, pipe):
    """hash_tag trimming on keys built from the tag bytes and their +-1
    neighbours (c ^ 1 next to c0 / c1: the bytes where a borrowing zero-byte
    test flags a false match, ADVICE r02 — ':;ab:' under '::', ')((x)' under
    '()'), against the oracle's byte loop (src/nc_server.c:665-677)."""
    import torch

    from twemproxy_amd import _lib as L

    c0, c1 = tag[0], tag[1]
    alpha = sorted({c0, c1, c0 ^ 1, c1 ^ 1, (c0 + 1) & 255, (c1 - 1) & 255, ord("a"), ord("x")})
    rng = np.random.default_rng(c0 * 256 + c1)
    keyset = [b":;ab:", b")((x)", b"$%$", b"{|}", b"::", b":;:", b";:;:", b"(()", b"()(x)"]
    keyset += [bytes(rng.choice(alpha, size=int(rng.integers(0, 24))).astype(np.uint8)) for _ in range(6000)]
    keys, off = t.pack_keys(keyset)
    kd, od = to_dev(keys, off, shift=1)
    L.lib().nc_gpuhash_set_tuning(0, 0, pipe)
    try:
        for p, nserver in pools(dist_fixture):
            kvals = np.array(p["ketama"]["values"], np.uint32)
            kidx = np.array(p["ketama"]["indices"], np.uint32)
            cd = t.continuum_device(kidx, kvals)
            for m in (1, 3, 6, 10):
                got = t.server_idx_device(m, "ketama", kd, od, cd, nserver, hash_tag=tag)
                torch.cuda.synchronize()
                want = oracle.server_idx_batch(m, 0, kvals, kidx, nserver, tag, keys, off)
                np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want,
                                              err_msg=f"tag={tag} {t.HASH_NAMES[m]} nserver={nserver}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


def test_ketama_lookup_table(gpu, oracle, dist_fixture):
    """ketama on the grouped pipeline: the continuum staged in LDS with its
    256-bucket index (the policy's choice up to 4,800 points and 256 servers;
    256- and 512-key tiles), the same index over the L2 continuum (bit 25), the 65536- and 4096-entry lookup tables in L2
    (bits 24 / 23, A/B), on batches of 64 Ki keys and more:
    every reference-built pool, a synthetic pool of 300 servers (48,000
    points, past 2^15 and past the LDS budget), one whose points crowd a few
    16-bit ranges, 256 servers (the u8 server bytes' limit) on exactly 4,800
    points and 4,801 points (just past the LDS limit) and on 1,280 / 1,281
    (the packed LDS continuum's limit), points sharing their top 24 bits with
    the keys' hashes (the packed search's full-value fallback), more packed
    pools (skewed, tiny, few or ~128 servers), hash tags, against the
    oracle's server_pool_idx."""
    import torch

    from twemproxy_amd import _lib as L

    spec = t.CONFIGS["C2"]["spec"]
    n = (1 << 17) + 3
    keys, off = t.synth_host(spec, 11, n)
    kd, od = to_dev(keys, off)
    shape = spec.shape(int(off[-1]))
    pools = [(np.array(p["ketama"]["values"], np.uint32), np.array(p["ketama"]["indices"], np.uint32), len(p["names"]))
             for p in dist_fixture["pools"]]
    rng = np.random.default_rng(3)
    big = np.sort(rng.integers(0, 1 << 32, size=48000, dtype=np.uint64)).astype(np.uint32)
    pools.append((big, rng.integers(0, 300, size=big.size).astype(np.uint32), 300))
    crowd = np.sort(np.concatenate([rng.integers(0, 1 << 18, size=700), rng.integers(0xfffc0000, 1 << 32, size=700),
                                    rng.integers(0, 1 << 32, size=40)]).astype(np.uint64)).astype(np.uint32)
    pools.append((crowd, rng.integers(0, 9, size=crowd.size).astype(np.uint32), 9))
    for npts in (4800, 4801, 1280, 1281):
        v = np.sort(rng.integers(0, 1 << 32, size=npts, dtype=np.uint64)).astype(np.uint32)
        pools.append((v, rng.integers(0, 256, size=npts).astype(np.uint32), 256))
    # the packed LDS continuum compares top 24 bits: points that share them
    # with the keys' own hashes (below, at and above the hash, and runs of
    # such points) must resolve on full values
    near = []
    for m in (6, 1, 10):
        h = oracle.batch(m, keys, off)[rng.choice(n, size=100, replace=False)].astype(np.int64)
        near += [h - 1, h, h + 1, (h & ~0xff) | rng.integers(0, 256, size=h.size), (h & ~0xff) | 0xff]
    near = np.unique(np.clip(np.concatenate(near), 0, (1 << 32) - 1)).astype(np.uint32)[:1280]
    pools.append((near, rng.integers(0, 200, size=near.size).astype(np.uint32), 200))
    # more packed continua (<= 1,280 points): server counts around 128, points
    # only in the top 1/256 of the ring, eight points, two servers, a crowd of
    # 700 points in one 2^22 bucket
    for npts, nsrv, lo, hi in ((1280, 100, 0, 1 << 32), (1280, 128, 0, 1 << 32), (1280, 131, 0, 1 << 32),
                               (1200, 9, 0xff000000, 1 << 32), (8, 8, 0, 1 << 32), (1279, 2, 0, 1 << 32)):
        v = np.sort(rng.integers(lo, hi, size=npts, dtype=np.uint64)).astype(np.uint32)
        pools.append((v, rng.integers(0, nsrv, size=npts).astype(np.uint32), nsrv))
    c1280 = np.sort(np.concatenate([rng.integers(0, 1 << 18, size=700), rng.integers(0, 1 << 32, size=580)])
                    .astype(np.uint64)).astype(np.uint32)
    pools.append((c1280, rng.integers(0, 9, size=c1280.size).astype(np.uint32), 9))
    try:
        for vals, idx, nserver in pools:
            cd = t.continuum_device(idx, vals)
            for m in (6, 1, 10):
                for tag in (None, b"{}"):
                    want = oracle.server_idx_batch(m, 0, vals, idx, nserver, tag, keys, off)
                    # grouped + 65536 / 4096 table in L2, grouped + bucket index over the L2 continuum,
                    # grouped + LDS continuum (256 / 512-key tiles), policy
                    # (bit 27: the 5-byte LDS continuum where the packed one fits)
                    for var in ((1 << 30) | (1 << 24), (1 << 30) | (1 << 23), (1 << 30) | (1 << 25),
                                (1 << 30) | (1 << 26), (1 << 30) | (1 << 27), 1 << 30, 0):
                        L.lib().nc_gpuhash_set_tuning(0, 0, var)
                        got = t.server_idx_device(m, "ketama", kd, od, cd, nserver, hash_tag=tag, shape=shape)
                        torch.cuda.synchronize()
                        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want,
                                                      err_msg=f"{t.HASH_NAMES[m]} tag={tag} nserver={nserver} {var}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)



def test_ketama_packed_top_hashes(gpu, oracle):
    """The packed LDS continuum ends in sentinels 0xffffff00 | point 0's
    server: a key whose hash has its top 24 bits all ones stops on a sentinel
    (or on a real point >= 0xffffff00) with the same top 24 bits and must
    resolve on full values — the wrap to point 0 past the last point, or the
    point itself. Keys with such fnv1a_64 hashes are found among 2^26 C2 keys
    on the device (about four), padded with 64 Ki ordinary C2 keys so the
    policy keeps the grouped pipeline; pools of 1,280 points (the packed
    limit) with the last point below those hashes, at them and above them,
    against the oracle's server_pool_idx."""
    import torch

    from twemproxy_amd import _lib as L

    spec = t.CONFIGS["C2"]["spec"]
    kd, od = t.synth_device(spec, 0, 1 << 26)
    h = t.hash_batch_device("fnv1a_64", kd, od).cpu().numpy().view(np.uint32)
    del kd, od
    torch.cuda.empty_cache()
    top = np.flatnonzero(h >= 0xffffff00)
    assert top.size >= 1, "no key of 2^26 hashes to >= 0xffffff00"
    special = []
    for i in top:
        k1, o1 = t.synth_host(spec, int(i), 1)
        special.append(bytes(k1[int(o1[0]):int(o1[1])]))
    hs = h[top].astype(np.int64)
    keys, off = t.synth_host(spec, 7, 1 << 16)
    ordinary = [bytes(keys[off[i]:off[i + 1]]) for i in range(off.size - 1)]
    keyset = ordinary[:30000] + special + ordinary[30000:] + special
    pk, po = t.pack_keys(keyset)
    kd, od = to_dev(pk, po)
    shape = t.shape_of(po)
    assert (oracle.batch(6, pk, po)[30000:30000 + len(special)] >= 0xffffff00).all()
    rng = np.random.default_rng(5)
    base = np.sort(rng.integers(0, 0xff000000, size=1280 - 8, dtype=np.uint64))
    pools = []
    for tail in ([], list(hs - 1), list(hs), list(hs + 1), [0xffffff00, 0xffffffff], [0xffffff00] * 3):
        v = np.sort(np.clip(np.concatenate([base, np.array(tail, np.int64)]), 0, 0xffffffff)).astype(np.uint32)
        pools.append((v, rng.integers(0, 8, size=v.size).astype(np.uint32)))
    try:
        for vals, idx in pools:
            cd = t.continuum_device(idx, vals)
            want = oracle.server_idx_batch(6, 0, vals, idx, 8, None, pk, po)
            for var in (0, 1 << 30, (1 << 30) | (1 << 27)):
                L.lib().nc_gpuhash_set_tuning(0, 0, var)
                got = t.server_idx_device(6, "ketama", kd, od, cd, 8, shape=shape)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want,
                                              err_msg=f"{vals[-3:]} var={var:#x}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)
