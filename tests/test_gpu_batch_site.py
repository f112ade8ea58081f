"""The batch site of INTEGRATION.md §2 compiled and run: integration/
nc_batch_site.c (msg_backend_hashes_submit / _poll, msg_backend_idx_batch)
built against the reference's own headers together with the reference's
request parsers, message and server code (oracle/Makefile `batch-site`,
oracle/batch_site_driver.c), with every hash_<name> resolved to
libnc_gpuhash.so. Each multi-key request of the fragment fixture is parsed by
the reference's parser into a struct msg of a client connection of a pool the
reference's ketama_update / modula_update built; the batch site's server
indices (one batch-ring batch per request, polled as the event loop would)
must equal msg_backend_idx per key (the fragment loops' call,
src/proto/nc_memcache.c:1326, src/proto/nc_redis.c:2876) and the indices the
pure reference build's memcache_fragment / redis_fragment produced
(tests/golden/proto_ref.json "fragments", every case)."""
import ctypes
import json
import os

import numpy as np
import pytest

import twemproxy_amd as t
from tests import proto_ref as P

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(HERE, "oracle", "_ref", "libbatch_site.so")
GOLDEN = os.path.join(HERE, "tests", "golden")

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

with open(os.path.join(GOLDEN, "proto_ref.json")) as f:
    DOC = json.load(f)


@pytest.fixture(scope="module")
def bs():
    if not os.path.exists(LIB):
        pytest.fail("oracle/_ref/libbatch_site.so is not built (make -C oracle batch-site, where /root/reference exists)")
    t.lib()  # libnc_gpuhash.so first: the batch site links against the same copy
    lib = ctypes.CDLL(LIB, mode=os.RTLD_LAZY)  # yaml / stats stay unresolved: never reached
    lib.rp_init.restype = ctypes.c_int
    lib.bs_request.restype = ctypes.c_int
    lib.bs_request.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p,
                               ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint32)]
    lib.bs_forget_probe.restype = ctypes.c_int
    lib.bs_forget_probe.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                    ctypes.c_void_p, ctypes.c_uint32]
    lib.bs_pipeline.restype = ctypes.c_int
    lib.bs_pipeline.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_uint32, ctypes.c_void_p]
    assert lib.rp_init() == DOC["mbuf_data_size"]
    return lib


@pytest.mark.parametrize("redis", [False, True], ids=["memcache", "redis"])
def test_batch_site_matches_fragment_loops(gpu, bs, dist_fixture, redis):
    reqs, _, _ = P.frag_requests(DOC, redis)
    kcap = 4096
    ref_idx = np.empty(kcap, np.uint32)
    got_idx = np.empty(kcap, np.uint32)
    polls = ctypes.c_uint32(0)
    nb, hk = ctypes.c_uint32(0), ctypes.c_uint32(0)
    checked = 0
    with t.Ring(0, nslots=4) as ring:
        for case in DOC["fragments"]["cases"]:
            pool = dist_fixture["pools"][case["pool"]]
            names = [n.encode() for n in pool["names"]]
            nserver = int(case["nserver"])
            assert nserver == len(names)
            c_names = (ctypes.c_char_p * nserver)(*names)
            c_lens = (ctypes.c_uint32 * nserver)(*[len(n) for n in names])
            c_w = (ctypes.c_uint32 * nserver)(*[int(w) for w in pool["weights"]])
            tag = case["tag"].encode()
            want = case["redis" if redis else "memcache"]
            for r, req in enumerate(reqs):
                n = bs.bs_request(int(redis), req, len(req), case["mode"], case["dist"], c_names, c_lens, c_w, nserver,
                                  tag, len(tag), ring._h, ref_idx.ctypes.data, got_idx.ctypes.data, kcap,
                                  ctypes.byref(polls), ctypes.byref(nb), ctypes.byref(hk))
                label = f"{'redis' if redis else 'memcache'} request {r} mode {case['mode']} dist {case['dist']} tag {tag!r}"
                assert n == len(want[r]["sidx"]), (label, n)
                assert ref_idx[:n].tolist() == want[r]["sidx"], label
                assert got_idx[:n].tolist() == want[r]["sidx"], label
                checked += n
    assert checked > 1000


def _pool(names, weights):
    n = len(names)
    return ((ctypes.c_char_p * n)(*names), (ctypes.c_uint32 * n)(*[len(x) for x in names]),
            (ctypes.c_uint32 * n)(*weights))


NAMES = [f"10.0.{i}.7:11211".encode() for i in range(7)]
WEIGHTS = [1, 2, 1, 3, 1, 1, 2]


def _expected(oracle, mode, dist, tag, keys):
    """server_pool_idx of each key by the oracle (pinned to the reference)"""
    kb = b"".join(keys)
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    if dist == 0:
        vals, idx = oracle.ketama_build(NAMES, WEIGHTS)
    else:
        vals, idx = None, oracle.modula_build(WEIGHTS)
    return oracle.server_idx_batch(mode, dist, vals, idx, len(NAMES), tag,
                                   np.frombuffer(kb, np.uint8) if kb else np.zeros(1, np.uint8), off)


@pytest.mark.parametrize("redis", [False, True], ids=["memcache", "redis"])
def test_batch_site_splits_large_requests(gpu, bs, oracle, redis):
    """a request with more keys or key bytes than one ring batch
    holds is cut into several ring batches (submitted as slots free up), and
    a key longer than a whole batch takes the library's per-key symbol; the
    indices equal the reference's per-key msg_backend_idx and the oracle's
    server_pool_idx"""
    rng = np.random.default_rng(71)
    nkeys = 60 if redis else 90  # the request fits one mbuf
    maxlen = 300 if redis else 250  # memcache caps keys at 250 B (src/proto/nc_memcache.c)
    lens = rng.integers(1, maxlen + 1, size=nkeys)
    keys = [bytes(rng.integers(0x21, 0x7f, size=int(n), dtype=np.uint8)) for n in lens]
    if redis:
        req = b"*%d\r\n$4\r\nmget\r\n" % (nkeys + 1) + b"".join(b"$%d\r\n%s\r\n" % (len(k), k) for k in keys)
    else:
        req = b"get " + b" ".join(keys) + b"\r\n"
    assert len(req) <= DOC["mbuf_data_size"]
    c_names, c_lens, c_w = _pool(NAMES, WEIGHTS)
    ref_idx = np.empty(nkeys, np.uint32)
    got_idx = np.empty(nkeys, np.uint32)
    polls, nb, hk = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_uint32(0)
    with t.Ring(0, nslots=3, max_keys=16, max_key_bytes=128) as ring:
        n = bs.bs_request(int(redis), req, len(req), 6, 0, c_names, c_lens, c_w, len(NAMES), b"", 0, ring._h,
                          ref_idx.ctypes.data, got_idx.ctypes.data, nkeys, ctypes.byref(polls), ctypes.byref(nb),
                          ctypes.byref(hk))
    assert n == nkeys
    want = _expected(oracle, 6, 0, b"", keys)
    assert ref_idx.tolist() == want.tolist()
    assert got_idx.tolist() == want.tolist()
    assert hk.value == int((lens > 128).sum()) > 0
    assert nb.value >= (nkeys - hk.value + 15) // 16 and nb.value > 3  # more batches than ring slots


def test_batch_site_forget_on_teardown(gpu, bs):
    """a msg torn down with its batches in flight forgets them;
    the ring then serves the slots again and never writes into the freed
    msg's hashes"""
    keys = [b"key%03d" % i for i in range(40)]
    req = b"get " + b" ".join(keys) + b"\r\n"
    c_names, c_lens, c_w = _pool(NAMES, WEIGHTS)
    with t.Ring(0, nslots=2, max_keys=16) as ring:
        rc = bs.bs_forget_probe(0, req, len(req), 6, 0, c_names, c_lens, c_w, len(NAMES), ring._h, 6)
    assert rc == 1


def _c5_streams(rng, redis, nconn, nreq, tag, multi_every=0):
    """per connection, nreq pipelined gets of Zipf 8-64 B printable keys
    (SURVEY.md §8d C5); every multi_every-th request a 3-key get/mget.
    Returns (stream bytes, per-connection offsets, per-connection list of
    (nkeys, key 0))"""
    ranks = np.arange(8, 65)
    p = 1.0 / (ranks - 7.0)
    p /= p.sum()
    out, soff, meta = [], [0], []
    for c in range(nconn):
        parts, reqs = [], []
        for r in range(nreq):
            nk = 3 if multi_every and r % multi_every == multi_every - 1 else 1
            ks = []
            for _ in range(nk):
                k = bytearray(rng.integers(0x21, 0x7f, size=int(rng.choice(ranks, p=p)), dtype=np.uint8))
                if tag and rng.random() < 0.3:  # a hash tag inside the key
                    i = int(rng.integers(0, len(k) - 3))
                    k[i], k[i + 3] = tag[0], tag[1]
                ks.append(bytes(k))
            if redis:
                cmd = b"get" if nk == 1 else b"mget"
                parts.append(b"*%d\r\n$%d\r\n%s\r\n" % (nk + 1, len(cmd), cmd) +
                             b"".join(b"$%d\r\n%s\r\n" % (len(k), k) for k in ks))
            else:
                parts.append(b"get " + b" ".join(ks) + b"\r\n")
            reqs.append((nk, ks[0]))
        s = b"".join(parts)
        out.append(s)
        soff.append(soff[-1] + len(s))
        meta.append(reqs)
    return b"".join(out), np.array(soff, np.uint64), meta


@pytest.mark.parametrize("redis", [False, True], ids=["memcache", "redis"])
@pytest.mark.parametrize("mode,dist,tag,read_bytes,multi", [
    (6, 0, b"", 16336, 0),        # C5: fnv1a_64 ketama, one mbuf per read
    (1, 1, b"{}", 1000, 7),       # md5 modula with a hash tag, short reads (repairs), multi-key requests between
])
def test_pipelined_single_key_site(gpu, bs, oracle, redis, mode, dist, tag, read_bytes, multi):
    """the pipelined single-key batch site compiled
    against the reference. 64 connections x 128 pipelined gets are read in
    mbuf-sized reads and parsed by the reference's own parser and split /
    repair steps; each request's forward is deferred into its connection's
    read batch, one ring batch per read, and forwarded in parse order once
    the batch is done. Every request's server index must equal the
    reference's per-message server_pool_idx (taken at parse time) and the
    oracle's; the per-connection forward order must be the parse order."""
    rng = np.random.default_rng(72 + mode + int(redis))
    nconn, nreq = 64, 128
    stream, soff, meta = _c5_streams(rng, redis, nconn, nreq, tag, multi)
    sbuf = np.frombuffer(stream, np.uint8).copy()
    c_names, c_lens, c_w = _pool(NAMES, WEIGHTS)
    cap = nconn * nreq
    o = {k: np.full(cap, 0xFFFFFFFF, np.uint32) for k in ("conn", "seq", "single", "idx", "ref")}
    stats = np.zeros(4, np.uint64)
    with t.Ring(0, nslots=16) as ring:
        n = bs.bs_pipeline(int(redis), sbuf.ctypes.data, soff.ctypes.data, nconn, read_bytes, mode, dist, c_names,
                           c_lens, c_w, len(NAMES), tag, len(tag), ring._h, o["conn"].ctypes.data,
                           o["seq"].ctypes.data, o["single"].ctypes.data, o["idx"].ctypes.data, o["ref"].ctypes.data,
                           cap, stats.ctypes.data)
        launches = ring.launches
    assert n == cap, n
    want = _expected(oracle, mode, dist, tag, [k for reqs in meta for _, k in reqs]).reshape(nconn, nreq)
    single = np.array([[nk == 1 for nk, _ in reqs] for reqs in meta])
    for c in range(nconn):
        sel = o["conn"][:n] == c
        seq = o["seq"][:n][sel]
        assert seq.tolist() == list(range(nreq)), c  # forwarded in parse order
        np.testing.assert_array_equal(o["ref"][:n][sel], want[c])
        np.testing.assert_array_equal(o["idx"][:n][sel], want[c])
        np.testing.assert_array_equal(o["single"][:n][sel].astype(bool), single[c])
    reads, batches = int(stats[0]), int(stats[1])
    assert reads >= nconn and batches >= reads // 2 and launches >= 1
