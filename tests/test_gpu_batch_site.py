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
                               ctypes.POINTER(ctypes.c_uint32)]
    assert lib.rp_init() == DOC["mbuf_data_size"]
    return lib


@pytest.mark.parametrize("redis", [False, True], ids=["memcache", "redis"])
def test_batch_site_matches_fragment_loops(gpu, bs, dist_fixture, redis):
    reqs, _, _ = P.frag_requests(DOC, redis)
    kcap = 4096
    ref_idx = np.empty(kcap, np.uint32)
    got_idx = np.empty(kcap, np.uint32)
    polls = ctypes.c_uint32(0)
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
                                  ctypes.byref(polls))
                label = f"{'redis' if redis else 'memcache'} request {r} mode {case['mode']} dist {case['dist']} tag {tag!r}"
                assert n == len(want[r]["sidx"]), (label, n)
                assert ref_idx[:n].tolist() == want[r]["sidx"], label
                assert got_idx[:n].tolist() == want[r]["sidx"], label
                checked += n
    assert checked > 1000
