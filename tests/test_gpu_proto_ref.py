"""The device key-extraction parsers and the fused server_pool_idx against
fixtures the COMPILED reference produced (tests/golden/proto_ref.json, from
redis_parse_req / memcache_parse_req / server_pool_idx built from
/root/reference's sources by tools/gen_proto_golden.py): same requests
accepted, same keys per request, same stopping point, same server index with
hash_tag."""
import numpy as np
import pytest

import twemproxy_amd as t
from tests import proto_ref as P

pytestmark = pytest.mark.gpu

DOC = P.load()


def dev(b: bytes):
    import torch

    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda() if b else \
        torch.zeros(0, dtype=torch.uint8, device="cuda")


def run(parser, e):
    import torch

    stream = P.stream_of(e)
    keys, off, kreq, status, info = parser.parse(dev(stream))
    torch.cuda.synchronize()
    o = off.cpu().numpy()
    kb = keys.cpu().numpy()
    key_bytes = [kb[o[i]: o[i + 1]].tobytes() for i in range(len(o) - 1)]
    P.check(e, info["nreqs"], info["first_error"], info["consumed"], status.cpu().numpy(), None, None,
            kreq.cpu().numpy(), key_bytes=key_bytes)
    return info


def test_redis_parser_matches_reference(gpu):
    with t.RedisParser(max_bytes=1 << 22, max_reqs=1 << 16, max_keys=1 << 16,
                       max_key_len=DOC["mbuf_data_size"]) as p:
        nk = sum(run(p, e)["nkeys"] for e in DOC["redis"])
    assert nk > 1000


def test_mc_parser_matches_reference(gpu):
    with t.McParser(max_bytes=1 << 22, max_reqs=1 << 16, max_keys=1 << 16) as p:
        nk = sum(run(p, e)["nkeys"] for e in DOC["memcache"])
    assert nk > 1000


@pytest.mark.parametrize("pipe", [0, 1 << 28, 1 << 29], ids=["policy", "ring", "workgroup"])
@pytest.mark.parametrize("wide", [False, True], ids=["narrow", "wide"])
def test_server_idx_matches_reference(gpu, dist_fixture, wide, pipe):
    import torch

    from twemproxy_amd import _lib as L

    keys, off = t.pack_keys(P.keys_of(DOC))
    buf = torch.zeros(keys.size + 64, dtype=torch.uint8, device="cuda")
    buf[: keys.size] = torch.from_numpy(keys).cuda()
    od = torch.from_numpy(off.astype(np.int64)).cuda()
    shape = (21 * (off.size - 1), 0, 64) if wide else None
    L.lib().nc_gpuhash_set_tuning(0, 0, pipe)  # bit 28: wave ring, bit 29: workgroup pipeline
    try:
        for c, p, vals, idx in P.server_idx_cases(DOC, dist_fixture):
            cd = t.continuum_device(idx, vals) if vals is not None else t.continuum_device(idx)
            dist = t.DIST_NAMES[c["dist"]]
            got = t.server_idx_device(c["mode"], dist, buf, od, cd, len(p["names"]),
                                      hash_tag=c["tag"].encode() or None, shape=shape)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), np.array(c["idx"], np.uint32),
                                          err_msg=f"mode {c['mode']} {dist} tag {c['tag']!r} pipe {pipe}")
    finally:
        L.lib().nc_gpuhash_set_tuning(0, 0, 0)


@pytest.mark.parametrize("redis", [False, True], ids=["memcache", "redis"])
def test_fragments_on_device_match_reference(gpu, dist_fixture, redis):
    """The batch site on the device: one pipelined stream of multi-key
    requests parsed by the device parser into a key CSR, the fused
    server_pool_idx over all of its keys in ONE launch, then the fragment
    plan (nc_gpuhash_frag_plan) and the fragments' bytes per request, against
    what the reference's own memcache_fragment / redis_fragment made of each
    request (tests/golden/proto_ref.json "fragments", every case)."""
    import torch

    reqs, stream, _ = P.frag_requests(DOC, redis)
    Parser = t.RedisParser if redis else t.McParser
    kw = {"max_key_len": DOC["mbuf_data_size"]} if redis else {}
    with Parser(max_bytes=1 << 20, max_reqs=1 << 12, max_keys=1 << 14, **kw) as p:
        kd, od, kreq, status, info = p.parse(dev(stream))
        torch.cuda.synchronize()
        assert info["first_error"] == len(reqs) and info["consumed"] == len(stream), info
        kr = kreq.cpu().numpy()[: info["nkeys"]]
        o = od.cpu().numpy()
        kb = kd.cpu().numpy()
        kbytes = [kb[o[i]: o[i + 1]].tobytes() for i in range(info["nkeys"])]
        by_req = [np.flatnonzero(kr == r) for r in range(len(reqs))]
        for case in DOC["fragments"]["cases"]:
            vals, idx, nserver = P.frag_pool(case, dist_fixture)
            cd = t.continuum_device(idx, vals) if vals is not None else t.continuum_device(idx)
            got = t.server_idx_device(case["mode"], t.DIST_NAMES[case["dist"]], kd, od, cd, nserver,
                                      hash_tag=case["tag"].encode() or None)
            torch.cuda.synchronize()
            sidx = got.cpu().numpy().view(np.uint32)
            P.check_fragments(case, redis, reqs, [[kbytes[j] for j in sel] for sel in by_req],
                              [sidx[sel] for sel in by_req])
