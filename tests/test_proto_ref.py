"""The oracle's restatements of the key-extraction parsers and of
server_pool_idx against fixtures the COMPILED reference produced
(tests/golden/proto_ref.json: redis_parse_req, memcache_parse_req and
server_pool_idx with hash_tag run from /root/reference's own sources by
tools/gen_proto_golden.py). CPU only; the device paths are checked against
the same fixtures in tests/test_gpu_proto_ref.py."""
import numpy as np
import pytest

from tests import proto_ref as P

DOC = P.load()


@pytest.mark.parametrize("i", range(len(DOC["redis"])))
def test_oracle_redis_parse_matches_reference(oracle, i):
    e = DOC["redis"][i]
    ks, kl, kr, st, info = oracle.redis_parse(P.stream_of(e), max_key_len=DOC["mbuf_data_size"])
    P.check(e, info["nparsed"], info["first_error"], info["consumed"], st, ks, kl, kr)


@pytest.mark.parametrize("i", range(len(DOC["memcache"])))
def test_oracle_mc_parse_matches_reference(oracle, i):
    e = DOC["memcache"][i]
    ks, kl, kr, st, info = oracle.mc_parse(P.stream_of(e))
    P.check(e, info["nparsed"], info["first_error"], info["consumed"], st, ks, kl, kr)


def test_fixture_covers_the_key_classes():
    types = {r["type"] for e in DOC["redis"] for r in e["reqs"] if r["keys"]}
    for ty in ("REQ_REDIS_GET", "REQ_REDIS_MGET", "REQ_REDIS_MSET", "REQ_REDIS_DEL", "REQ_REDIS_EXPIRE",
               "REQ_REDIS_HSET"):
        assert ty in types
    assert sum(len(e["reqs"]) for e in DOC["redis"]) > 1000
    assert {r["result"] for e in DOC["redis"] for r in e["reqs"]} >= {"OK", "ERROR", "AGAIN"}
    assert {r["type"] for e in DOC["memcache"] for r in e["reqs"]} >= {"REQ_MC_GET", "REQ_MC_GETS"}


def test_oracle_server_idx_matches_reference(oracle, dist_fixture):
    import twemproxy_amd as t

    keyset = P.keys_of(DOC)
    keys, off = t.pack_keys(keyset)
    n = 0
    for c, p, vals, idx in P.server_idx_cases(DOC, dist_fixture):
        tag = c["tag"].encode() or None
        got = oracle.server_idx_batch(c["mode"], c["dist"], vals, idx, len(p["names"]), tag, keys, off)
        np.testing.assert_array_equal(got, np.array(c["idx"], np.uint32),
                                      err_msg=f"mode {c['mode']} dist {c['dist']} tag {c['tag']!r}")
        n += 1
    assert n == len(DOC["server_idx"]["cases"]) >= 200


@pytest.mark.parametrize("ci", range(8))
@pytest.mark.parametrize("redis", [False, True], ids=["memcache", "redis"])
def test_fragments_match_reference(oracle, dist_fixture, redis, ci):
    """The batch site end to end on the host: the oracle's parser and
    server_pool_idx over a pipelined stream of multi-key requests, then
    nc_gpuhash_frag_plan and twemproxy_amd.fragment's copies, against what
    the reference's own memcache_fragment / redis_fragment made of each
    request (tests/golden/proto_ref.json "fragments")."""
    import twemproxy_amd as t

    case = DOC["fragments"]["cases"][ci]
    reqs, stream, bounds = P.frag_requests(DOC, redis)
    parse = oracle.redis_parse if redis else oracle.mc_parse
    ks, kl, kr, st, info = parse(stream)
    assert info["first_error"] == len(reqs) and info["consumed"] == len(stream)
    kbytes = [stream[int(s): int(s) + int(n)] for s, n in zip(ks, kl)]
    keys, off = t.pack_keys(kbytes)
    vals, idx, nserver = P.frag_pool(case, dist_fixture)
    sidx = oracle.server_idx_batch(case["mode"], case["dist"], vals, idx, nserver, case["tag"].encode() or None,
                                   keys, off)
    by_req = [np.flatnonzero(kr == r) for r in range(len(reqs))]
    P.check_fragments(case, redis, reqs, [[kbytes[j] for j in sel] for sel in by_req],
                      [sidx[sel] for sel in by_req])


def test_frag_plan_contract():
    from twemproxy_amd.fragment import frag_plan

    seq, srv, cnt = frag_plan([5, 1, 5, 3, 1], 8)
    assert seq.tolist() == [2, 0, 2, 1, 0] and srv.tolist() == [1, 3, 5] and cnt.tolist() == [2, 1, 2]
    seq, srv, cnt = frag_plan([], 4)
    assert seq.size == 0 and srv.size == 0
    import twemproxy_amd as t

    with pytest.raises(t.NcError):
        frag_plan([0, 4], 4)  # a server index >= nserver
