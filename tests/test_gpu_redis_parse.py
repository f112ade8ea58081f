"""Key extraction on the device for redis:
nc_gpuhash_redis_parse_device against the oracle's sequential restatement of
redis_parse_req (oracle_redis_parse; src/proto/nc_redis.c:460-1900) on the
reference's own request vectors (tests/golden/redis_req_cases.json, from
src/test_all.c:109-230), its failure rules, and random binary-safe pipelines
whose values hold false request starts; then the extracted CSR through the
hash kernels."""
import json
import os

import numpy as np
import pytest

import twemproxy_amd as t
from tests import redis_gen as G

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def dev(b: bytes):
    import torch

    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda() if b else \
        torch.zeros(0, dtype=torch.uint8, device="cuda")


def check(parser, oracle, stream: bytes):
    import torch

    keys, off, kreq, status, info = parser.parse(dev(stream))
    torch.cuda.synchronize()
    ks, kl, kr, st, oi = oracle.redis_parse(stream, max_key_len=parser.max_key_len)
    assert info["nreqs"] == oi["nparsed"], (info, oi)
    assert info["first_error"] == oi["first_error"], (info, oi)
    assert info["consumed"] == oi["consumed"]
    assert info["nkeys"] == oi["nkeys"]
    np.testing.assert_array_equal(status.cpu().numpy(), st)
    o = off.cpu().numpy()
    assert o[0] == 0 and len(o) == info["nkeys"] + 1
    kb = keys.cpu().numpy()
    want = [stream[int(a): int(a) + int(n)] for a, n in zip(ks, kl)]
    got = [kb[o[i]: o[i + 1]].tobytes() for i in range(len(o) - 1)]
    assert got == want
    np.testing.assert_array_equal(kreq.cpu().numpy().astype(np.uint32), kr)
    return keys, off, info


@pytest.fixture(scope="module")
def parser():
    p = t.RedisParser(max_bytes=1 << 24, max_reqs=1 << 20, max_keys=1 << 20)
    yield p
    p.close()


def golden():
    return [c["req"].encode("latin-1") for c in
            json.load(open(os.path.join(HERE, "golden", "redis_req_cases.json")))["cases"]]


def test_reference_vectors_one_by_one(gpu, oracle, parser):
    n_ok = 0
    for b in golden():
        _, _, info = check(parser, oracle, b)
        n_ok += info["nkeys"] > 0
    assert n_ok >= 60


def test_reference_vectors_pipelined(gpu, oracle, parser):
    """all of test_all.c's requests back to back: the first unsupported one stops the device parse"""
    cases = golden()
    supported = [b for b in cases if oracle.redis_parse(b)[3].tolist() == [0]]
    _, _, info = check(parser, oracle, b"".join(supported))
    assert info["nreqs"] == len(supported) and info["consumed"] == sum(map(len, supported))
    check(parser, oracle, b"".join(cases))


@pytest.mark.parametrize("stream", [
    b"",
    b"*2\r\n$3\r\nget\r\n$1\r\na\r\n",
    b"*2\r\n$3\r\nget\r\n$0\r\n\r\n",
    b"*2\r\n$3\r\nget\r\n$\r\n\r\n",
    b"*2\r\n$3\r\nget\r\n$1\r\na",
    b"*2\r\n$3\r\nget\r\n$1\r\na\r\n*2\r\n$3\r\nget",
    b"+2\r\n",
    b"*0\r\n",
    b"*2\r\n$0\r\n\r\n",
    b"*1\r\n$3\r\nget\r\n",
    b"*3\r\n$3\r\nget\r\n$1\r\na\r\n$1\r\nb\r\n",
    b"*2\r\n$6\r\nappend\r\n$1\r\na\r\n",
    b"*3\r\n$6\r\nappend\r\n$1\r\na\r\n$\r\n\r\n",
    b"*4\r\n$4\r\nmset\r\n$1\r\na\r\n$1\r\n1\r\n$1\r\nb\r\n",
    b"*2\r\n$3\r\nget\r\n$2\r\na\r\n",
    b"*2\r\n$3\r\nget\r\n$16336\r\n",
    b"*2\r\n$3\r\nget\r\n$16335\r\n" + b"k" * 16335 + b"\r\n",   # longest key below mbuf_data_size
    b"*2\r\n$3\r\ngex\r\n$1\r\na\r\n",
    b"*2\r\n$3\r\nget\r\n$1\r\na\r\nxyz",
    b"*2\r\n$3\r\nget\r\n$1\r\na\r\n$2\r\nzz\r\n",                  # next "request" starts with '$'
    b"*2\r\n$3\r\nGeT\r\n$3\r\n\r\n*\r\n*2\r\n$4\r\nMGET\r\n$1\r\n*\r\n",  # CR LF '*' inside keys
    b"*3\r\n$3\r\ndel\r\n$1\r\na\r\n$1\r\nb\r\n*5\r\n$4\r\nmset\r\n$1\r\nk\r\n$1\r\nv\r\n$1\r\nj\r\n$0\r\n\r\n",
])
def test_failure_rules(gpu, oracle, parser, stream):
    check(parser, oracle, stream)


@pytest.mark.parametrize("seed", range(6))
def test_random_pipelines(gpu, oracle, parser, seed):
    """binary-safe pipelines (values hold "\\r\\n*2\\r"), cut at a random byte
    for even seeds, a byte corrupted for odd ones"""
    rng = np.random.default_rng(100 + seed)
    b, reqs = G.stream(rng, 4000)
    if seed % 2 == 0:
        b = b[: int(rng.integers(len(b) // 2, len(b)))]
    else:
        b = bytearray(b)
        b[int(rng.integers(len(b) // 4, len(b)))] ^= 0x5A
        b = bytes(b)
    _, _, info = check(parser, oracle, b)
    assert info["nkeys"] > 0


def test_large_pipeline(gpu, oracle, parser):
    """~13 MiB, 100k requests: 20+ pointer-jumping rounds"""
    rng = np.random.default_rng(7)
    b, reqs = G.stream(rng, 100_000)
    assert len(b) < (1 << 24)
    _, _, info = check(parser, oracle, b)
    assert info["nreqs"] == len(reqs) and info["consumed"] == len(b)


def test_limits(gpu, oracle):
    import torch

    with t.RedisParser(max_bytes=64, max_reqs=4, max_keys=4) as p:
        with pytest.raises(t.NcError):
            p.parse(dev(b"*2\r\n$3\r\nget\r\n$1\r\na\r\n" * 4))  # 80 B > max_bytes
        with pytest.raises(t.NcError):
            p.parse(dev(b"*6\r\n$3\r\ndel\r\n$1\r\na\r\n$1\r\nb\r\n$1\r\nc\r\n$1\r\nd\r\n$1\r\ne\r\n"))  # 5 keys
        _, off, _, _, info = p.parse(dev(b"*3\r\n$3\r\ndel\r\n$1\r\na\r\n$1\r\nb\r\n"))
        torch.cuda.synchronize()
        assert info["nkeys"] == 2 and off.cpu().tolist() == [0, 1, 2]
    # exactly max_reqs ok requests, then a byte that starts no request: the
    # synthetic failing request does not count against max_reqs
    get = b"*2\r\n$3\r\nget\r\n$1\r\na\r\n"
    with t.RedisParser(max_bytes=256, max_reqs=4, max_keys=4) as p:
        _, off, _, status, info = p.parse(dev(get * 4 + b"x"))
        torch.cuda.synchronize()
        assert info["nkeys"] == 4 and info["first_error"] == 4 and info["nreqs"] == 5, info
        assert info["consumed"] == 4 * len(get)
        # the failing request has a status slot too (max_reqs + 1 entries)
        assert len(status) == info["nreqs"]
        assert status.cpu().tolist() == [0, 0, 0, 0, -1]  # NC_GPUHASH_REDIS_EINVAL
        _, _, _, oi = oracle.redis_parse(get * 4 + b"x")[1:]
        assert (oi["nkeys"], oi["first_error"], oi["consumed"]) == (4, 4, 4 * len(get)), oi


def test_extracted_keys_hash_like_the_host(gpu, oracle, parser):
    """parse -> fnv1a_64 / md5 / murmur on the extracted CSR == per-key host hash_t"""
    import torch

    rng = np.random.default_rng(3)
    b, reqs = G.stream(rng, 3000)
    keys = [k for a in reqs for k in G.keys_of(a)]
    kd, od, info = check(parser, oracle, b)
    assert info["nkeys"] == len(keys)
    for name in ("fnv1a_64", "md5", "murmur"):
        h = t.hash_batch_device(name, kd, od)
        torch.cuda.synchronize()
        assert h.cpu().numpy().view(np.uint32).tolist() == [t.hash_key(name, k) for k in keys], name
