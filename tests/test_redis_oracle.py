"""The oracle's restatement of redis_parse_req (oracle_redis_parse) against the
reference's own request vectors (tests/golden/redis_req_cases.json, from
src/test_all.c:109-230 by tools/gen_redis_golden.py) and the reference's
failure rules (src/proto/nc_redis.c, lines cited per case)."""
import json
import os

import numpy as np
import pytest

from tests import redis_gen as G

HERE = os.path.dirname(os.path.abspath(__file__))


def split_resp(b: bytes):
    """args of one well-formed multibulk request (test helper, independent of the oracle)"""
    assert b[:1] == b"*"
    p = b.index(b"\r\n")
    n = int(b[1:p])
    p += 2
    args = []
    for _ in range(n):
        q = b.index(b"\r\n", p)
        ln = int(b[p + 1:q])
        args.append(b[q + 2:q + 2 + ln])
        p = q + 2 + ln + 2
    assert p == len(b)
    return args


CLASS_OF = {**{c: 1 for c in G.ARG0}, **{c: 2 for c in G.ARG1}, **{c: 3 for c in G.ARGN},
            **{c: 4 for c in G.ARGX}, b"mset": 5}


def cases():
    return json.load(open(os.path.join(HERE, "golden", "redis_req_cases.json")))["cases"]


def test_reference_success_vectors(oracle):
    """Every request the reference's tests parse: the oracle accepts those in
    its key classes, with the keys SW_KEY would push, and hands the rest (-3)
    to the host parser."""
    n_ok = 0
    for c in cases():
        b = c["req"].encode("latin-1")
        args = split_resp(b)
        ks, kl, kr, st, info = oracle.redis_parse(b)
        if oracle.redis_class(c["type"].lower().encode()) == 0:
            assert list(st) == [-3], c
            assert info["consumed"] == 0 and info["nkeys"] == 0
            continue
        n_ok += 1
        assert list(st) == [0] and info["consumed"] == len(b), c
        got = [b[int(s): int(s) + int(n)] for s, n in zip(ks, kl)]
        assert got == G.keys_of(args), c
    assert n_ok >= 60


def test_class_table(oracle):
    for name, cls in CLASS_OF.items():
        assert oracle.redis_class(name) == cls
        assert oracle.redis_class(name.upper()) == cls  # str*icmp, src/proto/nc_proto.h:87
    for name in (b"auth", b"ping", b"eval", b"getrange", b"hincrby", b"quit", b"gex"):
        assert oracle.redis_class(name) == 0


@pytest.mark.parametrize("stream,status,nkeys,consumed", [
    (b"", [], 0, 0),
    (b"*2\r\n$3\r\nget\r\n$1\r\na\r\n", [0], 1, 20),
    (b"*2\r\n$3\r\nget\r\n$0\r\n\r\n", [0], 1, 19),            # empty key is a key (SW_KEY :1403-1435)
    (b"*2\r\n$3\r\nget\r\n$\r\n\r\n", [0], 1, 18),             # no digits: rlen 0 (SW_KEY_LEN :1362-1389)
    (b"*2\r\n$3\r\nget\r\n$1\r\na", [], 0, 0),                 # incomplete: left for the next read
    (b"*2\r\n$3\r\nget\r\n$1\r\na\r\n*2\r\n$3\r\nget", [0], 1, 20),
    (b"+2\r\n", [-1], 0, 0),                                   # not an array (:478-483)
    (b"*0\r\n", [-1], 0, 0),                                   # narg 0 (:497-499)
    (b"*2\r\n$0\r\n\r\n", [-1], 0, 0),                         # empty command (:533-535)
    (b"*1\r\n$3\r\nget\r\n", [-1], 0, 0),                      # narg 1 for a keyed command (:1347-1348)
    (b"*3\r\n$3\r\nget\r\n$1\r\na\r\n$1\r\nb\r\n", [-1], 1, 0),  # arg0 with an extra arg (:1441-1443)
    (b"*2\r\n$6\r\nappend\r\n$1\r\na\r\n", [-1], 1, 0),         # arg1 without its arg (:1446-1448)
    (b"*3\r\n$6\r\nappend\r\n$1\r\na\r\n$\r\n\r\n", [-1], 1, 0),  # arg without digits (:1502-1503)
    (b"*4\r\n$4\r\nmset\r\n$1\r\na\r\n$1\r\n1\r\n$1\r\nb\r\n", [-1], 1, 0),  # even narg (:1471-1472)
    (b"*2\r\n$3\r\nget\r\n$2\r\na\r\n", [-1], 0, 0),           # CR not where rlen says (:1415-1416)
    (b"*2\r\n$3\r\nget\r\n$16336\r\n", [-2], 0, 0),            # key >= mbuf_data_size (:1369-1375)
    (b"*2\r\n$3\r\ngex\r\n$1\r\na\r\n", [-3], 0, 0),           # unknown here: host parser
    (b"*2\r\n$3\r\nget\r\n$1\r\na\r\nxyz", [0, -1], 1, 20),    # garbage after a request
])
def test_failure_rules(oracle, stream, status, nkeys, consumed):
    ks, kl, kr, st, info = oracle.redis_parse(stream)
    assert list(st) == status
    assert info["consumed"] == consumed
    assert len(ks) == (nkeys if status[-1:] == [0] or not status else len(ks))
    if status and status[-1] != 0:
        assert info["first_error"] == len(status) - 1


def test_random_streams(oracle):
    rng = np.random.default_rng(11)
    for _ in range(20):
        b, reqs = G.stream(rng, int(rng.integers(1, 60)))
        ks, kl, kr, st, info = oracle.redis_parse(b)
        assert list(st) == [0] * len(reqs) and info["consumed"] == len(b)
        want = [(k, i) for i, a in enumerate(reqs) for k in G.keys_of(a)]
        got = [(b[int(s): int(s) + int(n)], int(r)) for s, n, r in zip(ks, kl, kr)]
        assert got == want
