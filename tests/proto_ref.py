"""The reference parsers' and server_pool_idx's own outputs
(tests/golden/proto_ref.json, written by tools/gen_proto_golden.py from the
compiled reference) and the rules that relate a batch key extraction — the
oracle's restatement or the device parser — to them.

The batch parsers report, for a stream: requests parsed (nreqs), the first
request not handled (first_error; == nreqs when all were), the bytes of
requests [0, first_error) (consumed), a status per parsed request (0 ok,
-1 syntax, -2 key length, -3 another command class), and the keys of
requests [0, first_error) with their request index. The reference parses one
request at a time: result OK / ERROR / AGAIN, type, consumed bytes, keypos
spans. They agree when
  - every request before first_error is OK in the reference, with the same
    start (running consumed) and the same key spans;
  - the request at first_error is, in the reference, an ERROR for status -1
    or -2, and anything for status -3 (the host parser takes over: the
    reference parses it, OK or not);
  - when first_error == nreqs and bytes remain, the reference's next request
    is not OK (AGAIN: incomplete, left for the next read; or it is the end of
    what the reference parsed).
"""
import base64
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "proto_ref.json")


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def stream_of(entry) -> bytes:
    return base64.b64decode(entry["stream_b64"])


def keys_of(doc):
    return [base64.b64decode(k) for k in doc["server_idx"]["keys_b64"]]


def check(entry, nreqs, first_error, consumed, statuses, kstart, klen, kreq, key_bytes=None):
    """assert a batch parse of stream_of(entry) agrees with the reference;
    with kstart None, key_bytes (the packed keys, in order) is compared with
    the bytes of the reference's spans instead of the spans themselves"""
    ref = entry["reqs"]
    stream = stream_of(entry)
    statuses = list(np.asarray(statuses).tolist())
    kreq = np.asarray(kreq).astype(np.int64)
    if kstart is not None:
        kstart, klen = (np.asarray(a).astype(np.int64) for a in (kstart, klen))
    assert len(statuses) == nreqs
    assert first_error <= nreqs
    pos = 0
    for i in range(first_error):
        assert i < len(ref), f"request {i}: the reference stopped before it"
        r = ref[i]
        assert r["result"] == "OK", f"request {i}: reference {r['result']} {r['type']}, batch ok"
        assert r["start"] == pos
        sel = np.flatnonzero(kreq == i)
        if kstart is not None:
            got = [[int(kstart[j]), int(kstart[j] + klen[j])] for j in sel]
            assert got == r["keys"], f"request {i} ({r['type']}): keys {got} != reference {r['keys']}"
        else:
            got = [key_bytes[j] for j in sel]
            want = [stream[a:b] for a, b in r["keys"]]
            assert got == want, f"request {i} ({r['type']}): keys {got!r} != reference {want!r}"
        pos += r["consumed"]
    assert consumed == pos
    assert int((kreq >= first_error).sum()) == 0
    if first_error < nreqs:
        st = statuses[first_error]
        assert st in (-1, -2, -3)
        if st in (-1, -2):
            assert first_error < len(ref) and ref[first_error]["result"] == "ERROR", \
                f"request {first_error}: batch status {st}, reference {ref[first_error] if first_error < len(ref) else None}"
    elif first_error < len(ref):
        assert ref[first_error]["result"] != "OK", f"request {first_error}: reference OK, batch stopped"


def server_idx_cases(doc, dist_fixture):
    """(case, pool, continuum values or None, indices) per reference case"""
    for c in doc["server_idx"]["cases"]:
        p = dist_fixture["pools"][c["pool"]]
        if c["dist"] == 0:
            vals = np.array(p["ketama"]["values"], np.uint32)
            idx = np.array(p["ketama"]["indices"], np.uint32)
        else:
            vals, idx = None, np.array(p["modula"]["indices"], np.uint32)
        yield c, p, vals, idx


def frag_requests(doc, redis: bool):
    """the fragment fixture's requests of one protocol, and the pipelined
    stream of all of them (request r at stream[bounds[r]:bounds[r + 1]])"""
    reqs = [base64.b64decode(r) for r in doc["fragments"]["redis_b64" if redis else "memcache_b64"]]
    bounds = np.concatenate([[0], np.cumsum([len(r) for r in reqs])]).astype(np.int64)
    return reqs, b"".join(reqs), bounds


def frag_pool(case, dist_fixture):
    """(continuum values or None, indices, nserver) of a fragment case's pool"""
    p = dist_fixture["pools"][case["pool"]]
    if case["dist"] == 0:
        return np.array(p["ketama"]["values"], np.uint32), np.array(p["ketama"]["indices"], np.uint32), len(p["names"])
    return None, np.array(p["modula"]["indices"], np.uint32), len(p["names"])


def check_fragments(case, redis: bool, reqs, keys_by_req, sidx_by_req):
    """every request of one fixture case: the server of each key, the key ->
    fragment map and the fragments' bytes against the reference's
    msg->fragment (twemproxy_amd.fragment, nc_gpuhash_frag_plan)"""
    from twemproxy_amd.fragment import fragments

    want = case["redis" if redis else "memcache"]
    nserver = int(case["nserver"])
    for r, (req, keys, sidx) in enumerate(zip(reqs, keys_by_req, sidx_by_req)):
        w = want[r]
        tag = f"{'redis' if redis else 'memcache'} request {r} mode {case['mode']} dist {case['dist']}"
        assert [int(x) for x in sidx] == w["sidx"], tag
        seq, frags = fragments(redis, req, keys, sidx, nserver)
        if not w["frags_b64"]:
            assert seq is None and frags == [], tag
            continue
        assert [int(x) for x in seq] == w["frag_seq"], tag
        assert frags == [base64.b64decode(f) for f in w["frags_b64"]], tag
