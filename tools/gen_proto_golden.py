"""Fixtures from the REAL reference request parsers and server_pool_idx
(oracle/_ref/libref_proto.so, `make -C oracle ref-proto`; only where
/root/reference exists) -> tests/golden/proto_ref.json.

  redis / memcache: request streams — test_all.c's request vectors, the
    failure-rule vectors of tests/test_gpu_{redis,mc}_parse.py and seeded random
    pipelines — parsed request after request the way test_all drives the
    parser (src/test_all.c:76-107): one mbuf holding the unparsed rest (at most
    mbuf_data_size() bytes), msg_get, req->parser. Per request: MSG_PARSE_*
    result, msg_type_t name, consumed bytes, and the keypos spans the parser
    pushed (src/proto/nc_redis.c:1362-1490, src/proto/nc_memcache.c:380-407)
    as absolute stream offsets. A stream stops at the first request that is
    not MSG_PARSE_OK.
  server_idx: server_pool_idx (src/nc_server.c:647-700) of tagged keys over
    the tests/golden/dist.json pools, every hash mode, ketama and modula,
    hash_tag none / "{}" / "$$" / "ab".
  fragments: multi-key requests — memcache get / gets, redis mget / del /
    touch / unlink / mset — each fragmented by the reference's own
    msg->fragment (memcache_fragment, src/proto/nc_memcache.c:1283-1389;
    redis_fragment, src/proto/nc_redis.c:2804-2924) from a client connection
    owned by a dist.json pool: per key the server msg_backend_idx picked and
    its fragment (frag_seq), and every fragment's bytes as sent.

Data only (inputs and the reference's outputs): run here, commit the JSON.
    make -C oracle ref-proto && python tools/gen_proto_golden.py
"""
import base64
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_proto.so")
OUT = os.path.join(ROOT, "tests", "golden", "proto_ref.json")
RESULTS = ["OK", "ERROR", "REPAIR", "AGAIN"]  # MSG_PARSE_* (src/nc_message.h:31-36)

REDIS_VECTORS = [
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
    b"*2\r\n$3\r\ngex\r\n$1\r\na\r\n",
    b"*2\r\n$3\r\nget\r\n$1\r\na\r\nxyz",
    b"*2\r\n$3\r\nget\r\n$1\r\na\r\n$2\r\nzz\r\n",
    b"*2\r\n$3\r\nGeT\r\n$3\r\n\r\n*\r\n*2\r\n$4\r\nMGET\r\n$1\r\n*\r\n",
    b"*3\r\n$3\r\ndel\r\n$1\r\na\r\n$1\r\nb\r\n*5\r\n$4\r\nmset\r\n$1\r\nk\r\n$1\r\nv\r\n$1\r\nj\r\n$0\r\n\r\n",
    b"*2\r\n$3\r\nget\r\n$16000\r\n" + b"k" * 16000 + b"\r\n",
]

MC_VECTORS = [
    b"get a\r\n",
    b"get a bb ccc\r\n",
    b"gets a\r\n  get   b  \r\n",
    b"get a\r\nget b",
    b"get \r\n",
    b"get\r\n",
    b"GET a\r\n",
    b"get\ta\r\n",
    b"get a\rb\r\n",
    b"get a\nb\r\n",
    b"get " + b"k" * 250 + b"\r\n",
    b"get " + b"k" * 251 + b"\r\n",
    b"get a\r\nset k 0 0 1\r\nx\r\nget b\r\n",
    b"get a\r\ndelete b\r\n",
    b"\r\nget a\r\n",
    b"get {user:1}:a x{}y\r\n",
]


class Ref:
    def __init__(self):
        lib = ctypes.CDLL(LIB, mode=os.RTLD_LAZY)
        lib.rp_init.restype = ctypes.c_int
        lib.rp_parse_one.restype = ctypes.c_int
        lib.rp_parse_one.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32] + [ctypes.c_void_p] * 6 + \
            [ctypes.c_uint32]
        lib.rp_type_name.argtypes = [ctypes.c_int32, ctypes.c_char_p, ctypes.c_uint32]
        lib.rp_fragment.restype = ctypes.c_int
        lib.rp_fragment.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                    ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                    ctypes.c_uint32, ctypes.c_void_p]
        lib.rp_server_idx.restype = ctypes.c_int
        lib.rp_server_idx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        self.lib = lib
        self.mbuf_data = lib.rp_init()

    def type_name(self, ty: int) -> str:
        b = ctypes.create_string_buffer(64)
        self.lib.rp_type_name(ty, b, 64)
        return b.value.decode()

    def parse_one(self, redis: bool, buf: bytes):
        res, ty, cons, err = (ctypes.c_int32(), ctypes.c_int32(), ctypes.c_uint32(), ctypes.c_int32())
        cap = 4096
        ks, ke = (ctypes.c_uint32 * cap)(), (ctypes.c_uint32 * cap)()
        nk = self.lib.rp_parse_one(1 if redis else 0, buf, len(buf), ctypes.byref(res), ctypes.byref(ty),
                                   ctypes.byref(cons), ctypes.byref(err), ks, ke, cap)
        assert 0 <= nk <= cap
        return {"result": RESULTS[res.value], "type": self.type_name(ty.value), "consumed": cons.value,
                "conn_err": err.value, "keys": [[ks[i], ke[i]] for i in range(nk)]}

    def parse_stream(self, redis: bool, stream: bytes):
        """requests one after another; key spans as absolute offsets"""
        reqs, pos = [], 0
        while pos < len(stream):
            window = stream[pos: pos + self.mbuf_data]
            r = self.parse_one(redis, window)
            # [-1, -1]: a span the reference pushed outside the request (COMMAND, LOLWUT)
            r["keys"] = [[s + pos, e + pos] if s != 0xFFFFFFFF else [-1, -1] for s, e in r["keys"]]
            r["start"] = pos
            reqs.append(r)
            if r["result"] != "OK" or r["consumed"] == 0:
                break
            pos += r["consumed"]
        return reqs

    def server_idx(self, mode, dist, names, weights, tag: bytes, keys):
        nb = [n.encode() for n in names]
        arr = (ctypes.c_char_p * len(nb))(*nb)
        lens = np.array([len(n) for n in nb], np.uint32)
        w = np.array(weights, np.uint32)
        off = np.zeros(len(keys) + 1, np.uint64)
        off[1:] = np.cumsum([len(k) for k in keys])
        kb = np.frombuffer(b"".join(keys) + b"\0", np.uint8)
        out = np.zeros(len(keys), np.uint32)
        rc = self.lib.rp_server_idx(mode, dist, arr, lens.ctypes.data, w.ctypes.data, len(nb), tag, len(tag),
                                    kb.ctypes.data, off.ctypes.data, len(keys), out.ctypes.data)
        assert rc == 0
        return out.tolist()


    def fragment(self, redis: bool, req: bytes, mode, dist, names, weights, tag: bytes):
        nb = [n.encode() for n in names]
        arr = (ctypes.c_char_p * len(nb))(*nb)
        lens = np.array([len(n) for n in nb], np.uint32)
        w = np.array(weights, np.uint32)
        kcap, pcap, fcap = 4096, 1 << 20, 1024
        sidx, fseq = np.zeros(kcap, np.uint32), np.zeros(kcap, np.uint32)
        payload, plen = np.zeros(pcap, np.uint8), np.zeros(fcap, np.uint32)
        nfrag = ctypes.c_uint32()
        nk = self.lib.rp_fragment(1 if redis else 0, req, len(req), mode, dist, arr, lens.ctypes.data, w.ctypes.data,
                                  len(nb), tag, len(tag), sidx.ctypes.data, fseq.ctypes.data, kcap,
                                  payload.ctypes.data, pcap, plen.ctypes.data, fcap, ctypes.byref(nfrag))
        assert nk > 0, req[:80]
        frags, pos = [], 0
        for n in plen[: nfrag.value].tolist():
            frags.append(b64(payload[pos: pos + n].tobytes()))
            pos += n
        return {"sidx": sidx[:nk].tolist(), "frag_seq": fseq[:nk].tolist() if nfrag.value else [],
                "frags_b64": frags}


def b64(b: bytes) -> str:
    return base64.b64encode(b).decode()


def mc_pipeline(rng, n):
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789:_-.{}ABC\x01\xff", dtype=np.uint8)
    reqs = []
    for _ in range(n):
        nk = int(rng.integers(1, 9))
        words = [rng.choice(alpha, size=int(min(250, 1 + rng.zipf(1.3)))).tobytes() for _ in range(nk)]
        sp = [b" " * int(rng.integers(1, 3)) for _ in range(nk)]
        cmd = b"gets" if rng.random() < 0.2 else b"get"
        reqs.append(b" " * int(rng.integers(0, 2)) + cmd + b"".join(s + w for s, w in zip(sp, words)) + b"\r\n")
    return b"".join(reqs)


def tagged_keys(rng, n):
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789:_-$", dtype=np.uint8)
    out = [b"", b"{}", b"{", b"}", b"}{", b"{a}", b"x{ab}y", b"{{a}}", b"a{b{c}d}e", b"{x}{y}", b"user:{42}:name",
           b"$$", b"$a$", b"a$bc$d", b"ab", b"xaby", b"abab", b"ba"]
    while len(out) < n:
        body = rng.choice(alpha, size=int(rng.integers(0, 40))).tobytes()
        if rng.random() < 0.5 and len(body) > 2:
            i = int(rng.integers(0, len(body) - 1))
            j = int(rng.integers(i, len(body)))
            o, c = [(b"{", b"}"), (b"$", b"$"), (b"a", b"b")][int(rng.integers(0, 3))]
            body = body[:i] + o + body[i:j] + c + body[j:]
        out.append(body)
    return out


def frag_requests(rng):
    """multi-key requests the fragment loops split: memcache get / gets, redis
    mget / del / touch / unlink (one key per argument) and mset (key, value
    pairs); 1..48 keys of tagged_keys shape, values binary"""
    mc, rd = [], []
    pool = [k for k in tagged_keys(rng, 400) if k and b" " not in k]
    for i in range(48):
        nk = 1 + (i % 48) if i < 40 else int(rng.integers(2, 48))
        ks = [pool[int(j)] for j in rng.integers(0, len(pool), size=nk)]
        mc.append((b"gets" if i % 5 == 4 else b"get") + b"".join(b" " + k for k in ks) + b"\r\n")
        cmd = [b"mget", b"del", b"touch", b"unlink", b"mset"][i % 5]
        if cmd == b"mset":
            args = []
            for k in ks[:24]:
                v = rng.integers(0, 256, size=int(rng.integers(0, 20)), dtype=np.uint8).tobytes()
                args += [k, v]
        else:
            args = ks
        rd.append(b"*%d\r\n$%d\r\n%s\r\n" % (len(args) + 1, len(cmd), cmd) +
                  b"".join(b"$%d\r\n%s\r\n" % (len(a), a) for a in args))
    return mc, rd


def main():
    from tests import redis_gen as G

    ref = Ref()
    rng = np.random.default_rng(20250)
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "redis_req_cases.json")))["cases"]
    redis_streams = [c["req"].encode("latin-1") for c in cases] + REDIS_VECTORS
    for seed in range(3):
        b, _ = G.stream(np.random.default_rng(500 + seed), 300)
        redis_streams.append(b)
    mc_streams = list(MC_VECTORS) + [mc_pipeline(np.random.default_rng(600 + s), 300) for s in range(3)]

    doc = {
        "source": "oracle/_ref/libref_proto.so: src/proto/nc_redis.c, src/proto/nc_memcache.c, src/nc_message.c, "
                  "src/nc_mbuf.c, src/nc_server.c compiled from /root/reference (tools/gen_proto_golden.py)",
        "mbuf_data_size": ref.mbuf_data,
        "redis": [{"stream_b64": b64(s), "reqs": ref.parse_stream(True, s)} for s in redis_streams],
        "memcache": [{"stream_b64": b64(s), "reqs": ref.parse_stream(False, s)} for s in mc_streams],
    }
    dist = json.load(open(os.path.join(ROOT, "tests", "golden", "dist.json")))
    keys = tagged_keys(rng, 300)
    sidx = []
    for pi, p in enumerate(dist["pools"][:3]):
        for mode in range(12):
            for d in (0, 1):
                for tag in (b"", b"{}", b"$$", b"ab"):
                    sidx.append({"pool": pi, "mode": mode, "dist": d, "tag": tag.decode(),
                                 "idx": ref.server_idx(mode, d, p["names"], p["weights"], tag, keys)})
    doc["server_idx"] = {"keys_b64": [b64(k) for k in keys], "cases": sidx}
    mc_reqs, rd_reqs = frag_requests(np.random.default_rng(7070))
    fcases = []
    for pi, mode, d, tag in ((0, 6, 0, b""), (1, 6, 0, b"{}"), (2, 1, 0, b""), (1, 10, 1, b""), (2, 3, 0, b"{}"),
                             (0, 9, 1, b"$$"), (1, 11, 0, b""), (2, 0, 1, b"{}")):
        p = dist["pools"][pi]
        fcases.append({"pool": pi, "mode": mode, "dist": d, "tag": tag.decode(), "nserver": len(p["names"]),
                       "memcache": [ref.fragment(False, r, mode, d, p["names"], p["weights"], tag) for r in mc_reqs],
                       "redis": [ref.fragment(True, r, mode, d, p["names"], p["weights"], tag) for r in rd_reqs]})
    doc["fragments"] = {"memcache_b64": [b64(r) for r in mc_reqs], "redis_b64": [b64(r) for r in rd_reqs],
                        "cases": fcases}
    with open(OUT, "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    nreq = sum(len(s["reqs"]) for s in doc["redis"]) + sum(len(s["reqs"]) for s in doc["memcache"])
    print(f"{len(doc['redis'])} redis + {len(doc['memcache'])} memcache streams, {nreq} requests, "
          f"{len(sidx)} server_idx cases -> {OUT} ({os.path.getsize(OUT)} bytes)", file=sys.stderr)


if __name__ == "__main__":
    main()
