"""RESP request streams for the redis key-extraction tests (CPU and GPU):
requests of every key class the device extracts, binary-safe values that
contain CR LF '*' (a false request start for the speculative parse), and the
failure kinds of redis_parse_req (src/proto/nc_redis.c)."""
import numpy as np

ARG0 = [b"get", b"incr", b"ttl", b"strlen", b"hgetall", b"llen", b"zcard", b"getdel"]
ARG1 = [b"expire", b"append", b"getset", b"hget", b"setnx", b"zscore", b"incrbyfloat"]
ARGN = [b"set", b"hset", b"sadd", b"zadd", b"exists", b"bitcount", b"restore", b"georadiusbymember"]
ARGX = [b"mget", b"del", b"unlink", b"touch"]


def bulk(b: bytes) -> bytes:
    return b"$%d\r\n%s\r\n" % (len(b), b)


def req(*args: bytes) -> bytes:
    return b"*%d\r\n" % len(args) + b"".join(bulk(a) for a in args)


def keys_of(args):
    """The keys twemproxy records for a request of these args (SW_KEY pushes)."""
    c = args[0].lower()
    if c in ARGX:
        return list(args[1:])
    if c == b"mset":
        return list(args[1::2])
    return [args[1]]


def blob(rng, n: int) -> bytes:
    """binary value; often holds "\\r\\n*" so a candidate request start appears inside it"""
    b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    if n >= 6 and rng.random() < 0.5:
        i = int(rng.integers(0, n - 5))
        b[i:i + 5] = b"\r\n*2\r"
    return bytes(b)


def random_request(rng):
    k = lambda: blob(rng, int(rng.integers(0, 40)))  # noqa: E731
    v = lambda: blob(rng, int(rng.integers(0, 120)))  # noqa: E731
    cls = int(rng.integers(0, 5))
    if cls == 0:
        args = [ARG0[rng.integers(len(ARG0))], k()]
    elif cls == 1:
        args = [ARG1[rng.integers(len(ARG1))], k(), v()]
    elif cls == 2:
        args = [ARGN[rng.integers(len(ARGN))], k()] + [v() for _ in range(int(rng.integers(0, 4)))]
    elif cls == 3:
        args = [ARGX[rng.integers(len(ARGX))]] + [k() for _ in range(int(rng.integers(1, 9)))]
    else:
        args = [b"mset"]
        for _ in range(int(rng.integers(1, 5))):
            args += [k(), v()]
    if rng.random() < 0.3:
        args[0] = args[0].upper()
    return list(args)


def stream(rng, nreq: int):
    """nreq valid requests; returns (bytes, [args per request])"""
    reqs = [random_request(rng) for _ in range(nreq)]
    return b"".join(req(*a) for a in reqs), reqs
