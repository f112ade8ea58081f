"""The batch sites' second half: multi-key requests split into per-server
fragments from server indices computed in one batch.

twemproxy's fragment loops — memcache_fragment_retrieval
(/root/reference/src/proto/nc_memcache.c:1283-1370) and redis_fragment_argx
(/root/reference/src/proto/nc_redis.c:2804-2898) — call msg_backend_idx
(src/nc_message.c:461-467) once per key, then copy each key into the
sub-message of its server. With the indices of every key of a read computed
at once (nc_gpuhash_server_idx_device over the device parser's key CSR), what
is left is the plan (nc_gpuhash_frag_plan: key -> fragment, fragments in
ascending server order) and the copies, which this module restates
byte for byte as the reference builds them:

  memcache  "get " / "gets " + each key followed by one space + CRLF
            (memcache_append_key, nc_memcache.c:1257-1277; prefix and CRLF
            nc_memcache.c:1349-1366);
  redis     "*<narg+1>\\r\\n$<n>\\r\\n<cmd>\\r\\n" + "$<len>\\r\\n<key>\\r\\n" per
            key (redis_append_key, nc_redis.c:2708-2763), mset's values copied
            as they arrived (redis_copy_bulk) — narg counts keys and values
            (nc_redis.c:2870-2889).

A one-key request is not fragmented (memcache_should_fragment,
nc_memcache.c:104-118; redis_fragment, nc_redis.c:2903).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L

# command name as the reference prepends it (nc_redis.c:2875-2889), keyed by
# the lower-cased command of the original request
REDIS_FRAG_CMDS = {b"mget": b"mget", b"del": b"del", b"mset": b"mset", b"touch": b"touch", b"unlink": b"unlink"}


def frag_plan(sidx, nserver: int):
    """(frag_seq, frag_server, frag_nkeys) of one request through
    nc_gpuhash_frag_plan."""
    s = np.ascontiguousarray(np.asarray(sidx, dtype=np.uint32))
    n = int(s.size)
    cap = max(1, min(n, int(nserver)))
    seq = np.empty(max(1, n), np.uint32)
    srv = np.empty(cap, np.uint32)
    cnt = np.empty(cap, np.uint32)
    nf = L.lib().nc_gpuhash_frag_plan(s.ctypes.data, n, int(nserver), seq.ctypes.data, srv.ctypes.data,
                                      cnt.ctypes.data)
    if nf < 0:
        raise L.NcError(ctypes.get_errno(), "nc_gpuhash_frag_plan")
    return seq[:n], srv[:nf], cnt[:nf]


def _resp_args(req: bytes) -> list[bytes]:
    """the bulk strings of one RESP request, in order (the command first)"""
    p = req.index(b"\r\n")
    narg = int(req[1:p])
    p += 2
    args = []
    for _ in range(narg):
        q = req.index(b"\r\n", p)
        n = int(req[p + 1: q])
        args.append(req[q + 2: q + 2 + n])
        p = q + 2 + n + 2
    return args


def fragments(redis: bool, req: bytes, keys, sidx, nserver: int):
    """The fragments the reference sends for one multi-key request `req`
    whose keys (request order) are `keys` and go to servers `sidx`:
    (frag_seq, [fragment bytes, ...]), or (None, []) when the reference does
    not fragment the request."""
    keys = [bytes(k) for k in keys]
    if len(keys) <= 1:
        return None, []
    if redis:
        args = _resp_args(req)
        cmd = REDIS_FRAG_CMDS.get(args[0].lower())
        if cmd is None:
            return None, []
        step = 2 if cmd == b"mset" else 1
        if args[1::step] != keys:
            raise ValueError("keys are not the request's key arguments")
    else:
        word = req.lstrip(b" ").split(b" ", 1)[0]
        if word not in (b"get", b"gets"):
            return None, []
    seq, _srv, cnt = frag_plan(sidx, nserver)
    body = [[] for _ in range(len(cnt))]
    narg = [0] * len(cnt)
    for i, key in enumerate(keys):
        f = int(seq[i])
        if redis:
            body[f].append(b"$%d\r\n%s\r\n" % (len(key), key))
            narg[f] += 1
            if step == 2:
                val = args[2 + 2 * i]
                body[f].append(b"$%d\r\n%s\r\n" % (len(val), val))
                narg[f] += 1
        else:
            body[f].append(key + b" ")
    out = []
    for f in range(len(cnt)):
        if redis:
            out.append(b"*%d\r\n$%d\r\n%s\r\n" % (narg[f] + 1, len(cmd), cmd) + b"".join(body[f]))
        else:
            out.append(word + b" " + b"".join(body[f]) + b"\r\n")
    return seq, out
