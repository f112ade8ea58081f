#!/usr/bin/env python3
"""Device key extraction (nc_gpuhash_mc_parse_device) on pipelined GET
streams: C5's batch (64 connections x 128 pipelined "get <key>\\r\\n", C2
Zipf printable keys) and a 2^22-request stream for throughput, then the
extracted keys through fnv1a_64 and the fused server_idx. Then the redis
parser (nc_gpuhash_redis_parse_device) on the same keys as RESP GETs and on a
mixed binary-safe pipeline (tests/redis_gen.py). Prints JSON lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def get_stream(t, np, nreq, seed=5):
    """b"get <key>\\r\\n" x nreq, keys from the C5 generator, assembled with numpy."""
    spec = t.SynthSpec.zipf(seed, charset=t.BYTES_PRINTABLE)
    kh, oh = t.synth_host(spec, 0, nreq)
    lens = np.diff(oh).astype(np.int64)
    rl = lens + 6
    ro = np.zeros(nreq + 1, np.int64)
    np.cumsum(rl, out=ro[1:])
    buf = np.empty(int(ro[-1]), np.uint8)
    for j, c in enumerate(b"get "):
        buf[ro[:-1] + j] = c
    # key bytes: scatter each key after its "get "
    idx = np.repeat(ro[:-1] + 4 - oh[:-1].astype(np.int64), lens) + np.arange(int(oh[-1]), dtype=np.int64)
    buf[idx] = kh[: int(oh[-1])]
    buf[ro[1:] - 2] = 13
    buf[ro[1:] - 1] = 10
    return buf, int(oh[-1])


def main():
    import numpy as np
    import torch

    import twemproxy_amd as t

    with t.McParser(max_bytes=1 << 30, max_reqs=1 << 23, max_keys=1 << 23) as ps:
        for nreq in (64 * 128, 1 << 22):
            buf, kbytes = get_stream(t, np, nreq)
            sd = torch.from_numpy(buf).cuda()
            for _ in range(3):
                ps.parse(sd)
            torch.cuda.synchronize()
            reps = 20 if nreq < 100000 else 5
            t0 = time.perf_counter()
            for _ in range(reps):
                keys, off, kreq, status, info = ps.parse(sd)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            assert info["nkeys"] == nreq and info["first_error"] == nreq
            h = t.hash_batch_device("fnv1a_64", keys, off)
            torch.cuda.synchronize()
            hv = h.cpu().numpy().view(np.uint32)
            rng = np.random.default_rng(0)
            bad = 0
            o = off.cpu().numpy()
            kb = keys.cpu().numpy()
            for i in rng.integers(0, nreq, size=64):
                bad += int(hv[i]) != t.hash_key("fnv1a_64", kb[o[i]: o[i + 1]].tobytes())
            print(json.dumps({"workload": f"{nreq} pipelined 'get <key>' requests (C5 keys)",
                              "stream_bytes": int(buf.size), "key_bytes": kbytes,
                              "parse_ms_wall": round(dt * 1e3, 4),
                              "stream_gb_s": round(buf.size / dt / 1e9, 2), "mreq_s": round(nreq / dt / 1e6, 1),
                              "sample_hash_mismatches": bad}), flush=True)


def resp_get_stream(t, np, nreq, seed=5):
    """RESP "*2 $3 get $<len> <key>" x nreq over the same C5 keys"""
    spec = t.SynthSpec.zipf(seed, charset=t.BYTES_PRINTABLE)
    kh, oh = t.synth_host(spec, 0, nreq)
    kb = kh.tobytes()
    parts = []
    for i in range(nreq):
        k = kb[int(oh[i]): int(oh[i + 1])]
        parts.append(b"*2\r\n$3\r\nget\r\n$%d\r\n%s\r\n" % (len(k), k))
    return np.frombuffer(b"".join(parts), np.uint8).copy(), int(oh[-1])


def timed(torch, ps, sd, reps):
    for _ in range(3):
        ps.parse(sd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = ps.parse(sd)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def redis_main():
    import numpy as np
    import torch

    import twemproxy_amd as t
    from tests import redis_gen as G

    with t.RedisParser(max_bytes=1 << 30, max_reqs=1 << 23, max_keys=1 << 23) as ps:
        for nreq in (64 * 128, 1 << 21):
            buf, kbytes = resp_get_stream(t, np, nreq)
            sd = torch.from_numpy(buf).cuda()
            dt, (keys, off, kreq, status, info) = timed(torch, ps, sd, 20 if nreq < 100000 else 5)
            assert info["nkeys"] == nreq and info["first_error"] == nreq
            print(json.dumps({"workload": f"redis: {nreq} pipelined RESP GETs (C5 keys)",
                              "stream_bytes": int(buf.size), "key_bytes": kbytes,
                              "parse_ms_wall": round(dt * 1e3, 4),
                              "stream_gb_s": round(buf.size / dt / 1e9, 2), "mreq_s": round(nreq / dt / 1e6, 1)}),
                  flush=True)
        rng = np.random.default_rng(1)
        b, reqs = G.stream(rng, 200_000)
        sd = torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()
        dt, (keys, off, kreq, status, info) = timed(torch, ps, sd, 5)
        assert info["nreqs"] == len(reqs) and info["consumed"] == len(b)
        print(json.dumps({"workload": "redis: 200000 mixed binary-safe requests (tests/redis_gen.py, seed 1)",
                          "stream_bytes": len(b), "nkeys": info["nkeys"], "parse_ms_wall": round(dt * 1e3, 4),
                          "stream_gb_s": round(len(b) / dt / 1e9, 2), "mreq_s": round(len(reqs) / dt / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    if "--redis" in sys.argv:
        redis_main()
        sys.exit(0)
    main()
