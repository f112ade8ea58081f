"""The batch ring (nc_gpuhash_ring, include/nc_gpuhash.h 3d): small batches
served by resident worker workgroups (one per lane) polling mapped host
memory, no HIP call per batch. Every result against the oracle; the workers'
life cycle (one launch per lane for a burst, leaving after an idle 10 ms and relaunching on demand,
stopping on destroy) and the limits."""
import threading
import time

import numpy as np
import pytest

import twemproxy_amd as t

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]


def batch(rng, nkeys, maxlen=300, total=30000):
    """one mbuf-like buffer of keys (0..maxlen bytes, every byte value) and
    their (start, end) spans; at most `total` key bytes"""
    lens = rng.integers(0, maxlen + 1, size=nkeys)
    lens = lens[np.cumsum(lens) <= total]
    gaps = rng.integers(0, 5, size=lens.size)  # bytes between keys, as "get " / "\r\n" would be
    buf = rng.integers(0, 256, size=int((lens + gaps).sum()) + 64, dtype=np.uint8)
    spans, pos = [], 0
    for n, g in zip(lens.tolist(), gaps.tolist()):
        pos += g
        spans.append((pos, pos + n))
        pos += n
    return buf, spans


def want(oracle, mode, buf, spans):
    keys, off = t.pack_keys([buf[s:e].tobytes() for s, e in spans])
    return oracle.batch(mode, keys, off)


def test_ring_every_mode_matches_oracle(gpu, oracle):
    rng = np.random.default_rng(31)
    with t.Ring(0, nslots=4) as r:
        for m in range(12):
            for nk in (1, 7, 64, 585, 1500):
                buf, spans = batch(rng, nk)
                tk, out = r.submit_spans(m, buf, spans)
                r.wait(tk)
                np.testing.assert_array_equal(out, want(oracle, m, buf, spans), err_msg=f"{t.HASH_NAMES[m]} {nk}")
        assert r.launches == 2  # one worker per lane served the whole burst


def test_ring_single_slot_single_lane(gpu, oracle):
    """nslots=1: one lane, every batch through the same slot"""
    rng = np.random.default_rng(34)
    with t.Ring(0, nslots=1) as r:
        for i in range(50):
            buf, spans = batch(rng, int(rng.integers(1, 900)), maxlen=40)
            tk, out = r.submit_spans(i % 12, buf, spans)
            r.wait(tk)
            np.testing.assert_array_equal(out, want(oracle, i % 12, buf, spans))
        assert r.launches == 1


def test_ring_pipelined_in_order(gpu, oracle):
    """nslots batches in flight, polled; a full ring refuses the next submit
    (BlockingIOError) until its slot's batch is done"""
    rng = np.random.default_rng(32)
    nslots = 4
    with t.Ring(0, nslots=nslots) as r:
        pending = []
        for i in range(200):
            buf, spans = batch(rng, int(rng.integers(1, 700)), maxlen=64)
            while True:
                try:
                    tk, out = r.submit_spans("fnv1a_64", buf, spans)
                    break
                except BlockingIOError:
                    tk0, out0, b0, s0 = pending.pop(0)
                    r.wait(tk0)
                    np.testing.assert_array_equal(out0, want(oracle, 6, b0, s0))
            pending.append((tk, out, buf, spans))
            if len(pending) > nslots:
                # the submit reused the oldest batch's slot: that batch was
                # finished and delivered on the way
                tk0, out0, b0, s0 = pending.pop(0)
                assert r.poll(tk0)
                np.testing.assert_array_equal(out0, want(oracle, 6, b0, s0))
        for tk, out, buf, spans in pending:
            while not r.poll(tk):
                pass
            np.testing.assert_array_equal(out, want(oracle, 6, buf, spans))


def test_ring_worker_leaves_and_returns(gpu, oracle):
    """the worker leaves after 10 ms of an empty ring and the next submit
    relaunches it; batches right around the leaving point are not lost"""
    rng = np.random.default_rng(33)
    with t.Ring(0, nslots=2) as r:
        for rep in range(3):
            buf, spans = batch(rng, 300)
            tk, out = r.submit_spans("md5", buf, spans)
            r.wait(tk)
            np.testing.assert_array_equal(out, want(oracle, 1, buf, spans))
            time.sleep(0.05)
        assert r.launches == 3
        # submits spaced around the idle limit
        for gap in (0.008, 0.009, 0.010, 0.011, 0.012):
            time.sleep(gap)
            buf, spans = batch(rng, 100)
            tk, out = r.submit_spans("crc32", buf, spans)
            r.wait(tk)
            np.testing.assert_array_equal(out, want(oracle, 3, buf, spans))


def test_ring_limits_and_empty(gpu):
    with t.Ring(0, nslots=2, max_keys=100, max_key_bytes=1000) as r:
        buf = np.zeros(4096, np.uint8)
        with pytest.raises(t.NcError):
            r.submit_spans("fnv1a_64", buf, [(0, 1)] * 101)  # more keys than max_keys
        with pytest.raises(t.NcError):
            r.submit_spans("fnv1a_64", buf, [(0, 600), (600, 1200)])  # more bytes than max_key_bytes
        tk, out = r.submit_spans("fnv1a_64", buf, [])
        r.wait(tk)
        assert out.size == 0
        tk, out = r.submit_spans("jenkins", buf, [(0, 0), (0, 13)])
        r.wait(tk)
        assert out.tolist() == [t.hash_key("jenkins", b""), t.hash_key("jenkins", bytes(13))]


def test_ring_destroy_with_worker_running(gpu):
    """destroy right after a submit: the worker stops at its next poll and the
    call returns (no wait for the idle limit or a hang)"""
    buf = np.arange(256, dtype=np.uint8)
    t0 = time.perf_counter()
    for _ in range(5):
        r = t.Ring(0, nslots=2)
        r.submit_spans("fnv1a_64", buf, [(0, 10), (10, 200)])
        r.close()
    assert time.perf_counter() - t0 < 5.0


def test_ring_shared_by_threads(gpu, oracle):
    """four threads submit and wait on one ring (its mutex): every batch's
    hashes are its own, none lost or delivered twice"""
    errors = []
    with t.Ring(0, nslots=4) as r:
        def worker(seed):
            rng = np.random.default_rng(seed)
            try:
                for _ in range(40):
                    buf, spans = batch(rng, int(rng.integers(1, 400)), maxlen=48)
                    while True:
                        try:
                            tk, out = r.submit_spans("fnv1a_64", buf, spans)
                            break
                        except BlockingIOError:
                            time.sleep(0)
                    r.wait(tk)
                    np.testing.assert_array_equal(out, want(oracle, 6, buf, spans))
            except Exception as e:  # reported by the main thread
                errors.append(e)
        th = [threading.Thread(target=worker, args=(40 + i,)) for i in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join(60)
        assert not any(x.is_alive() for x in th)
    assert not errors, errors[0]


def test_ring_rejects_spans_outside_the_buffer(gpu):
    with t.Ring(0, nslots=2) as r:
        buf = np.zeros(100, np.uint8)
        for bad in ([(0, 101)], [(-1, 5)], [(10, 5)]):
            with pytest.raises(ValueError):
                r.submit_spans("fnv1a_64", buf, bad)
