"""The batch ring (nc_gpuhash_ring, include/nc_gpuhash.h 3d): small batches
served by one resident launch (a workgroup per lane) polling its staging, no
HIP call per batch. Every result against the oracle; the launch's life cycle
(one launch for a burst, ending after an idle 10 ms or 2 s and relaunching on
demand, stopping on destroy), the lane and thread shapes, the ticket space
across 2^31 and 2^32 batches, and the limits. Every test runs twice: with the
batches staged in device memory written through the PCIe BAR
(NC_GPUHASH_RING_STAGING=device; the default for rings of 1 or 2 lanes on a
large-BAR device such as the MI355X) and in mapped host memory
(NC_GPUHASH_RING_STAGING=host; the default for 4 lanes and more), and a
third time with device staging and the hashes published by a release
instead of stored write-through (NC_GPUHASH_RING_WT=0)."""
import ctypes
import threading
import time

import numpy as np
import pytest

import twemproxy_amd as t

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]


@pytest.fixture(autouse=True, params=["device", "host", "device-release"])
def staging(request, monkeypatch):
    """the staging every ring of the test is created with (read at create);
    "device-release": device staging with the hashes stored plainly and
    published by a system-scope release (NC_GPUHASH_RING_WT=0, the A/B of the
    default write-through stores)"""
    st = request.param.split("-")[0]
    monkeypatch.setenv("NC_GPUHASH_RING_STAGING", st)
    if request.param.endswith("-release"):
        monkeypatch.setenv("NC_GPUHASH_RING_WT", "0")
    else:
        monkeypatch.delenv("NC_GPUHASH_RING_WT", raising=False)
    return st


def test_ring_staging_is_the_one_asked_for(gpu, staging):
    # MI355X exposes its whole HBM through a large BAR (tools/probes/bar_probe.hip)
    with t.Ring(0, nslots=2) as r:
        assert r.staging == staging


@pytest.mark.parametrize("lanes,want", [(1, "device"), (2, "device"), (4, "host"), (8, "host")])
def test_ring_default_staging(gpu, staging, monkeypatch, lanes, want):
    monkeypatch.delenv("NC_GPUHASH_RING_STAGING")
    with t.Ring(0, nslots=8, lanes=lanes) as r:
        assert r.staging == want


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
    # batches and expected hashes first: the burst below has no host gap
    # near the 10 ms idle limit
    work = []
    for m in range(12):
        for nk in (1, 7, 64, 585, 1500):
            buf, spans = batch(rng, nk)
            work.append((m, nk, buf, spans, want(oracle, m, buf, spans)))
    with t.Ring(0, nslots=4) as r:
        outs = []
        for m, nk, buf, spans, _ in work:
            tk, out = r.submit_spans(m, buf, spans)
            r.wait(tk)
            outs.append(out)
        launches = r.launches
    for (m, nk, _, _, w), out in zip(work, outs):
        np.testing.assert_array_equal(out, w, err_msg=f"{t.HASH_NAMES[m]} {nk}")
    assert launches == 1  # one launch (a workgroup per lane) served the whole burst


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


@pytest.mark.parametrize("lanes", [1, 2])
def test_ring_tiny_batches(gpu, oracle, lanes):
    """batches of 0..9 keys, every mode, one and two lanes"""
    rng = np.random.default_rng(77 + lanes)
    work = []
    for nk in list(range(10)) * 2:
        buf, spans = batch(rng, nk, maxlen=90)
        m = int(rng.integers(0, 12))
        work.append((m, buf, spans, want(oracle, m, buf, spans)))
    with t.Ring(0, nslots=4, lanes=lanes, threads=1024) as r:
        for m, buf, spans, w in work:
            tk, out = r.submit_spans(m, buf, spans)
            r.wait(tk)
            np.testing.assert_array_equal(out, w, err_msg=f"{t.HASH_NAMES[m]} {len(spans)}")


def test_ring_create_while_another_runs(gpu, oracle):
    """a ring created while another ring's resident worker serves a steady
    stream neither waits for that worker (its set-up synchronises only its
    own stream) nor disturbs it"""
    rng = np.random.default_rng(91)
    buf, spans = batch(rng, 300, maxlen=60)
    w = want(oracle, 6, buf, spans)
    stop = threading.Event()
    errors, served = [], [0]
    with t.Ring(0, nslots=2, lanes=1) as a:
        def feed():
            try:
                while not stop.is_set():
                    tk, out = a.submit_spans(6, buf, spans)
                    a.wait(tk)
                    np.testing.assert_array_equal(out, w)
                    served[0] += 1
            except Exception as e:  # noqa: BLE001 - reported below
                errors.append(e)
        th = threading.Thread(target=feed)
        th.start()
        try:
            time.sleep(0.2)  # the worker is resident and busy
            t0 = time.perf_counter()
            with t.Ring(0, nslots=2, lanes=1) as b:
                took = time.perf_counter() - t0
                tk, out = b.submit_spans(6, buf, spans)
                b.wait(tk)
                np.testing.assert_array_equal(out, w)
        finally:
            stop.set()
            th.join(30)
    assert not errors, errors[0]
    assert served[0] > 100
    assert took < 0.5, f"ring create took {took:.3f} s beside a running worker"


def test_ring_rejects_spans_outside_the_buffer(gpu):
    with t.Ring(0, nslots=2) as r:
        buf = np.zeros(100, np.uint8)
        for bad in ([(0, 101)], [(-1, 5)], [(10, 5)]):
            with pytest.raises(ValueError):
                r.submit_spans("fnv1a_64", buf, bad)


@pytest.mark.parametrize("lanes,threads", [(1, 256), (1, 512), (1, 1024), (2, 256), (2, 512), (2, 1024), (3, 1024),
                                           (4, 256), (8, 256), (8, 1024)])
def test_ring_lane_shapes(gpu, oracle, lanes, threads):
    """every lane count and workgroup size, batches pipelined over 8 slots"""
    rng = np.random.default_rng(50 + lanes * 7 + threads)
    work = []
    for i in range(80):
        buf, spans = batch(rng, int(rng.integers(0, 1200)), maxlen=70)
        work.append((i % 12, buf, spans, want(oracle, i % 12, buf, spans)))
    done = []
    with t.Ring(0, nslots=8, lanes=lanes, threads=threads) as r:
        assert r.lanes == lanes
        pending = []
        for m, buf, spans, w in work:
            while True:
                try:
                    tk, out = r.submit_spans(m, buf, spans)
                    break
                except BlockingIOError:
                    tk0, out0, w0 = pending.pop(0)
                    r.wait(tk0)
                    done.append((out0, w0))
            pending.append((tk, out, w))
        for tk, out, w in pending:
            r.wait(tk)
            done.append((out, w))
        launches = r.launches
    assert len(done) == len(work)
    for out, w in done:
        np.testing.assert_array_equal(out, w)
    assert launches == 1


@pytest.mark.parametrize("start", [2**31 - 21, 2**32 - 23, 2**33 + 5])
@pytest.mark.parametrize("nslots", [3, 4])
def test_ring_ticket_wrap(gpu, oracle, start, nslots):
    """a ring that has already numbered `start` batches: across 2^31 (the
    ticket's 31 bits wrap) and 2^32 (a 32-bit count would wrap), with slot
    counts that do (4) and do not (3) divide 2^32, every batch's hashes are
    its own, a delivered ticket polls done, and an unissued ticket is an
    error, never NC_OK"""
    rng = np.random.default_rng(start % 1000 + nslots)
    with t.Ring(0, nslots=nslots) as r:
        r.debug_start_seq(start)
        with pytest.raises(t.NcError):
            r.poll(start & 0x7FFFFFFF)  # not issued yet
        pending, tickets = [], []
        for i in range(60):
            m = (i * 5) % 12
            buf, spans = batch(rng, int(rng.integers(1, 400)), maxlen=40)
            while True:
                try:
                    tk, out = r.submit_spans(m, buf, spans)
                    break
                except BlockingIOError:
                    tk0, out0, b0, s0, m0 = pending.pop(0)
                    r.wait(tk0)
                    np.testing.assert_array_equal(out0, want(oracle, m0, b0, s0))
            assert tk == (start + i) & 0x7FFFFFFF
            tickets.append(tk)
            pending.append((tk, out, buf, spans, m))
        for tk, out, buf, spans, m in pending:
            r.wait(tk)
            np.testing.assert_array_equal(out, want(oracle, m, buf, spans))
        for tk in tickets:  # all delivered, the oldest through their slots' reuse
            assert r.poll(tk)
        with pytest.raises(t.NcError):
            r.poll((start + 60) & 0x7FFFFFFF)  # the next ticket: not issued
        with pytest.raises(t.NcError):
            r.poll((start - 1) & 0x7FFFFFFF)  # before the ring's first batch
        with pytest.raises(t.NcError):
            r.debug_start_seq(0)  # only a fresh ring


def test_ring_pending_batch_never_polls_done(gpu, oracle):
    """while no worker runs (debug hold), a submitted batch polls NC_EAGAIN
    every time; released, the same ticket completes with its own hashes"""
    rng = np.random.default_rng(61)
    with t.Ring(0, nslots=3) as r:
        r.debug_hold(True)
        items = []
        for m in (6, 1, 3):
            buf, spans = batch(rng, 200, maxlen=50)
            tk, out = r.submit_spans(m, buf, spans)
            items.append((tk, out, buf, spans, m))
        t_end = time.perf_counter() + 0.05
        while time.perf_counter() < t_end:
            for tk, *_ in items:
                assert not r.poll(tk)
        with pytest.raises(BlockingIOError):
            r.submit_spans(6, *batch(rng, 10))  # every slot pending
        assert r.launches == 0
        r.debug_hold(False)
        for tk, out, buf, spans, m in items:
            r.wait(tk)
            np.testing.assert_array_equal(out, want(oracle, m, buf, spans))
        assert r.launches == 1


def test_ring_relaunch_under_steady_load(gpu, oracle):
    """a launch lives at most 2 s even while batches keep coming: it ends and
    the next submit or poll relaunches it, with no batch lost"""
    rng = np.random.default_rng(62)
    bufs = [batch(rng, 300, maxlen=40) for _ in range(8)]
    wants = [want(oracle, 6, b, s) for b, s in bufs]
    with t.Ring(0, nslots=4) as r:
        t_end = time.perf_counter() + 2.6
        i = 0
        while time.perf_counter() < t_end:
            buf, spans = bufs[i % 8]
            tk, out = r.submit_spans("fnv1a_64", buf, spans)
            r.wait(tk)
            np.testing.assert_array_equal(out, wants[i % 8])
            i += 1
        assert r.launches >= 2, (r.launches, i)


def test_ring_c_rejects_inverted_and_null_spans(gpu, oracle):
    """the C entry point itself (below the Python checks): a span with end <
    start, or a NULL start, is EINVAL before anything is staged; the ring
    then serves the next batch normally"""
    lib = t._lib.lib()
    buf = (ctypes.c_uint8 * 256)(*range(256))
    base = ctypes.addressof(buf)
    with t.Ring(0, nslots=2) as r:
        out = (ctypes.c_uint32 * 4)()
        tk = ctypes.c_int(-1)
        for bad in ([(base + 10, base + 5)], [(base, base + 4), (base + 100, base + 99)], [(0, 8)]):
            spans = (t._lib.NcKeySpan * len(bad))()
            for i, (s0, e0) in enumerate(bad):
                spans[i].start = s0
                spans[i].end = e0
            rc = lib.nc_gpuhash_ring_submit_spans(r._h, 6, spans, len(bad), ctypes.addressof(out), ctypes.byref(tk))
            assert rc == t._lib.NC_ERROR and ctypes.get_errno() == 22, (bad, rc)
        tk2, out2 = r.submit_spans("fnv1a_64", np.frombuffer(bytes(buf), np.uint8), [(0, 10), (10, 40)])
        r.wait(tk2)
        assert tk2 == 0  # the refused submits took no ticket
        assert out2.tolist() == [t.hash_key("fnv1a_64", bytes(range(10))), t.hash_key("fnv1a_64", bytes(range(10, 40)))]


def test_ring_life_limit_with_every_slot_in_flight(gpu, oracle):
    """the 2 s life limit under pipelined load: every slot stays submitted
    (more than one batch per lane in flight, so a lane always finds its next
    batch published when it polls) for 2.6 s; the launch must still end and
    be relaunched, with every result equal to the oracle's"""
    import collections

    rng = np.random.default_rng(64)
    bufs = [batch(rng, 200, maxlen=40) for _ in range(8)]
    wants = [want(oracle, 6, b, s) for b, s in bufs]
    nslots = 16
    with t.Ring(0, nslots=nslots, lanes=4) as r:
        inflight = collections.deque()
        t_end = time.perf_counter() + 2.6
        i = checked = 0
        while time.perf_counter() < t_end:
            if len(inflight) == nslots:
                tk, out, j = inflight.popleft()
                r.wait(tk)
                np.testing.assert_array_equal(out, wants[j])
                checked += 1
            buf, spans = bufs[i % 8]
            tk, out = r.submit_spans("fnv1a_64", buf, spans)
            inflight.append((tk, out, i % 8))
            i += 1
        while inflight:
            tk, out, j = inflight.popleft()
            r.wait(tk)
            np.testing.assert_array_equal(out, wants[j])
            checked += 1
        assert r.launches >= 2, (r.launches, checked)
        assert checked == i


def test_ring_forget_drops_the_copy(gpu, oracle):
    """a forgotten ticket's batch still runs, its slot is reused normally,
    and its output array is never written (its owner freed it)"""
    rng = np.random.default_rng(65)
    with t.Ring(0, nslots=2) as r:
        buf, spans = batch(rng, 50, maxlen=30)
        r.debug_hold(True)
        tk, out = r.submit_spans("fnv1a_64", buf, spans)
        out[:] = 7
        r.forget(tk)
        r.debug_hold(False)
        r.wait(tk)
        assert (out == 7).all()
        # the slots go on serving: three more batches reuse both slots
        for _ in range(3):
            b2, s2 = batch(rng, 40, maxlen=30)
            tk2, o2 = r.submit_spans("murmur", b2, s2)
            r.wait(tk2)
            np.testing.assert_array_equal(o2, want(oracle, 10, b2, s2))
        with pytest.raises(Exception):
            r.forget(123456)  # never issued
