"""Host-side batch API on the GPU: synchronous nc_hashkit_batch, the
asynchronous context (submit / poll / wait), keypos-style spans, and the
error returns of SURVEY.md §8b.3."""
import numpy as np
import pytest

import twemproxy_amd as t

pytestmark = pytest.mark.gpu


def test_hashkit_batch_sync(gpu, corpus):
    keys, off, expected = corpus
    for m in range(12):
        np.testing.assert_array_equal(t.hash_batch_host(m, keys, off), expected[m])
    assert t.hash_keys("fnv1a_64", [b"apple"]) == [1488911807]


def test_hashkit_batch_grows_context(gpu, oracle):
    keys, off = t.synth_host(t.SynthSpec.zipf(9), 0, 300000)
    np.testing.assert_array_equal(t.hash_batch_host("murmur", keys, off), oracle.batch(10, keys, off))


def test_context_async_slots(gpu, oracle):
    with t.Context(max_keys=4096, max_key_bytes=1 << 20, nslots=2) as ctx:
        batches = [t.synth_host(t.SynthSpec.zipf(20 + i), 0, 3000) for i in range(6)]
        tickets = []
        for i, (k, o) in enumerate(batches[:2]):
            tickets.append(ctx.submit("fnv1a_64", k, o))
        # a third submit while both slots are in flight returns NC_EAGAIN, unless
        # a slot already completed (then it is recycled and its output delivered)
        try:
            tickets.append(ctx.submit("fnv1a_64", *batches[2]))
            third = True
        except BlockingIOError:
            third = False
        for tk, out in tickets:
            ctx.wait(tk)
        for (k, o), (_, out) in zip(batches[: len(tickets)], tickets):
            np.testing.assert_array_equal(out, oracle.batch(6, k, o))
        # poll loop over the rest, the way core_loop would
        pending = []
        for k, o in batches[(3 if third else 2):]:
            while True:
                try:
                    pending.append((ctx.submit("md5", k, o), k, o))
                    break
                except BlockingIOError:
                    for (tk, _), _, _ in pending:
                        ctx.poll(tk)
        for (tk, out), k, o in pending:
            while not ctx.poll(tk):
                pass
            np.testing.assert_array_equal(out, oracle.batch(1, k, o))


def test_context_spans_from_mbuf(gpu, oracle):
    """Keys borrowed from a 16 KiB mbuf-like buffer as (start, end) spans."""
    rng = np.random.default_rng(5)
    mbuf = rng.integers(0x21, 0x7F, size=16336, dtype=np.uint8)
    spans, pos = [], 0
    while True:
        n = int(rng.integers(1, 64))
        if pos + n + 2 > mbuf.size:
            break
        spans.append((pos, pos + n))
        pos += n + 2  # "\r\n"-like separator between keys
    with t.Context(max_keys=2048, max_key_bytes=1 << 16) as ctx:
        tk, out = ctx.submit_spans("fnv1a_64", mbuf, spans)
        ctx.wait(tk)
    want = [oracle.hash(6, mbuf[s:e].tobytes()) for s, e in spans]
    assert out.tolist() == want


def test_context_limits(gpu):
    with t.Context(max_keys=16, max_key_bytes=64) as ctx:
        k, o = t.pack_keys([b"x" * 10] * 17)
        with pytest.raises(t.NcError):  # NC_ENOMEM: too many keys
            ctx.submit("md5", k, o)
        k, o = t.pack_keys([b"x" * 65])
        with pytest.raises(t.NcError):  # NC_ENOMEM: too many bytes
            ctx.submit("md5", k, o)
        with pytest.raises(ValueError):
            ctx.submit("sha1", k, o)


@pytest.mark.parametrize("zc", [1 << 14, 1 << 40])
def test_context_zero_copy(gpu, oracle, zc):
    """Zero-copy batches (kernel over mapped pinned staging) and copied ones
    mixed in one context, every mode, ragged sizes, spans."""
    with t.Context(max_keys=20000, max_key_bytes=1 << 20, nslots=3, zero_copy_bytes=zc) as ctx:
        for i, n in enumerate((1, 255, 798, 3000, 20000)):
            k, o = t.synth_host(t.SynthSpec.zipf(40 + i, charset=t.BYTES_PRINTABLE), 0, n)
            for m in range(12):
                tk, out = ctx.submit(m, k, o)
                ctx.wait(tk)
                np.testing.assert_array_equal(out, oracle.batch(m, k, o), err_msg=f"n={n} mode={m}")


def test_context_shared_by_worker_threads(gpu, oracle):
    """one context, 4 threads each submitting and polling its
    own batches (slot state is under the context's lock). Every output must be
    delivered to its own batch exactly, whichever thread recycles the slot."""
    import threading

    batches = [t.synth_host(t.SynthSpec.zipf(100 + i), 0, 700 + 37 * i) for i in range(4 * 12)]
    want = [oracle.batch(6 if i % 2 == 0 else 1, k, o) for i, (k, o) in enumerate(batches)]
    errors = []
    with t.Context(max_keys=4096, max_key_bytes=1 << 18, nslots=3) as ctx:
        def worker(w):
            try:
                for j in range(w, len(batches), 4):
                    k, o = batches[j]
                    while True:
                        try:
                            tk, out = ctx.submit("fnv1a_64" if j % 2 == 0 else "md5", k, o)
                            break
                        except BlockingIOError:
                            pass
                    while not ctx.poll(tk):
                        pass
                    if not np.array_equal(out, want[j]):
                        errors.append(j)
            except Exception as e:  # reported below, never swallowed
                errors.append(repr(e))

        threads = [threading.Thread(target=worker, args=(w,)) for w in range(4)]
        for th in threads:
            th.start()
        for th in threads:
            th.join(120)
        assert not any(th.is_alive() for th in threads)
    assert errors == []


@pytest.mark.parametrize("chunk", [(1000, 1 << 14, 2), (4096, 1 << 16, 3), (1 << 20, 1 << 24, 4)],
                         ids=["tiny2", "small3", "big4"])
def test_pinned_pipe_matches_oracle(gpu, oracle, chunk):
    """nc_gpuhash_batch_pinned over torch-pinned host CSRs: many chunks
    (keys cut by the key and byte limits), mixed lengths incl. empty and long
    keys, every mode, against the oracle."""
    import torch

    ck, cb, depth = chunk
    keys_np, off_np = t.synth_host(t.SynthSpec.uniform(77, 0, 700), 0, 30001)
    keys = torch.from_numpy(keys_np).pin_memory()
    off = torch.from_numpy(off_np.astype(np.int64)).pin_memory()
    out = torch.empty(30001, dtype=torch.int32).pin_memory()
    with t.Pipe(0, ck, cb, depth) as p:
        for m in range(12):
            want = oracle.batch(m, keys_np, off_np)
            out.fill_(0)
            p.hash(m, keys, off, out, shape=t.shape_of(off_np))
            np.testing.assert_array_equal(out.numpy().view(np.uint32), want,
                                          err_msg=f"mode {t.HASH_NAMES[m]} chunk={chunk}")


def test_pinned_pipe_registered_numpy_and_limits(gpu, oracle):
    """host_register'ed numpy buffers (a proxy pinning its mbuf arena), a
    batch whose offsets do not start at 0, and a key longer than a chunk."""
    import torch

    keys_np, off_np = t.synth_host(t.CONFIGS["C2"]["spec"], 5, 50000)
    off_np = off_np + np.uint64(0)  # own copy
    out = np.zeros(50000 - 7, dtype=np.uint32)
    for a in (keys_np, off_np, out):
        t.host_register(a.ctypes.data, a.nbytes)
    try:
        with t.Pipe(0, 1 << 12, 1 << 15, 2) as p:
            sub = off_np[7:]  # offsets[0] != 0
            p.hash("fnv1a_64", keys_np.ctypes.data, sub.ctypes.data, out.ctypes.data, nkeys=sub.size - 1)
            np.testing.assert_array_equal(out, oracle.batch(6, keys_np, off_np)[7:])
        big, boff = t.pack_keys([b"x" * 5000])
        with t.Pipe(0, 16, 4096, 2) as p:
            bk = torch.from_numpy(big).pin_memory()
            bo = torch.from_numpy(boff.astype(np.int64)).pin_memory()
            bout = torch.empty(1, dtype=torch.int32).pin_memory()
            with pytest.raises(t.NcError):
                p.hash("md5", bk, bo, bout)
            # good chunks first, then the key no chunk holds: the error comes
            # back only after every queued chunk finished (pipe_drain), so the
            # hashes before the failing key are all in `out` already
            small = [b"s%03d" % i for i in range(200)]
            mk, mo = t.pack_keys(small + [b"y" * 5000])
            mkt = torch.from_numpy(mk).pin_memory()
            mot = torch.from_numpy(mo.astype(np.int64)).pin_memory()
            mout = torch.zeros(201, dtype=torch.int32).pin_memory()
            with pytest.raises(t.NcError):
                p.hash("md5", mkt, mot, mout)
            assert mout.numpy().view(np.uint32)[:200].tolist() == [t.hash_key(1, k) for k in small]
    finally:
        for a in (keys_np, off_np, out):
            t.host_unregister(a.ctypes.data)


def test_pinned_pipe_rejects_short_buffers(gpu):
    """Pipe.hash on pinned tensors: a short `out` or a key buffer without
    NC_GPUHASH_PAD raises before any copy; the same tensors, right-sized,
    hash."""
    import torch

    keys_np, off_np = t.pack_keys([b"k%d" % i for i in range(100)])
    keys = torch.from_numpy(keys_np).pin_memory()
    off = torch.from_numpy(off_np.astype(np.int64)).pin_memory()
    out = torch.zeros(100, dtype=torch.int32).pin_memory()
    with t.Pipe(0, 64, 4096, 2) as p:
        with pytest.raises(ValueError):
            p.hash("fnv1a_64", keys, off, out[:99])
        with pytest.raises(ValueError):
            p.hash("fnv1a_64", keys[: int(off_np[-1])], off, out)
        assert int(out.abs().sum()) == 0  # nothing was written
        p.hash("fnv1a_64", keys, off, out)
    assert out.numpy().view(np.uint32).tolist() == [t.hash_key(6, b"k%d" % i) for i in range(100)]


def test_probe_mix_contract():
    """nc_gpuhash_probe_mix: a positive rate for every policy, EINVAL for an
    output buffer below ceil(bytes / 32768) * 4096 or an unknown policy."""
    import ctypes

    import torch

    import twemproxy_amd as t
    from twemproxy_amd import _lib as L

    buf = torch.randint(0, 256, (1 << 24,), dtype=torch.uint8, device="cuda")
    for pol in range(4):
        assert t.probe_mix_gbs(buf, 2, policy=pol) > 0
    need = -(-buf.numel() // 32768) * 4096
    wout = torch.empty(need, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(65536, dtype=torch.int32, device="cuda")
    ms = ctypes.c_float(0.0)
    f = L.lib().nc_gpuhash_probe_mix
    assert f(buf.data_ptr(), buf.numel(), wout.data_ptr(), need - 16, sink.data_ptr(), None, 0, 1,
             ctypes.byref(ms)) != 0
    assert f(buf.data_ptr(), buf.numel(), wout.data_ptr(), need, sink.data_ptr(), None, 4, 1, ctypes.byref(ms)) != 0
    assert f(buf.data_ptr(), buf.numel(), wout.data_ptr(), need, sink.data_ptr(), None, 0, 1, ctypes.byref(ms)) == 0
