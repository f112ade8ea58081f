#!/usr/bin/env python3
"""Generate the golden fixtures from the REAL reference hashkit.

Run in the build container (where /root/reference exists):

    make -C oracle ref && python tests/golden/make_golden.py

It loads oracle/_ref/libref_hashkit.so — twemproxy's own src/hashkit sources
compiled where they lie under /root/reference (oracle/Makefile) plus the thin
oracle/ref_driver.c — and writes only numbers (inputs and expected outputs):

  kat.json      the 12 "apple" KATs and 2 ketama_hash KATs of
                src/test_all.c:41-60, plus the SURVEY.md Appendix A pattern table
  corpus.npz    1024 keys of 0..300 random bytes x 12 modes
  digests.json  sha256 of the reference's u32 outputs over the synthetic
                configs C1/C2/C3/C5 (full size) and a C4 prefix, with sha256 of the
                generated inputs to pin the generator
  dist.json     ketama / modula continua built by the reference's own
                ketama_update / modula_update and dispatch results for sample hashes
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)

from twemproxy_amd import hashkit as hk  # noqa: E402  (input generator only)

REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_hashkit.so")


def load_ref():
    ref = ctypes.CDLL(REF_SO)
    ref.ref_hash.restype = ctypes.c_uint32
    ref.ref_hash.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    ref.ref_ketama_hash.restype = ctypes.c_uint32
    ref.ref_ketama_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
    ref.ref_hash_batch.restype = ctypes.c_int
    ref.ref_hash_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_void_p, ctypes.c_int]
    ref.ref_build_continuum.restype = ctypes.c_int
    ref.ref_build_continuum.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    ref.ref_dispatch.restype = ctypes.c_uint32
    ref.ref_dispatch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    assert ref.ref_nmodes() == 12
    return ref


def ref_batch(ref, mode, keys, offsets, threads=8):
    n = offsets.size - 1
    out = np.empty(n, dtype=np.uint32)
    rc = ref.ref_hash_batch(mode, keys.ctypes.data, offsets.ctypes.data, n, out.ctypes.data, threads)
    assert rc == 0
    return out


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def digest_sets() -> dict:
    """label -> (spec, keys, modes) of digests.json: every mode on C1, C2 and
    C3 (each C2 mode's shape-policy pipeline is checked at 2^26 keys)"""
    c = hk.CONFIGS
    return {"C1": (c["C1"]["spec"], c["C1"]["nkeys"], hk.HASH_NAMES),
            "C2": (c["C2"]["spec"], c["C2"]["nkeys"], hk.HASH_NAMES),
            "C3": (c["C3"]["spec"], c["C3"]["nkeys"], hk.HASH_NAMES),
            "C4_prefix_2^20": (c["C4"]["spec"], 1 << 20, ("md5", "crc32")),
            "C5": (c["C5"]["spec"], c["C5"]["nkeys"], ("fnv1a_64",)),
            "UNI_0_600": (hk.SynthSpec.uniform(6, 0, 600), 1 << 16, hk.HASH_NAMES)}


def digest_entry(ref, spec, n, modes, label, t0) -> dict:
    kb, ob = hk.synth_host(spec, 0, n)
    entry = {"spec": spec.__dict__, "nkeys": n, "key_bytes": int(ob[-1]),
             "sha256_keys": sha(kb[: int(ob[-1])]), "sha256_offsets": sha(ob), "modes": {}}
    for name in modes:
        out = ref_batch(ref, hk.HASH_NAMES.index(name), kb, ob)
        entry["modes"][name] = {"sha256": sha(out), "head": [int(x) for x in out[:8]],
                                "xor": int(np.bitwise_xor.reduce(out)), "sum": int(out.astype(np.uint64).sum())}
    print(f"  {label}: {n} keys, {time.time() - t0:.1f}s", flush=True)
    return entry


def main() -> None:
    ref = load_ref()
    t0 = time.time()
    if len(sys.argv) > 2 and sys.argv[1] == "--digests":
        # refresh only the named digests.json entries (e.g. --digests C2)
        path = os.path.join(HERE, "digests.json")
        digests = json.load(open(path))
        sets = digest_sets()
        for label in sys.argv[2:]:
            spec, n, modes = sets[label]
            digests[label] = digest_entry(ref, spec, n, modes, label, t0)
        with open(path, "w") as f:
            json.dump(digests, f, indent=1)
        return

    # 1. KATs (src/test_all.c:41-60) and the Appendix A pattern table
    apple = {name: int(ref.ref_hash(m, b"apple", 5)) for m, name in enumerate(hk.HASH_NAMES)}
    ket = {str(a): int(ref.ref_ketama_hash(b"server1-8", 9, a)) for a in range(4)}
    pattern = bytes(((i * 131 + 7) & 0xFF) for i in range(512))
    lens = [0, 1, 2, 3, 4, 5, 7, 8, 11, 12, 13, 24, 25, 55, 56, 63, 64, 65, 119, 120, 127, 128, 129, 250, 300, 511]
    table = {str(n): [int(ref.ref_hash(m, pattern[:n], n)) for m in range(12)] for n in lens}
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"source": "oracle/_ref (reference src/hashkit compiled from /root/reference)",
                   "modes": list(hk.HASH_NAMES), "apple": apple, "ketama_server1-8": ket,
                   "pattern": "buf[i] = (i*131+7) & 0xff", "pattern_table": table}, f, indent=1)

    # 2. random corpus, every byte value, lengths 0..300
    rng = random.Random(20240611)
    keys = [bytes(rng.randrange(256) for _ in range(rng.choice((rng.randrange(0, 20), rng.randrange(0, 301)))))
            for _ in range(1024)]
    buf, off = hk.pack_keys(keys)
    exp = np.stack([ref_batch(ref, m, buf, off, 1) for m in range(12)])
    np.savez_compressed(os.path.join(HERE, "corpus.npz"), keys=buf, offsets=off, expected=exp)

    # 3. full-size synthetic configs
    digests = {label: digest_entry(ref, spec, n, modes, label, t0) for label, (spec, n, modes) in digest_sets().items()}
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=1)

    # 4. distributions built by the reference's ketama_update / modula_update
    dist = []
    sets = [
        ([b"127.0.0.1:11211", b"127.0.0.1:11212"], [1, 1]),
        ([b"server%d" % i for i in range(1, 9)], [1] * 8),
        ([b"10.0.0.%d:6379" % i for i in range(1, 6)], [1, 2, 3, 1, 5]),
        ([b"cache-%02d.example.com:11211" % i for i in range(20)], [(i % 4) + 1 for i in range(20)]),
    ]
    sample_hashes = np.array([rng.getrandbits(32) for _ in range(2000)] + [0, 1, 0xFFFFFFFF], dtype=np.uint32)
    for names, weights in sets:
        n = len(names)
        cn = (ctypes.c_char_p * n)(*names)
        cl = (ctypes.c_uint32 * n)(*[len(x) for x in names])
        cw = (ctypes.c_uint32 * n)(*weights)
        rec = {"names": [x.decode() for x in names], "weights": weights}
        for d, dname in enumerate(("ketama", "modula")):
            cap = 200000
            vals = np.zeros(cap, dtype=np.uint32)
            idxs = np.zeros(cap, dtype=np.uint32)
            np_ = ref.ref_build_continuum(d, cn, cl, cw, n, vals.ctypes.data, idxs.ctypes.data, cap)
            assert np_ > 0
            vals, idxs = vals[:np_], idxs[:np_]
            disp = [int(ref.ref_dispatch(d, vals.ctypes.data, idxs.ctypes.data, np_, int(h))) for h in sample_hashes]
            rec[dname] = {"values": vals.tolist(), "indices": idxs.tolist(), "dispatch": disp}
        dist.append(rec)
    with open(os.path.join(HERE, "dist.json"), "w") as f:
        json.dump({"sample_hashes": sample_hashes.tolist(), "pools": dist}, f)
    print(f"done in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
