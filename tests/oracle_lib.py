"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_hashkit.so")


def ensure_built() -> None:
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if path == ORACLE_SO:
            ensure_built()
        lib = ctypes.CDLL(path)
        lib.oracle_hash.restype = ctypes.c_uint32
        lib.oracle_hash.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
        lib.oracle_ketama_hash.restype = ctypes.c_uint32
        lib.oracle_ketama_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        lib.oracle_hash_batch.restype = ctypes.c_int
        lib.oracle_hash_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_int]
        lib.oracle_time_batch.restype = ctypes.c_double
        lib.oracle_time_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        lib.oracle_ketama_build.restype = ctypes.c_int
        lib.oracle_ketama_build.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint32]
        lib.oracle_mc_parse.restype = ctypes.c_int
        lib.oracle_mc_parse.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.oracle_redis_parse.restype = ctypes.c_int
        lib.oracle_redis_parse.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]
        lib.oracle_redis_class.restype = ctypes.c_int
        lib.oracle_redis_class.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        lib.oracle_ketama_build_live.restype = ctypes.c_int
        lib.oracle_ketama_build_live.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint32),
                                                 ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p, ctypes.c_uint32,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        lib.oracle_ketama_dispatch.restype = ctypes.c_uint32
        lib.oracle_ketama_dispatch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        lib.oracle_modula_build.restype = ctypes.c_int
        lib.oracle_modula_build.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_uint32]
        lib.oracle_modula_dispatch.restype = ctypes.c_uint32
        lib.oracle_modula_dispatch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        lib.oracle_server_idx_batch.restype = ctypes.c_int
        lib.oracle_server_idx_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        self.lib = lib

    def hash(self, mode: int, key: bytes) -> int:
        return int(self.lib.oracle_hash(mode, key, len(key)))

    def ketama_hash(self, key: bytes, alignment: int) -> int:
        return int(self.lib.oracle_ketama_hash(key, len(key), alignment))

    def batch(self, mode: int, keys: np.ndarray, offsets: np.ndarray, threads: int = 0) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        out = np.empty(n, dtype=np.uint32)
        if threads <= 0:
            threads = min(os.cpu_count() or 1, 16)
        rc = self.lib.oracle_hash_batch(mode, keys.ctypes.data, offsets.ctypes.data, n, out.ctypes.data, threads)
        assert rc == 0
        return out

    def time_batch(self, mode: int, keys: np.ndarray, offsets: np.ndarray, threads: int, reps: int) -> float:
        n = offsets.size - 1
        out = np.empty(n, dtype=np.uint32)
        return float(self.lib.oracle_time_batch(mode, keys.ctypes.data, offsets.ctypes.data, n,
                                                out.ctypes.data, threads, reps))

    def ketama_build(self, names: list[bytes], weights: list[int], live=None) -> tuple[np.ndarray, np.ndarray]:
        n = len(names)
        cap = 160 * n * n + 16
        vals = np.zeros(cap, dtype=np.uint32)
        idx = np.zeros(cap, dtype=np.uint32)
        lv = None if live is None else (ctypes.c_uint8 * n)(*[1 if x else 0 for x in live])
        cnt = self.lib.oracle_ketama_build_live((ctypes.c_char_p * n)(*names),
                                                (ctypes.c_uint32 * n)(*map(len, names)),
                                                (ctypes.c_uint32 * n)(*weights), lv, n, vals.ctypes.data,
                                                idx.ctypes.data, cap)
        assert cnt >= 0
        return vals[:cnt], idx[:cnt]

    def ketama_dispatch(self, vals: np.ndarray, idx: np.ndarray, h: int) -> int:
        return int(self.lib.oracle_ketama_dispatch(vals.ctypes.data, idx.ctypes.data, vals.size, h))

    def modula_build(self, weights: list[int]) -> np.ndarray:
        cap = sum(weights) + 1
        idx = np.zeros(cap, dtype=np.uint32)
        cnt = self.lib.oracle_modula_build((ctypes.c_uint32 * len(weights))(*weights), len(weights),
                                           idx.ctypes.data, cap)
        assert cnt >= 0
        return idx[:cnt]

    def mc_parse(self, stream: bytes, max_keys: int = 1 << 20, max_reqs: int = 1 << 20):
        """memcache retrieval-request stream -> (key spans [(start, len)], key_req, statuses, info)."""
        buf = np.frombuffer(stream, dtype=np.uint8) if len(stream) else np.zeros(1, np.uint8)
        ks = np.zeros(max_keys, np.uint64)
        kl = np.zeros(max_keys, np.uint32)
        kr = np.zeros(max_keys, np.uint32)
        st = np.zeros(max_reqs, np.int32)
        out = (ctypes.c_uint64 * 4)()
        rc = self.lib.oracle_mc_parse(buf.ctypes.data, len(stream), max_keys, ks.ctypes.data, kl.ctypes.data,
                                      kr.ctypes.data, st.ctypes.data, max_reqs, ctypes.byref(out, 0),
                                      ctypes.byref(out, 8), ctypes.byref(out, 16), ctypes.byref(out, 24))
        assert rc == 0
        nk, nr = int(out[0]), int(out[1])
        info = {"nkeys": nk, "nparsed": nr, "first_error": int(out[2]), "consumed": int(out[3])}
        return ks[:nk], kl[:nk], kr[:nk], st[:nr], info

    def redis_parse(self, stream: bytes, max_key_len: int = 16336, max_keys: int = 1 << 20,
                    max_reqs: int = 1 << 20):
        """RESP request stream -> (key starts, key lengths, key_req, statuses, info), like mc_parse."""
        buf = np.frombuffer(stream, dtype=np.uint8) if len(stream) else np.zeros(1, np.uint8)
        ks = np.zeros(max_keys, np.uint64)
        kl = np.zeros(max_keys, np.uint32)
        kr = np.zeros(max_keys, np.uint32)
        st = np.zeros(max_reqs, np.int32)
        out = (ctypes.c_uint64 * 4)()
        rc = self.lib.oracle_redis_parse(buf.ctypes.data, len(stream), max_key_len, max_keys, ks.ctypes.data,
                                         kl.ctypes.data, kr.ctypes.data, st.ctypes.data, max_reqs,
                                         ctypes.byref(out, 0), ctypes.byref(out, 8), ctypes.byref(out, 16),
                                         ctypes.byref(out, 24))
        assert rc == 0
        nk, nr = int(out[0]), int(out[1])
        info = {"nkeys": nk, "nparsed": nr, "first_error": int(out[2]), "consumed": int(out[3])}
        return ks[:nk], kl[:nk], kr[:nk], st[:nr], info

    def redis_class(self, name: bytes) -> int:
        return self.lib.oracle_redis_class(name, len(name))

    def modula_dispatch(self, idx: np.ndarray, h: int) -> int:
        return int(self.lib.oracle_modula_dispatch(idx.ctypes.data, idx.size, h))

    def server_idx_batch(self, mode: int, dist: int, vals, idx, nserver: int, tag, keys: np.ndarray,
                         offsets: np.ndarray) -> np.ndarray:
        """server_pool_idx per key (src/nc_server.c:647-700); vals may be None for modula."""
        idx = np.ascontiguousarray(idx, dtype=np.uint32)
        vals = idx if vals is None else np.ascontiguousarray(vals, dtype=np.uint32)
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        out = np.empty(n, dtype=np.uint32)
        rc = self.lib.oracle_server_idx_batch(mode, dist, vals.ctypes.data, idx.ctypes.data, idx.size, nserver, tag,
                                              keys.ctypes.data, offsets.ctypes.data, n, out.ctypes.data)
        assert rc == 0
        return out


class RefHashkit:
    """The real reference hashkit (oracle/_ref), when it has been built."""

    def __init__(self, path: str = REF_SO):
        lib = ctypes.CDLL(path)
        lib.ref_hash_batch.restype = ctypes.c_int
        lib.ref_hash_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_int]
        lib.ref_time_batch.restype = ctypes.c_double
        lib.ref_time_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        self.lib = lib

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_SO)

    def batch(self, mode: int, keys: np.ndarray, offsets: np.ndarray, threads: int = 1) -> np.ndarray:
        n = offsets.size - 1
        out = np.empty(n, dtype=np.uint32)
        assert self.lib.ref_hash_batch(mode, keys.ctypes.data, offsets.ctypes.data, n, out.ctypes.data, threads) == 0
        return out

    def time_batch(self, mode: int, keys: np.ndarray, offsets: np.ndarray, threads: int, reps: int) -> float:
        n = offsets.size - 1
        out = np.empty(n, dtype=np.uint32)
        return float(self.lib.ref_time_batch(mode, keys.ctypes.data, offsets.ctypes.data, n, out.ctypes.data,
                                             threads, reps))

    def build_continuum(self, dist: int, names: list[bytes], weights: list[int]) -> tuple[np.ndarray, np.ndarray]:
        """The reference's own ketama_update (dist 0) / modula_update (1) over
        all-live servers (oracle/ref_driver.c ref_build_continuum)."""
        n = len(names)
        cap = 160 * n * n + sum(weights) + 16
        vals = np.zeros(cap, dtype=np.uint32)
        idx = np.zeros(cap, dtype=np.uint32)
        f = self.lib.ref_build_continuum
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint32),
                      ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_uint32]
        cnt = f(dist, (ctypes.c_char_p * n)(*names), (ctypes.c_uint32 * n)(*map(len, names)),
                (ctypes.c_uint32 * n)(*weights), n, vals.ctypes.data, idx.ctypes.data, cap)
        assert cnt >= 0
        return vals[:cnt], idx[:cnt]
