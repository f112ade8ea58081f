"""The drop-in claim of INTEGRATION.md §1, executed (CPU): the reference's own
src/hashkit/nc_ketama.c and nc_modula.c (compiled where they lie under
/root/reference, no reference hash algorithm object) linked with
oracle/link_compat.c against libnc_gpuhash.so's per-key symbols
(oracle/Makefile target `link-compat`).

- every hash_<name> and md5_signature is an undefined dynamic symbol of the
  program, so the library provides it;
- the checks of test_hash_algorithms (src/test_all.c:41-60) pass;
- the reference's ketama_update / modula_update, running on the library's
  md5_signature, build the same continua as the compiled reference hashkit;
- server_pool_hash + dispatch (src/nc_server.c:630-700) through the
  reference's hash_t table order gives the oracle's server indices.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from tests.oracle_lib import Oracle, RefHashkit

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "link_compat")
NAMES = ("one_at_a_time", "md5", "crc16", "crc32", "crc32a", "fnv1_64", "fnv1a_64", "fnv1_32", "fnv1a_32",
         "hsieh", "murmur", "jenkins")


@pytest.fixture(scope="module")
def exe():
    if not os.path.isdir("/root/reference/src/hashkit"):
        pytest.skip("needs /root/reference (the reference's ketama/modula sources)")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "link-compat"], check=True)
    return EXE


def run(exe, *args):
    p = subprocess.run([exe, *args], capture_output=True, text=True, check=True, timeout=60)
    return json.loads(p.stdout)


def test_hash_symbols_come_from_the_library(exe):
    dyn = subprocess.run(["nm", "-D", exe], capture_output=True, text=True, check=True).stdout.split("\n")
    undef = {ln.split()[-1] for ln in dyn if ln.strip().startswith("U ")}
    for name in NAMES:
        assert "hash_" + name in undef, name
    assert "md5_signature" in undef
    # and nothing in the program itself defines one
    full = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    defined = {ln.split()[-1] for ln in full.split("\n") if len(ln.split()) == 3 and ln.split()[1] in "TtWw"}
    assert not defined & ({"hash_" + n for n in NAMES} | {"md5_signature"})
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
    assert "libnc_gpuhash.so" in ldd


def test_test_all_hash_algorithms(exe):
    """src/test_all.c:41-60 expected values (tests/golden/kat.json holds the
    same numbers, produced by the compiled reference)."""
    got = run(exe, "kat")
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))
    assert got["kat"] == kat["apple"]
    assert got["kat"]["fnv1a_64"] == 1488911807 and got["kat"]["md5"] == 3195025439
    assert got["ketama_hash"] == [3853726576, 2667054752]


@pytest.mark.parametrize("dist", ["ketama", "modula"])
@pytest.mark.parametrize("weights", [[1, 1], [1, 2, 1, 1, 3], [5] * 9, [1, 3, 2, 7, 1, 1, 4, 2, 9, 1, 1, 1]])
def test_reference_continuum_and_dispatch(exe, dist, weights):
    got = run(exe, "pool", dist, str(len(weights)), *map(str, weights))
    names = [f"10.0.{s}.1:11211".encode() for s in range(len(weights))]
    vals = np.array(got["values"], np.uint32)
    idx = np.array(got["indices"], np.uint32)
    if RefHashkit.available():  # the compiled reference, all of its own hashkit
        ref = RefHashkit()
        rv, ri = ref.build_continuum(0 if dist == "ketama" else 1, names, weights)
        np.testing.assert_array_equal(vals, rv)
        np.testing.assert_array_equal(idx, ri)
    oracle = Oracle()
    if dist == "ketama":
        ov, oi = oracle.ketama_build(names, weights)
        np.testing.assert_array_equal(vals, ov)
        np.testing.assert_array_equal(idx, oi)
    keys = [b"key:%d" % i for i in range(4096)]
    buf = np.frombuffer(b"".join(keys) + bytes(64), np.uint8)
    off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=off[1:])
    for m, name in enumerate(NAMES):
        want = oracle.server_idx_batch(m, 0 if dist == "ketama" else 1, vals if dist == "ketama" else None, idx,
                                       len(weights), None, buf, off)
        np.testing.assert_array_equal(np.array(got["server_idx"][name], np.uint32), want, err_msg=f"{dist} {name}")
