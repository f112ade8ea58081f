"""bench.py's output contract on the device at reduced sizes: one JSON line
with the driver's fields, the roofline and cpu_baseline objects, every
secondary leg, and no PMC traffic borrowed from the full-size profiles."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


@pytest.fixture(scope="module")
def run(tmp_path_factory):
    import torch  # noqa: F401  (pages the image in before the child's own import)

    detail = str(tmp_path_factory.mktemp("bench") / "detail.json")
    cmd = [sys.executable, "-u", os.path.join(HERE, "bench.py"), "--steps", "3", "--warmup", "1",
           "--nkeys", str(1 << 20), "--c4-nkeys", str(1 << 16), "--cpu-sample", str(1 << 16), "--detail-out", detail]
    p = subprocess.run(cmd, cwd=HERE, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    rows = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(rows) == 1, p.stdout[-2000:]
    # the driver keeps the last 2000 characters of stdout + stderr: the line
    # ends with every kernel leg, and a plain run writes nothing on stderr
    # beyond the runtime's own notices
    assert len(p.stderr) < 600, p.stderr[-1000:]
    return rows[0], json.load(open(detail))


@pytest.fixture(scope="module")
def line(run):
    return json.loads(run[0])


def test_tail_holds_every_leg(run):
    tail = run[0][-1800:]
    for k in ('"c4_shard":', '"c3_md5":', '"c3_crc32":', '"server_idx_ketama":', '"md5":', '"c3_fnv1a_64":',
              '"north_star":'):
        assert k in tail, k


def test_driver_fields(line):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 3 and line["warmup"] == 1
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert line["higher_is_better"] is True and line["scaling"] == "weak"
    assert line["dtype"] == "u8" and line["unit"] == "Mkeys/s"
    assert "workload" in line["config"] and line["config"]["nkeys_per_gpu"] == 1 << 20
    # value is the wall clock over the K steps: keys / (ms_per_step) within rounding
    assert abs(line["value"] - (1 << 20) / (line["ms_per_step"] * 1e-3) / 1e6) <= 0.02 * line["value"] + 0.2


def test_roofline(line):
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert rf["achieved"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["traffic"] is None  # the committed PMC profiles are of 2^26 keys, not 2^20
    assert rf["alg_bytes_per_launch"] == line["config"]["key_bytes_rank0"] + 12 * (1 << 20)
    # the same-run mix ceiling (reads + 12.5 % writes; at this size the
    # buffer sits in the caches, so no ordering against the read probe)
    assert rf["mix_ceiling_gbs"] > 0
    assert abs(rf["frac_of_mix_ceiling"] - rf["achieved"] / rf["mix_ceiling_gbs"]) < 1e-3


def test_cpu_baseline(line):
    cb = line["cpu_baseline"]
    assert "error" not in cb, cb
    assert cb["value"] > 0 and cb["unit"] == "Mkeys/s" and cb["cores"] >= 1
    assert cb["kind"] in ("reference", "port") and cb["sample"]


def test_secondary_legs(line):
    for k in ("md5", "server_idx_ketama", "c3_fnv1a_64", "c3_crc32", "c3_md5", "c4_shard",
              "redis_key_extraction", "c5_e2e"):
        assert k in line, k
        assert "error" not in line[k], line[k]
    assert line["md5"]["roofline"]["bound"] == "valu" and line["md5"]["roofline_hbm"]["bound"] == "hbm"
    for k in ("md5", "c3_fnv1a_64", "c3_crc32", "c3_md5", "server_idx_ketama"):
        assert line[k]["kernel_ms"] > 0
    for mode in ("md5", "crc32", "fnv1a_64"):
        assert line["c4_shard"][mode]["kernel_ms"] > 0
        # no PMC traffic borrowed from the full-size profiles, in the line or the detail file
        assert "traffic_over_alg" not in line["c4_shard"][mode]["roofline"]


def test_detail_record(run):
    detail = run[1]
    for mode in ("md5", "crc32", "fnv1a_64"):
        assert detail["c4_shard"][mode]["roofline"]["traffic"] is None
    assert len(detail["c5_e2e"]["gpu"]) >= 2


def test_north_star_and_summary(line):
    ns = line["north_star"]
    assert ns["kernel_ms"] == line["c3_fnv1a_64"]["kernel_ms"] and ns["frac"] == line["c3_fnv1a_64"]["roofline"]["frac"]
    assert ns["target_frac"] == 0.70 and ns["met"] == (ns["frac"] >= 0.70)
    # the line is a summary: per-depth C5 rows live in the detail file only
    assert "gpu" not in line["c5_e2e"] and line["c5_e2e"]["mismatches"] == 0
    # 2^20 keys has no reference digest ("unpinned"); a mismatch would be named in "bad"
    assert line["parity"]["all"] in ("ok", "unpinned") and line["parity"]["bad"] == []
