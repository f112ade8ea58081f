"""The printed bench line keeps every kernel leg inside the driver's record.

The driver stores the last 2000 characters of a bench run's output (stdout,
then stderr), so `bench.summarize` orders the line with the kernel legs and
the north-star object last. This feeds it a record shaped like a full N = 1
run (the round-6 r06d figures, `profiles/r06d_bench.json`) and checks the
tail. CPU only: bench.py imports no torch at module level.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402


def _rf(frac, **kw):
    return {"bound": "hbm", "achieved": 5000.1, "peak": 8000.0, "unit": "GB/s", "frac": frac,
            "traffic": 9618684518, "traffic_over_alg": 1.0696, **kw}


def _full_record():
    res = json.load(open(os.path.join(os.path.dirname(HERE), "profiles", "r06d_bench.json")))["plain_run"]
    res = {k: v for k, v in res.items() if k in (
        "metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "gb_per_s_hashed", "kernel_ms_rank0", "kernel_ms_max",
        "variant", "roofline", "redis_key_extraction", "e2e_c2", "c4_ingest")}
    md5_rf = {"bound": "valu", "achieved": 30.894, "peak": 78.643, "unit": "Tlane-op/s", "frac": 0.3928,
              "frac_of_md5_compute_ceiling": 0.6792, "clock_mhz": 2160.0,
              "frac_of_md5_compute_ceiling_at_clock": 0.7505}
    res["md5"] = {"kernel_ms": 0.7297, "value": 91527.9, "unit": "Mkeys/s", "roofline": md5_rf,
                  "roofline_hbm": _rf(0.36)}
    res["server_idx_ketama"] = {"kernel_ms": 0.4682, "value": 142416.9, "unit": "Mkeys/s", "roofline": _rf(0.5611)}
    res["c3_fnv1a_64"] = {"kernel_ms": 0.5239, "value": 127754.0, "unit": "Mkeys/s", "roofline": _rf(0.7045)}
    res["c3_crc32"] = {"kernel_ms": 0.54, "value": 123854.5, "unit": "Mkeys/s", "roofline": _rf(0.6835),
                       "roofline_lds": {"bound": "lds", "frac": 0.2023, "achieved": 1.0, "peak": 2.0}}
    res["c3_md5"] = {"kernel_ms": 0.5934, "value": 112484.8, "unit": "Mkeys/s",
                     "roofline": dict(md5_rf, frac=0.4659), "roofline_hbm": _rf(0.622)}
    res["c4_shard"] = {m: {"kernel_ms": 1.79, "value": 18681.2, "unit": "Mkeys/s", "roofline": _rf(0.627)}
                       for m in ("md5", "crc32", "fnv1a_64")}
    res["c4_shard"]["md5"]["roofline_valu"] = md5_rf
    row = {"point": "gpu", "path": "ring (resident worker)", "staging": "device", "depth": 8, "lanes": 8,
           "threads": 1024, "batches": 320245, "keys_per_batch": 585.1, "submit_to_done_us": 9.71,
           "mkeys_s": 468.46, "mismatches": 0, "worker_launches": 1}
    res["c5_e2e"] = {"host_per_key": {"point": "host", "path": "host", "mkeys_s": 80.81},
                     "gpu": [dict(row, depth=d) for d in (1, 2, 4, 8, 16)] * 3,
                     "ring_best_depth_ge2_le20us": row, "mismatches": 0}
    res["parity"] = {"all": "ok", "per_rank": {k: ["ok"] for k in (
        "C2/fnv1a_64", "C2/md5", "C3/fnv1a_64", "C3/crc32", "C3/md5", "C4/md5", "C4/crc32", "C4/fnv1a_64")}}
    res["cpu_baseline"] = {"value": 1918.12, "unit": "Mkeys/s", "cores": 256, "kind": "reference",
                           "sample": "first 16777216 keys of the same workload (324040181 key bytes), fnv1a_64, "
                                     "best of 5 after a warm-up, per-key hash_t calls on 256 pthreads",
                           "threads_share": 16, "cpu_model": "AMD EPYC 9575F 64-Core Processor",
                           "detail": {"fnv1a_64": {"mkeys_s_1threads": 77.12},
                                      "md5": {"mkeys_s_256threads": 202.84}}}
    return res


def test_line_tail_holds_every_leg():
    line = bench.summarize(_full_record(), "gpurun_out/bench_detail.json")
    text = json.dumps(line, separators=(",", ":"))
    tail = text[-bench.TAIL_CHARS:]
    for needle in ('"c3_fnv1a_64":{"kernel_ms":0.5239', '"md5":{"kernel_ms":0.7297',
                   '"server_idx_ketama":{"kernel_ms":0.4682', '"c3_crc32":{"kernel_ms":0.54',
                   '"c3_md5":{"kernel_ms"', '"c4_shard":{"md5":{"kernel_ms"', '"north_star":{',
                   '"frac":0.7045', '"over_hash":'):
        assert needle in tail, (needle, len(text))
    back = json.loads(text)
    assert back["c3_fnv1a_64"]["roofline"]["frac"] == 0.7045
    assert back["north_star"]["met"] is True
    # the contract fields still lead the line
    assert list(back)[:3] == ["metric", "value", "unit"]
    assert back["roofline"]["frac"] and back["cpu_baseline"]["kind"] == "reference"
