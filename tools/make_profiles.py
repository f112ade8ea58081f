#!/usr/bin/env python3
"""Turn one tools/gpu_profile_round.sh output directory into the committed
profiles/ artifacts of a round:

  profiles/<round>_bench_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `python3 bench.py`
  profiles/<round>_bench_phases.json        per-phase kernel averages from the same trace, next
                                            to bench.py's own HIP-event kernel time
  profiles/<round>_bench.json               the bench line of the plain run (and the one under rocprof)
  profiles/pmc_<round>.json                 FETCH_SIZE / WRITE_SIZE per launch -> HBM bytes
                                            (gfx950 correction: read = 2 x FETCH_SIZE KB; MI355X_MICROARCH.md)
  profiles/<round>_e2e.jsonl                end-to-end host batch benchmark (tools/nc_e2e_bench)

    python tools/make_profiles.py gpurun_out/r01r r01
    python tools/make_profiles.py --modes gpurun_out/r01s r01   (tools/gpu_modes.sh output ->
                                                                 profiles/<round>_modes_c3.json)
"""
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "tools"))
from pmc_summary import counters  # noqa: E402

# bench.py's launch order on one GPU: (label, timed launches) -- see bench.py main(). Each phase
# starts with a time-bounded untimed spin-up and W warm-ups, so only its last `timed` dispatches count.
BENCH_PHASES = [("C2 fnv1a_64", 20), ("C2 md5", 10), ("C2 server_idx ketama", 10), ("C3 fnv1a_64", 20),
                ("C3 crc32", 20), ("C3 md5", 10), ("C4 md5", 10), ("C4 crc32", 10), ("C4 fnv1a_64", 10)]
# the PMC passes of tools/gpu_profile_round.sh: (config dir name, bench workload key, mode)
PMC_LEGS = [("C2", "C2", "fnv1a_64"), ("C2", "C2", "md5"), ("C2", "C2", "server_idx"), ("C3", "C3", "fnv1a_64"),
            ("C3", "C3", "crc32"), ("C3", "C3", "md5"), ("C4S", "C4", "md5"), ("C4S", "C4", "crc32"),
            ("C4S", "C4", "fnv1a_64")]
HASH_KERNELS = ("nc_hash_kernel", "nc_md5_", "nc_bytes_direct", "nc_bytes_short")


def is_hash_kernel(name):
    return any(k in name for k in HASH_KERNELS)


def hash_phases(trace_csv):
    """consecutive runs of nc_hash_kernel dispatches, split where another kernel
    runs; the launches bench.py's clock_under makes beside the clock sampler
    (after a leg's timed region, round 6) are dropped, sampler included"""
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    samp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "clock_sampler" in r["Kernel_Name"]]

    def beside_sampler(r):
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        return any(a <= t1 and t0 <= b for a, b in samp)

    rows = [r for r in rows if "clock_sampler" not in r["Kernel_Name"] and not beside_sampler(r)]
    runs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if is_hash_kernel(name):
            short = name.replace("void (anonymous namespace)::", "").split("(")[0]
            if cur is None or cur["kernel"] != short:
                cur = {"kernel": short, "ns": []}
                runs.append(cur)
            cur["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        else:
            cur = None
    return runs


MODE_NAMES = ["one_at_a_time", "md5", "crc16", "crc32", "crc32a", "fnv1_64", "fnv1a_64", "fnv1_32", "fnv1a_32",
              "hsieh", "murmur", "jenkins"]


def modes(src, rnd):
    """all 12 modes on C3: in-process sweep (3 variants), kernel-trace stats and PMC bytes per launch"""
    import re

    dst = os.path.join(HERE, "profiles")
    rows = [json.loads(l) for l in open(os.path.join(src, "sweep.log")) if l.startswith("{")]
    probe = [r for r in rows if "probe_read_gbs" in r]
    alg = 2 ** 31 + 12 * 2 ** 26
    res = {"workload": "C3: 2^26 x 32 B keys, bytes 0x00-0xFF (seed 3)", "alg_bytes_per_launch": alg,
           "hbm_peak_gbs": 8000.0, "probe_read_gbs": probe[0]["probe_read_gbs"] if probe else None,
           "modes": {}}
    for r in rows:
        if "mode" not in r:
            continue
        key = f"grid{r['grid_cap']}_sort{r['sort']}_var{r['var']}"
        m = res["modes"].setdefault(r["mode"], {"sweep_ms_median": {}})
        m["sweep_ms_median"][key] = r["ms_median"]
    def mode_of_kernel(name):
        """hash mode of a kernel name: the first template argument, or md5 for its own kernels"""
        if "nc_md5_" in name:
            return "md5"
        mm = re.search(r"(?:nc_hash_kernel(?:_rs|_wr)?|nc_bytes_direct_kernel|nc_bytes_short_kernel)<(?:mode=)?(\d+)", name)
        return MODE_NAMES[int(mm.group(1))] if mm else None

    stats = os.path.join(src, "trace", "modes_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        name = mode_of_kernel(r["Name"])
        if name:
            res["modes"][name]["trace_kernel"] = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            res["modes"][name]["trace_kernel"] = res["modes"][name]["trace_kernel"].split("(")[0]
            res["modes"][name]["trace_avg_ms_auto"] = round(float(r["AverageNs"]) / 1e6, 4)
            res["modes"][name]["trace_calls"] = int(r["Calls"])
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for k, v in counters(os.path.join(src, f"pmc_{ctr}", "pmc_counter_collection.csv")).items():
            name = mode_of_kernel(k)
            if name:
                res["modes"][name][ctr + "_KB"] = v[ctr]
    for name, m in res["modes"].items():
        v0 = m["sweep_ms_median"].get("grid0_sort0_var0")  # var 0 = the shape policy's choice
        if v0:
            m["alg_gbs_auto"] = round(alg / (v0 * 1e-3) / 1e9, 1)
            m["frac_auto"] = round(m["alg_gbs_auto"] / 8000.0, 4)
        if "FETCH_SIZE_KB" in m and "WRITE_SIZE_KB" in m:
            m["hbm_bytes_per_launch"] = round(2.0 * m["FETCH_SIZE_KB"] * 1024 + m["WRITE_SIZE_KB"] * 1024)
            m["traffic_over_alg"] = round(m["hbm_bytes_per_launch"] / alg, 4)
    json.dump(res, open(os.path.join(dst, f"{rnd}_modes_c3.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


def main():
    if sys.argv[1] == "--modes":
        return modes(sys.argv[2], sys.argv[3])
    src, rnd = sys.argv[1], sys.argv[2]
    dst = os.path.join(HERE, "profiles")
    os.makedirs(dst, exist_ok=True)
    prof = os.path.join(src, "prof")
    shutil.copy(os.path.join(prof, "bench_kernel_stats.csv"), os.path.join(dst, f"{rnd}_bench_kernel_stats.csv"))

    bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
    under = json.loads(open(os.path.join(src, "bench_under_rocprof.json")).read().strip().splitlines()[-1])
    # (a launch or two of clock_under's that started before its sampler can
    # remain as a short run of its own: no leg has fewer than 5 dispatches)
    runs = [r for r in hash_phases(os.path.join(prof, "bench_kernel_trace.csv")) if len(r["ns"]) >= 5]
    # the device-resident legs come first; the end-to-end legs after them
    # launch the hash kernel per chunk, between copies (more runs)
    if len(runs) < len(BENCH_PHASES):
        raise SystemExit(f"expected {len(BENCH_PHASES)} hash-kernel phases, found {len(runs)}")
    runs = runs[: len(BENCH_PHASES)]
    event_ms = {"C2 fnv1a_64": under["kernel_ms_rank0"], "C2 md5": under["md5"]["kernel_ms"],
                "C2 server_idx ketama": under["server_idx_ketama"]["kernel_ms"],
                "C3 fnv1a_64": under["c3_fnv1a_64"]["kernel_ms"], "C3 crc32": under["c3_crc32"]["kernel_ms"],
                "C3 md5": under["c3_md5"]["kernel_ms"]}
    for m in ("md5", "crc32", "fnv1a_64"):
        if "c4_shard" in under:
            event_ms[f"C4 {m}"] = under["c4_shard"][m]["kernel_ms"]
    phases = []
    for (label, timed), run in zip(BENCH_PHASES, runs):
        ns = run["ns"]
        assert len(ns) > timed, (label, len(ns))
        t = ns[-timed:]
        ph = {"phase": label, "kernel": run["kernel"], "dispatches": len(ns), "timed": len(t),
              "avg_ms_timed": round(sum(t) / len(t) / 1e6, 4), "min_ms": round(min(t) / 1e6, 4),
              "max_ms": round(max(t) / 1e6, 4)}
        if label in event_ms:
            ph["bench_hip_event_ms"] = event_ms[label]
            ph["rel_diff"] = round(ph["avg_ms_timed"] / event_ms[label] - 1.0, 4)
        phases.append(ph)
    json.dump({"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py", "phases": phases},
              open(os.path.join(dst, f"{rnd}_bench_phases.json"), "w"), indent=1)
    json.dump({"plain_run": bench, "under_rocprof": under}, open(os.path.join(dst, f"{rnd}_bench.json"), "w"),
              indent=1)

    pmc = {"note": "per launch of the hash kernel; hbm_read = 2 x FETCH_SIZE x 1024 (gfx950 reports half "
                   "of a 16-B/lane stream, MI355X_MICROARCH.md HBM section), hbm_write = WRITE_SIZE x 1024; "
                   "one counter per rocprofv3 pass; inputs as bench.py (tools/pmc_run.py, variant 0:0:0)",
           "workloads": {}}
    for cdir, cfg, mode in PMC_LEGS:
        rec = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(src, f"pmc_{cdir}_{mode}_{ctr}", "pmc_counter_collection.csv")
            if not os.path.exists(d):
                continue
            hk = {k: v for k, v in counters(d).items() if is_hash_kernel(k)}
            if not hk:
                continue
            k, v = max(hk.items(), key=lambda kv: kv[1]["_dispatches"])  # the leg's kernel (5 launches)
            rec["kernel"] = k
            rec[ctr + "_KB"] = v[ctr]
            rec["dispatches"] = v["_dispatches"]
        if "FETCH_SIZE_KB" in rec and "WRITE_SIZE_KB" in rec:
            rd = 2.0 * rec["FETCH_SIZE_KB"] * 1024.0
            wr = rec["WRITE_SIZE_KB"] * 1024.0
            rec.update(hbm_read_bytes=round(rd), hbm_write_bytes=round(wr), hbm_bytes_per_launch=round(rd + wr))
            pmc["workloads"].setdefault(cfg, {})[mode] = rec
    json.dump(pmc, open(os.path.join(dst, f"pmc_{rnd}.json"), "w"), indent=1)
    for name in ("e2e", "c5"):
        f = os.path.join(src, f"{name}.jsonl")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(dst, f"{rnd}_{name}.jsonl"))
    print(json.dumps(phases, indent=1))
    print(json.dumps(pmc["workloads"], indent=1))


if __name__ == "__main__":
    main()
