#!/usr/bin/env python3
"""Committed PMC records from one tools/gpu_pmc_round.sh output directory.

    python tools/pmc_records.py gpurun_out/pmc_r03h profiles/r03h_bench.json C2:server_idx C2:md5 \
        > profiles/pmc_r03h.json

For every CFG:MODE it merges the four passes (<CFG>_<MODE>_0_p1..p4: FETCH_SIZE,
WRITE_SIZE and the two SQ groups, one rocprofv3 run each) of the hash kernel
(the dispatch with the most FETCH_SIZE), and derives what DESIGN.md quotes:
  hbm_read_bytes   = 2 x FETCH_SIZE x 1024 (gfx950 reports half, MI355X_MICROARCH.md)
  hbm_write_bytes  = WRITE_SIZE x 1024
  traffic_over_alg = (read + write) / the bench leg's algorithmic bytes
  kernel_cycles_per_xcd = GRBM_GUI_ACTIVE / 8
  valu_inst_per_simd_cycle = SQ_INSTS_VALU / (1024 SIMDs x kernel cycles)
  valu_issue_frac  = that x 3.5 (mean issue cycles of the VALU mix, measured
                     with tools/probes/md5_rate.hip: VOP3 ~4.2, VOP2 ~2.4)
  wait_any_over_wave_cycles = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  lds_bank_conflict_cycles_per_cu = SQ_LDS_BANK_CONFLICT / 256
  valu_lane_inst_over_alg_ops = 64 x SQ_INSTS_VALU / the leg's alg_ops_per_launch
                     (md5: 324 lane-ops per 64-byte block)
The algorithmic bytes (and md5 ops) come from the bench line's legs.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from pmc_summary import counters  # noqa: E402

SKIP = ("rocprim", "at::native", "__amd_rocclr")


def hash_kernel(res):
    cands = {k: v for k, v in res.items() if k and not any(s in k for s in SKIP)}
    return max(cands, key=lambda k: cands[k].get("FETCH_SIZE", 0.0)) if cands else None


def record(d, tag, alg):
    rec, kern = {}, None
    for p in (1, 2, 3, 4):
        path = os.path.join(d, f"{tag}_p{p}")
        csvs = [os.path.join(r, f) for r, _, fs in os.walk(path) for f in fs if f.endswith("counter_collection.csv")]
        if not csvs:
            continue
        res = counters(csvs[0])
        k = kern or hash_kernel(res)
        if k is None or k not in res:
            continue
        kern = k
        rec.update({c: round(v, 1) for c, v in res[k].items()
                    if not c.startswith("_") and c not in ("hbm_read_bytes_corrected", "hbm_write_bytes")})
    if kern is None:
        return None
    out = {"kernel": kern, **rec}
    if "FETCH_SIZE" in rec and "WRITE_SIZE" in rec:
        rd, wr = round(2 * rec["FETCH_SIZE"] * 1024), round(rec["WRITE_SIZE"] * 1024)
        out.update({"hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                    "alg_bytes_per_launch": alg, "traffic_over_alg": round((rd + wr) / alg, 4) if alg else None})
    if "GRBM_GUI_ACTIVE" in rec:
        cyc = rec["GRBM_GUI_ACTIVE"] / 8
        out["kernel_cycles_per_xcd"] = round(cyc)
        if "SQ_INSTS_VALU" in rec:
            v = rec["SQ_INSTS_VALU"] / (1024 * cyc)
            out["valu_inst_per_simd_cycle"] = round(v, 4)
            out["valu_issue_frac"] = round(3.5 * v, 3)
    if "SQ_WAIT_ANY" in rec and "SQ_WAVE_CYCLES" in rec:
        out["wait_any_over_wave_cycles"] = round(rec["SQ_WAIT_ANY"] / rec["SQ_WAVE_CYCLES"], 4)
    if "SQ_LDS_BANK_CONFLICT" in rec:
        out["lds_bank_conflict_cycles_per_cu"] = round(rec["SQ_LDS_BANK_CONFLICT"] / 256)
    return out


def leg_of(line, cfg, mode):
    """the bench line's leg for CFG:MODE (C4S = the C4 shard)"""
    if cfg == "C2":
        return {"fnv1a_64": line, "md5": line.get("md5"), "server_idx": line.get("server_idx_ketama")}.get(mode)
    if cfg == "C3":
        return line.get(f"c3_{mode}")
    if cfg in ("C4", "C4S"):
        return line.get("c4_shard", {}).get(mode)
    return None


def roofs(leg):
    return [leg[k] for k in ("roofline_hbm", "roofline", "roofline_valu") if isinstance(leg.get(k), dict)] if leg else []


def main():
    d, bench = sys.argv[1], json.load(open(sys.argv[2]))
    line = bench.get("plain_run", bench)
    work = {}
    for spec in sys.argv[3:]:
        cfg, mode = spec.split(":")
        rf = roofs(leg_of(line, cfg, mode))
        alg = next((r["alg_bytes_per_launch"] for r in rf if "alg_bytes_per_launch" in r), None)
        ops = next((r["alg_ops_per_launch"] for r in rf if "alg_ops_per_launch" in r), None)
        r = record(d, f"{cfg}_{mode}_0", alg)
        if r:
            if ops and "SQ_INSTS_VALU" in r:
                # md5: lane instructions issued (64 per wave instruction) over
                # the algorithm's 324 per 64-byte block
                r["valu_lane_inst_over_alg_ops"] = round(64 * r["SQ_INSTS_VALU"] / ops, 4)
            work.setdefault("C4" if cfg == "C4S" else cfg, {})[mode] = r
    print(json.dumps({"note": "per launch of the hash kernel; " + __doc__.split("derives what DESIGN.md quotes:")[0]
                      .strip().splitlines()[0] + " (tools/pmc_records.py)", "source": d, "workloads": work}, indent=1))


if __name__ == "__main__":
    main()
