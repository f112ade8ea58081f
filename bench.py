#!/usr/bin/env python3
"""Benchmark of the MI355X batched key hasher (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts N rank processes itself)
    torchrun --nproc-per-node N ... bench.py --gpus N ...   (one rank per GPU, RCCL)

Headline (BASELINE.json configs[1]): fnv1a_64 over 2^26
keys per GPU with Zipf lengths 8-64 B (s = 1.0), synthetic bytes 0x00-0xFF,
device-resident. A step = one kernel pass over one rank's batch. For N > 1
rank 0 generates all N x 2^26 keys and scatters byte-balanced ranges over
RCCL (grouped point-to-point); scatter time is reported separately and is
not part of `value` (weak scaling: fixed keys per GPU).

Rank 0 prints ONE JSON line (a summary whose last ~1800 characters hold every
kernel leg and the north-star object; the full record goes to
--detail-out). `value` = total keys hashed by all ranks per
second (Mkeys/s) over K timed steps, max over ranks. Beside it, each timed
with HIP events on the launch stream:
  md5         the same C2 keys (the metric's second mode), against the VALU
              issue ceiling as well as HBM;
  c3_*        2^26 x 32 B keys (configs[2]; the north-star 70 % target is
              quoted on fnv1a_64 here), crc32 with its LDS traffic, md5;
  c4_shard    one GPU's share of configs[3]: 2^25 x 256 B keys, md5, crc32
              and fnv1a_64; for N > 1 rank 0 generates all N shards and
              scatters them over RCCL first (configs[3]'s root scatter);
  server_idx  fused hash -> ketama dispatch on the C2 keys (§8f.1);
  redis_key_extraction  2^20 pipelined RESP GETs parsed on the device (§8f.4);
  c5_e2e      the pipelined GET replay (configs[4]) through the host batch
              API and the batch ring, PCIe-inclusive (tools/nc_c5_replay);
  cpu_baseline  the reference hashkit compiled from /root/reference, timed on
              this host (rank 0, N = 1).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md chip table
VALU_PEAK = 78.6432e12  # lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz (one wave64 op per 2 cycles)
LDS_PEAK_GBS = 78643.2  # ds_read_b32: 128 B/clk/CU x 256 CUs x 2.4 GHz (MI355X_MICROARCH.md LDS table)
MD5_OPS_PER_BLOCK = 324  # 64 steps x 5 VALU ops (F, 2 adds, rotate, add) + 4 state adds
SPINUP_S = 0.5  # untimed launches before the warm-up steps (clock ramp)
METRIC = "Mkeys/s + GB/s hashed (device-resident), fnv1a_64 & md5, 1/2/4/8 MI355X"


VERBOSE = False  # --verbose: progress notes on stderr (the driver's 2000-character tail takes stderr too)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def note(*a):
    if VERBOSE:
        log(*a)


T0 = time.monotonic()


class Record(dict):
    """the bench record; with --verbose each leg's arrival is a progress note
    (a long multi-rank run otherwise prints nothing until its line)"""

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        note(f"bench.py rank {os.environ.get('RANK', '0')}: {k} at {time.monotonic() - T0:.1f} s")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--nkeys", type=int, default=1 << 26, help="C2 keys per GPU")
    p.add_argument("--c4-nkeys", type=int, default=1 << 25, help="C4 keys per GPU (256 B each)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--no-extra", action="store_true", help="skip every secondary leg")
    p.add_argument("--no-c4", action="store_true", help="skip the C4 shard leg")
    p.add_argument("--cpu-sample", type=int, default=1 << 24, help="keys in the CPU baseline sample")
    p.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                   help="process-group backend for N > 1 (nccl = RCCL; gloo stages the scatter through host memory)")
    p.add_argument("--same-device", action="store_true",
                   help="every rank on cuda:0: the one-GPU rehearsal of the N > 1 code (tests/test_gpu_bench_dist.py)")
    p.add_argument("--launch-check", action="store_true",
                   help="start the ranks, rendezvous over gloo and report them; no device work (tests/test_launch.py)")
    p.add_argument("--detail-out", default=None,
                   help="where rank 0 writes the full record (default gpurun_out/bench_detail.json when that "
                        "directory exists); the printed line is its summary")
    p.add_argument("--verbose", action="store_true", help="progress notes on stderr")
    a = p.parse_args()
    global VERBOSE
    VERBOSE = a.verbose
    return a


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_devices() -> int:
    """GPUs this process may use. torch.cuda.device_count() does not
    initialise the GPU on this image, so the launching parent may call it."""
    import torch

    return torch.cuda.device_count()


def spawn_ranks(args) -> int | None:
    """`python3 bench.py --gpus N` with no launcher around it: start N fresh
    rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one per
    GPU) before this process touches any GPU, pass their output through, and
    return the worst child exit code. Returns None when this process is
    itself the rank to run (N = 1, or a launcher such as torch.distributed.run
    already set WORLD_SIZE — which must then equal --gpus)."""
    import signal

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            log(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
            return 2
        return None
    if args.gpus < 1:
        log(f"bench.py: --gpus {args.gpus} < 1")
        return 2
    if not args.same_device:
        ndev = visible_devices()
        if args.gpus > ndev:
            log(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) are visible")
            return 2
    if args.gpus == 1:
        return None
    port = str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]], env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    # a rank that fails leaves its peers blocked in a collective: give them a
    # grace period, then stop them (their exact PIDs, never a pattern)
    failed_at = None
    while any(p.poll() is None for p in procs):
        if failed_at is None and any(p.poll() not in (None, 0) for p in procs):
            failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > float(os.environ.get("NC_BENCH_GRACE_S", 30)):
            stop()
            for p in procs:
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.1)
    for p in procs:
        p.wait()
    # the first rank to fail names the job's failure (the ranks stopped after
    # it exit by SIGTERM)
    first = next((p.returncode for p in sorted(procs, key=lambda p: p.returncode in (-15, 143))
                  if p.returncode != 0), 0)
    return first if first >= 0 else 128 - first


def launch_check(args, world: int, rank: int, local: int) -> None:
    """--launch-check: the rendezvous the bench's ranks make, on gloo, with
    no device work; rank 0 prints every rank's view of the job."""
    import torch.distributed as dist

    if os.environ.get("NC_BENCH_FAIL_RANK") == str(rank):  # tests/test_launch.py: a rank that dies early
        sys.exit(3)
    me = {"rank": rank, "local_rank": local, "world": world, "pid": os.getpid()}
    views = [me]
    if world > 1:
        dist.init_process_group("gloo")
        views = [None] * world
        dist.all_gather_object(views, me)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "gpus_arg": args.gpus, "ranks": views}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def timed_steps(t, torch, mode, keys, off, out, steps, warmup, dist_on, shape=None, launch=None, key_end=None):
    """W untimed + K timed launches; wall time bracketed by barrier+sync,
    kernel time by HIP events recorded on the launch stream. `shape` is what
    the packer knows (key bytes, min/max length): it picks the pipeline.
    `launch(stream)` replaces the hash launch (the fused dispatch leg)."""
    if launch is None:
        def launch(stream=None):
            t.hash_batch_device(mode, keys, off, out, stream=stream, shape=shape, key_end=key_end)
    # device clocks ramp up under load: the first ~20 launches of a cold GPU
    # run 5-50 % slow (tools/timing_check.py), so spin for SPINUP_S untimed
    # before the W warm-up steps
    t_end = time.perf_counter() + SPINUP_S
    while time.perf_counter() < t_end:
        for _ in range(10):
            launch()
        torch.cuda.synchronize()
    for _ in range(warmup):
        launch()
    torch.cuda.synchronize()
    if dist_on:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        launch(stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    return wall, kern_ms


COMM_DEV = "cuda"  # where the small all-reduces live: cuda for nccl (RCCL), cpu for gloo


def max_over_ranks(torch, x: float, dist_on: bool) -> float:
    if not dist_on:
        return x
    import torch.distributed as dist

    v = torch.tensor([x], dtype=torch.float64, device=COMM_DEV)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return float(v.item())


def sum_over_ranks(torch, x: float, dist_on: bool) -> float:
    if not dist_on:
        return x
    import torch.distributed as dist

    v = torch.tensor([x], dtype=torch.float64, device=COMM_DEV)
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    return float(v.item())


def roofline(alg_bytes: float, kern_ms: float, traffic):
    """achieved = algorithmic bytes per launch / measured launch time; traffic =
    HBM bytes per launch from PMC counters (None when not measured)."""
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic["bytes_per_launch"] if traffic else None,
         "alg_bytes_per_launch": int(alg_bytes)}
    if traffic:
        r["traffic_source"] = traffic["source"]
        r["traffic_over_alg"] = round(traffic["bytes_per_launch"] / alg_bytes, 4)
    return r


def md5_ops(torch, off) -> float:
    """algorithmic VALU lane-ops of md5 over a batch: 324 per 64-byte block,
    floor((len + 8) / 64) + 1 blocks per key (the padding and the 64-bit
    length, src/hashkit/nc_md5.c:249-274)."""
    lens = off[1:] - off[:-1]
    return float(((lens + 8) // 64 + 1).sum().item()) * MD5_OPS_PER_BLOCK


def valu_roofline(ops: float, kern_ms: float, ceiling, clock_mhz=None):
    """md5's VALU roofline; with the clock the leg ran at (clock_under) also
    the ceiling scaled to that clock: the probe's rate x clock / the probe's
    own clock (the probe, VALU alone, holds ~2.37 GHz; the hash kernels,
    VALU under HBM traffic, run at 1.9-2.2 GHz)"""
    achieved = ops / (kern_ms * 1e-3)
    r = {"bound": "valu", "achieved": round(achieved / 1e12, 3), "peak": round(VALU_PEAK / 1e12, 3),
         "unit": "Tlane-op/s", "frac": round(achieved / VALU_PEAK, 4), "alg_ops_per_launch": int(ops),
         "ops_per_block": MD5_OPS_PER_BLOCK}
    if ceiling:
        r["md5_compute_ceiling"] = ceiling
        r["frac_of_md5_compute_ceiling"] = round(achieved / (ceiling["tlane_ops_s"] * 1e12), 4)
    if clock_mhz:
        r["clock_mhz"] = clock_mhz
        r["frac_of_peak_at_clock"] = round(achieved / (VALU_PEAK * clock_mhz / 2400.0), 4)
        if ceiling and ceiling.get("clock_mhz"):
            r["frac_of_md5_compute_ceiling_at_clock"] = round(
                achieved / (ceiling["tlane_ops_s"] * 1e12 * clock_mhz / ceiling["clock_mhz"]), 4)
    return r


def clock_under(t, torch, launch, samples=3000, gap=2000, tries=4):
    """Median shader clock (MHz) while `launch(stream)` runs back to back:
    one sampler wave (nc_gpuhash_probe_clock_sampler, launched first on its
    own high-priority stream) stamps s_memtime against the 100 MHz
    s_memrealtime every 20 us for 60 ms. Run after a leg's timed region,
    never inside it: md5 runs below the 2.4 GHz the VALU peak assumes (the
    board's power limit under VALU + HBM load, profiles/r06c_clock.json), and
    its compute ceiling is read at the clock it actually ran at. Two streams
    can land on one hardware queue, where the work would wait for the
    sampler and the sampler would see an idle GPU: a window the work did not
    fill (fewer launches than the window holds) is measured again on fresh
    streams; None if no try overlapped."""
    from twemproxy_amd import _lib as L

    dev = torch.cuda.current_device()
    buf = torch.zeros(2 * samples, dtype=torch.int64, device=dev)
    for attempt in range(tries):
        s_samp = torch.cuda.Stream(priority=-1)
        s_work = torch.cuda.Stream()
        torch.cuda.synchronize()
        L.check(L.lib().nc_gpuhash_probe_clock_sampler(buf.data_ptr(), samples, gap, s_samp.cuda_stream),
                "nc_gpuhash_probe_clock_sampler")
        done = torch.cuda.Event()
        done.record(s_samp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s_work)
        t0 = time.perf_counter()
        n = 0
        while not done.query() and time.perf_counter() - t0 < 5.0:
            with torch.cuda.stream(s_work):
                for _ in range(4):
                    launch(s_work)
                    n += 1
            s_work.synchronize()
        e1.record(s_work)
        torch.cuda.synchronize()
        a = buf.cpu().numpy().astype(np.int64)
        dc, dr = np.diff(a[0::2]), np.diff(a[1::2])
        window_ms = float(a[-1] - a[1]) / 1e5
        work_ms = e0.elapsed_time(e1)
        mhz = dc[dr > 0] / dr[dr > 0] * 100.0
        mid = mhz[int(0.1 * mhz.size): int(0.9 * mhz.size)]
        med = float(np.median(mid if mid.size else mhz))
        # the work must have been running for the whole window, and longer:
        # launches only stop once the sampler is done
        ok = n > 8 and work_ms >= 0.9 * window_ms
        note(f"clock_under try {attempt}: {n} launches over {work_ms:.1f} ms, window {window_ms:.1f} ms, "
            f"median {med:.1f} MHz{'' if ok else ' (no overlap: again)'}")
        if ok:
            return round(med, 1)
    return None


def md5_ceiling():
    """Compute-only md5 rate on this GPU (tools/probes/md5_rate: the kernel's
    61-step block on register-resident words, no memory traffic): the ceiling
    the VALU fraction is read against — md5's steps are half VOP3 ops, which
    issue at half the rate the nominal peak assumes."""
    exe = os.path.join(HERE, "tools", "probes", "md5_rate")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe], capture_output=True, text=True, timeout=60, check=True).stdout
    except Exception:
        return None
    rows = [r for r in (json.loads(l) for l in out.splitlines() if l.startswith("{")) if "ns_per_round_per_simd" in r]
    best = min(rows, key=lambda r: r["ns_per_round_per_simd"], default=None)
    if best is None:
        return None
    # one round = 64 lanes x one 61-step final block (61 x 5 ops + 1 add)
    ops = 64 * (61 * 5 + 1)
    c = {"tlane_ops_s": round(ops * 1024 / (best["ns_per_round_per_simd"] * 1e-9) / 1e12, 3),
         "source": f"tools/probes/md5_rate.hip (fastest of its step forms: form {best['form']}, "
                   f"{best['waves_per_simd']} waves/SIMD{', after 300 ms of sustained load' if best.get('sustained') else ''})"}
    if best.get("clock_mhz"):
        c["clock_mhz"] = best["clock_mhz"]
    return c


def read_ceiling(t, rf, buf):
    """Same-run STREAM-style read ceiling over the key buffer:
    the achievable HBM read rate on this box, after the timed region, with
    default and with non-temporal loads (the hash kernels stream with nt),
    and the read+write mix of a hash kernel (profiles/r03_cache_policy_ab.md)."""
    probe = t.probe_read_gbs(buf, 20)
    rf["read_ceiling_gbs"] = round(probe, 1)
    rf["frac_of_read_ceiling"] = round(rf["achieved"] / probe, 4)
    probe_nt = t.probe_read_gbs(buf, 20, nt=True)
    rf["read_ceiling_nt_gbs"] = round(probe_nt, 1)
    rf["frac_of_read_ceiling_nt"] = round(rf["achieved"] / probe_nt, 4)
    # a hash kernel also writes (4 B per key: ~12 % of C2's bytes); the mix
    # probe is the nt read plus one nt 16-B store per 128 B read
    mix = t.probe_mix_gbs(buf, 20)
    rf["mix_ceiling_gbs"] = round(mix, 1)
    rf["frac_of_mix_ceiling"] = round(rf["achieved"] / mix, 4)


SHARD_DIGESTS = os.path.join(HERE, "tests", "golden", "shard_digests.json")
_digests = None


def _load_digests():
    """{cfg: [entry, ...]}: the full-size entry ("configs") and the reduced
    sizes the multi-rank rehearsal runs at ("small", keyed by keys per rank)"""
    global _digests
    if _digests is None:
        _digests = {}
        try:
            d = json.load(open(SHARD_DIGESTS))
        except (OSError, ValueError):
            return
        for cfg, e in d.get("configs", {}).items():
            _digests.setdefault(cfg, []).append(e)
        for cfg, by_n in d.get("small", {}).items():
            _digests.setdefault(cfg, []).extend(by_n.values())


def digest_ranks(cfg: str, n_per_rank: int, world: int):
    """per-rank digest records of `cfg` at this size and N, or None"""
    _load_digests()
    for e in _digests.get(cfg, []):
        if e["n_per_rank"] == n_per_rank and str(world) in e["N"]:
            return e["N"][str(world)]
    return None


def rank_parity(torch, cfg: str, mode: str, out, first: int, nk: int, n_per_rank: int, world: int, rank: int):
    """This rank's outputs against the compiled reference's digest of its
    shard (tests/golden/shard_digests.json, made by
    tests/golden/make_shard_digests.py): "ok", "MISMATCH", or "unpinned"
    when this run's sizes or N have no digest. Outside every timed region."""
    import hashlib

    ranks = digest_ranks(cfg, n_per_rank, world)
    if ranks is None:
        return "unpinned"
    want = ranks[rank]
    if want["keys"] != [first, first + nk] or mode not in want:
        return "MISMATCH (key range)"
    got = hashlib.sha256(out[:nk].cpu().numpy().tobytes()).hexdigest()
    return "ok" if got == want[mode] else "MISMATCH"


def gather_parity(torch, status: str, dist_on: bool) -> list:
    """every rank's status, in rank order (on every rank)"""
    if not dist_on:
        return [status]
    import torch.distributed as dist

    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, status)
    return out


PROFILED_NKEYS = {"C2": 1 << 26, "C3": 1 << 26, "C4": 1 << 25}  # tools/pmc_run.py sizes
RUN_NKEYS = dict(PROFILED_NKEYS)  # this run's nominal keys per GPU (--nkeys / --c4-nkeys)


def load_traffic(kernel_mode: str, workload: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this
    workload (profiles/pmc_*.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950
    correction), or None when no such measurement exists or the batch is not
    the profiled size (PROFILED_NKEYS)."""
    import glob

    if PROFILED_NKEYS.get(workload) != RUN_NKEYS.get(workload):
        return None
    best = None
    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        rec = d.get("workloads", {}).get(workload, {}).get(kernel_mode)
        if rec and "hbm_bytes_per_launch" in rec:
            best = {"bytes_per_launch": rec["hbm_bytes_per_launch"], "source": os.path.relpath(path, HERE)}
    return best


def online_cores() -> int:
    """sysconf(_SC_NPROCESSORS_ONLN), bounded by this process's CPU affinity
    (SURVEY.md §8d / BASELINE.md: all online host cores)."""
    n = os.sysconf("SC_NPROCESSORS_ONLN")
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    return max(1, min(int(n), 256))  # oracle/ref_driver.c runs at most 256 pthreads


def cpu_baseline(t, spec, n, mode_names, reps=5):
    """Reference hashkit (oracle/_ref, compiled from /root/reference) or, when
    that build is absent, the repo's C restatement, timed on this host: one
    thread, and every online core (best of `reps` after a warm-up, per-key
    hash_t calls over byte-balanced contiguous ranges, BASELINE.md:40-44).
    The figure at the job's own CPU share (OMP_NUM_THREADS, 16 on the GPU
    box) is reported beside it."""
    from tests.oracle_lib import Oracle, RefHashkit

    if RefHashkit.available():
        impl, kind = RefHashkit(), "reference"
    else:
        impl, kind = Oracle(), "port"
    keys, off = t.synth_host(spec, 0, n)
    nbytes = int(off[-1])
    cores = online_cores()
    share = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or cores))
    res = {}
    for name in mode_names:
        m = t.HASH_NAMES.index(name)
        r = {}
        for th in sorted({1, share, cores}):
            s = impl.time_batch(m, keys, off, th, reps)
            r[f"mkeys_s_{th}threads"] = round(n / s / 1e6, 2)
            r[f"gbs_{th}threads"] = round(nbytes / s / 1e9, 3)
        res[name] = r
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    head = res[mode_names[0]]
    return {"value": head[f"mkeys_s_{cores}threads"], "unit": "Mkeys/s", "cores": cores, "kind": kind,
            "sample": f"first {n} keys of the same workload ({nbytes} key bytes), {mode_names[0]}, "
                      f"best of {reps} after a warm-up, per-key hash_t calls on {cores} pthreads (all online "
                      f"cores) over byte-balanced ranges; 1 thread, the job's {share}-thread CPU share and md5 "
                      f"alongside",
            "threads_share": share, "cpu_model": cpu_model, "detail": res}


def leg(t, torch, mode, keys, off, out, steps, warmup, dist_on, shape, key_end, nk, kb, workload, traffic_key):
    """one timed mode on one resident batch: value (all ranks), kernel ms, HBM roofline"""
    w, k = timed_steps(t, torch, mode, keys, off, out, steps, warmup, dist_on, shape, key_end=key_end)
    w = max_over_ranks(torch, w, dist_on)
    kmax = max_over_ranks(torch, k, dist_on)
    return {"workload": workload, "value": round(sum_over_ranks(torch, float(nk), dist_on) * steps / w / 1e6, 1),
            "unit": "Mkeys/s",
            "gb_per_s_hashed": round(sum_over_ranks(torch, float(kb), dist_on) * steps / w / 1e9, 2),
            "kernel_ms": round(k, 4), "kernel_ms_max": round(kmax, 4), "steps": steps,
            "variant": t.pick_variant(mode, nk, shape),
            "roofline": roofline(kb + 12.0 * nk, k, load_traffic(mode, traffic_key))}


def main():
    args = parse()
    rc = spawn_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    if args.launch_check:
        return launch_check(args, world, rank, local)
    import torch

    global COMM_DEV
    ndev = torch.cuda.device_count()
    if local >= ndev or (not args.same_device and world > ndev):
        log(f"bench.py: rank {rank} needs cuda:{local} of {world} ranks but {ndev} GPU(s) are visible")
        sys.exit(2)
    torch.cuda.set_device(local)
    dist_on = world > 1
    if dist_on:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
            COMM_DEV = "cpu"
    import twemproxy_amd as t
    from twemproxy_amd.shard import scatter_shards

    spec = t.CONFIGS["C2"]["spec"]
    n_local = args.nkeys
    RUN_NKEYS.update(C2=args.nkeys, C3=args.nkeys, C4=args.c4_nkeys)
    dev = torch.device("cuda", local)
    ceiling = md5_ceiling() if (rank == 0 and not args.no_extra) else None

    def resident(spec_, n_per_rank):
        """a config's keys on every rank before any timed region: generated
        locally at N = 1; at N > 1 generated on rank 0 and scattered"""
        if not dist_on:
            k_, o_ = t.synth_device(spec_, 0, n_per_rank, device=dev)
            return k_, o_, 0, None
        import torch.distributed as dist

        fk = fo = None
        if rank == 0:
            fk, fo = t.synth_device(spec_, 0, n_per_rank * world, device=dev)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        k_, o_, first_ = scatter_shards(fk, fo, dev)
        torch.cuda.synchronize()
        dist.barrier()
        sc = {"ms": round((time.perf_counter() - t0) * 1e3, 2),
              "root_egress_bytes": int(fk.numel() + fo.numel() * 8) if rank == 0 else 0,
              "how": (f"rank 0 -> every rank, one grouped batch_isend_irecv per round of <= 1 GiB pieces "
                      f"({'RCCL point-to-point over xGMI' if args.backend == 'nccl' else 'gloo, host-staged'})")}
        del fk, fo
        torch.cuda.empty_cache()
        return k_, o_, first_, sc

    # ---- headline: fnv1a_64 on C2
    keys, off, first, scatter = resident(spec, n_local)
    nk = off.numel() - 1
    key_bytes = int(off[-1].item())
    out = torch.empty(nk, dtype=torch.int32, device=dev)
    shape = spec.shape(key_bytes)
    wall, kern_ms = timed_steps(t, torch, "fnv1a_64", keys, off, out, args.steps, args.warmup, dist_on, shape,
                                key_end=key_bytes)
    wall = max_over_ranks(torch, wall, dist_on)
    kern_ms_max = max_over_ranks(torch, kern_ms, dist_on)
    total_keys = sum_over_ranks(torch, float(nk), dist_on) * args.steps
    total_bytes = sum_over_ranks(torch, float(key_bytes), dist_on) * args.steps
    value = total_keys / wall / 1e6
    alg = key_bytes + 12.0 * nk  # key bytes + u64 offset + u32 hash per key
    rf = roofline(alg, kern_ms, load_traffic("fnv1a_64", "C2"))
    read_ceiling(t, rf, keys)

    note(f"bench.py rank {rank}: C2 headline at {time.monotonic() - T0:.1f} s")
    res = Record({
        "metric": METRIC, "value": round(value, 1), "unit": "Mkeys/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 counter generator, SURVEY.md §8d seeds 2-5)",
        "config": {"workload": f"C2: fnv1a_64 over {n_local} keys per GPU, Zipf lengths 8-64 B (s=1.0, "
                               "mean ~19.3 B), bytes 0x00-0xFF, device-resident",
                   "hash": "fnv1a_64", "nkeys_per_gpu": n_local, "key_bytes_rank0": key_bytes,
                   "parallelism": f"shard{world}" if world > 1 else "single"},
        "gb_per_s_hashed": round(total_bytes / wall / 1e9, 2),
        "kernel_ms_rank0": round(kern_ms, 4), "kernel_ms_max": round(kern_ms_max, 4),
        "variant": t.pick_variant("fnv1a_64", nk, shape),
        "roofline": rf,
    })
    if scatter:
        res["scatter"] = scatter
    parity = {}

    def check(cfg, mode, out_, first_, nk_, per_rank):
        parity[f"{cfg}/{mode}"] = gather_parity(
            torch, rank_parity(torch, cfg, mode, out_, first_, nk_, per_rank, world, rank), dist_on)

    check("C2", "fnv1a_64", out, first, nk, n_local)

    if not args.no_extra:
        # ---- md5 on the same keys: HBM and VALU rooflines
        s5 = max(5, args.steps // 2)
        m = leg(t, torch, "md5", keys, off, out, s5, 1, dist_on, shape, key_bytes, nk, key_bytes,
                "C2 keys, md5", "C2")
        m["roofline_hbm"] = m.pop("roofline")
        clk = clock_under(t, torch, lambda st: t.hash_batch_device("md5", keys, off, out, stream=st, shape=shape,
                                                                   key_end=key_bytes))
        m["roofline"] = valu_roofline(md5_ops(torch, off), m["kernel_ms"], ceiling, clk)  # md5's binding ceiling
        res["md5"] = m
        check("C2", "md5", out, first, nk, n_local)
        # ---- fused server_pool_idx: fnv1a_64 + ketama_dispatch over
        # a synthetic sorted continuum of 8 servers x 160 points (LDS-staged)
        rng = np.random.default_rng(9)
        cvals = np.sort(rng.integers(0, 1 << 32, size=8 * 160, dtype=np.uint64)).astype(np.uint32)
        cidx = rng.integers(0, 8, size=cvals.size).astype(np.uint32)
        cont = t.continuum_device(cidx, cvals, device=dev)
        sidx = max(5, args.steps // 2)
        wd, kdd = timed_steps(t, torch, None, None, None, None, sidx, 1, dist_on, launch=lambda stream=None:
                              t.server_idx_device("fnv1a_64", "ketama", keys, off, cont, 8, out=out, stream=stream,
                                                  shape=shape, key_end=key_bytes))
        wd = max_over_ranks(torch, wd, dist_on)
        res["server_idx_ketama"] = {
            "workload": "C2 keys, fnv1a_64 + ketama_dispatch, 8 servers x 160 points (LDS-staged continuum)",
            "value": round(sum_over_ranks(torch, float(nk), dist_on) * sidx / wd / 1e6, 1), "unit": "Mkeys/s",
            "kernel_ms": round(kdd, 4), "roofline": roofline(alg, kdd, load_traffic("server_idx", "C2"))}
    del keys, off, out
    torch.cuda.empty_cache()

    if not args.no_extra:
        # ---- C3 shape: fnv1a_64 (the 70 % target), crc32 (+ its LDS traffic), md5
        c3 = t.CONFIGS["C3"]["spec"]
        keys3, off3, first3, sc3 = resident(c3, n_local)
        nk3 = off3.numel() - 1
        kb3 = int(off3[-1].item())
        out3 = torch.empty(nk3, dtype=torch.int32, device=dev)
        sh3 = c3.shape(kb3)
        f3 = leg(t, torch, "fnv1a_64", keys3, off3, out3, args.steps, args.warmup, dist_on, sh3, kb3, nk3, kb3,
                 f"C3: fnv1a_64 over {n_local} x 32 B keys per GPU", "C3")
        read_ceiling(t, f3["roofline"], keys3)
        res["c3_fnv1a_64"] = f3
        check("C3", "fnv1a_64", out3, first3, nk3, n_local)
        c = leg(t, torch, "crc32", keys3, off3, out3, args.steps, args.warmup, dist_on, sh3, kb3, nk3, kb3,
                f"C3: crc32 over {n_local} x 32 B keys per GPU", "C3")
        # one 4-byte table lookup per key byte (slicing-by-4 or -8; the policy's
        # short-key kernel uses slicing-by-8 in 8 copies)
        lds_bytes = kb3 * 4.0
        lds_gbs = lds_bytes / (c["kernel_ms"] * 1e-3) / 1e9
        c["roofline_lds"] = {"bound": "lds", "achieved": round(lds_gbs, 1), "peak": LDS_PEAK_GBS, "unit": "GB/s",
                             "frac": round(lds_gbs / LDS_PEAK_GBS, 4), "lds_bytes_per_launch": int(lds_bytes),
                             "note": "table reads only: 1 ds_read_b32 per key byte over 8 table copies"}
        res["c3_crc32"] = c
        check("C3", "crc32", out3, first3, nk3, n_local)
        m3 = leg(t, torch, "md5", keys3, off3, out3, max(5, args.steps // 2), 1, dist_on, sh3, kb3, nk3, kb3,
                 f"C3: md5 over {n_local} x 32 B keys per GPU", "C3")
        m3["roofline_hbm"] = m3.pop("roofline")
        clk3 = clock_under(t, torch, lambda st: t.hash_batch_device("md5", keys3, off3, out3, stream=st, shape=sh3,
                                                                    key_end=kb3))
        m3["roofline"] = valu_roofline(md5_ops(torch, off3), m3["kernel_ms"], ceiling, clk3)
        res["c3_md5"] = m3
        check("C3", "md5", out3, first3, nk3, n_local)
        if sc3:
            res["c3_scatter"] = sc3
        del keys3, off3, out3
        torch.cuda.empty_cache()

    if not args.no_extra and not args.no_c4:
        # ---- C4 shard: 256-byte keys, one GPU's share of configs[3] (scattered from rank 0 at N > 1)
        c4 = t.CONFIGS["C4"]["spec"]
        n4 = args.c4_nkeys
        keys4, off4, first4, sc4 = resident(c4, n4)
        nk4 = off4.numel() - 1
        kb4 = int(off4[-1].item())
        out4 = torch.empty(nk4, dtype=torch.int32, device=dev)
        sh4 = c4.shape(kb4)
        r4 = {"workload": f"C4 shard: {n4} x 256 B keys per GPU (BASELINE configs[3] is 2^28 keys over 8 GPUs)"}
        for mode in ("md5", "crc32", "fnv1a_64"):
            x = leg(t, torch, mode, keys4, off4, out4, 10, 1, dist_on, sh4, kb4, nk4, kb4, mode, "C4")
            x.pop("workload")
            if mode == "md5":
                clk4 = clock_under(t, torch, lambda st: t.hash_batch_device("md5", keys4, off4, out4, stream=st,
                                                                            shape=sh4, key_end=kb4))
                x["roofline_valu"] = valu_roofline(md5_ops(torch, off4), x["kernel_ms"], ceiling, clk4)
            r4[mode] = x
            check("C4", mode, out4, first4, nk4, n4)
        if sc4:
            r4["scatter"] = sc4
        res["c4_shard"] = r4
        del keys4, off4, out4
        torch.cuda.empty_cache()

    # ---- redis key extraction, rank 0: 2^20 pipelined RESP GETs over
    # the first C2 keys (binary-safe), parsed on the device into the CSR above
    if rank == 0 and not args.no_extra:
        try:
            res["redis_key_extraction"] = redis_leg(t, torch, np, spec, dev)
        except Exception as e:  # reported beside the headline, never instead of it
            res["redis_key_extraction"] = {"error": repr(e)}

    # ---- end to end from pinned host memory (PCIe-inclusive; never `value`):
    # the whole C2 batch on rank 0 at N = 1, and the §8e alternative ingest —
    # every rank pulls its own C4 shard H2D from pinned host memory and hashes it
    if not args.no_extra:
        if world == 1 and rank == 0:
            try:
                d2 = digest_ranks("C2", args.nkeys, 1)
                res["e2e_c2"] = e2e_leg(t, torch, "C2", spec, 0, args.nkeys, "fnv1a_64", dev, d2[0] if d2 else None,
                                        world, rank, dist_on)
            except Exception as e:
                res["e2e_c2"] = {"error": repr(e)}
        if not args.no_c4:
            try:
                n4 = args.c4_nkeys
                d4 = digest_ranks("C4", n4, world)
                res["c4_ingest"] = e2e_leg(t, torch, "C4 shard (per rank)", t.CONFIGS["C4"]["spec"], rank * n4, n4, "md5",
                                           dev, d4[rank] if d4 else None, world, rank, dist_on,
                                           chunk=(1 << 20, 1 << 28, 3))
            except Exception as e:
                res["c4_ingest"] = {"error": repr(e)}

    # ---- C5 pipelined GET replay through the host batch API (rank 0, N = 1)
    if rank == 0 and world == 1 and not args.no_extra:
        res["c5_e2e"] = c5_leg()

    # ---- every rank's outputs against the reference's per-shard digests
    flat = [v for st in parity.values() for v in st]
    res["parity"] = {"all": "ok" if flat and all(v == "ok" for v in flat) else
                     ("unpinned" if all(v == "unpinned" for v in flat) else "FAIL"),
                     "per_rank": parity,
                     "source": "tests/golden/shard_digests.json (sha256 of the compiled reference's outputs per rank)"}

    # ---- CPU baseline (rank 0, N = 1)
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            res["cpu_baseline"] = cpu_baseline(t, spec, args.cpu_sample, ["fnv1a_64", "md5"])
        except Exception as e:  # reported, never substituted for the GPU number
            res["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        path = args.detail_out
        if path is None and os.path.isdir(os.path.join(HERE, "gpurun_out")):
            path = os.path.join(HERE, "gpurun_out", "bench_detail.json")
        line = summarize(res, os.path.relpath(path, HERE) if path else None)
        if path:
            with open(path, "w") as f:
                json.dump(res, f, indent=1)
        print(json.dumps(line, separators=(",", ":")), flush=True)
    if dist_on:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


NORTH_STAR_FRAC = 0.70  # BASELINE.json north_star: >= 70 % of HBM peak on C3 fnv1a_64


TAIL_CHARS = 1800  # the driver keeps the last 2000 characters of stdout + stderr


def _rf(r: dict | None, keep=("bound", "frac", "traffic_over_alg", "clock_mhz",
                              "frac_of_md5_compute_ceiling_at_clock")) -> dict | None:
    if r is None:
        return None
    return {k: r[k] for k in keep if k in r}


def _leg(x: dict | None, extra=()) -> dict | None:
    """one leg of the full record, cut to kernel time and roofline fraction
    (rate, achieved/peak/traffic stay in the detail file)"""
    if x is None:
        return None
    if "error" in x:
        return {"error": x["error"][:200]}
    s = {k: x[k] for k in ("kernel_ms",) if k in x}
    if "roofline" in x:
        s["roofline"] = _rf(x["roofline"])
    for k in extra:
        if k in x:
            s[k] = _rf(x[k])
    return s


def summarize(res: dict, detail_path: str | None) -> dict:
    """The printed line. The driver parses the whole line but keeps only the
    last ~2000 characters of output in its record, so the order is: the
    contract fields, the headline roofline, cpu_baseline, parity and the
    end-to-end legs first; then every kernel leg cut to kernel time, rate and
    roofline fraction, ending with the C2 md5 leg, C3 fnv1a_64 and the
    north-star object, so that the record's tail holds all of them
    (`TAIL_CHARS`, checked by tests/test_bench_line.py). The whole record,
    per-depth C5 rows and ceilings included, goes to `detail_path`."""
    line = {k: res[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                                "gb_per_s_hashed", "kernel_ms_rank0", "kernel_ms_max", "variant", "roofline")
            if k in res}
    if "cpu_baseline" in res:
        cb = res["cpu_baseline"]
        line["cpu_baseline"] = cb if "error" in cb else {
            **{k: cb[k] for k in ("value", "unit", "cores", "kind", "sample", "threads_share", "cpu_model")},
            "mkeys_s_1thread": cb["detail"]["fnv1a_64"].get("mkeys_s_1threads"),
            "md5_mkeys_s_all_cores": cb["detail"].get("md5", {}).get(f"mkeys_s_{cb['cores']}threads")}
    par = res["parity"]
    line["parity"] = {"all": par["all"], "legs": len(par["per_rank"]),
                      "ranks": max((len(v) for v in par["per_rank"].values()), default=0),
                      "bad": sorted(k for k, v in par["per_rank"].items() if any(x not in ("ok", "unpinned") for x in v))}
    line["detail"] = detail_path
    r = res.get("redis_key_extraction")
    if r:
        line["redis_key_extraction"] = r if "error" in r else {k: r[k] for k in ("ms_per_parse_wall", "mreq_s")}
    for k in ("e2e_c2", "c4_ingest"):
        e = res.get(k)
        if e:
            line[k] = {kk: e[kk] for kk in ("ms", "value", "unit", "h2d_gbs", "frac_of_h2d_probe", "parity", "error")
                       if kk in e}
    c5 = res.get("c5_e2e")
    if c5:
        if "error" in c5:
            line["c5_e2e"] = c5
        else:
            def pt(r_):
                return None if r_ is None else {k: r_[k] for k in ("depth", "lanes", "threads", "staging",
                                                                   "submit_to_done_us", "us_per_batch", "mkeys_s")
                                                if k in r_}
            # one batch in flight: the faster worker shape (256- or 1024-thread lanes)
            ring1 = max((r_ for r_ in c5["gpu"] if r_["path"].startswith("ring") and r_["depth"] == 1),
                        key=lambda r_: r_["mkeys_s"], default=None)
            line["c5_e2e"] = {"host_per_key": pt(c5["host_per_key"]), "ring_depth1": pt(ring1),
                              "ring_best_depth_ge2_le20us": pt(c5["ring_best_depth_ge2_le20us"]),
                              "points": len(c5["gpu"]), "mismatches": c5["mismatches"]}
    for k in ("scatter", "c3_scatter"):
        if k in res:
            line[k] = res[k]
    # ---- the kernel legs: these make up the record's tail
    if "c4_shard" in res:
        c4 = res["c4_shard"]
        line["c4_shard"] = {m: _leg(c4[m], ("roofline_valu",)) for m in ("md5", "crc32", "fnv1a_64") if m in c4}
        if "scatter" in c4:
            line["c4_shard"]["scatter"] = c4["scatter"]
    for k in ("c3_md5", "c3_crc32"):
        if k in res:
            line[k] = _leg(res[k], ("roofline_lds", "roofline_hbm"))
    if "server_idx_ketama" in res:
        s = _leg(res["server_idx_ketama"])
        if "kernel_ms" in s and res.get("kernel_ms_rank0"):
            s["over_hash"] = round(s["kernel_ms"] / res["kernel_ms_rank0"] - 1.0, 4)
        line["server_idx_ketama"] = s
    if "md5" in res:
        line["md5"] = _leg(res["md5"], ("roofline_hbm",))
    if "c3_fnv1a_64" in res:
        line["c3_fnv1a_64"] = _leg(res["c3_fnv1a_64"])
    c3 = res.get("c3_fnv1a_64")
    if c3 and "roofline" in c3:
        rf = c3["roofline"]
        line["north_star"] = {"workload": "C3 fnv1a_64", "kernel_ms": c3["kernel_ms"],
                              "frac": rf["frac"], "target_frac": NORTH_STAR_FRAC,
                              "met": rf["frac"] >= NORTH_STAR_FRAC, "traffic": rf.get("traffic"),
                              "traffic_over_alg": rf.get("traffic_over_alg")}
    return line


def h2d_probe(torch, src, dev, reps=3):
    """Same-run PCIe H2D ceiling: GB/s of one hipMemcpyAsync of the pinned
    host tensor `src` into device memory (best of `reps`)."""
    dst = torch.empty(src.numel(), dtype=src.dtype, device=dev)
    best = None
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src, non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del dst
    return src.numel() * src.element_size() / (best * 1e-3) / 1e9


def pinned_copy(torch, x):
    h = torch.empty(x.numel(), dtype=x.dtype).pin_memory()
    h.copy_(x)
    return h


def e2e_leg(t, torch, cfg, spec, first, n, mode, dev, digest_rank, world, rank, dist_on, reps=3,
            chunk=(1 << 22, 1 << 26, 3)):
    """End to end from a host CSR in pinned memory: chunked
    H2D -> kernel -> D2H over the whole batch (nc_gpuhash_batch_pinned, three
    streams), the caller's buffers used in place. The inputs are generated on
    the device and copied into pinned host tensors before any timing; the
    outputs land in pinned host memory and are checked against the compiled
    reference's digest. Beside it the same run's H2D ceiling (one large
    hipMemcpyAsync)."""
    import hashlib

    kd, od = t.synth_device(spec, first, n, device=dev)
    kb = int(od[-1].item())
    keys_h = pinned_copy(torch, kd)
    off_h = pinned_copy(torch, od)
    out_h = torch.empty(n, dtype=torch.int32).pin_memory()
    del kd, od
    torch.cuda.empty_cache()
    probe = h2d_probe(torch, keys_h, dev)
    h2d_bytes = kb + 8 * (n + 1)
    shape = spec.shape(kb)
    res = {"workload": f"{cfg}: {n} keys ({kb} key bytes) in pinned host memory -> {mode} -> hashes in pinned "
                       f"host memory", "h2d_bytes": h2d_bytes, "d2h_bytes": 4 * n,
           "h2d_probe_gbs": round(probe, 2),
           "chunk": {"keys": chunk[0], "bytes": chunk[1], "depth": chunk[2]}}
    with t.Pipe(torch.cuda.current_device(), *chunk) as p:
        try:
            p.hash(mode, keys_h, off_h, out_h, shape=shape)  # warm-up
            if dist_on:
                import torch.distributed as dist

                dist.barrier()
            best = None
            for _ in range(reps):
                t0 = time.perf_counter()
                p.hash(mode, keys_h, off_h, out_h, shape=shape)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            wall = max_over_ranks(torch, best, dist_on)
            got = hashlib.sha256(out_h.numpy().tobytes()).hexdigest()
            res.update({"ms": round(wall * 1e3, 2),
                        "value": round(sum_over_ranks(torch, float(n), dist_on) / wall / 1e6, 1), "unit": "Mkeys/s",
                        "h2d_gbs": round(h2d_bytes / best / 1e9, 2),
                        "frac_of_h2d_probe": round(h2d_bytes / best / 1e9 / probe, 4),
                        "parity": "ok" if digest_rank and got == digest_rank.get(mode) else
                                  ("unpinned" if not digest_rank else "MISMATCH")})
        except Exception as e:  # reported beside the headline, never instead of it
            res["error"] = repr(e)
    del keys_h, off_h, out_h
    return res


def c5_leg(seconds=0.4):
    """tools/nc_c5_replay: 64 x 128 pipelined GETs read into 16,336-byte mbufs
    with repair, one mbuf's keys per batch: the context path (submit_spans,
    depth 1/2/4, copy and zero-copy) and the batch ring (no HIP call per
    batch, depth 1/2/4/8), next to the per-key host hash of the same spans."""
    exe = os.path.join(HERE, "tools", "nc_c5_replay")
    if not os.path.exists(exe):
        return {"error": "tools/nc_c5_replay not built"}
    try:
        p = subprocess.run([exe, str(seconds)], capture_output=True, text=True, timeout=120)
    except Exception as e:
        return {"error": repr(e)}
    rows = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    if p.returncode != 0 or not rows:
        return {"error": f"rc {p.returncode}", "stderr": p.stderr[-400:]}
    host = [r for r in rows if r["point"] == "host_per_key"]
    gpu = [r for r in rows if r["point"] == "gpu"]
    return {"workload": "C5: 64 connections x 128 pipelined 'get <key>\\r\\n' (Zipf 8-64 B printable keys) read "
                        "into 16,336-byte mbufs with repair; one mbuf's keys per batch (nc_gpuhash_submit_spans "
                        "or the batch ring); host->device->host, fnv1a_64",
            "host_per_key": host[0] if host else None, "gpu": gpu,
            # the fastest ring point with >= 2 batches in flight and submit -> done <= 20 us
            "ring_best_depth_ge2_le20us": max((r for r in gpu if r["path"].startswith("ring") and r["depth"] >= 2
                                               and r["submit_to_done_us"] <= 20.0),
                                              key=lambda r: r["mkeys_s"], default=None),
            "mismatches": int(sum(r["mismatches"] for r in gpu))}


def redis_leg(t, torch, np, spec, dev, nreq=1 << 20, reps=10):
    """nc_gpuhash_redis_parse_device over nreq "*2 $3 get $<len> <key>" requests
    (wall time per parse, host syncs included: the counts size the launches)."""
    kh, oh = t.synth_host(spec, 0, nreq)
    kb = kh.tobytes()
    stream = b"".join(b"*2\r\n$3\r\nget\r\n$%d\r\n%s\r\n" % (int(oh[i + 1] - oh[i]), kb[int(oh[i]): int(oh[i + 1])])
                      for i in range(nreq))
    sd = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).to(dev)
    with t.RedisParser(max_bytes=len(stream) + 16, max_reqs=nreq + 1, max_keys=nreq + 1) as ps:
        for _ in range(2):
            ps.parse(sd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            keys, off, _, _, info = ps.parse(sd)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        if info["nkeys"] != nreq or info["consumed"] != len(stream):
            raise AssertionError(f"redis parse: {info}")
        o = off.cpu().numpy()
        if not np.array_equal(o, oh.astype(np.int64)):
            raise AssertionError("redis parse: key offsets differ from the generator's")
        if not np.array_equal(keys[: int(oh[-1])].cpu().numpy(), kh[: int(oh[-1])]):
            raise AssertionError("redis parse: key bytes differ from the generator's")
    return {"workload": f"{nreq} pipelined RESP GETs over the first C2 keys", "stream_bytes": len(stream),
            "ms_per_parse_wall": round(dt * 1e3, 4), "stream_gb_s": round(len(stream) / dt / 1e9, 2),
            "mreq_s": round(nreq / dt / 1e6, 1)}


if __name__ == "__main__":
    main()
