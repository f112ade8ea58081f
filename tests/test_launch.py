"""bench.py's own launcher (spawn_ranks) on CPU: `python3 bench.py --gpus N`
with no torch.distributed.run around it starts N rank processes with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set, and they meet over gloo
(--launch-check: the rendezvous only, no device work). A --gpus that
disagrees with the launcher's WORLD_SIZE, or asks for more GPUs than are
visible, exits non-zero before any rank runs. The GPU form of the same
launch, with every leg and per-rank parity, is tests/test_gpu_bench_dist.py."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(HERE, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], cwd=HERE, capture_output=True, text=True,
                          timeout=timeout, env=env)


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_starts_n_ranks(n):
    p = _run(["--gpus", str(n), "--backend", "gloo", "--same-device", "--launch-check"])
    assert p.returncode == 0, p.stderr[-3000:]
    rows = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(rows) == 1, p.stdout  # rank 0 alone prints
    r = json.loads(rows[0])
    assert r["n_gpus"] == n and r["gpus_arg"] == n
    assert [v["rank"] for v in r["ranks"]] == list(range(n))
    assert all(v["world"] == n and v["local_rank"] == 0 for v in r["ranks"])  # --same-device
    assert len({v["pid"] for v in r["ranks"]}) == n  # one fresh process per rank


def test_one_gpu_runs_in_process():
    p = _run(["--gpus", "1", "--same-device", "--launch-check"])
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["n_gpus"] == 1 and r["ranks"][0]["pid"] > 0


def test_launcher_world_mismatch_fails():
    p = _run(["--gpus", "4", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_more_gpus_than_visible_fails():
    import torch

    n = torch.cuda.device_count() + 1
    p = _run(["--gpus", str(n), "--launch-check"])
    assert p.returncode != 0 and "visible" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_failing_rank_fails_the_job():
    # rank 1 dies before the rendezvous (a test hook in launch_check): rank 0
    # is left waiting for it, so the parent must stop rank 0 after the grace
    # period and return rank 1's failure, not hang or report success
    p = _run(["--gpus", "2", "--backend", "gloo", "--same-device", "--launch-check"],
             {"NC_BENCH_FAIL_RANK": "1", "NC_BENCH_GRACE_S": "2"}, timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
