"""bench.py's multi-rank code on the one-GPU box: bench.py starts itself as
2 ranks (`python3 bench.py --gpus 2`, no launcher: spawn_ranks), and
`torch.distributed.run` starts it as 2 ranks (the driver's form) (``--backend gloo --same-device``: both ranks on
cuda:0, the scatter staged through host memory) at reduced sizes. Every
N > 1 branch of bench.py runs — the process group, rank 0's generation and
the root scatter of C2/C3/C4 (resident()), the max/sum over ranks, the
all_gather of per-rank parity, c4_ingest on every rank — so only the RCCL
transport itself is left for the driver's 8-GPU run. Every rank's outputs are
checked against the compiled reference's per-rank digests at these sizes
(tests/golden/shard_digests.json "small", tests/golden/make_shard_digests.py
--small): parity must read "ok" for both ranks, never "unpinned"."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2
NKEYS = 1 << 16     # C2 / C3 keys per rank (a "small" digest size)
C4_NKEYS = 1 << 12  # C4 keys per rank

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(420)]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module", params=["self", "torchrun"])
def run(request, tmp_path_factory):
    import torch  # noqa: F401  (pages the image in before the children's own imports)

    detail = str(tmp_path_factory.mktemp("bench") / "detail.json")
    launcher = [] if request.param == "self" else [
        "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={WORLD}",
        "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
    cmd = [sys.executable, *launcher,
           os.path.join(HERE, "bench.py"), "--gpus", str(WORLD), "--steps", "3", "--warmup", "1",
           "--nkeys", str(NKEYS), "--c4-nkeys", str(C4_NKEYS), "--backend", "gloo", "--same-device",
           "--detail-out", detail]
    # 64 KiB scatter messages: the C4 shard's 1 MiB goes in 16 rounds, as
    # an 8 GiB shard does in 1 GiB pieces on the 8-GPU node
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"),
               NC_SCATTER_MAX_MSG_BYTES=str(1 << 16))
    p = subprocess.run(cmd, cwd=HERE, capture_output=True, text=True, timeout=400, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    rows = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(rows) == 1, p.stdout[-2000:]  # rank 0 alone prints
    return json.loads(rows[0]), json.load(open(detail))


@pytest.fixture(scope="module")
def line(run):
    return run[0]


def test_driver_fields_at_n2(line):
    assert line["n_gpus"] == WORLD and line["scaling"] == "weak"
    assert line["config"]["parallelism"] == f"shard{WORLD}"
    # value = keys of ALL ranks per second of the max-over-ranks wall time
    assert abs(line["value"] - WORLD * NKEYS / (line["ms_per_step"] * 1e-3) / 1e6) <= 0.02 * line["value"] + 0.2
    assert line["kernel_ms_max"] >= line["kernel_ms_rank0"] > 0
    assert "cpu_baseline" not in line and "c5_e2e" not in line and "e2e_c2" not in line  # rank 0 at N = 1 only


def test_every_rank_parity_ok(run):
    line, full = run
    assert line["parity"] == {"all": "ok", "legs": 8, "ranks": WORLD, "bad": []}, line["parity"]
    par = full["parity"]
    assert par["all"] == "ok", par
    want = {"C2/fnv1a_64", "C2/md5", "C3/fnv1a_64", "C3/crc32", "C3/md5", "C4/md5", "C4/crc32", "C4/fnv1a_64"}
    assert set(par["per_rank"]) == want
    for k, st in par["per_rank"].items():
        assert st == ["ok"] * WORLD, (k, st)


def test_scatter_reported(line):
    for sc in (line["scatter"], line["c3_scatter"], line["c4_shard"]["scatter"]):
        assert sc["ms"] > 0 and "gloo" in sc["how"]
    # rank 0 sends every shard but its own; the report is rank 0's egress:
    # the whole batch (keys + offsets) it generated
    assert line["scatter"]["root_egress_bytes"] > WORLD * NKEYS * 8


def test_legs_at_n2(line):
    for k in ("md5", "server_idx_ketama", "c3_fnv1a_64", "c3_crc32", "c3_md5"):
        assert "error" not in line[k], line[k]
        assert line[k]["kernel_ms"] > 0
    for mode in ("md5", "crc32", "fnv1a_64"):
        assert line["c4_shard"][mode]["kernel_ms"] > 0
    ing = line["c4_ingest"]
    assert "error" not in ing, ing
    assert ing["parity"] == "ok", ing  # every rank's own C4 shard, pulled H2D, against its digest
