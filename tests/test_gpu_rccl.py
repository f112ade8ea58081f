"""RCCL's point-to-point path on one GPU (the 8-GPU scaling run's transport,
exercised before the driver's run): tests/rccl_selfcheck.py in a fresh
process — init_process_group("nccl"), device-tensor batch_isend_irecv of
shard._pieces()-cut buffers (self send/receive, 4 KiB pieces), scatter_shards
at world size 1, and bench.py's CUDA-tensor all_reduce / barrier /
all_gather_object. Reference analogue: the per-key shard choice of
src/nc_server.c:647-700, which the scatter feeds."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(240)]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_p2p_pieces_and_collectives():
    env = dict(os.environ, NC_SCATTER_MAX_MSG_BYTES=str(1 << 12), MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, os.path.join(HERE, "tests", "rccl_selfcheck.py"), str(_free_port())],
                       cwd=HERE, capture_output=True, text=True, timeout=200, env=env)
    rows = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and rows, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    r = json.loads(rows[-1])
    assert r["backend"] == "nccl" and r["ok"], r
    assert r["pieces"] >= 4 and r["piece_bytes"] == 1 << 12
