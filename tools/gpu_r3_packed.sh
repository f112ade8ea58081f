#!/bin/bash
# Round 3: the packed LDS ketama continuum — dispatch parity tests, then the
# fused server_idx on C2 against the 5-byte continuum, in one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03packed
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dispatch.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 400 python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --tags none,{} \
    --pipes policy,grouped,grouped8,grouped_5b --rounds 5 > "$O/ab_sidx.jsonl" 2> "$O/ab_sidx.err" \
    || { tail -20 "$O/ab_sidx.err"; exit 1; }
cat "$O/ab_sidx.jsonl"
