#!/bin/bash
# The batch ring on the GPU box: its tests, then the C5 replay (every path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_ring}; mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 100 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_ring.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -8 $O/tests.log
timeout -k 10 120 tools/nc_c5_replay 0.4 > $O/c5.jsonl 2> $O/c5.err || { cat $O/c5.err; exit 1; }
cat $O/c5.jsonl
