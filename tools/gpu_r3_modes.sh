#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 500 python3 tools/ab.py --configs C2 --modes all --variants 0 --rounds 3 --iters 10 > $O/c2_all.jsonl 2> $O/c2_all.err || { tail $O/c2_all.err; exit 1; }
bash tools/gpu_modes.sh r03m_c3 || exit $?
echo modes done
