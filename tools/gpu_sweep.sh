#!/bin/bash
# GPU parity tests, then a variant sweep; stops at the first failure.
#   usage: tools/gpu_sweep.sh <tag> <sweep args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/sweep.py "$@" > "$OUT/sweep.log" 2>&1
rc=$?; echo "sweep rc=$rc"
[ $rc -eq 0 ] || { tail -5 "$OUT/sweep.log"; exit $rc; }
