#!/bin/bash
# GPU-box check: smoke, GPU parity tests, one bench line, optional rocprof.
# Every GPU step has its own time limit; any non-zero exit ends the script
# before the next GPU step.
#   usage: tools/gpu_check.sh [tag] [--prof]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"

step() {  # name limit cmd...
    local name=$1 limit=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 5 "$OUT/$name.log"
    return $rc
}

step smoke 400 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
# any failure stops the script: a failing GPU test can hide a device fault
step pytest_gpu 900 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider || exit $?
step bench 600 python3 bench.py --steps 20 --warmup 3 || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
if [ "${2:-}" = "--prof" ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu || exit $?
fi
echo "done"
