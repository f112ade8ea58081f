#!/bin/bash
# GPU steps for one gpurun call, each under its own time limit, stopping at the first failure.
#   tools/gpu_step.sh TAG "pytest args" [bench] [sweep-args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
if [ -n "${2:-}" ]; then
    timeout -k 10 600 python3 -u -m pytest $2 -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
    tail -2 "$OUT/pytest.log"
fi
if [ "${3:-}" = "bench" ]; then
    timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 3 --no-cpu > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
    grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
fi
if [ -n "${4:-}" ]; then
    shift 3
    bash tools/gpu_lensweep.sh "$(basename "$OUT")/sw" "$@" || exit 1
fi
echo done
