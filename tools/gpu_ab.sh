#!/bin/bash
# GPU-box A/B of launch variants (tools/ab.py), optionally after the GPU tests.
#   usage: tools/gpu_ab.sh TAG CONFIGS MODES VARIANTS [--tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p "$O"
if [ "${5:-}" = "--tests" ]; then
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
        --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
    tail -2 "$O/pytest_gpu.log"
fi
timeout -k 10 600 python3 tools/ab.py --configs "$2" --modes "$3" --variants "$4" --rounds 3 --iters 10 \
    > "$O/ab.jsonl" 2> "$O/ab.err" || { tail -20 "$O/ab.err"; exit 1; }
python3 -c "
import json,sys
for l in open('$O/ab.jsonl'):
    r=json.loads(l); print(r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r['check'])"
