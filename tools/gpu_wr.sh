#!/bin/bash
# Wave-ring kernel check: parity tests for the new variants, then an
# in-process A/B sweep against the workgroup pipelines.  usage: tools/gpu_wr.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-wr}
mkdir -p "$OUT"
step() {  # name limit cmd...
    local name=$1 limit=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 4 "$OUT/$name.log"
    return $rc
}
step parity 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 \
    -k "wavering or ragged or long_keys or offsets or edge or variants_agree or kats" || exit $?
step sweep 600 python3 -u tools/sweep.py --modes fnv1a_64,md5 --configs C2,C3 --rounds 3 --iters 20 \
    --variants 0:0:0,0:0:32,0:0:128,0:0:384,0:0:640,0:0:896 || exit $?
echo done
