#!/bin/bash
# Full-size race screen: every launch variant listed is compared key-by-key
# with variant 0 at several grid sizes (tools/diag_variant.py), after the GPU
# parity suite. Stops at the first failure.   usage: tools/gpu_screen.sh <tag> <variants...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -n 3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for c in C2 C3; do for v in "$@"; do for g in 1024 1536 2048; do
    echo "== $c $v $g" >> "$OUT/screen.log"
    timeout -k 5 90 python3 tools/diag_variant.py $c fnv1a_64 $v $g > "$OUT/one.log" 2>&1
    rc=$?; grep -v amdgpu.ids "$OUT/one.log" | head -12 >> "$OUT/screen.log"; [ $rc -eq 0 ] || exit $rc
done; done; done
grep -c "mismatches=0" "$OUT/screen.log"
