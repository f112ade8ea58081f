#!/bin/bash
# Kernel choice by key length: workgroup pipeline vs wave ring shapes, fnv1a_64 (and md5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-lsw}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u tools/sweep.py --modes ${2:-fnv1a_64} --configs ${3:-F8,F16,F24,C2,U8-64,C3,F48,F64,F128,F256} \
    --rounds 3 --iters 10 --variants ${4:-0:0:0,0:0:32,0:1:0,0:0:2176,0:0:896,0:0:3968,0:0:2432} > "$OUT/sweep.log" 2>&1
rc=$?; tail -n 2 "$OUT/sweep.log"; exit $rc
