#!/bin/bash
# Experiment sweep (fnv1a_64): wave-ring shapes x {4 waves/WG, pair, pinned deep reads}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sx}
mkdir -p "$OUT"
V=0:0:0,0:0:32
for b in 3968 2176 2432; do for f in 0 16384 4096 20480; do V="$V,0:0:$((b + f))"; done; done
timeout -k 10 900 python3 -u tools/sweep.py --modes ${3:-fnv1a_64} --configs ${2:-C2,C3} --rounds 3 --iters 20 \
    --variants "$V" > "$OUT/sweep.log" 2>&1
rc=$?; tail -n 2 "$OUT/sweep.log"; exit $rc
