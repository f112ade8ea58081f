#!/bin/bash
# Ring-shape sweep of the wave-ring kernel (variant bits 8-10) against the
# workgroup pipelines, one process.     usage: tools/gpu_sweep_wr.sh <tag> [modes]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-swr}
mkdir -p "$OUT"
V=0:0:0,0:0:32
for k in 0 1 2 3 4 5 6 7; do V="$V,0:0:$((128 + k * 256))"; done
V="$V,0:0:136,0:0:$((136 + 768)),0:0:$((136 + 1792)),0:0:8"
timeout -k 10 900 python3 -u tools/sweep.py --modes "${2:-fnv1a_64}" --configs C2,C3 --rounds 3 --iters 20 \
    --variants "$V" > "$OUT/sweep.log" 2>&1
rc=$?; tail -n 3 "$OUT/sweep.log"; exit $rc
