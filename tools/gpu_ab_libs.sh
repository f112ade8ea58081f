#!/bin/bash
# Same-box A/B of library builds (tools/ab.py --lib), interleaved A B A B.
#   usage: tools/gpu_ab_libs.sh TAG CONFIGS MODES VARIANTS LIB_A LIB_B [REPS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p "$O"
for i in $(seq 1 "${7:-2}"); do
    for lib in "$5" "$6"; do
        tag=$(basename "$lib" .so)
        timeout -k 10 300 python3 tools/ab.py --configs "$2" --modes "$3" --variants "$4" --rounds 3 --iters 10 \
            --lib "$lib" > "$O/ab_${tag}_$i.jsonl" 2> "$O/ab_${tag}_$i.err" || { tail -20 "$O/ab_${tag}_$i.err"; exit 1; }
        python3 -c "
import json
for l in open('$O/ab_${tag}_$i.jsonl'):
    r=json.loads(l); print('$tag', r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r['check'])"
    done
done
