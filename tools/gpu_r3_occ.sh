#!/bin/bash
# Round 3 DIAGNOSTIC: the grouped fnv1a_64 pipeline on C2 at three workgroups
# per CU (6400 B of unused dynamic LDS, variant bit 29) and at four with a
# 5 KiB smaller slab budget (bit 30), against the policy, A/B/C/A/B/C.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03occ
mkdir -p "$O"
timeout -k 10 400 python3 tools/ab.py --configs C2 --modes fnv1a_64 \
    --variants 0,775946240,1312817152,0:0,775946240:0,1312817152:0 --rounds 5 --iters 10 \
    > "$O/ab.jsonl" 2> "$O/ab.err" || { tail -20 "$O/ab.err"; exit 1; }
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    r=json.loads(l); print(r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r['check'])"
