#!/bin/bash
# Round 3: md5 direct pipeline, offsets with the default cache policy
# (variant bit 29) against the policy, A/B/A/B in one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03md5off
mkdir -p "$O"
timeout -k 10 500 python3 tools/ab.py --configs C2,C3 --modes md5 --variants 0,537395200,0:0,537395200:0 --rounds 7 \
    --iters 10 > "$O/ab_md5.jsonl" 2> "$O/ab_md5.err" || { tail -20 "$O/ab_md5.err"; exit 1; }
timeout -k 10 300 python3 tools/ab.py --configs C3 --modes crc32 --variants 0,547880960,0:0,547880960:0 --rounds 5 \
    --iters 10 > "$O/ab_crc.jsonl" 2> "$O/ab_crc.err" || { tail -20 "$O/ab_crc.err"; exit 1; }
python3 -c "
import json
for f in ('ab_md5','ab_crc'):
    for l in open('$O/'+f+'.jsonl'):
        r=json.loads(l); print(r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r['check'])"
