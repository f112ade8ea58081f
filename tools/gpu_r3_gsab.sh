#!/bin/bash
# A/B of the grouped pipeline's DMA addressing (bit 29) and sort scan (bit 30), same process
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 500 python3 tools/ab.py --configs C2 --modes fnv1a_64,murmur,fnv1_32 --variants 239075328,775946240,1312817152,1849688064,239075328 --rounds 5 --iters 10 > $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes one_at_a_time --variants 234881024,1845493760,234881024 --rounds 5 --iters 10 >> $O/ab.jsonl 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    r=json.loads(l); print(r['config'], r['mode'], r['var'], r['ms_median'], r['ms_min'], r['check'])"
