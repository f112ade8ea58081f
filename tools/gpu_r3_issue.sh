#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 500 python3 tools/ab.py --configs C2 --modes fnv1a_64,murmur,fnv1_32 --variants 239075328,507510784,239075328,507510784 --rounds 5 --iters 10 > $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes one_at_a_time --variants 234881024,503316480,234881024 --rounds 5 --iters 10 >> $O/ab.jsonl 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    r=json.loads(l); print(r['config'], r['mode'], r['var'], r['ms_median'], r['ms_min'], r['check'])"
