#!/bin/bash
# Round 3: cache-policy A/Bs (variant bits 29-30): the direct pipelines' offsets
# with the default policy; the grouped fnv1a_64 with default-policy stores /
# DMAs; and the read / read-nt / read+write mix probes side by side.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03knt
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/probe_mix.py > "$O/probes.jsonl" 2> "$O/probes.err" || { tail -20 "$O/probes.err"; exit 1; }
cat "$O/probes.jsonl"
timeout -k 10 400 python3 tools/ab.py --configs C3 --modes crc32,crc16 --variants 0,547880960 --rounds 5 --iters 10 \
    > "$O/ab_crc.jsonl" 2> "$O/ab_crc.err" || { tail -20 "$O/ab_crc.err"; exit 1; }
timeout -k 10 400 python3 tools/ab.py --configs C2,C3 --modes md5 --variants 0,537395200 --rounds 5 --iters 10 \
    > "$O/ab_md5.jsonl" 2> "$O/ab_md5.err" || { tail -20 "$O/ab_md5.err"; exit 1; }
timeout -k 10 400 python3 tools/ab.py --configs C2 --modes fnv1a_64 --variants 0,775946240,1312817152,1849688064 \
    --rounds 5 --iters 10 > "$O/ab_gs.jsonl" 2> "$O/ab_gs.err" || { tail -20 "$O/ab_gs.err"; exit 1; }
python3 -c "
import json
for f in ('ab_crc','ab_md5','ab_gs'):
    for l in open('$O/'+f+'.jsonl'):
        r=json.loads(l); print(r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r['check'])"
