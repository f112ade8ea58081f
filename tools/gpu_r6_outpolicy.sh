#!/bin/bash
# The hash outputs' store policy (nc_out_policy.h) A/B on one box: the
# default build (nt) against abl/out_plain.so and abl/out_sc1.so
# (tools/build_ablib.sh NAME "-DNC_OUT_POLICY=1|2"), alternated twice, each
# on the bench's configs and modes (tools/ab.py: outputs checked against the
# first variant and sampled keys against the host symbols).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06zi_outpolicy}; mkdir -p $O
for r in 1 2; do
  for lib in default out_plain out_sc1; do
    L=""; [ $lib != default ] && L="--lib abl/$lib.so"
    timeout -k 10 240 python3 tools/ab.py --configs ${CONFIGS:-C2,C3,C4S} --modes ${MODES:-fnv1a_64,md5,crc32} \
        --rounds 3 --iters 10 --spinup 1.5 $L > $O/${lib}_$r.jsonl 2> $O/${lib}_$r.err || { tail -5 $O/${lib}_$r.err; exit 1; }
    echo "$lib $r $(python3 -c "
import json,sys
for l in open('$O/${lib}_$r.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('config'), d.get('mode'), d.get('ms_median'), d.get('check', d.get('ok')), end='; ')
")"
  done
done
