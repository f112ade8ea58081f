#!/bin/bash
# C4 shard: the lines kernels at fewer resident waves per CU (A/B bits 27-28).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_occ}; mkdir -p $O
for rep in 1 2; do
timeout -k 10 300 python3 tools/ab.py --configs C4S --modes md5 --variants 4718592,138936320,273154048 --rounds 3 --iters 10 \
    > $O/md5_$rep.jsonl 2> $O/md5_$rep.err || { tail -20 $O/md5_$rep.err; exit 1; }
timeout -k 10 300 python3 tools/ab.py --configs C4S --modes fnv1a_64,crc32 --variants 15204352,149422080 --rounds 3 --iters 10 \
    > $O/bytes_$rep.jsonl 2> $O/bytes_$rep.err || { tail -20 $O/bytes_$rep.err; exit 1; }
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/*.jsonl')):
    for l in open(f):
        r=json.loads(l); print(f.split('/')[-1], r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r.get('hbm_frac'),r['check'])"
