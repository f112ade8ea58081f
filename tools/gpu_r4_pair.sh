#!/bin/bash
# md5 on long keys: one key per lane (nc_md5_lines_kernel) vs two
# (nc_md5_lines2_kernel, variant bit 27), parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_pair}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "direct_ragged or c4" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
timeout -k 10 300 python3 tools/ab.py --configs C4S --modes md5 --variants 4718592,138936320,13107200,147324928 --rounds 3 --iters 10 \
    > $O/md5_$rep.jsonl 2> $O/md5_$rep.err || { tail -20 $O/md5_$rep.err; exit 1; }
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/md5_*.jsonl')):
    for l in open(f):
        r=json.loads(l); print(f.split('/')[-1], r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r.get('hbm_frac'),r['check'])"
