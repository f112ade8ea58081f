#!/bin/bash
# C4 shard crcs on the line image: 16 waves x 8 table copies (policy) vs 12 waves x 16 copies (bit 28).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_r16}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "direct_ragged" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
timeout -k 10 300 python3 tools/ab.py --configs C4S --modes crc32,crc16 --variants 15204352,283639808 --rounds 3 --iters 10 \
    > $O/crc_$rep.jsonl 2> $O/crc_$rep.err || { tail -20 $O/crc_$rep.err; exit 1; }
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/crc_*.jsonl')):
    for l in open(f):
        r=json.loads(l); print(f.split('/')[-1], r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r.get('hbm_frac'),r['check'])"
