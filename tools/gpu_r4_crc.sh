#!/bin/bash
# C3 / C4 shard crc A/B: slicing-by-4 (8 copies) vs the byte table (one copy per bank).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_crc}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k direct_ragged > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/ab.py --configs C3 --modes crc32,crc16,crc32a --variants 0,279445504 --rounds 3 --iters 10 \
    > $O/c3.jsonl 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
timeout -k 10 300 python3 tools/ab.py --configs C4S --modes crc32,crc16 --variants 0,283639808 --rounds 3 --iters 10 \
    > $O/c4.jsonl 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
timeout -k 10 300 python3 tools/ab.py --configs C4S --modes md5 --variants 4718592,524288,8912896,13107200 --rounds 3 --iters 10 \
    > $O/c4md5.jsonl 2> $O/c4md5.err || { tail -20 $O/c4md5.err; exit 1; }
python3 -c "
import json
for f in ('$O/c3.jsonl','$O/c4.jsonl','$O/c4md5.jsonl'):
    for l in open(f):
        r=json.loads(l); print(r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r.get('hbm_frac'),r['check'])"
