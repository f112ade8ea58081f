#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "md5 or digest or golden or kat or corpus or policy" > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 400 python3 tools/ab.py --configs C2 --modes md5 --variants 0,524288,18874368,19922944,25165824,26214400 --rounds 3 --iters 10 > $O/ab_md5.jsonl 2> $O/ab_md5.err || { tail $O/ab_md5.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab_md5.jsonl'):
    r=json.loads(l); print(r['config'], r['mode'], r['var'], r['ms_median'], r['ms_min'], r['check'])"
bash tools/gpu_sidx.sh r03z_sidx
