#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dispatch.py tests/test_gpu_proto_ref.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
S="python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64,md5 --dists ketama --tags none,{} --pipes policy,grouped3,workgroup --rounds 5"
timeout -k 10 200 $S > $O/sidx_new1.jsonl 2>$O/sidx.err && timeout -k 10 200 $S --lib tools/ablib/libnc_gpuhash_sidx_bkt256.so > $O/sidx_old.jsonl 2>>$O/sidx.err && timeout -k 10 200 $S > $O/sidx_new2.jsonl 2>>$O/sidx.err || { tail $O/sidx.err; exit 1; }
cat $O/sidx_new1.jsonl $O/sidx_old.jsonl $O/sidx_new2.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['lib'], r['config'], r['mode'], r['tag'], r['ms'], set(r['check'].values()))"
timeout -k 10 300 python3 tools/ab.py --configs C2 --modes fnv1a_64 --variants 239075328,239075328:2048,239075328:2560,239075328:3584,239075328:4096,239075328 --rounds 5 --iters 10 > $O/grid.jsonl 2> $O/grid.err || { tail $O/grid.err; exit 1; }
python3 -c "
import json
for l in open('$O/grid.jsonl'):
    r=json.loads(l); print(r['mode'], r['var'], r['ms_median'], r['ms_min'], r['check'])"
