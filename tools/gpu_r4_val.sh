#!/bin/bash
# The crc pipeline A/B on C3 (direct vs wave ring, byte-serial or slicing-by-4,
# vs workgroup pipelines), then the round validation (smoke, GPU tests, bench +
# rocprof, PMC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04d}
timeout -k 10 300 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "wave_ring_ragged" > gpurun_out/${TAG}_ring_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_ring_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_ring_tests.log
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python3 tools/ab.py --configs C3 --modes crc32 --variants 0,896,128,2176,2944,32,262176 --rounds 3 --iters 10 \
    > $O/c3crc_pipes.jsonl 2> $O/c3crc_pipes.err || { tail -20 $O/c3crc_pipes.err; exit 1; }
python3 -c "
import json
for l in open('$O/c3crc_pipes.jsonl'):
    r=json.loads(l); print(r['config'],r['mode'],r['var'],r['ms_median'],r['ms_min'],r.get('hbm_frac'),r['check'])"
bash tools/gpu_validate_round.sh $TAG C2:md5 C3:md5 C4S:md5 C3:crc32 C4S:crc32 C2:fnv1a_64 || exit $?
