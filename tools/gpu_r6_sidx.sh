#!/bin/bash
# round 6: the packed ketama continuum's 1024-bucket index — parity, then a
# same-process A/B against the u16[512] index and the plain hash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06g}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dispatch.py tests/test_gpu_proto_ref.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --pipes policy,grouped_idx512,plain_hash \
    --rounds 5 > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
