#!/bin/bash
# server_idx parity (dispatch + reference fixtures) and the A/B of the ketama pipelines
#   usage: tools/gpu_sidx.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dispatch.py tests/test_gpu_proto_ref.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/ab_sidx.py --configs C2,C3 --modes fnv1a_64 --dists ketama,modula --tags none,{} > $O/sidx.jsonl 2> $O/sidx.err || { tail $O/sidx.err; exit 1; }
python3 -c "
import json
for l in open('$O/sidx.jsonl'):
    r=json.loads(l); print(r['config'], r['dist'], r['tag'], r['ms'], set(r['check'].values()))"
