#!/bin/bash
# server_idx parity + A/B of the ketama pipelines, then PMC passes of the
# bench legs (tools/gpu_pmc_round.sh)
#   usage: tools/gpu_sidx_pmc.sh TAG PMC_TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dispatch.py tests/test_gpu_proto_ref.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/ab_sidx.py --configs C2 --modes fnv1a_64 --dists ketama --tags none,{} > $O/sidx.jsonl 2> $O/sidx.err || { tail $O/sidx.err; exit 1; }
cat $O/sidx.jsonl
bash tools/gpu_pmc_round.sh $2 C2:probe_read C2:probe_read_nt C2:fnv1a_64 C2:md5 C2:server_idx C3:crc32 C4S:md5
