#!/bin/bash
# round 6: the N = 4 bench path at FULL size on one GPU (gloo, every rank on
# cuda:0, launched by bench.py itself): every rank's outputs against the
# reference's N = 4 per-rank digests. Times are meaningless (four ranks share
# one GPU); the point is the data path at the driver's sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06n}; mkdir -p $O
timeout -k 20 1000 python3 bench.py --gpus 4 --backend gloo --same-device --steps 3 --warmup 1 --no-cpu --verbose \
    --detail-out $O/detail.json > $O/bench_n4.log 2>&1
rc=$?
tail -c 3000 $O/bench_n4.log
exit $rc
